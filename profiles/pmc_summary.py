#!/usr/bin/env python3
"""Fold the rocprofv3 passes of profiles/collect.sh into profiles/<tag>_summary.json and copy the
kernel-trace stats CSV to profiles/<tag>_kernel_stats.csv.

HBM traffic per launch follows MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
(KiB, from TCC_EA0 requests) come from separate passes; on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced streaming reads, so traffic = 2 * FETCH_SIZE + WRITE_SIZE (bytes). The
Infinity Cache is counted, not excluded."""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    """'void k_conv1<2, true, 3>(ConvArgs)' -> 'k_conv1<2, true, 3>'"""
    name = re.sub(r'^void\s+', '', name)
    return re.sub(r'\(.*$', '', name).strip()


def counters(d):
    f = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not f:
        return {}
    per = defaultdict(lambda: defaultdict(list))
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            per[short(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} | {'dispatches': max(len(v) for v in cs.values())}
            for k, cs in per.items()}


def main(out, tag):
    res = {'tag': tag, 'kernels': {}}
    stats = glob.glob(os.path.join(out, 'stats', '**', '*kernel_stats.csv'), recursive=True)
    if stats:
        dst = os.path.join(ROOT, 'profiles', f'{tag}_kernel_stats.csv')
        shutil.copy(stats[0], dst)
        with open(stats[0]) as fh:
            for r in csv.DictReader(fh):
                k = short(r['Name'])
                res['kernels'].setdefault(k, {})['trace'] = {
                    'calls': int(r['Calls']), 'total_ns': float(r['TotalDurationNs']),
                    'avg_ns': float(r['AverageNs']), 'pct': float(r['Percentage'])}
    fetch, write, sq = (counters(os.path.join(out, p)) for p in ('fetch', 'write', 'sq'))
    for k in set(fetch) | set(write) | set(sq):
        e = res['kernels'].setdefault(k, {})
        if k in fetch and k in write:
            fb = fetch[k]['FETCH_SIZE'] * 1024.0
            wb = write[k]['WRITE_SIZE'] * 1024.0
            e['hbm'] = {'fetch_size_bytes': fb, 'write_size_bytes': wb, 'traffic_bytes': 2.0 * fb + wb,
                        'dispatches': min(fetch[k]['dispatches'], write[k]['dispatches'])}
        if k in sq:
            s = sq[k]
            e['sq'] = s
            if s.get('SQ_INSTS_MFMA'):
                e['sq']['valu_per_mfma'] = s.get('SQ_INSTS_VALU', 0.0) / s['SQ_INSTS_MFMA']
            if s.get('SQ_WAVE_CYCLES'):
                e['sq']['active_frac'] = s.get('SQ_ACTIVE_INST_ANY', 0.0) / s['SQ_WAVE_CYCLES']
                e['sq']['wait_frac'] = s.get('SQ_WAIT_ANY', 0.0) / s['SQ_WAVE_CYCLES']
    # per kernel symbol (template instantiations summed): the granularity of bench.py's roofline
    sym = {}
    for k, e in res['kernels'].items():
        name = re.sub(r'<.*$', '', k.split('::')[-1])
        d = sym.setdefault(name, {'calls': 0, 'total_ns': 0.0, 'hbm_bytes': 0.0, 'hbm_dispatches': 0})
        t = e.get('trace')
        if t:
            d['calls'] += t['calls']
            d['total_ns'] += t['total_ns']
        h = e.get('hbm')
        if h:
            d['hbm_bytes'] += h['traffic_bytes'] * h['dispatches']
            d['hbm_dispatches'] += h['dispatches']
    for d in sym.values():
        d['avg_ns'] = d['total_ns'] / d['calls'] if d['calls'] else None
        d['traffic_bytes_per_launch'] = d['hbm_bytes'] / d['hbm_dispatches'] if d['hbm_dispatches'] else None
    res['symbols'] = sym
    dst = os.path.join(ROOT, 'profiles', f'{tag}_summary.json')
    with open(dst, 'w') as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    for k, e in sorted(res['kernels'].items(), key=lambda kv: -kv[1].get('trace', {}).get('total_ns', 0)):
        t = e.get('trace', {})
        h = e.get('hbm', {})
        print(f"{k[:48]:48s} calls {t.get('calls', 0):5d} avg {t.get('avg_ns', 0) / 1e3:8.2f} us "
              f"traffic/launch {h.get('traffic_bytes', 0) / 1e6:8.2f} MB  "
              f"valu/mfma {e.get('sq', {}).get('valu_per_mfma', 0):6.2f}")
    print('wrote', dst)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else 'r01')
