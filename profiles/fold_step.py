#!/usr/bin/env python3
"""Fold a rocprofv3 kernel trace of bench.py --mode train: the last full step (between k_adam
launches), its busy time, and per backward coupling layer (split at k_coup_bw) the span, launch count
and the kernels by total time."""
import csv
import glob
import os
import sys


def main(d):
    rows = []
    for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ad = [i for i, r in enumerate(rows) if 'k_adam' in r['Kernel_Name']]
    st = rows[ad[-2] + 1:ad[-1] + 1]
    t0, t1 = int(st[0]['Start_Timestamp']), int(st[-1]['End_Timestamp'])
    iv = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in st)
    busy, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f'step: {len(st)} launches, span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us')
    nm = lambda r: r['Kernel_Name'].split('(')[0].replace('void ', '').replace('cnf::', '')
    fw = next(i for i, r in enumerate(st) if 'k_nll_grad' in r['Kernel_Name'])
    print(f'forward_train: {fw} launches, {(int(st[fw]["Start_Timestamp"]) - t0) / 1e3:.1f} us')
    cb = [i for i, r in enumerate(st) if 'k_coup_bw' in r['Kernel_Name']]
    # a layer's launches: from after the previous layer's last scatter to its own last scatter
    ends = [i for i, r in enumerate(st) if 'k_scatter_add_u1c' in r['Kernel_Name']][1::2]
    start = fw
    for j, e in enumerate(ends):
        seg = st[start:e + 1]
        a, b = int(seg[0]['Start_Timestamp']), max(int(r['End_Timestamp']) for r in seg)
        tot = {}
        for r in seg:
            tot[nm(r)] = tot.get(nm(r), 0) + (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        top = ', '.join(f'{k} {v:.0f}' for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:4])
        print(f'bwd #{j:2d}: {len(seg):3d} launches, span {(b - a) / 1e3:7.1f} us | {top}')
        start = e + 1


if __name__ == '__main__':
    main(sys.argv[1])
