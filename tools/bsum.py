"""Summarise a bench.py JSON line: value, step, per-kernel times."""
import json
import sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d['roofline']
    print(f, d['value'], 'img/s', d['ms_per_step'], 'ms', 'median', d.get('step_ms_median'), 'dom', r['kernel'], r['frac'])
    for k, v in r['per_kernel'].items():
        print(f'   {k:12s} {v["ms_per_step"]:.4f} ms/step  {v["launches"]:3d} x {v["avg_launch_us"]:.2f} us  frac {v["frac"]}')
    for k, v in r.get('per_role', {}).items():
        print(f'      {k:28s} {v["ms_per_step"]:.4f} ms/step  {v["launches"]:3d} x {v["avg_launch_us"]:.2f} us')
