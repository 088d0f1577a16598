#!/bin/bash
# round 5: nt (non-temporal) policy on conv_b's read-once t2 loads (A/B), and the cfg4 B=32 per-kernel breakdown
set -o pipefail
bash profiles/sessions/r5_ab.sh r5nt cfg2 "base nt2 nt3" --inflight 1 || exit 1
timeout -k 10 300 python3 bench.py --config cfg4 --batch 32 --steps 10 --warmup 3 --no-cpu-baseline --inflight 2 > gpurun_out/r5nt/cfg4_b32.json 2> gpurun_out/r5nt/cfg4_b32.err || { tail gpurun_out/r5nt/cfg4_b32.err; exit 1; }
python3 -c "
import json
d = json.load(open('gpurun_out/r5nt/cfg4_b32.json'))
print('cfg4 B=32', d['value'], d['step_ms_median'], 'serving', d['serving']['value'] if d.get('serving') else None)
for k, v in sorted(d['roofline']['per_role'].items(), key=lambda kv: -kv[1]['ms_per_step']):
    print(f'  {k:28s} {v[\"ms_per_step\"]:.4f} ms/step  {v[\"launches\"]:3d} x {v[\"avg_launch_us\"]:.2f} us')"
grep "^#  " gpurun_out/r5nt/cfg4_b32.err | head -70 > gpurun_out/r5nt/cfg4_b32_launches.txt
