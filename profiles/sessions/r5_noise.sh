#!/bin/bash
# round 5: the fused input-noise forward -- its GPU tests, then the bench with and without --noise 0.98
set -o pipefail
out=gpurun_out/r5noise; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_transforms.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/plain_$rep.json 2> $out/plain_$rep.err || { tail $out/plain_$rep.err; exit 1; }
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --noise 0.98 $([ $rep = 2 ] || echo --no-cpu-baseline) > $out/noise_$rep.json 2> $out/noise_$rep.err || { tail $out/noise_$rep.err; exit 1; }
  python3 -c "
import json
for k in ('plain_$rep', 'noise_$rep'):
    d = json.load(open('$out/' + k + '.json'))
    print(k, d['value'], d['step_ms_median'], d['config'].get('input_noise'), d.get('bits_per_dim'), d.get('bits_per_dim_ref'))"
done
