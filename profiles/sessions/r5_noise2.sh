#!/bin/bash
# round 5: fused logit + noise input preparation -- GPU tests, bench --noise 0.98 --logit 0.01, training bench
set -o pipefail
out=gpurun_out/r5noise2; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_transforms.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --noise 0.98 --logit 0.01 > $out/noise.json 2> $out/noise.err || { tail $out/noise.err; exit 1; }
python3 -c "
import json
d = json.load(open('$out/noise.json'))
print(d['value'], d['step_ms_median'], d['config'].get('input_noise'), d.get('bits_per_dim'), d.get('bits_per_dim_ref'))"
timeout -k 10 300 python3 bench.py --mode train --steps 10 --warmup 3 > $out/train.json 2> $out/train.err || { tail $out/train.err; exit 1; }
cat $out/train.json
