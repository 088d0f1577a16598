#!/bin/bash
# round 5: LN partial slots folded by the consumers up to 256 per image (no k_ln_merge on the 64x64
# layers) -- cfg4 B=32 / B=128 and cfg5 B=64 against a merge above 256 slots (CNF_LN_MERGE=256), then parity
set -o pipefail
out=gpurun_out/r5lnm; mkdir -p $out
for cb in "cfg4 32" "cfg4 128" "cfg5 64" "cfg2 64"; do
  set -- $cb
  for m in default 256; do
    if [ $m = default ]; then unset CNF_LN_MERGE; else export CNF_LN_MERGE=$m; fi
    timeout -k 10 300 python3 bench.py --config $1 --batch $2 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --inflight 1 > $out/$1_$2_$m.json 2> $out/$1_$2_$m.err || { tail $out/$1_$2_$m.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/$1_$2_$m.json')); print('$1 B=$2 merge=$m', d['value'], d['step_ms_median'])"
  done
done
unset CNF_LN_MERGE
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_train.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; tail -3 $out/tests.log
