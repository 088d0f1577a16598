#!/bin/bash
# round 5: streamed conv_out + coupling law in one launch (k_out_law) against the tap GEMM + k_coupling
# pair (CNF_OUT_LAW=0), cfg2 / cfg3 / ref_default forward, then the parity and training suites
set -o pipefail
out=gpurun_out/r5olaw; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/parity.log 2>&1; rc=$?; tail -3 $out/parity.log; [ $rc = 0 ] || exit 1
for cb in "cfg2 64" "cfg3 64" "ref_default 32"; do
  set -- $cb
  for m in 1 0 1 0; do
    export CNF_OUT_LAW=$m
    timeout -k 10 300 python3 bench.py --config $1 --batch $2 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --inflight 1 > $out/$1_$2_$m.json 2> $out/$1_$2_$m.err || { tail $out/$1_$2_$m.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/$1_$2_$m.json')); print('$1 B=$2 out_law=$m', d['value'], d['step_ms_median'])"
  done
done
unset CNF_OUT_LAW
timeout -k 10 900 python -u -m pytest tests/test_train.py tests/test_transforms.py tests/test_capi.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; tail -3 $out/tests.log
