#!/bin/bash
# round 5: the streamed grouped stage's independent launches (k_gc groups, tap-mode branches) over the
# caller's stream + two side streams (CNF_GC_CONC=0: one stream) -- parity, then cfg4 / cfg5 A/B
set -o pipefail
out=gpurun_out/r5conc; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "cfg4 or cfg5 or cfg2" > $out/parity.log 2>&1; rc=$?; tail -3 $out/parity.log; [ $rc = 0 ] || exit 1
for cb in "cfg4 32" "cfg4 128" "cfg5 64" "cfg2 64"; do
  set -- $cb
  for m in 1 0 1 0; do
    timeout -k 10 300 env CNF_GC_CONC=$m python3 bench.py --config $1 --batch $2 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --inflight 1 > $out/$1_$2_$m.json 2> $out/$1_$2_$m.err || { tail $out/$1_$2_$m.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/$1_$2_$m.json')); print('$1 B=$2 conc=$m', d['value'], d['step_ms_median'])"
  done
done
