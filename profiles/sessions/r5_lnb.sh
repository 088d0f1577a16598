#!/bin/bash
# round 5: k_lnb_apply with 8-image load batches issued before its sums preamble -- gradient tests,
# train step (thin kernels on / off), and the step's kernel stats
set -o pipefail
root=$PWD; out=$root/gpurun_out/r5lnb; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_train.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit 1
for m in 1 0 1 0; do
  timeout -k 10 300 env CNF_TCONV_THIN=$m CNF_WGRAD_THIN=$m python3 bench.py --mode train --steps 10 --warmup 3 > $out/train_$m.json 2> $out/train_$m.err || { tail $out/train_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/train_$m.json')); print('thin=$m', d['ms_per_step'], d['value'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/step -o run -- python3 $root/bench.py --mode train --steps 3 --warmup 1 > $out/step.log 2>&1 || { echo "trace failed"; tail $out/step.log; exit 1; }
python3 $root/profiles/fold_step.py $out/step > $out/fold.txt && head -3 $out/fold.txt
grep -h "lnb_apply\|lnb_gsum\|thin" $out/step/*kernel_stats.csv | cut -c1-150
