#!/bin/bash
# round 5: thin-channel training kernels (k_tconv_thin: conv_out data gradient / conv_in recompute;
# k_wgrad_thin: conv_out weight gradient) -- gradient tests, then the train step against the MFMA
# kernels for those convs (CNF_TCONV_THIN=0 CNF_WGRAD_THIN=0), alternating, and a layer trace
set -o pipefail
root=$PWD; out=$root/gpurun_out/r5thin; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_train.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit 1
for m in 1 0 1 0; do
  timeout -k 10 300 env CNF_TCONV_THIN=$m CNF_WGRAD_THIN=$m python3 bench.py --mode train --steps 10 --warmup 3 > $out/train_$m.json 2> $out/train_$m.err || { tail $out/train_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/train_$m.json')); print('thin=$m', d['ms_per_step'], d['value'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $out/l2 -o run -- python3 $root/profiles/train_layer_trace.py cfg2 64 2 > $out/l2.log 2>&1 || { echo "trace failed"; tail $out/l2.log; exit 1; }
python3 $root/profiles/train_layer_trace.py --fold $out/l2 > $out/l2.txt && sed -n 55,75p $out/l2.txt
