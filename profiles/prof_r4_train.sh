#!/bin/bash
# Per-dispatch kernel traces of one coupling layer's training backward at cfg2 B=64 (a streamed 32x32
# layer and an LDS 16x16 layer), and rocprofv3 stats of the whole training step.
#   bash profiles/prof_r4_train.sh TAG
set -o pipefail
tag=${1:-r4t}
root=$PWD
out=$root/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for ci in 2 0; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $out/l$ci -o run -- python3 $root/profiles/train_layer_trace.py cfg2 64 $ci > $out/l$ci.log 2>&1 || { echo "layer $ci trace failed"; tail $out/l$ci.log; exit 1; }
  python3 $root/profiles/train_layer_trace.py --fold $out/l$ci > $out/l$ci.txt || exit 1
  tail -25 $out/l$ci.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/step -o run -- python3 $root/bench.py --mode train --steps 3 --warmup 1 > $out/step.log 2>&1 || { echo "train step trace failed"; tail $out/step.log; exit 1; }
tail -2 $out/step.log
