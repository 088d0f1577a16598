#!/bin/bash
# per-dispatch trace of one streamed layer's training backward (cfg2 B=64, coupling 2), alone on the GPU
set -o pipefail
root=$PWD; out=$root/gpurun_out/r5ltr; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $out/l2 -o run -- python3 $root/profiles/train_layer_trace.py cfg2 64 2 > $out/l2.log 2>&1 || { echo "trace failed"; tail $out/l2.log; exit 1; }
python3 $root/profiles/train_layer_trace.py --fold $out/l2 > $out/l2.txt && head -60 $out/l2.txt
