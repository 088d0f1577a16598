#!/bin/bash
# rocprofv3 kernel-trace stats of the cfg2 training step (bench.py --mode train), on the GPU box
set -o pipefail
root=$PWD; out=$root/gpurun_out/${1:-ptr}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/train -o run -- python3 $root/bench.py --mode train --steps 3 --warmup 1 > $out/train.log 2>&1 || { echo "train failed"; tail $out/train.log; exit 1; }
echo done
