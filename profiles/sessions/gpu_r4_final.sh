#!/bin/bash
# round-4 closing call: the GPU suite, the three bench lines, the training step's kernel stats and per-layer
# fold.   bash profiles/sessions/gpu_r4_final.sh TAG
set -o pipefail
tag=${1:-r4f}
bash profiles/sessions/gpu_r4.sh $tag || exit 1
root=$PWD
out=$root/gpurun_out/${tag}_prof
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/train -o run -- python3 $root/bench.py --mode train --steps 4 --warmup 1 > $out/train.log 2>&1 || { echo "train stats failed"; tail $out/train.log; exit 1; }
cd $root
python3 profiles/fold_step.py $out/train > $out/fold.txt && cat $out/fold.txt
