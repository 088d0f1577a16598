#!/bin/bash
# rocprofv3 kernel trace of the training step (bench.py --mode train), folded per coupling layer.
#   bash profiles/prof_r4_step.sh TAG
set -o pipefail
tag=${1:-r4s}
root=$PWD
out=$root/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/step -o run -- python3 $root/bench.py --mode train --steps 3 --warmup 1 > $out/step.log 2>&1 || { echo "train step trace failed"; tail $out/step.log; exit 1; }
cd $root
python3 profiles/fold_step.py $out/step > $out/fold.txt && cat $out/fold.txt
