#!/bin/bash
# training-step kernel trace (cfg2 B=64) folded per backward layer
set -o pipefail
root=$PWD; out=$root/gpurun_out/r5trf; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/step -o run -- python3 $root/bench.py --mode train --steps 3 --warmup 1 > $out/step.log 2>&1 || { echo "trace failed"; tail $out/step.log; exit 1; }
python3 $root/profiles/fold_step.py $out/step > $out/fold.txt && cat $out/fold.txt
