#!/bin/bash
# isolated kernel durations of the training step: rocprofv3 kernel trace with every launch serialised
# (AMD_SERIALIZE_KERNEL=3), folded per layer
set -o pipefail
root=$PWD
out=$root/gpurun_out/r4serial
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/step -o run -- python3 $root/bench.py --mode train --steps 3 --warmup 1 > $out/step.log 2>&1 || { echo "serial trace failed"; tail $out/step.log; exit 1; }
cd $root
python3 profiles/fold_step.py $out/step > $out/fold.txt && cat $out/fold.txt
