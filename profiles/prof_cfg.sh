#!/bin/bash
# rocprofv3 kernel-trace stats of the cfg5 and cfg4 forward benches (run on the GPU box from the repo root)
set -o pipefail
root=$PWD; out=$root/gpurun_out/${1:-p45}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for c in cfg5 cfg4; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$c -o run -- python3 $root/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > $out/$c.log 2>&1 || { echo "$c failed"; tail $out/$c.log; exit 1; }
done
echo done
