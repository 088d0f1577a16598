#!/bin/bash
# 1-GPU anchors at the per-GPU batches the strong-scaling runs put on each GPU (BASELINE configs[3]:
# cfg4 256 global over 8 / 4 / 2 GPUs -> 32 / 64 / 128; configs[4]: cfg5 512 over 8 -> 64), with the
# CPU leg, plus rocprofv3 kernel-trace stats of each.   bash profiles/prof_r4_anchors.sh TAG
set -o pipefail
tag=${1:-r5c}
root=$PWD
out=$root/gpurun_out/$tag
mkdir -p $out
for cb in cfg4:32 cfg4:64 cfg4:128 cfg5:64 ref_default:32 cfg3:128; do
  c=${cb%%:*}; b=${cb##*:}
  timeout -k 10 300 python3 bench.py --config $c --batch $b --steps 20 --warmup 3 > $out/${c}_b$b.json 2> $out/${c}_b$b.err || { echo "$c B=$b failed"; tail $out/${c}_b$b.err; exit 1; }
  head -c 400 $out/${c}_b$b.json; echo
done
cd /tmp && export TMPDIR=/tmp
for cb in cfg4:32 cfg5:64; do
  c=${cb%%:*}; b=${cb##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats_${c}_b$b -o run -- python3 $root/bench.py --config $c --batch $b --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > $out/stats_${c}_b$b.log 2>&1 || { echo "stats $c failed"; tail $out/stats_${c}_b$b.log; exit 1; }
done
echo anchors done
