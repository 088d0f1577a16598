#!/bin/bash
# Profile collection on the GPU box (run from the repo root):  bash profiles/collect.sh TAG
#  1. rocprofv3 --kernel-trace --stats of the bench command (graph replay, as timed)
#  2-4. separate --pmc passes (never combined with sys/runtime traces): FETCH_SIZE, WRITE_SIZE,
#     SQ issue/wait counters, each with --kernel-trace only, on the eager (no-graph) bench path
#  5. --kernel-trace --stats of the training step (bench.py --mode train)
# then profiles/pmc_summary.py folds them into profiles/TAG_summary.json (+ the stats CSV copy).
# Only gpurun_out/ comes back from the box: re-run the fold in the container afterwards,
#   python3 profiles/pmc_summary.py gpurun_out/prof_TAG TAG
set -o pipefail
tag=${1:-r01}
root=$PWD
out=$root/gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
B="$root/bench.py --no-cpu-baseline --no-roofline --inflight 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- python3 $B --steps 20 --warmup 5 > $out/stats.log 2>&1 || { echo "stats pass failed"; tail $out/stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o run -- python3 $B --steps 3 --warmup 1 --no-graph > $out/fetch.log 2>&1 || { echo "fetch pass failed"; tail $out/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o run -- python3 $B --steps 3 --warmup 1 --no-graph > $out/write.log 2>&1 || { echo "write pass failed"; tail $out/write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU --kernel-trace --output-format csv -d $out/sq -o run -- python3 $B --steps 3 --warmup 1 --no-graph > $out/sq.log 2>&1 || { echo "sq pass failed"; tail $out/sq.log; exit 1; }
# the training step (forward_train + backward + Adam), kernel trace only
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/train -o run -- python3 $root/bench.py --mode train --steps 3 --warmup 1 > $out/train.log 2>&1 || { echo "train pass failed"; tail $out/train.log; exit 1; }
cd $root
python3 profiles/pmc_summary.py $out $tag
