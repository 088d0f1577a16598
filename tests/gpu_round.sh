#!/bin/bash
# GPU-box session: parity tests, bench line, rocprofv3 kernel-trace summary of the same bench.
# usage (from repo root, on the GPU box): bash tests/gpu_round.sh TAG
set -o pipefail
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > $out/tests.log 2>&1 || { echo "tests failed"; tail -20 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
root=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/prof -o run -- python3 $root/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $root/$out/prof_bench.json 2> $root/$out/prof_bench.err || { echo "rocprof failed"; tail -20 $root/$out/prof_bench.err; exit 1; }
find $root/$out/prof -name "*stats*" | head
