#!/bin/bash
# round-4 GPU session: risky new shapes first (own short limit), then the whole GPU suite, then the bench
# usage (repo root, GPU box): bash profiles/sessions/gpu_r4.sh TAG [pytest -k expr for the first step]
set -o pipefail
tag=${1:-r4}
out=gpurun_out/$tag
mkdir -p $out
if [ -n "$2" ]; then
  timeout -k 10 240 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$2" > $out/first.log 2>&1 || { echo "first step failed"; tail -40 $out/first.log; exit 1; }
  tail -3 $out/first.log
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > $out/tests.log 2>&1 || { echo "tests failed"; tail -40 $out/tests.log; exit 1; }
tail -25 $out/tests.log
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 python bench.py --mode inverse > $out/inverse.json 2> $out/inverse.err || { echo "inverse bench failed"; tail -20 $out/inverse.err; exit 1; }
cat $out/inverse.json
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > $out/train.json 2> $out/train.err || { echo "train bench failed"; tail -20 $out/train.err; exit 1; }
cat $out/train.json
