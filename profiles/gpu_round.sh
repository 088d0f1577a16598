#!/bin/bash
# GPU-box session: parity tests, bench line, rocprofv3 kernel-trace summary of the same bench.
# usage (from repo root, on the GPU box): bash profiles/gpu_round.sh TAG [pytest -k expr]
set -o pipefail
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
sel=()
[ -n "$2" ] && sel=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${sel[@]}" > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
if [ -n "$CNF_ROUND_TRAIN" ]; then
  timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 2 > $out/train.json 2> $out/train.err || { echo "train bench failed"; tail -20 $out/train.err; exit 1; }
  cat $out/train.json
fi
