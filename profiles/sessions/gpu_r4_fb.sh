#!/bin/bash
# training tests + train bench (gpu_r4_tt.sh), the forward parity tests, and the forward bench
set -o pipefail
tag=${1:-r4fb}
out=gpurun_out/$tag
mkdir -p $out
bash profiles/sessions/gpu_r4_tt.sh $tag || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/parity.log 2>&1 || { echo "parity failed"; grep -E "FAIL|Error" $out/parity.log | tail -20; exit 1; }
tail -1 $out/parity.log
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail $out/bench.err; exit 1; }
head -c 300 $out/bench.json; echo
