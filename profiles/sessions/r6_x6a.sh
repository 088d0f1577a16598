set -o pipefail
out=gpurun_out/x6a; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
tail -30 $out/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 0 > $out/bench.json 2> $out/bench.err
tail -c 600 $out/bench.json
