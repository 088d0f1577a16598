set -o pipefail
out=gpurun_out/r6i; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for c in "cfg4 32" "cfg5 64" "cfg2 64"; do
  set -- $c
  timeout -k 10 300 python bench.py --config $1 --batch $2 --steps 20 --warmup 3 --no-cpu-baseline --inflight 0 > $out/b.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/b.json'));print('$c', d['value'], d['ms_per_step'])"
done
