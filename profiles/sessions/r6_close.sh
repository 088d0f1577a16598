set -o pipefail
# closing run (k_gc image pairs off, generic k_pw / k_gc at 64x64 and above): smoke, the GPU suite, the cfg5
# more times, forward and training bench lines
out=gpurun_out/r6close; mkdir -p $out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "(cfg5 or cfg4) and (ragged or deterministic or roundtrip_bench)" > $out/rep$r.log 2>&1; echo "repeat $r rc=$?"; tail -1 $out/rep$r.log
done
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > $out/train.json 2> $out/train.err || { tail -20 $out/train.err; exit 1; }
python -c "
import json
for f in ('bench','train'):
    d=json.load(open('$out/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)"
