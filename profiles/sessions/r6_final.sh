set -o pipefail
out=gpurun_out/r6final; mkdir -p $out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > $out/train.json 2> $out/train.err || { tail -20 $out/train.err; exit 1; }
python -c "
import json
for f in ('bench','train'):
    d=json.load(open('$out/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)"
