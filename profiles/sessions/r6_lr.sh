set -o pipefail
# LeakyReLU as v_maximum3_f32 (no inline asm) with cin folded again in k_pw and without the extra
# k_gc barrier: the presets that showed run-to-run differences, three runs each, then the GPU suite
# and the bench
out=gpurun_out/r6lr; mkdir -p $out; : > $out/d.log
for c in "cfg2 64" "cfg5 2" "cfg5 4" "cfg4 32" "cfg3 16"; do
  timeout -k 10 200 python -u profiles/diag/diag_nondet.py $c '' >> $out/d.log 2>&1 || { cat $out/d.log; exit 1; }
done
cat $out/d.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 0 > $out/b$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/b$i.json'));print(d['value'], d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['per_role'].items()})"
done
