set -o pipefail
out=gpurun_out/r6d; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k test_deterministic > $out/det.log 2>&1 || { tail -30 $out/det.log; exit 1; }
tail -3 $out/det.log
for o in '' 'GENERIC=2' '' 'GENERIC=2'; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 0 --debug-options "$o" > $out/ab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/ab.json'));print('[$o]', d['value'], d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['per_role'].items()})"
done
bash profiles/collect.sh r06
