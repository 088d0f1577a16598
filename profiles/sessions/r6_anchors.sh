set -o pipefail
# cfg4 / cfg5 anchors at their 8-GPU shares on the final build (generic k_pw / k_gc by default at 64x64+)
# against the specialised kernels (GENERIC=0)
out=gpurun_out/r6anch; mkdir -p $out
for c in "cfg4 32" "cfg4 128" "cfg5 64"; do
  set -- $c
  for o in '' 'GENERIC=0'; do
    timeout -k 10 300 python bench.py --config $1 --batch $2 --no-cpu-baseline --inflight 0 --debug-options "$o" > $out/a.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$out/a.json'));print('$1 B=$2 [$o]', d['value'], d['ms_per_step'])"
  done
done
