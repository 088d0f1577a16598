set -o pipefail
out=gpurun_out/r6k; mkdir -p $out
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for lib in libcnf_hip.so libcnf_ablw.so libcnf_ablb.so libcnf_hip.so; do
  CNF_LIB=$L/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --inflight 0 > $out/b.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/b.json'));print('$lib', d['value'], d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['per_role'].items() if 'k_gc' in k})"
done
