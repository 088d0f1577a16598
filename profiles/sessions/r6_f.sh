set -o pipefail
out=gpurun_out/r6f; mkdir -p $out
export CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_diag.so
run() { timeout -k 10 200 env "$@" python bench.py --no-cpu-baseline --inflight 0 > $out/ab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/ab.json'));print('$*', d['value'], d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['per_role'].items() if 'k_pw' in k or 'k_gc' in k})"; }
run X=0
run CNF_PW_IPW_RES=2
run CNF_PW_IPW_RES=8
run CNF_PW_IPW=2
run CNF_PW_IPW=8
run CNF_GC_IPW=1
run CNF_GC_IPW=4
run X=0
