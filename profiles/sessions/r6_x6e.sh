set -o pipefail
out=gpurun_out/x6e; mkdir -p $out; : > $out/sid.log
export CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_diag.so
for sid in 26 27 28 29 30; do
  CNF_PW_ONLY_SID=$sid timeout -k 10 120 python -u profiles/diag/diag_opts_err.py cfg5 1 '' >> $out/sid.log 2>&1 || exit 1
  echo "^ sid $sid" >> $out/sid.log
done
cat $out/sid.log
unset CNF_LIB
timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 0 > $out/bench.json 2> $out/bench.err
python -c "
import json
d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['per_role'].items()})"
