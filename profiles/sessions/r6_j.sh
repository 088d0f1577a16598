set -o pipefail
out=gpurun_out/r6j; mkdir -p $out; : > $out/nd.log
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for spec in "cfg4 32" "cfg3 16" "ref_default 8" "cfg5 2"; do
  timeout -k 10 300 python -u profiles/diag/diag_nondet.py $spec '' >> $out/nd.log 2>&1 || exit 1
done
cat $out/nd.log
for c in "cfg4 32" "cfg4 128" "cfg3 128"; do
  set -- $c
  for lib in libcnf_hip.so libcnf_nohalves.so libcnf_hip.so libcnf_nohalves.so; do
    CNF_LIB=$L/$lib timeout -k 10 300 python bench.py --config $1 --batch $2 --steps 20 --warmup 3 --no-cpu-baseline --inflight 0 > $out/b.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$out/b.json'));print('$lib $c', d['value'], d['ms_per_step'])"
  done
done
