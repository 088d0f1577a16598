set -o pipefail
out=gpurun_out/r6h; mkdir -p $out
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for spec in "cfg5 4" "cfg4 32" "cfg3 16"; do
  set -- $spec
  timeout -k 10 200 python -u profiles/diag/diag_dump.py $1 $2 $out/${1}_pairs.npz > /dev/null 2>&1 || exit 1
  CNF_LIB=$L/libcnf_nopairs.so timeout -k 10 200 python -u profiles/diag/diag_dump.py $1 $2 $out/${1}_single.npz > /dev/null 2>&1 || exit 1
  python -c "
import numpy as np
a=np.load('$out/${1}_pairs.npz'); b=np.load('$out/${1}_single.npz')
print('$spec', {k: bool(np.array_equal(a[k], b[k])) for k in a.files})"
done
timeout -k 10 300 python -u profiles/diag/diag_nondet.py cfg5 4 '' >> $out/nd.log 2>&1 || exit 1
timeout -k 10 300 python -u profiles/diag/diag_nondet.py cfg4 32 '' >> $out/nd.log 2>&1 || exit 1
cat $out/nd.log
for c in "cfg4 32" "cfg5 64"; do
  set -- $c
  timeout -k 10 300 python bench.py --config $1 --batch $2 --steps 20 --warmup 3 --no-cpu-baseline --inflight 0 > $out/b.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/b.json'));print('pairs $c', d['value'], d['ms_per_step'])"
  CNF_LIB=$L/libcnf_nopairs.so timeout -k 10 300 python bench.py --config $1 --batch $2 --steps 20 --warmup 3 --no-cpu-baseline --inflight 0 > $out/b.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/b.json'));print('single $c', d['value'], d['ms_per_step'])"
done
