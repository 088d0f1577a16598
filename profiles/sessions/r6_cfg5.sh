set -o pipefail
# the cfg5 GPU parity cases, twice per library: default, no k_ln_merge (consumers fold every slot),
# generic k_pw / k_gc (GENERIC=6 default) -- which one, if any, removes the intermittent cfg5 B = 64 failure
out=gpurun_out/r6cfg5; mkdir -p $out
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for r in 1 2; do
  for v in hip nomerge gen; do
    CNF_LIB=$L/libcnf_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "cfg5" > $out/${v}_$r.log 2>&1
    echo "[$v run $r] rc=$? $(tail -1 $out/${v}_$r.log)"
  done
done
