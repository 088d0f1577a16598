set -o pipefail
# the cfg5 B = 64 ragged-batch case alone, six runs per library (default / no k_ln_merge / generic)
out=gpurun_out/r6cfg5b; mkdir -p $out
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for r in 1 2 3 4 5 6; do
  for v in hip nomerge gen; do
    CNF_LIB=$L/libcnf_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 150 --timeout-method thread -k "ragged and cfg5" > $out/${v}_$r.log 2>&1
    echo "[$v run $r] rc=$? $(tail -1 $out/${v}_$r.log)"
  done
done
