set -o pipefail
# which kernel needs the generic instantiations: auto GENERIC=2 (k_pw only) / 4 (k_gc only) at 64x64+,
# the cfg5 B = 64 and cfg4 B = 32 ragged cases, six and three runs
out=gpurun_out/r6g24; mkdir -p $out
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for r in 1 2 3 4 5 6; do
  for v in g2 g4; do
    k="ragged and cfg5"; [ $r -gt 3 ] && k="ragged and (cfg5 or cfg4)"
    CNF_LIB=$L/libcnf_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 150 --timeout-method thread -k "$k" > $out/${v}_$r.log 2>&1
    echo "[$v run $r] rc=$? $(tail -1 $out/${v}_$r.log)"
  done
done
