set -o pipefail
out=gpurun_out/x6v; mkdir -p $out; : > $out/d.log
export CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_diag.so
for d in 0 2 4 6; do
  echo "pw diag $d (sid 28 only, gc generic)" >> $out/d.log
  CNF_PW_DIAG=$d CNF_PW_ONLY_SID=28 timeout -k 10 120 python -u profiles/diag/diag_nondet.py cfg5 1 GENERIC=4 >> $out/d.log 2>&1 || exit 1
done
cat $out/d.log
