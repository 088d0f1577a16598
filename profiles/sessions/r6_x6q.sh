set -o pipefail
out=gpurun_out/x6q; mkdir -p $out; : > $out/d.log
export CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_diag.so
for sid in 11 12 13 14 15 999; do
  echo "gc sid $sid" >> $out/d.log
  CNF_GC_ONLY_SID=$sid timeout -k 10 120 python -u profiles/diag/diag_nondet.py cfg5 2 GENERIC=2 >> $out/d.log 2>&1 || exit 1
done
cat $out/d.log
