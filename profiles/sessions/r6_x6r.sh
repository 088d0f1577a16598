set -o pipefail
out=gpurun_out/x6r; mkdir -p $out; : > $out/d.log
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for b in 1 3 4 8; do
  echo "gc sid 11 B=$b" >> $out/d.log
  CNF_LIB=$L/libcnf_diag.so CNF_GC_ONLY_SID=11 timeout -k 10 120 python -u profiles/diag/diag_nondet.py cfg5 $b GENERIC=2 >> $out/d.log 2>&1 || exit 1
done
echo "pw sid 28 PP_RUNTIME, gc generic" >> $out/d.log
CNF_LIB=$L/libcnf_diag2.so CNF_PW_ONLY_SID=28 timeout -k 10 120 python -u profiles/diag/diag_nondet.py cfg5 2 GENERIC=4 >> $out/d.log 2>&1 || exit 1
echo "pw sid 28 const, gc generic, B=1" >> $out/d.log
CNF_LIB=$L/libcnf_diag.so CNF_PW_ONLY_SID=28 timeout -k 10 120 python -u profiles/diag/diag_nondet.py cfg5 1 GENERIC=4 >> $out/d.log 2>&1 || exit 1
cat $out/d.log
