set -o pipefail
out=gpurun_out/x6x; mkdir -p $out; : > $out/d.log
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for m in 1 2 4 8; do
  echo "pp runtime group $m" >> $out/d.log
  CNF_LIB=$L/libcnf_pp$m.so timeout -k 10 150 python -u profiles/diag/diag_nondet.py cfg2 64 '' >> $out/d.log 2>&1 || exit 1
done
cat $out/d.log
