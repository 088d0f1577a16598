set -o pipefail
out=gpurun_out/x6u; mkdir -p $out; : > $out/d.log
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for x in 1 2 3; do
  echo "X$x" >> $out/d.log
  CNF_LIB=$L/libcnf_x$x.so timeout -k 10 200 python -u profiles/diag/diag_nondet.py cfg5 2 GENERIC=2 >> $out/d.log 2>&1 || exit 1
done
cat $out/d.log
