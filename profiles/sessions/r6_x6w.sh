set -o pipefail
out=gpurun_out/x6w; mkdir -p $out; : > $out/d.log
timeout -k 10 200 python -u profiles/diag/diag_nondet.py cfg2 64 '' GENERIC=2 GENERIC=4 GENERIC=6 GENERIC=8 >> $out/d.log 2>&1 || exit 1
echo "diag gc ipw 1" >> $out/d.log
CNF_GC_IPW=1 CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_diag.so timeout -k 10 200 python -u profiles/diag/diag_nondet.py cfg2 64 '' GENERIC=2 >> $out/d.log 2>&1 || exit 1
cat $out/d.log
