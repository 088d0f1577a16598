set -o pipefail
out=gpurun_out/x6k; mkdir -p $out; : > $out/d.log
echo "diag2 GENERIC=2" >> $out/d.log
CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_diag2.so timeout -k 10 120 python -u profiles/diag/diag_opts_err.py cfg5 2 GENERIC=2 GENERIC=2 '' >> $out/d.log 2>&1 || exit 1
echo "diag2 ONLY_SID=999" >> $out/d.log
CNF_PW_ONLY_SID=999 CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_diag2.so timeout -k 10 120 python -u profiles/diag/diag_opts_err.py cfg5 2 '' '' >> $out/d.log 2>&1 || exit 1
cat $out/d.log
