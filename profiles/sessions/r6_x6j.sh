set -o pipefail
out=gpurun_out/x6j; mkdir -p $out; : > $out/d.log
export CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_diag2.so
CNF_PW_ONLY_SID=28 timeout -k 10 120 python -u profiles/diag/diag_opts_err.py cfg5 2 '' '' >> $out/d.log 2>&1 || exit 1
cat $out/d.log
