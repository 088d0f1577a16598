set -o pipefail
out=gpurun_out/x6g; mkdir -p $out; : > $out/sid.log
export CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_diag.so
for rep in 1 2; do
  CNF_PW_ONLY_SID=28 timeout -k 10 120 python -u profiles/diag/diag_opts_err.py cfg5 1 '' '' >> $out/sid.log 2>&1 || exit 1
done
CNF_PW_ONLY_SID=28 timeout -k 10 120 python -u profiles/diag/diag_opts_err.py cfg5 2 '' >> $out/sid.log 2>&1 || exit 1
CNF_PW_ONLY_SID=18 timeout -k 10 120 python -u profiles/diag/diag_opts_err.py cfg4 4 '' >> $out/sid.log 2>&1 || exit 1
cat $out/sid.log
