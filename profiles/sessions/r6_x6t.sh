set -o pipefail
out=gpurun_out/x6t; mkdir -p $out; : > $out/d.log
export CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_diag.so
echo "sync all" >> $out/d.log
CNF_SYNC_ALL=1 timeout -k 10 200 python -u profiles/diag/diag_nondet.py cfg5 2 '' GENERIC=2 GENERIC=4 >> $out/d.log 2>&1 || exit 1
echo "gc ipw 1" >> $out/d.log
CNF_GC_IPW=1 timeout -k 10 200 python -u profiles/diag/diag_nondet.py cfg5 2 GENERIC=2 >> $out/d.log 2>&1 || exit 1
cat $out/d.log
