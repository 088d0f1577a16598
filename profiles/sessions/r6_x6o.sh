set -o pipefail
out=gpurun_out/x6o; mkdir -p $out; : > $out/d.log
L=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_diag.so
timeout -k 10 240 python -u profiles/diag/diag_nondet.py cfg5 2 'GENERIC=2,LAYOUT=3' 'GENERIC=2,LAYOUT=4' 'GENERIC=2,LAYOUT=0' 'GENERIC=4,LAYOUT=3' 'GENERIC=4,LAYOUT=5' >> $out/d.log 2>&1 || exit 1
echo "diag ONLY_SID=999" >> $out/d.log
CNF_PW_ONLY_SID=999 CNF_LIB=$L timeout -k 10 120 python -u profiles/diag/diag_nondet.py cfg5 2 GENERIC=4 >> $out/d.log 2>&1 || exit 1
echo "diag ONLY_SID=28" >> $out/d.log
CNF_PW_ONLY_SID=28 CNF_LIB=$L timeout -k 10 120 python -u profiles/diag/diag_nondet.py cfg5 2 GENERIC=4 >> $out/d.log 2>&1 || exit 1
cat $out/d.log
