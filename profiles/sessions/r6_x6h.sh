set -o pipefail
out=gpurun_out/x6h; mkdir -p $out
export CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_diag.so
CNF_PW_ONLY_SID=28 timeout -k 10 200 python -u profiles/diag/diag_layer_map.py cfg5 2 2 '' GENERIC=2 > $out/map.log 2>&1; cat $out/map.log
