set -o pipefail
# localise the intermittent cfg5 difference (ragged B = 64 test, 7.7e-3): specialised k_gc (GENERIC=4)
# and k_pw (GENERIC=2) instantiations off in turn, three forwards each; then the k_lnb_apply session
out=gpurun_out/r6loc; mkdir -p $out
timeout -k 10 400 python -u profiles/diag/diag_nondet.py cfg5 8 '' GENERIC=4 GENERIC=2 GENERIC=6 2>&1 | grep -v amdgpu.ids | tee $out/d.log || exit 1
timeout -k 10 300 python -u profiles/diag/diag_nondet.py cfg5 16 '' GENERIC=4 2>&1 | grep -v amdgpu.ids | tee -a $out/d.log || exit 1
bash profiles/sessions/r6_lnb.sh
