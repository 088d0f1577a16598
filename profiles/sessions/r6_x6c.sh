set -o pipefail
out=gpurun_out/x6c; mkdir -p $out
timeout -k 10 300 python -u profiles/diag/diag_opts_err.py cfg5 1 '' GENERIC=2 GENERIC=4 GENERIC=8 > $out/cfg5.log 2>&1; cat $out/cfg5.log
