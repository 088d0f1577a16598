set -o pipefail
out=gpurun_out/x6b; mkdir -p $out
timeout -k 10 300 python -u profiles/diag/diag_opts_err.py cfg5 1 > $out/cfg5.log 2>&1; cat $out/cfg5.log
timeout -k 10 300 python -u profiles/diag/diag_opts_err.py cfg4 2 '' GENERIC=1 > $out/cfg4.log 2>&1; cat $out/cfg4.log
