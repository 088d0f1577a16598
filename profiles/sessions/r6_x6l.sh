set -o pipefail
out=gpurun_out/x6l; mkdir -p $out; : > $out/d.log
timeout -k 10 150 python -u profiles/diag/diag_opts_err.py cfg5 2 '' '' GENERIC=2 GENERIC=2 GENERIC=4 GENERIC=8 >> $out/d.log 2>&1 || exit 1
timeout -k 10 150 python -u profiles/diag/diag_layerwise.py cfg5 2 GENERIC=2 '' >> $out/d.log 2>&1 || exit 1
cat $out/d.log
