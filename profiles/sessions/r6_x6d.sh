set -o pipefail
out=gpurun_out/x6d; mkdir -p $out
timeout -k 10 300 python -u profiles/diag/diag_layerwise.py cfg5 1 GENERIC=2 '' > $out/lw.log 2>&1; cat $out/lw.log
