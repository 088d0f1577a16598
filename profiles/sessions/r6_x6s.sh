set -o pipefail
out=gpurun_out/x6s; mkdir -p $out; : > $out/d.log
timeout -k 10 240 python -u profiles/diag/diag_nondet.py cfg5 2 '' GENERIC=2 GENERIC=4 >> $out/d.log 2>&1 || exit 1
cat $out/d.log
