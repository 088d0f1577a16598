set -o pipefail
out=gpurun_out/x6n; mkdir -p $out; : > $out/d.log
timeout -k 10 240 python -u profiles/diag/diag_nondet.py cfg5 2 GENERIC=6 GENERIC=10 GENERIC=12 GENERIC=14 'GENERIC=6,LAYOUT=3' >> $out/d.log 2>&1 || exit 1
timeout -k 10 240 python -u profiles/diag/diag_nondet.py cfg5 1 '' GENERIC=14 >> $out/d.log 2>&1 || exit 1
cat $out/d.log
