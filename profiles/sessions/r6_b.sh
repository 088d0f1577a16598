set -o pipefail
out=gpurun_out/r6b; mkdir -p $out; : > $out/nd.log
timeout -k 10 200 python -u profiles/diag/diag_nondet.py cfg5 2 '' GENERIC=1 >> $out/nd.log 2>&1 || exit 1
timeout -k 10 200 python -u profiles/diag/diag_nondet.py cfg5 4 '' >> $out/nd.log 2>&1 || exit 1
timeout -k 10 200 python -u profiles/diag/diag_nondet.py cfg4 4 '' >> $out/nd.log 2>&1 || exit 1
timeout -k 10 200 python -u profiles/diag/diag_nondet.py cfg2 8 '' >> $out/nd.log 2>&1 || exit 1
cat $out/nd.log
CNF_ROUND_TRAIN=1 bash profiles/gpu_round.sh r6b
