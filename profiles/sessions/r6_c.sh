set -o pipefail
out=gpurun_out/r6c; mkdir -p $out; : > $out/nd.log
for spec in "cfg2 64" "cfg5 1" "cfg5 2" "cfg5 4" "cfg4 32" "ref_default 32" "cfg3 16"; do
  timeout -k 10 200 python -u profiles/diag/diag_nondet.py $spec '' >> $out/nd.log 2>&1 || exit 1
done
cat $out/nd.log
grep -q "e-0[1-4]" $out/nd.log && { echo "NONDET OR ERROR"; exit 1; }
CNF_ROUND_TRAIN=1 bash profiles/gpu_round.sh r6c
