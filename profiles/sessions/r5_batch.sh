#!/bin/bash
# round 5: the batch-dependence bisection (profiles/diag/diag_batch.py) on cfg2 / cfg3 with knobs
set -o pipefail
out=gpurun_out/r5_batch
mkdir -p $out
for cfg in cfg3 cfg2; do
  for knobs in "" "CNF_PW_IPW=1 CNF_PW_IPW_RES=1" "CNF_GC_IPW=1" "CNF_PW_GENERIC=1" "CNF_GC_GENERIC=1" "CNF_NETLDS_GENERIC=1" "CNF_FUSE_COUPLING=0"; do
    timeout -k 10 120 python profiles/diag/diag_batch.py $cfg 67 $knobs >> $out/log.txt 2>&1 || { echo "failed: $cfg $knobs"; tail -20 $out/log.txt; exit 1; }
  done
done
cat $out/log.txt
