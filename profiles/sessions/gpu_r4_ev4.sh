#!/bin/bash
set -o pipefail
tag=${1:-r4ev4}
out=gpurun_out/$tag
mkdir -p $out
for v in 256 4096; do
ROC_SIGNAL_POOL_SIZE=$v timeout -k 10 200 python profiles/diag/diag_train_host.py > $out/host_sp$v.txt 2>&1 || { echo "diag failed"; tail $out/host_sp$v.txt; exit 1; }
echo "signal pool $v"; cat $out/host_sp$v.txt
done
DEBUG_CLR_MAX_BATCH_SIZE=4096 timeout -k 10 200 python profiles/diag/diag_train_host.py > $out/host_mb.txt 2>&1 || { echo "diag failed"; tail $out/host_mb.txt; exit 1; }
echo "max batch 4096"; cat $out/host_mb.txt
