#!/bin/bash
set -o pipefail
tag=${1:-r4ev2}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 200 python profiles/diag/diag_train_host.py > $out/host.txt 2>&1 || { echo "diag failed"; tail $out/host.txt; exit 1; }
cat $out/host.txt
CNF_TRAIN_NETORDER=1 timeout -k 10 200 python profiles/diag/diag_train_host.py > $out/host_rev.txt 2>&1 || { echo "diag rev failed"; tail $out/host_rev.txt; exit 1; }
cat $out/host_rev.txt
CNF_TRAIN_NETORDER=1 bash profiles/prof_r4_step.sh ${tag}_s || exit 1
