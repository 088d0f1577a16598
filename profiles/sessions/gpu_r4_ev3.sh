#!/bin/bash
set -o pipefail
tag=${1:-r4ev3}
out=gpurun_out/$tag
mkdir -p $out
CNF_TRAIN_EVFLAGS=0 timeout -k 10 200 python profiles/diag/diag_train_host.py > $out/host_ev0.txt 2>&1 || { echo "diag failed"; tail $out/host_ev0.txt; exit 1; }
cat $out/host_ev0.txt
CNF_TRAIN_WSTREAM=0 timeout -k 10 200 python profiles/diag/diag_train_host.py > $out/host_ws0.txt 2>&1 || { echo "diag ws0 failed"; tail $out/host_ws0.txt; exit 1; }
cat $out/host_ws0.txt
CNF_TRAIN_WSTREAM=0 bash profiles/prof_r4_step.sh ${tag}_s > /dev/null || exit 1
