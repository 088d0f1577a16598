#!/bin/bash
# round 5: k_net_lds phase stamps (generic stamps instantiation), then the k_pw stagger A/B
set -o pipefail
CNF_STAMPS=1 timeout -k 10 200 python3 profiles/diag/diag_stamps.py > gpurun_out/r5stamps.txt 2>&1 || { tail gpurun_out/r5stamps.txt; exit 1; }
cat gpurun_out/r5stamps.txt
bash profiles/sessions/r5_ab.sh r5stg cfg2 "base stg24 stg60" --inflight 1
