#!/bin/bash
# round 5: per-workgroup stamps of conv_b / conv_a / k_gc (profiles/diag/diag_wg_stamps.py), the A/B of
# the lrelu-only build against the default, then the GPU suite on the default build
set -o pipefail
out=gpurun_out/r5st; mkdir -p $out
L=arl_conditional_normalizing_flows_amd/lib
for v in st2 st1 gcst; do
  echo "== $v" | tee -a $out/stamps.txt
  CNF_LIB=$L/var_$v.so timeout -k 10 120 python3 profiles/diag/diag_wg_stamps.py cfg2 >> $out/stamps.txt 2>&1 || { tail -20 $out/stamps.txt; exit 1; }
done
cat $out/stamps.txt
bash profiles/sessions/r5_ab.sh r5ab2 cfg2 "base lra" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; tail -3 $out/tests.log
