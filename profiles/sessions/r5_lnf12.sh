#!/bin/bash
# LN partial slots folded by the consumers up to 768 per image (-DCNF_LN_FETCH=12 variant lib) against
# 512 (default): cfg4 B=32 / B=128 (k_ln_merge launches of the 64x64 layers' grouped stages), cfg2, cfg5
set -o pipefail
out=gpurun_out/r5lnf12; mkdir -p $out
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for cb in "cfg4 32" "cfg4 128" "cfg5 64" "cfg2 64"; do
  set -- $cb
  for v in def lnf12 def lnf12; do
    if [ $v = def ]; then lib=$L/libcnf_hip.so; else lib=$L/var_$v.so; fi
    timeout -k 10 300 env CNF_LIB=$lib python3 bench.py --config $1 --batch $2 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --inflight 1 > $out/r.json 2> $out/r.err || { tail $out/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/r.json')); print('$1 B=$2 $v', d['value'], d['step_ms_median'])"
  done
done
