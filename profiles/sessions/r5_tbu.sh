#!/bin/bash
# k_tconv_band staging: quads per thread and load batch 4 (default) / 8 / 16 (variant libs), train step
set -o pipefail
root=$PWD; out=$root/gpurun_out/r5tbu; mkdir -p $out
L=$root/arl_conditional_normalizing_flows_amd/lib
for v in def tbu8 tbu16 def tbu8 tbu16; do
  if [ $v = def ]; then lib=$L/libcnf_hip.so; else lib=$L/var_$v.so; fi
  timeout -k 10 300 env CNF_LIB=$lib python3 bench.py --mode train --steps 10 --warmup 3 > $out/$v.json 2> $out/$v.err || { tail $out/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$v.json')); print('$v', d['ms_per_step'], d['value'])"
done
