#!/bin/bash
# k_out_law per-launch times (bench per_role) for the 64- and 128-pixel tiles, cfg2 B=64
set -o pipefail
out=gpurun_out/r5olaw2; mkdir -p $out
for ks in 2 1 0; do
  if [ $ks = 0 ]; then export CNF_OUT_LAW=0; else export CNF_OUT_LAW_KS=$ks; fi
  timeout -k 10 300 python3 bench.py --config cfg2 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline --inflight 1 > $out/ks$ks.json 2> $out/ks$ks.err || { tail $out/ks$ks.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/ks$ks.json')); print('ks=$ks', d['value'], d['step_ms_median'])
for k,v in d['per_role'].items(): print('   ', k, v['avg_launch_us'], v['launches'])"
done
