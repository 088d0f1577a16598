#!/bin/bash
# images per workgroup of the streamed kernels, re-swept on the round-5 kernels (cfg2 B=64)
set -o pipefail
out=gpurun_out/r5ipw; mkdir -p $out
for kv in "X=0" "CNF_PW_IPW_RES=2" "CNF_PW_IPW_RES=8" "CNF_PW_IPW=2" "CNF_PW_IPW=8" "CNF_GC_IPW=1" "CNF_GC_IPW=3" "X=0"; do
  timeout -k 10 300 env $kv python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --inflight 1 > $out/r.json 2> $out/r.err || { tail $out/r.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/r.json')); r=d['roofline']['per_role']
print('$kv', d['value'], d['step_ms_median'], ' '.join(f'{k}={v[\"avg_launch_us\"]}' for k,v in list(r.items())[:4]))"
done
