#!/bin/bash
# HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) against the default, cfg2 / cfg4 forward
set -o pipefail
out=gpurun_out/r5ka; mkdir -p $out
for cb in "cfg2 64" "cfg4 32"; do
  set -- $cb
  for m in 0 1 0 1; do
    timeout -k 10 300 env HIP_FORCE_DEV_KERNARG=$m python3 bench.py --config $1 --batch $2 --steps 20 --warmup 5 --no-cpu-baseline --inflight 1 > $out/$1_$m.json 2> $out/$1_$m.err || { tail $out/$1_$m.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$out/$1_$m.json')); r=d['roofline']['per_role']
print('$1 B=$2 devkernarg=$m', d['value'], d['step_ms_median'], ' '.join(f'{k}={v[\"avg_launch_us\"]}' for k,v in list(r.items())[:5]))"
  done
done
timeout -k 10 300 env HIP_FORCE_DEV_KERNARG=1 python3 bench.py --mode train --steps 10 --warmup 3 > $out/train_1.json 2>/dev/null && python3 -c "import json; d=json.load(open('$out/train_1.json')); print('train devkernarg=1', d['ms_per_step'])"
