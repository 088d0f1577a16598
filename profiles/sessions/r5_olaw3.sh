#!/bin/bash
# k_out_law with one staging batch (U=18, 286 VGPRs: one workgroup per CU) / two batches (U=9
# variant lib) against the tap GEMM + k_coupling pair, cfg2 B=64, per-launch times
set -o pipefail
out=gpurun_out/r5olaw3; mkdir -p $out
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --config cfg2 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline --inflight 1 > $out/$n.json 2> $out/$n.err || { tail $out/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/$n.json')); print('$n', d['value'], d['step_ms_median'])
for k,v in d['roofline']['per_role'].items():
    if 'out' in k or 'coupling' in k: print('   ', k, v['avg_launch_us'], v['launches'])"
}
run u18 CNF_OUT_LAW=1
run u9 CNF_OUT_LAW=1 CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/var_olu9.so
run off CNF_OUT_LAW=0
run u18b CNF_OUT_LAW=1
