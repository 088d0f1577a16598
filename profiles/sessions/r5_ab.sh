#!/bin/bash
# round 5: A/B of library builds (lib/var_NAME.so, tools/variant.sh) on the forward bench, interleaved
# twice; prints images/s and the per-role in-stream kernel times.
# usage: bash profiles/sessions/r5_ab.sh TAG CONFIG "base var1 var2 ..." [extra bench args]
set -o pipefail
tag=$1; cfg=$2; vars=$3; shift 3
out=gpurun_out/$tag; mkdir -p $out
lib=arl_conditional_normalizing_flows_amd/lib
for rep in 1 2; do
  for v in $vars; do
    if [ "$v" = base ]; then L=$lib/libcnf_hip.so; else L=$lib/var_$v.so; fi
    CNF_LIB=$L timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline "$@" > $out/${v}_$rep.json 2> $out/${v}_$rep.err || { echo "$v failed"; tail -20 $out/${v}_$rep.err; exit 1; }
    python3 - $out/${v}_$rep.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
pr = d['roofline']['per_role']
print(f"{sys.argv[2]:>8} {d['value']:9.1f} img/s {d['step_ms_median']:.4f} ms | " +
      ' '.join(f"{k.replace('k_pw<','').replace('>','')}={v['avg_launch_us']:.2f}" for k, v in pr.items()), flush=True)
PY
  done
done
