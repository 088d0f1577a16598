#!/bin/bash
# per-kernel stats of the training step under environment variants:  bash profiles/sessions/gpu_r4_abl.sh TAG "ENV=.." ...
set -o pipefail
tag=$1; shift
root=$PWD
out=$root/gpurun_out/$tag
mkdir -p $out
i=0
for envs in "$@"; do
  i=$((i+1))
  echo "== $envs"
  cd /tmp && export TMPDIR=/tmp
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/v$i -o run -- python3 $root/bench.py --mode train --steps 4 --warmup 1 > $out/v$i.log 2>&1 || { echo "variant $envs failed"; tail $out/v$i.log; exit 1; }
  cd $root
  grep '"metric"' $out/v$i.log | head -c 200; echo
  python3 profiles/kstats.py $(ls $out/v$i/*kernel_stats.csv $out/v$i/*/*kernel_stats.csv 2>/dev/null | head -1) 5
done
