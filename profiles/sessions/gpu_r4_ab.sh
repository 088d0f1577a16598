#!/bin/bash
# A/B of environment knobs on the training step:  bash profiles/sessions/gpu_r4_ab.sh TAG "ENV1=.. ENV2=.." "ENV1=.." ...
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python profiles/diag/diag_train_host.py > $out/host_$i.txt 2>&1 || { echo "diag $envs failed"; tail $out/host_$i.txt; exit 1; }
  echo "== $envs"; grep -v amdgpu.ids $out/host_$i.txt | tail -3
  env $envs timeout -k 10 200 python bench.py --mode train --steps 20 --warmup 3 > $out/train_$i.json 2> $out/train_$i.err || { echo "bench $envs failed"; tail $out/train_$i.err; exit 1; }
  head -c 220 $out/train_$i.json; echo
done
