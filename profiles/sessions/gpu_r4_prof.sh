#!/bin/bash
# Round-4 profile call: kernel stats + PMC passes + training stats (profiles/collect.sh), the
# per-GPU-batch anchors with their rocprof stats, then a 2-rank rehearsal of the training bench on
# one GPU (gloo).   bash profiles/sessions/gpu_r4_prof.sh TAG
set -o pipefail
tag=${1:-r04}
root=$PWD
out=$root/gpurun_out/$tag
mkdir -p $out
bash profiles/collect.sh $tag || exit 1
bash profiles/prof_r4_anchors.sh ${tag}_anch || exit 1
cd $root
CNF_BENCH_DEVICE=0 CNF_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --mode train \
  --steps 5 --warmup 2 > $out/train_2rank.json 2> $out/train_2rank.err || { echo "2-rank train failed"; tail $out/train_2rank.err; exit 1; }
cat $out/train_2rank.json
echo r4 profile call done
