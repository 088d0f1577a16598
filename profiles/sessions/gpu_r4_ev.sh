#!/bin/bash
# training-step stream check: train bench, the per-layer step profile (queue overlap per layer), and the
# 2-rank gloo rehearsal with and without the overlapped all-reduce.   bash profiles/sessions/gpu_r4_ev.sh TAG
set -o pipefail
tag=${1:-r4ev}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > $out/train.json 2> $out/train.err || { echo "train bench failed"; tail -20 $out/train.err; exit 1; }
cat $out/train.json
bash profiles/prof_r4_step.sh ${tag}_s || exit 1
for ov in 1 0; do
CNF_GRAD_OVERLAP=$ov CNF_BENCH_DEVICE=0 CNF_BENCH_BACKEND=gloo timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --mode train \
  --steps 3 --warmup 1 > $out/train_2rank_ov$ov.json 2> $out/train_2rank_ov$ov.err || { echo "2-rank train failed"; tail $out/train_2rank_ov$ov.err; exit 1; }
head -c 300 $out/train_2rank_ov$ov.json; echo
done
