#!/bin/bash
# same-box A/B of the dual-store conv_a: forward bench (default vs CNF_LIB=$1), the training tests,
# then the train bench with each library
set -o pipefail
alt=$1
bash profiles/sessions/gpu_r4_fwdab.sh $alt || exit 1
bash profiles/sessions/gpu_r4_tt.sh r4dual || exit 1
CNF_LIB=$alt timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > gpurun_out/r4dual/train_ab.json 2> gpurun_out/r4dual/train_ab.err || { echo "train ab failed"; exit 1; }
cat gpurun_out/r4dual/train_ab.json
