#!/bin/bash
# the training GPU tests in full (gradients, bitwise reproducibility, forward_train == forward), the train bench
set -o pipefail
tag=${1:-r4tt}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_train.py tests/test_comm.py tests/test_training_driver.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error" $out/tests.log | tail -30; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > $out/train.json 2> $out/train.err || { echo "train bench failed"; tail -20 $out/train.err; exit 1; }
cat $out/train.json
