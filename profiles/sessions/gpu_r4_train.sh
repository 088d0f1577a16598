#!/bin/bash
# training-path GPU session: gradient parity (fused LDS backward and the multi-kernel one), the
# training bench, the host-enqueue diagnostic.   bash profiles/sessions/gpu_r4_train.sh TAG
set -o pipefail
tag=${1:-r4tr}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_train.py tests/test_comm.py tests/test_training_driver.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error" $out/tests.log | tail -30; exit 1; }
grep -E "worst|PASS|FAIL" $out/tests.log | tail -30
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > $out/train.json 2> $out/train.err || { echo "train bench failed"; tail -20 $out/train.err; exit 1; }
cat $out/train.json
timeout -k 10 120 python profiles/train_host_time.py cfg2 64 > $out/host.txt 2>&1 || { echo "host diag failed"; tail $out/host.txt; exit 1; }
cat $out/host.txt
