#!/bin/bash
# quick training check: cfg2 gradient parity, the train bench, the per-layer step profile.  bash profiles/sessions/gpu_r4_tq.sh TAG
set -o pipefail
tag=${1:-r4tq}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_train.py -m gpu -x -v --timeout 300 --timeout-method thread -k "gradients_match_oracle and (cfg2 or small or narrow)" > $out/tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error" $out/tests.log | tail -30; exit 1; }
grep -E "worst|PASS|FAIL" $out/tests.log | tail -12
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > $out/train.json 2> $out/train.err || { echo "train bench failed"; tail -20 $out/train.err; exit 1; }
cat $out/train.json
bash profiles/prof_r4_step.sh ${tag}_s
CNF_LDSBWD_STAMPS=1 timeout -k 10 120 python profiles/diag/diag_bwd_stamps.py > gpurun_out/$tag/stamps.txt 2>&1 || { echo "stamps failed"; tail gpurun_out/$tag/stamps.txt; exit 1; }
cat gpurun_out/$tag/stamps.txt
