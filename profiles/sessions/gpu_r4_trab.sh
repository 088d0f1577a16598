#!/bin/bash
# the training GPU tests, then a same-box A/B of the train bench: the default library against
# CNF_LIB=$1, twice each, alternating
set -o pipefail
alt=$1
out=gpurun_out/r4trab
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_train.py tests/test_comm.py tests/test_training_driver.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error" $out/tests.log | tail -30; exit 1; }
tail -1 $out/tests.log
for i in 1 2; do
  for lib in default $alt; do
    if [ $lib = default ]; then env=""; else env="CNF_LIB=$lib"; fi
    env $env timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > $out/tr_$i.json 2> $out/tr_$i.err || { echo "train bench failed"; tail $out/tr_$i.err; exit 1; }
    echo "$(basename $lib) $(python3 -c "import json;d=json.loads(open('$out/tr_$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done
