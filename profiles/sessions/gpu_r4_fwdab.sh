#!/bin/bash
# same-box A/B of the forward bench: the default library against CNF_LIB=$1, twice each, alternating
set -o pipefail
alt=$1
for i in 1 2; do
  for lib in default $alt; do
    if [ $lib = default ]; then env=""; else env="CNF_LIB=$lib"; fi
    env $env timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/fwdab_$i.json 2> gpurun_out/fwdab_$i.err || { echo "bench failed"; tail gpurun_out/fwdab_$i.err; exit 1; }
    echo "$lib $(python3 -c "import json;d=json.loads(open('gpurun_out/fwdab_$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  done
done
