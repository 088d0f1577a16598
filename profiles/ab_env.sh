#!/bin/bash
# A/B of an environment knob on the forward bench: bash profiles/ab_env.sh OUT CONFIG VAR "v1 v2 ..."
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for v in $4; do
env $3=$v timeout -k 10 300 python3 bench.py --config $2 --steps 3 --warmup 1 --no-cpu-baseline > $out/$2_$v.json 2> $out/$2_$v.err || { echo "$2 $3=$v failed"; tail $out/$2_$v.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/$2_$v.json'));print('$2 $3=$v', d['value'], d['ms_per_step'])"
done
