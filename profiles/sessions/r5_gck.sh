#!/bin/bash
# cfg4 B=32 / cfg5 B=64: the grouped stage's plan knobs (polyphase k_gc groups, tap-mode dilation floor)
set -o pipefail
out=gpurun_out/r5gck; mkdir -p $out
for cb in "cfg4 32" "cfg5 64"; do
  set -- $cb
  for kv in "X=0" "CNF_GC_POLY=0" "CNF_GC_TAP_DMIN=16" "CNF_GC_TAP_DMIN=2" "X=0" "CNF_GC_POLY=0"; do
    timeout -k 10 300 env $kv python3 bench.py --config $1 --batch $2 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --inflight 1 > $out/$1_$2.json 2> $out/$1_$2.err || { tail $out/$1_$2.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/$1_$2.json')); print('$1 B=$2 $kv', d['value'], d['step_ms_median'])"
  done
done
