#!/bin/bash
# per-launch in-stream kernel times of the cfg5 and cfg4 forward benches (bench.py's stderr table)
set -o pipefail
out=gpurun_out/${1:-ck}; mkdir -p $out
for c in cfg5 cfg4; do
timeout -k 10 300 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $out/$c.json 2> $out/$c.err || { echo "$c failed"; tail $out/$c.err; exit 1; }
done
echo done
