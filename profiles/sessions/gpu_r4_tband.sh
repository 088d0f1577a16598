#!/bin/bash
# same-box sweep of the band data-gradient kernel's knobs on the train bench
set -o pipefail
out=gpurun_out/r4tband
mkdir -p $out
run() {
  local tag=$1; shift
  timeout -k 10 300 env "$@" python bench.py --mode train --steps 10 --warmup 3 > $out/$tag.json 2> $out/$tag.err || { echo "$tag failed"; tail $out/$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
}
run def CNF_X=0
run mw128 CNF_TBAND_MINWG=128
run mw512 CNF_TBAND_MINWG=512
run mw64 CNF_TBAND_MINWG=64
run mw1024 CNF_TBAND_MINWG=1024
run def2 CNF_X=0
