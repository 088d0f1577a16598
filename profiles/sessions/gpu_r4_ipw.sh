#!/bin/bash
# same-box sweep of the streamed kernels' images-per-workgroup at cfg2 B=64 (forward bench)
set -o pipefail
out=gpurun_out/r4ipw
mkdir -p $out
run() {
  local tag=$1; shift
  timeout -k 10 300 env "$@" python bench.py --no-cpu-baseline --no-roofline > $out/$tag.json 2> $out/$tag.err || { echo "$tag failed"; tail $out/$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
}
run def CNF_X=0
run res2 CNF_PW_IPW_RES=2
run res8 CNF_PW_IPW_RES=8
run a2 CNF_PW_IPW=2
run a8 CNF_PW_IPW=8
run gc2 CNF_GC_IPW=2
run gc4 CNF_GC_IPW=4
run gc8 CNF_GC_IPW=8
run def2 CNF_X=0
