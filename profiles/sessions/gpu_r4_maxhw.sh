#!/bin/bash
# measured alternative to k_net_lds's one-CU-per-(image, net) layers: stream the larger layers through
# k_pw/k_gc (CNF_NETLDS_MAXHW) at cfg2 B=64 and ref_default B=32, forward and train, same box
set -o pipefail
out=gpurun_out/r4maxhw
mkdir -p $out
run() {   # tag env... -- bench args
  local tag=$1; shift

  timeout -k 10 300 env "$@" > $out/$tag.json 2> $out/$tag.err || { echo "$tag failed"; tail $out/$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
}
B="python bench.py --no-cpu-baseline --no-roofline"
run cfg2_def CNF_X=0 $B
run cfg2_s256 CNF_NETLDS_MAXHW=128 $B
run cfg2_s64 CNF_NETLDS_MAXHW=32 $B
run ref_def CNF_X=0 $B --config ref_default
run ref_s CNF_NETLDS_MAXHW=128 $B --config ref_default
run ref_s2 CNF_NETLDS_MAXHW=32 $B --config ref_default
run tr_def CNF_X=0 $B --mode train --steps 10 --warmup 3
run tr_s256 CNF_NETLDS_MAXHW=128 $B --mode train --steps 10 --warmup 3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_s256 -o run -- python3 bench.py --no-cpu-baseline --no-roofline --steps 50 > $out/prof_s256.log 2>&1 || { echo prof failed; exit 1; }
echo done
