set -o pipefail
out=gpurun_out/x6m; mkdir -p $out; : > $out/d.log
timeout -k 10 240 python -u profiles/diag/diag_nondet.py cfg5 2 '' GC=0 LAYOUT=3 LAYOUT=5 LAYOUT=6 PW=0 GENERIC=1 FUSE_COUPLING=0 'GC=0,LAYOUT=0' >> $out/d.log 2>&1 || exit 1
cat $out/d.log
