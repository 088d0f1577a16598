set -o pipefail
# LeakyReLU form A/B on the shipped kernels (cin at run time, k_gc image barrier): lr3w the round-5
# inline asm, lr0w fmaxf, lr2w v_maximum3 (both compiler-visible): determinism + oracle error, then
# the cfg2 forward bench alternating
out=gpurun_out/r6lr3; mkdir -p $out; : > $out/d.log
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for v in lr3w lr0w lr2w; do
  for c in "cfg2 64" "cfg3 16" "cfg5 2"; do
    echo "[$v]" >> $out/d.log
    CNF_LIB=$L/libcnf_$v.so timeout -k 10 200 python -u profiles/diag/diag_nondet.py $c '' 2>&1 | grep -v amdgpu.ids >> $out/d.log || { cat $out/d.log; exit 1; }
  done
done
cat $out/d.log
for r in 1 2; do
  for v in lr3w lr0w lr2w; do
    CNF_LIB=$L/libcnf_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 0 > $out/b_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$out/b_$v.json'));print('$v', d['value'], d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['per_role'].items()})"
  done
done
