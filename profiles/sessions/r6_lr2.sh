set -o pipefail
# LeakyReLU forms A/B (cnf_device.h CNF_LRELU: 0 fmaxf, 1 select, 2 v_maximum3 builtin, 3 the round-5 asm;
# lr0w: fmaxf with cin at run time and the extra k_gc barrier): run-to-run and oracle error, three runs each
out=gpurun_out/r6lr2; mkdir -p $out; : > $out/d.log
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for v in hip lr3 lr0 lr1 lr0w; do
  for c in "cfg2 64" "cfg3 16"; do
    echo "[$v]" >> $out/d.log
    CNF_LIB=$L/libcnf_$v.so timeout -k 10 200 python -u profiles/diag/diag_nondet.py $c '' 2>&1 | grep -v amdgpu.ids >> $out/d.log || { cat $out/d.log; exit 1; }
  done
done
cat $out/d.log
