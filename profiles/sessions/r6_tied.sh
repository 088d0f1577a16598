set -o pipefail
# bf16x6 chains as one tied-accumulator asm statement (cnf_device.h mfma_x6): with the two round-6
# workarounds (default build) and without them (tiednw: cin folded, no k_gc image barrier)
out=gpurun_out/r6tied; mkdir -p $out; : > $out/d.log
L=$PWD/arl_conditional_normalizing_flows_amd/lib
for v in tiednw hip; do
  for c in "cfg2 64" "cfg3 16" "cfg5 8" "cfg4 32"; do
    echo "[$v]" >> $out/d.log
    CNF_LIB=$L/libcnf_$v.so timeout -k 10 200 python -u profiles/diag/diag_nondet.py $c '' 2>&1 | grep -v amdgpu.ids >> $out/d.log || { cat $out/d.log; exit 1; }
  done
done
cat $out/d.log
for v in tiednw hip; do
  CNF_LIB=$L/libcnf_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "roundtrip_bench_batches or deterministic or ragged" > $out/t_$v.log 2>&1; echo "[$v] pytest rc=$?"; tail -1 $out/t_$v.log
done
for r in 1 2; do
  for v in tiednw hip; do
    CNF_LIB=$L/libcnf_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 0 > $out/b_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$out/b_$v.json'));print('$v', d['value'], d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['per_role'].items()})"
  done
done
