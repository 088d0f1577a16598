set -o pipefail
# k_lnb_apply with one load round trip (eight images' loads + gamma issued with the per-image sums):
# the training GPU tests, two training bench lines, and the training-step kernel stats
out=gpurun_out/r6lnb; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_train.py tests/test_comm.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 --no-cpu-baseline > $out/train$r.json 2> $out/train$r.err || { tail -20 $out/train$r.err; exit 1; }
  python -c "import json;d=json.load(open('$out/train$r.json'));print('train', d['value'], d['ms_per_step'])"
done
root=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/prof -o run -- python3 $root/bench.py --mode train --steps 3 --warmup 1 --no-cpu-baseline > $root/$out/prof.log 2>&1 || { tail $root/$out/prof.log; exit 1; }
cd $root; find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/train_kernel_stats.csv \;
ls -la $out
