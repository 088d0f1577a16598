set -o pipefail
root=$PWD; out=$root/gpurun_out/r6g; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg5 -o run -- python3 $root/bench.py --config cfg5 --batch 64 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --inflight 0 > $out/cfg5prof.log 2>&1 || { echo "prof failed"; tail $out/cfg5prof.log; exit 1; }
echo done
