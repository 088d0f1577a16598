set -o pipefail
root=$PWD; out=$root/gpurun_out/r6e; mkdir -p $out
for spec in "cfg4 32" "cfg4 128" "cfg5 64" "ref_default 32" "cfg3 128"; do
  set -- $spec
  timeout -k 10 300 python3 bench.py --config $1 --batch $2 --steps 20 --warmup 3 --no-cpu-baseline --inflight 2 > $out/$1_b$2.json 2> $out/$1_b$2.err || { echo "$spec failed"; tail $out/$1_b$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/$1_b$2.json'));print('$spec', d['value'], d['ms_per_step'], d.get('serving',{}).get('value'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg4 -o run -- python3 $root/bench.py --config cfg4 --batch 32 --steps 5 --warmup 1 --no-cpu-baseline --no-roofline --inflight 0 > $out/cfg4prof.log 2>&1 || { echo "prof failed"; tail $out/cfg4prof.log; exit 1; }
echo done
