#!/bin/bash
# k_gc per-instantiation stats + SQ counters of one config's forward (cfg5 by default), on the GPU box
set -o pipefail
c=${2:-cfg5}
root=$PWD; out=$root/gpurun_out/${1:-gcp}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
B="$root/bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-graph"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- python3 $B > $out/stats.log 2>&1 || { echo "stats failed"; tail $out/stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU --kernel-trace --output-format csv -d $out/sq -o run -- python3 $B > $out/sq.log 2>&1 || { echo "sq failed"; tail $out/sq.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/sq2 -o run -- python3 $B > $out/sq2.log 2>&1 || { echo "sq2 failed"; tail $out/sq2.log; exit 1; }
echo done
