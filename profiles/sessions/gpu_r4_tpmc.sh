#!/bin/bash
# PMC passes over the training step (each its own run, --kernel-trace only):  bash profiles/sessions/gpu_r4_tpmc.sh TAG
set -o pipefail
tag=${1:-r4tpmc}
root=$PWD
out=$root/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
B="$root/bench.py --mode train --steps 2 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU --kernel-trace --output-format csv -d $out/sq -o run -- python3 $B > $out/sq.log 2>&1 || { echo "sq pass failed"; tail $out/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $out/lds -o run -- python3 $B > $out/lds.log 2>&1 || { echo "lds pass failed"; tail $out/lds.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o run -- python3 $B > $out/fetch.log 2>&1 || { echo "fetch pass failed"; tail $out/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o run -- python3 $B > $out/write.log 2>&1 || { echo "write pass failed"; tail $out/write.log; exit 1; }
cd $root
python3 profiles/pmc_kernels.py $out/sq $out/lds $out/fetch $out/write
