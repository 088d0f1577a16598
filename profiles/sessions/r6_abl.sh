set -o pipefail
mkdir -p gpurun_out/abl
timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 0 > gpurun_out/abl/def.json 2> gpurun_out/abl/def.err && \
CNF_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/libcnf_abl.so timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 0 > gpurun_out/abl/abl.json 2> gpurun_out/abl/abl.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 0 > gpurun_out/abl/def2.json 2> gpurun_out/abl/def2.err
