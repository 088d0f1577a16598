#!/bin/bash
# round 5: shared-tile k_pw (CNF_PW_SH builds, 2 / 3 image streams) -- A/B on cfg2, then the parity suite on sh2
set -o pipefail
bash profiles/sessions/r5_ab.sh r5sh cfg2 "base sh2 sh3" || exit 1
CNF_LIB=arl_conditional_normalizing_flows_amd/lib/var_sh2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5sh/tests_sh2.log 2>&1; tail -3 gpurun_out/r5sh/tests_sh2.log
