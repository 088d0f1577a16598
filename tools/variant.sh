#!/bin/bash
# build a diagnostic / A-B variant of the library into lib/var_NAME.so (then rebuild the default)
# usage: tools/variant.sh NAME "-DFOO=1 -DBAR"
set -e
cd "$(dirname "$0")/.."
CNF_EXTRA_FLAGS="$2" python -c "from arl_conditional_normalizing_flows_amd import _build; _build.build()"
cp arl_conditional_normalizing_flows_amd/lib/libcnf_hip.so arl_conditional_normalizing_flows_amd/lib/var_$1.so
python -c "from arl_conditional_normalizing_flows_amd import _build; _build.build()"
