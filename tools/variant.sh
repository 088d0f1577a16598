#!/bin/bash
# build a diagnostic / A-B variant of the library into lib/var_NAME.so (the default build is untouched)
# usage: tools/variant.sh NAME "-DFOO=1 -DBAR"
set -e
cd "$(dirname "$0")/.."
CNF_BUILD_LIB=$PWD/arl_conditional_normalizing_flows_amd/lib/var_$1.so CNF_EXTRA_FLAGS="$2" \
  python -c "from arl_conditional_normalizing_flows_amd import _build; _build.build()"
