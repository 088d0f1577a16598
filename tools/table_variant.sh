#!/bin/bash
# build lib/var_NAME.so with shape tables generated under the environment settings ENV... (plan knobs
# that change launch shapes, e.g. CNF_GC_POLY_NW=16), then restore the committed tables and rebuild the
# default library. Run the variant with the same ENV and CNF_LIB=.../var_NAME.so.
# usage: tools/table_variant.sh NAME VAR=VALUE [VAR=VALUE ...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
C=arl_conditional_normalizing_flows_amd/csrc
env "$@" python $C/gen_netlds_shapes.py
CNF_EXTRA_FLAGS="-DCNF_VARIANT_$name" python -c "from arl_conditional_normalizing_flows_amd import _build; _build.build()"
cp arl_conditional_normalizing_flows_amd/lib/libcnf_hip.so arl_conditional_normalizing_flows_amd/lib/var_$name.so
git checkout $C/cnf_gc_shapes.inc $C/cnf_pw_shapes.inc $C/cnf_netlds_shapes.inc
python -c "from arl_conditional_normalizing_flows_amd import _build; _build.build()"
