#!/bin/bash
# Host AddressSanitizer + UndefinedBehaviorSanitizer build of libcnf_hip.so (host code only: every
# -fsanitize= sits behind -Xarch_host, the gfx950 device code is built as usual), then the C-ABI
# tests that need no GPU (plan creation, workspace layouts, host dry runs of the forward / inverse,
# the t1 / t2 layout and shape-table debug entry points, the toy and transform argument checks)
# run against it. CPU only; the sanitizer build never goes to the GPU box.
#   bash tools/host_sanitize.sh
set -eo pipefail
root=$(cd "$(dirname "$0")/.." && pwd)
cd "$root"
lib=$root/arl_conditional_normalizing_flows_amd/build/asan/libcnf_hip_asan.so
mkdir -p "$(dirname "$lib")"
export CNF_EXTRA_FLAGS="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer -g"
export CNF_EXTRA_LDFLAGS="-fsanitize=address,undefined -shared-libsan"
CNF_BUILD_LIB=$lib python3 -c "import sys; sys.path.insert(0, '.'); from arl_conditional_normalizing_flows_amd import _build; print(_build.build())"
asan_rt=$(/opt/rocm/bin/hipcc -print-file-name=libclang_rt.asan-x86_64.so)
# leaks: python and torch hold allocations at exit that are not the library's
CNF_LIB=$lib LD_PRELOAD=$asan_rt ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  python3 -m pytest -x -q -p no:cacheprovider tests/test_capi.py tests/test_toy.py tests/test_transforms.py "$@"
