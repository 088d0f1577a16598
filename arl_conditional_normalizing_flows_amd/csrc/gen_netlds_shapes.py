#!/usr/bin/env python3
"""Generate cnf_netlds_shapes.inc, cnf_gc_shapes.inc and cnf_pw_shapes.inc. The first holds the k_net_lds "shape words" (NETSHAPE_WORDS ints: every
launch-independent field of NetLdsArgs except the mask) of the LDS-resident coupling layers of the
presets in SPECIALISE. cnf_netlds.hip compiles one shape-specialised instantiation per entry, with
those words as compile-time constants; launch_net_lds picks it when a launch's words match and
otherwise runs the generic kernel, so a stale table is never wrong, only slower (and
tests/test_capi.py fails on it). The second holds the GcShape (branch geometry, tile, strides) of the
streamed layers' k_gc launches, used the same way by cnf_stream.hip; the third the PwShape of every
k_pw launch of the forward, taken from a host-only dry run of it (cnf_debug_pw_shapes).

    python arl_conditional_normalizing_flows_amd/csrc/gen_netlds_shapes.py [--check]

Needs a built libcnf_hip.so (plan creation is host-only: no GPU)."""
from __future__ import annotations

import ctypes as C
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))

from arl_conditional_normalizing_flows_amd import _lib  # noqa: E402
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402

# BASELINE.json configs[1] (the benchmark), configs[2], the reference's default, configs[3], configs[4]
SPECIALISE = ('cfg2', 'cfg3', 'ref_default', 'cfg4', 'cfg5')
OUT = HERE / 'cnf_netlds_shapes.inc'
OUT_GC = HERE / 'cnf_gc_shapes.inc'
OUT_PW = HERE / 'cnf_pw_shapes.inc'
PW_BATCH = 64                 # the benchmark batch (k_pw shapes do not depend on it: ipw and B stay runtime)
PW_MASK_WORDS = 2             # PwShape ends with the two uint32 stored-channel masks and st_compact
GC_BRANCH_WORDS = 18          # GcBranch: 16 ints, then the two uint32 division magics
GC_MAXBR = 8
CNF_LAYER_COUPLING = 0
CAP = 2048
W2 = 7   # words of [off_y, stamp_off): off_y, off_t1, off_t2, off_w, off_k, off_ks, maxnr
M1 = 123  # int members in [offs_per_net, zero_bias) (any further word is alignment padding before zero_bias)


def _plan(lib, cfg):
    arr = lambda v: (C.c_int * len(v))(*[int(x) for x in v])
    keep = [arr(cfg.squeeze_factor_block_list), arr(cfg.ResNeXt_block_list), arr(cfg.num_kernels_list),
            arr(cfg.cardinality_list)]
    desc = _lib.cnf_flow_desc(cfg.io_shape[0], cfg.io_shape[1], cfg.io_shape[2], cfg.x_d,
                              len(cfg.squeeze_factor_block_list), *keep, cfg.lambda_y, cfg.ksize,
                              int(cfg.LAYER_NORM), int(cfg.DILATIONS), {'reference': 0, 'intended': 1}[cfg.group_mode])
    plan = C.c_void_p()
    _lib.check(lib.cnf_plan_create(C.byref(desc), C.byref(plan)), 'plan')
    return plan, keep


def shapes(lib):
    lib.cnf_debug_netlds_shape.restype = C.c_int
    lib.cnf_debug_netlds_shape.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.c_int]
    out = []
    for name in SPECIALISE:
        plan, _keep = _plan(lib, PRESETS[name])
        info = _lib.cnf_layer_info()
        buf = (C.c_int * CAP)()
        for i in range(lib.cnf_plan_num_layers(plan)):
            _lib.check(lib.cnf_plan_layer_info(plan, i, C.byref(info)), 'layer info')
            if info.kind != CNF_LAYER_COUPLING:
                continue
            n = lib.cnf_debug_netlds_shape(plan, info.coupling_index, buf, CAP)
            if n < 0:
                raise RuntimeError('cnf_debug_netlds_shape failed')
            w = tuple(buf[j] for j in range(n))
            if n and w not in out:
                out.append(w)
        lib.cnf_plan_destroy(plan)
    return out


def gc_shapes(lib):
    """k_gc shapes as a dry run of the B-image forward launches them (GcArgs::s)"""
    lib.cnf_debug_gc_launch_shapes.restype = C.c_int
    lib.cnf_debug_gc_launch_shapes.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.c_int]
    out = []
    for name in SPECIALISE:
        plan, _keep = _plan(lib, PRESETS[name])
        buf = (C.c_int * (CAP * 8))()
        n = lib.cnf_debug_gc_launch_shapes(plan, PW_BATCH, buf, CAP * 8)
        if n < 0:
            raise RuntimeError('cnf_debug_gc_launch_shapes failed: ' + lib.cnf_last_error().decode())
        nw = lib.cnf_debug_gc_words()   # GCSHAPE_WORDS
        for g0 in range(0, n, nw):
            w = tuple(buf[g0 + j] for j in range(nw))
            if w not in out:
                out.append(w)
        lib.cnf_plan_destroy(plan)
    return out


def pw_shapes(lib):
    lib.cnf_debug_pw_shapes.restype = C.c_int
    lib.cnf_debug_pw_shapes.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.c_int]
    out = []
    for name in SPECIALISE:
        plan, _keep = _plan(lib, PRESETS[name])
        buf = (C.c_int * (CAP * 8))()
        n = lib.cnf_debug_pw_shapes(plan, PW_BATCH, buf, CAP * 8)
        if n < 0:
            raise RuntimeError('cnf_debug_pw_shapes failed: ' + lib.cnf_last_error().decode())
        nw = lib.cnf_debug_pw_words()  # PWSHAPE_WORDS
        for i in range(0, n, nw):
            w = tuple(buf[i + j] for j in range(nw))
            if w not in out:
                out.append(w)
        lib.cnf_plan_destroy(plan)
    return out


def render_pw(sh):
    lines = ['// Generated by gen_netlds_shapes.py from dry runs of the ' + ', '.join(SPECIALISE) + ' forward: do not edit.',
             '// One k_pw PwShape (cnf_kernels.h) per shape-specialised instantiation.',
             f'#define CNF_PW_NSHAPES {len(sh)}',
             f'constexpr PwShape kPwShapes[{max(1, len(sh))}] = {{']
    for w in sh or [None]:
        if w is None:
            lines.append('    {},')
            continue
        k = len(w) - PW_MASK_WORDS - 2   # ..., st_mask_lo, st_mask_hi, st_compact, in_mapped
        lines.append('    {' + ', '.join([str(x) for x in w[:k]] + [f'{x & 0xffffffff}u' for x in w[k:k + 2]] +
                                       [str(x) for x in w[k + 2:]]) + '},')
    lines.append('};')
    return '\n'.join(lines) + '\n'


def render_gc(sh):
    lines = ['// Generated by gen_netlds_shapes.py from the plans of ' + ', '.join(SPECIALISE) + ': do not edit.',
             '// One k_gc GcShape (cnf_kernels.h) per shape-specialised instantiation.',
             f'#define CNF_GC_NSHAPES {len(sh)}',
             f'constexpr GcShape kGcShapes[{max(1, len(sh))}] = {{']
    for w in sh or [None]:
        if w is None:
            lines.append('    {},')
            continue
        vals = []
        for i, x in enumerate(w):
            if i < GC_MAXBR * GC_BRANCH_WORDS and i % GC_BRANCH_WORDS >= GC_BRANCH_WORDS - 2:
                vals.append(f'{x & 0xffffffff}u')
            else:
                vals.append(str(x))
        lines.append('    {' + ', '.join(vals) + '},')
    lines.append('};')
    return '\n'.join(lines) + '\n'


def render(sh):
    lines = ['// Generated by gen_netlds_shapes.py from the plans of ' + ', '.join(SPECIALISE) + ': do not edit.',
             '// One k_net_lds shape (NETSHAPE_WORDS ints, see cnf_kernels.h) per shape-specialised instantiation.',
             f'#define CNF_NETLDS_NSHAPES {len(sh)}']
    rows = max(1, len(sh))
    lines.append(f'constexpr int kNetShapeWords[{rows}][NETSHAPE_WORDS] = {{')
    for w in sh or [(0,)]:
        lines.append('    {' + ', '.join(str(x) for x in w) + '},')
    lines.append('};')
    # the same shapes as NetLdsArgs aggregates (declaration order, brace elision): u, so[2], params,
    # aux, offs, [offs_per_net, zero_bias) words, zero_bias, [off_y, stamp_off) words, stamp_off
    lines.append(f'constexpr NetLdsArgs kNetShapes[{rows}] = {{')
    for w in sh or [None]:
        if w is None:
            lines.append('    {},')
            continue
        w1, w2 = w[:M1], w[-W2:]
        lines.append('    {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, ' + ', '.join(str(x) for x in w1) +
                     ', nullptr, ' + ', '.join(str(x) for x in w2) + ', 0},')
    lines.append('};')
    return '\n'.join(lines) + '\n'


def main():
    lib = _lib.load()
    sh, gsh, psh = shapes(lib), gc_shapes(lib), pw_shapes(lib)
    outs = [(OUT, render(sh), len(sh)), (OUT_GC, render_gc(gsh), len(gsh)), (OUT_PW, render_pw(psh), len(psh))]
    if '--check' in sys.argv:
        bad = [f.name for f, text, _ in outs if (f.read_text() if f.exists() else '') != text]
        if bad:
            print(f'{", ".join(bad)} stale: rerun {Path(__file__).name}', file=sys.stderr)
            return 1
        return 0
    for f, text, n in outs:
        f.write_text(text)
        print(f'wrote {f} ({n} shapes)')
    return 0


if __name__ == '__main__':
    sys.exit(main())
