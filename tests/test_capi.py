"""CPU: the C-ABI library loads, exports every symbol include/cnf.h declares, and its host-side
plan (cFlow.__init__ restated in C++) agrees with the oracle. No GPU compute here."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

from arl_conditional_normalizing_flows_amd import _lib
from arl_conditional_normalizing_flows_amd.config import PRESETS
from oracle.cflow_np import OracleCFlow

ROOT = Path(__file__).resolve().parents[1]


def _header_symbols():
    txt = (ROOT / 'include' / 'cnf.h').read_text()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(cnf_[a-z0-9_]+)\s*\(', txt)))


def test_all_header_symbols_exported(lib):
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f'{s} not exported'
    assert sorted(_lib.EXPORTED_SYMBOLS) == syms


def _plan(lib, kw, group_mode=0):
    arr = lambda v: (C.c_int * len(v))(*v)
    keep = [arr(kw['squeeze_factor_block_list']), arr(kw['ResNeXt_block_list']), arr(kw['num_kernels_list']),
            arr(kw['cardinality_list'])]
    d = _lib.cnf_flow_desc(*kw['io_shape'], kw['x_d'], len(keep[0]), *keep, 100.0, 3, 1, 1, group_mode)
    p = C.c_void_p()
    rc = lib.cnf_plan_create(C.byref(d), C.byref(p))
    return rc, p, keep


@pytest.mark.parametrize('name', list(PRESETS))
@pytest.mark.parametrize('gm', ['reference', 'intended'])
def test_plan_matches_oracle(lib, name, gm):
    kw = PRESETS[name].kwargs()
    kw.pop('group_mode')
    rc, p, keep = _plan(lib, kw, 0 if gm == 'reference' else 1)
    assert rc == 0, lib.cnf_last_error()
    try:
        o = OracleCFlow(**kw, group_mode=gm)
        buf = C.create_string_buffer(256)
        off, nd, sh = C.c_int64(), C.c_int(), (C.c_int * 4)()
        got, exp_off = [], 0
        for i in range(lib.cnf_plan_num_param_tensors(p)):
            assert lib.cnf_plan_param_tensor(p, i, buf, 256, C.byref(off), C.byref(nd), sh) == 0
            got.append((buf.value.decode(), tuple(sh[j] for j in range(nd.value))))
            assert off.value == exp_off
            exp_off += int(np.prod(got[-1][1])) if got[-1][1] else 1
        assert got == [(n, tuple(s)) for n, s in o.specs]
        assert lib.cnf_plan_num_params(p) == o.num_params()
        assert lib.cnf_plan_num_layers(p) == len(o.layers)
        info = _lib.cnf_layer_info()
        for li, e in enumerate(o.layers):
            assert lib.cnf_plan_layer_info(p, li, C.byref(info)) == 0
            assert info.kind == {'coupling': 0, 'squeeze': 1, 'factor': 2}[e.kind]
            assert (info.h, info.w, info.d) == tuple(e.shape)
            if e.kind == 'coupling':
                c = e.coupling
                assert (info.mask, info.hc, info.wc, info.dc1, info.dc2, info.num_kernels, info.cardinality) == \
                       (c.mask, c.hc, c.wc, c.dc1, c.dc2, c.nk, c.card)
                assert [info.dilations[i] for i in range(info.num_dilations)] == c.dilations
            if e.kind == 'factor':
                assert info.num_prev_factors == e.num_prev_factors
        assert lib.cnf_plan_workspace_bytes(p, 4) > 0
    finally:
        lib.cnf_plan_destroy(p)


@pytest.mark.parametrize('bad,msg', [
    (dict(io_shape=[5, 4, 2]), 'divisible by 2'),
    (dict(cardinality_list=[3]), 'cardinality'),
    (dict(num_kernels_list=[5]), 'kernels'),
    (dict(squeeze_factor_block_list=[2]), 'allowed entries'),
])
def test_plan_rejects_like_reference_asserts(lib, bad, msg):
    kw = dict(io_shape=[8, 8, 2], x_d=1, squeeze_factor_block_list=[0], ResNeXt_block_list=[1],
              num_kernels_list=[4], cardinality_list=[2])
    kw.update(bad)
    rc, p, _ = _plan(lib, kw)
    assert rc == -1
    assert msg in lib.cnf_last_error().decode()


def test_aux_pack_map_is_grouped_kernel_gather(lib):
    """The aux image (dense grouped-conv weights) is exactly the per-group Conv2D kernels placed
    block-wise (reference mode: all groups share the input slice)."""
    kw = PRESETS['small'].kwargs()
    kw.pop('group_mode')
    rc, p, keep = _plan(lib, kw)
    assert rc == 0
    assert lib.cnf_plan_aux_floats(p) > 0
    lib.cnf_plan_destroy(p)


def test_version(lib):
    assert b'gfx950' in lib.cnf_version()


def test_fused_net_plan(lib):
    """k_net_lds covers every cfg2 coupling layer whose s,t net fits one CU's 160 KiB LDS image
    (all but the four 32x32 channel-mask layers); CNF_NETLDS=0 forces the streamed path."""
    import os
    kw = PRESETS['cfg2'].kwargs()
    kw.pop('group_mode')

    def fused():
        rc, p, keep = _plan(lib, kw)
        assert rc == 0
        out = []
        for i in range(lib.cnf_plan_num_layers(p)):
            li = _lib.cnf_layer_info()
            assert lib.cnf_plan_layer_info(p, i, C.byref(li)) == 0
            if li.kind == 0:
                out.append((li.hc * li.wc, li.num_kernels, li.fused_net))
        lib.cnf_plan_destroy(p)
        return out

    f = fused()
    assert len(f) == 16
    assert [x[2] for x in f] == [0 if (hw == 1024 and nk == 64) else 1 for hw, nk, _ in f]
    os.environ['CNF_NETLDS'] = '0'
    try:
        assert all(x[2] == 0 for x in fused())
    finally:
        os.environ.pop('CNF_NETLDS')


def test_netlds_shape_table_is_current(lib):
    """The shape-specialised k_net_lds instantiations are compiled from cnf_netlds_shapes.inc; the
    table must equal the shapes the current plan produces for the benchmark configuration (a stale
    table is not wrong, the launcher falls back to the generic kernel, but it loses the speed)."""
    import subprocess
    import sys
    root = Path(__file__).resolve().parent.parent
    gen = root / 'arl_conditional_normalizing_flows_amd' / 'csrc' / 'gen_netlds_shapes.py'
    r = subprocess.run([sys.executable, str(gen), '--check'], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
