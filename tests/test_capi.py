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


def _plan(lib, kw, group_mode=0, options=None):
    arr = lambda v: (C.c_int * len(v))(*v)
    keep = [arr(kw['squeeze_factor_block_list']), arr(kw['ResNeXt_block_list']), arr(kw['num_kernels_list']),
            arr(kw['cardinality_list'])]
    d = _lib.cnf_flow_desc(*kw['io_shape'], kw['x_d'], len(keep[0]), *keep, 100.0, 3, 1, 1, group_mode,
                           options.encode() if options else None)
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


def _weight_map(lib, p, which):
    n = lib.cnf_plan_weight_map(p, which, None, 0)
    assert n > 0
    buf = (C.c_int64 * n)()
    assert lib.cnf_plan_weight_map(p, which, buf, n) == n
    return np.frombuffer(buf, dtype=np.int64).copy()


@pytest.mark.parametrize('name', ['small', 'cfg2', 'ref_default'])
@pytest.mark.parametrize('gm', ['reference', 'intended'])
def test_grouped_conv_images_are_the_per_group_kernels(lib, name, gm):
    """The dense image of every grouped dilated stage (the one the kernels' packed images and the
    training path are built from) is exactly the card per-group Conv2D kernels
    (conv_cINN_base_functions.py:389-411) placed block-wise: output channel n = j*_d + o of branch d
    comes from group j's kernel [tap][c - in_offset_j][o] — in reference mode every group reads the
    LAST _d-channel slice (the Lambda closure quirk), in intended mode slice j — and is
    zero elsewhere. Checked entry by entry against the oracle's parameter table. The packed kernel
    image then holds every conv element (each grouped kernel element equally often) and no LN or
    tanh parameter."""
    kw = PRESETS[name].kwargs()
    kw.pop('group_mode')
    rc, p, keep = _plan(lib, kw, 0 if gm == 'reference' else 1)
    assert rc == 0
    try:
        o = OracleCFlow(**kw, group_mode=gm)
        offs, at = {}, 0
        for n_, s_ in o.specs:
            offs[n_] = (at, s_)
            at += int(np.prod(s_)) if s_ else 1
        bw = _weight_map(lib, p, 1)
        pad4 = lambda v: (v + 3) // 4 * 4
        pos = 0

        def take(taps, cin, cout, kernel_idx, bias_idx):
            nonlocal pos
            w = bw[pos:pos + taps * cin * cout].reshape(taps, cin, cout)
            pos += taps * cin * cout
            b = bw[pos:pos + pad4(cout)]
            pos += pad4(cout)
            assert np.array_equal(w, kernel_idx)
            assert np.array_equal(b[:cout], bias_idx) and np.all(b[cout:] == -1)

        def plain(nm, taps, cin, cout):
            k0, _ = offs[nm + '.kernel']
            b0, _ = offs[nm + '.bias']
            take(taps, cin, cout, k0 + np.arange(taps * cin * cout).reshape(taps, cin, cout), b0 + np.arange(cout))

        n_grouped = 0
        for c in o.coupling_specs:
            for net in ('A', 'b'):
                q = f'c{c.index}.{net}'
                plain(f'{q}.conv_in', 9, c.dc1, c.nk)
                for r in range(c.R):
                    plain(f'{q}.rb{r}.conv_a', 1, c.nk, c.nk)
                    for bi, br in enumerate(c.branches):
                        lo = min(br.in_offsets)
                        cin = max(br.in_offsets) + br.width - lo
                        cout = len(br.in_offsets) * br.width
                        exp = -np.ones((9, cin, cout), np.int64)
                        bias = np.zeros(cout, np.int64)
                        for j, off in enumerate(br.in_offsets):
                            k0, shp = offs[f'{q}.rb{r}.gc.d{bi}.g{j}.kernel']
                            assert tuple(shp) == (3, 3, br.width, br.width)
                            kk = k0 + np.arange(9 * br.width * br.width).reshape(9, br.width, br.width)
                            exp[:, off - lo:off - lo + br.width, j * br.width:(j + 1) * br.width] = kk
                            bias[j * br.width:(j + 1) * br.width] = offs[f'{q}.rb{r}.gc.d{bi}.g{j}.bias'][0] + \
                                np.arange(br.width)
                        if gm == 'reference' and len(br.in_offsets) > 1:
                            assert len(set(br.in_offsets)) == 1 and cin == br.width   # all groups: last slice
                        take(9, cin, cout, exp, bias)
                        n_grouped += 1
                    plain(f"{q}.rb{r}.conv_b", 1, c.gc_channels, c.nk)
                plain(f'{q}.conv_out', 9, c.nk, c.dc2)
        assert pos == bw.size and n_grouped > 0
        # the packed kernel image: conv elements only, each grouped kernel element equally often
        aux = _weight_map(lib, p, 0)
        assert aux.size == lib.cnf_plan_aux_floats(p)
        specs = {f'c{c.index}': c for c in o.coupling_specs}
        cnt = np.bincount(aux[aux >= 0], minlength=o.num_params())
        for n_, (k0, s_) in offs.items():
            size = int(np.prod(s_)) if s_ else 1
            seg = cnt[k0:k0 + size]
            if n_.endswith('.kernel') or n_.endswith('.bias'):
                assert seg.min() >= 1, n_
                if '.gc.' in n_:
                    assert seg.min() == seg.max(), n_
            elif '.ln2.' in n_ and seg.max() > 0:
                # streamed layers store t1 compactly (only the grouped branches' input windows): their
                # LN2 gamma/beta are gathered once into that layout, the same channels at every pixel
                c = specs[n_.split('.')[0]]
                used = np.zeros(c.nk, np.int64)
                for br in c.branches:
                    for off in br.in_offsets:
                        used[off:off + br.width] = 1
                rows = seg.reshape(-1, c.nk)
                assert used.sum() < c.nk and np.array_equal(rows, np.broadcast_to(used, rows.shape)), n_
            elif '.ln3.' in n_ and seg.max() > 0:
                # t2 split into its k_gc groups' sub-tensors (mapped layout): LN3 gamma/beta gathered
                # once into it, a permutation of the channels at every pixel
                assert seg.min() == 1 and seg.max() == 1, n_
            else:
                assert seg.max() == 0, n_
    finally:
        lib.cnf_plan_destroy(p)


def test_version(lib):
    assert b'gfx950' in lib.cnf_version()


def test_fused_net_plan(lib):
    """k_net_lds covers every cfg2 coupling layer whose s,t net fits one CU's 160 KiB LDS image
    (all but the four 32x32 channel-mask layers); the debug option NETLDS=0 forces the streamed path."""
    kw = PRESETS['cfg2'].kwargs()
    kw.pop('group_mode')

    def fused(options=None):
        rc, p, keep = _plan(lib, kw, options=options)
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
    assert all(x[2] == 0 for x in fused('NETLDS=0'))


# every environment variable an earlier build of the library read (rounds 1-5): the library reads none now
OLD_KNOBS = ['CNF_CO_TAPMAX', 'CNF_FUSE_COUPLING', 'CNF_GC', 'CNF_GC_CONC', 'CNF_GC_GENERIC', 'CNF_GC_IPW',
             'CNF_GC_POLY', 'CNF_GC_POLY_NW', 'CNF_GC_TAPGROUP', 'CNF_GC_TAP_DMIN', 'CNF_GC_TH', 'CNF_LDSBWD_STAMPS',
             'CNF_LDS_BWD', 'CNF_LDS_SPLIT', 'CNF_LN2_MASK', 'CNF_LNR_FUSE', 'CNF_LN_MERGE', 'CNF_NETLDS',
             'CNF_NETLDS_DUMP', 'CNF_NETLDS_GENERIC', 'CNF_NETLDS_MAXHW', 'CNF_NETLDS_VERBOSE', 'CNF_NETLDS_WIDE',
             'CNF_OUT_LAW', 'CNF_OUT_LAW_KS', 'CNF_PW', 'CNF_PW_ALIGNED', 'CNF_PW_GENERIC', 'CNF_PW_IPW',
             'CNF_PW_IPW_RES', 'CNF_PW_SH', 'CNF_STAMPS', 'CNF_T1_COMPACT', 'CNF_T2_MAP', 'CNF_TAP_PW',
             'CNF_TBAND_ALLTAPS_KB', 'CNF_TBAND_MINWG', 'CNF_TCONV_BAND', 'CNF_TCONV_THIN', 'CNF_TRAIN_EVFLAGS',
             'CNF_TRAIN_INTERLEAVE', 'CNF_TRAIN_SAVE', 'CNF_TRAIN_VALU', 'CNF_TRAIN_WSTREAM', 'CNF_WGRAD_DIRECT',
             'CNF_WGRAD_THIN', 'CNF_WG_ABL']


def test_library_reads_no_environment():
    """Configuration is the plan descriptor's (debug_options), never the process environment: the
    library's sources name no getenv outside the -DCNF_DIAG diagnostic builds (the GPU test
    test_gpu_parity.py::test_old_knobs_change_nothing runs a forward with every old variable set)."""
    root = Path(__file__).resolve().parent.parent / 'arl_conditional_normalizing_flows_amd' / 'csrc'
    for f in sorted(root.glob('*.[ch]*')):
        depth = 0   # inside '#ifdef CNF_DIAG'
        for ln, line in enumerate(f.read_text().splitlines(), 1):
            t = line.strip()
            if t.startswith('#if'):
                depth = depth + 1 if (depth or 'CNF_DIAG' in t) else 0
            elif t.startswith('#endif') and depth:
                depth -= 1
            elif 'getenv' in t and not t.startswith('//'):
                assert depth > 0, f'{f.name}:{ln}: getenv outside a CNF_DIAG build: {t}'


def test_debug_options_are_validated(lib):
    kw = PRESETS['small'].kwargs()
    kw.pop('group_mode')
    for bad in ('NOPE=1', 'NETLDS', 'NETLDS=x', 'LDS_BWD=3'):
        rc, p, keep = _plan(lib, kw, options=bad)
        assert rc == -1 and not p.value, bad
        assert b'debug_options' in lib.cnf_last_error()
    rc, p, keep = _plan(lib, kw, options='NETLDS=0,GC=0,LAYOUT=3')
    assert rc == 0
    lib.cnf_plan_destroy(p)


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


def test_forward_rejects_aliased_xy_zy(lib):
    """cnf_flow_forward / _inverse / _forward_train are out-of-place (cnf.h): an aliased call is
    refused before anything is launched (so this runs without a GPU)."""
    kw = PRESETS['tiny'].kwargs()
    kw.pop('group_mode')
    rc, p, keep = _plan(lib, kw)
    assert rc == 0
    try:
        a, b = 1 << 40, 2 << 40   # never dereferenced
        assert lib.cnf_flow_forward(p, a, a, b, b, a, a, 2, None) == -1
        assert b'alias' in lib.cnf_last_error()
        assert lib.cnf_flow_inverse(p, a, a, b, b, a, 2, None) == -1
        assert lib.cnf_flow_forward_train(p, a, a, b, b, a, a, 2, None) == -1
        c = 3 << 40
        # the noisy-input forward: xy, xy_noisy and zy pairwise distinct
        assert lib.cnf_flow_forward_noise(p, a, a, b, 0.0, 0.98, 1, 0, b, c, a, a, 2, None) == -1
        assert lib.cnf_flow_forward_noise(p, a, a, b, 0.0, 0.98, 1, 0, c, c, a, a, 2, None) == -1
        assert lib.cnf_flow_forward_noise(p, a, a, b, 0.0, 0.98, 1, 0, c, b, a, a, 2, None) == -1
        assert b'alias' in lib.cnf_last_error()
        d = 4 << 40
        assert lib.cnf_flow_forward_noise(p, a, a, b, 0.7, 0.98, 1, 0, c, d, a, a, 2, None) == -1   # logit_a
        assert b'logit_a' in lib.cnf_last_error()
    finally:
        lib.cnf_plan_destroy(p)


@pytest.mark.parametrize('name', ['cfg2', 'cfg3', 'ref_default', 'cfg4', 'cfg5', 'small'])
def test_t1_layout_is_dense_per_consumer(lib, name):
    """Streamed layers store t1 as one sub-tensor per consumer (cnf_plan.cpp, Coupling::t1_map): every
    branch window starts 16-byte aligned with its sub-tensor's pixel stride, the per-channel store map
    agrees with the branch windows, exactly the channels the branches read are stored, and every
    (pixel, channel) of the image has its own float inside the image's t1_cs floats per pixel."""
    kw = PRESETS[name].kwargs()
    kw.pop('group_mode')
    rc, p, keep = _plan(lib, kw)
    assert rc == 0
    lib.cnf_debug_t1_layout.restype = C.c_int
    lib.cnf_debug_t1_layout.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.c_int]
    o = OracleCFlow(**kw)
    compact_seen = 0
    try:
        for c in o.coupling_specs:
            buf = (C.c_int * 512)()
            n = lib.cnf_debug_t1_layout(p, c.index, buf, 512)
            assert n >= 2
            w = list(buf[:n])
            compact, cs = w[0], w[1]
            nb = len(c.branches)
            br = [w[2 + 4 * i: 6 + 4 * i] for i in range(nb)]
            if not compact:
                assert cs == c.nk and all(b[0] == b[2] and b[1] == c.nk for b in br)
                continue
            compact_seen += 1
            tmap = np.array(w[2 + 4 * nb:2 + 4 * nb + 128]).reshape(64, 2)
            used = set()
            for off, pcs, cin_off, cin in br:
                assert off % 4 == 0 and pcs % 4 == 0 and 0 < cin <= pcs
                for ch in range(cin_off, cin_off + cin):
                    assert tuple(tmap[ch]) == (off + ch - cin_off, pcs)
                    used.add(ch)
            assert set(np.nonzero(tmap[:, 0] >= 0)[0].tolist()) == used
            hw = c.hc * c.wc
            idx = np.concatenate([tmap[ch, 0] + np.arange(hw) * tmap[ch, 1] for ch in sorted(used)])
            assert idx.min() >= 0 and idx.max() < hw * cs
            assert np.unique(idx).size == idx.size
    finally:
        lib.cnf_plan_destroy(p)
    if name in ('cfg2', 'cfg5'):
        assert compact_seen > 0


@pytest.mark.parametrize('name', ['cfg2', 'cfg4', 'cfg5', 'small'])
def test_t2_layout_is_dense_per_producer(lib, name):
    """When several launches produce t2 (cfg4 / cfg5), it holds one dense sub-tensor per producer
    (Coupling::t2_*): each branch's output slice has its own pixel stride, conv_b's quad map agrees
    with the slices, and every (pixel, channel) of the image has its own float among its t2_cs floats
    per pixel. cfg2's single k_gc group keeps the plain layout."""
    kw = PRESETS[name].kwargs()
    kw.pop('group_mode')
    rc, p, keep = _plan(lib, kw)
    assert rc == 0
    lib.cnf_debug_t2_layout.restype = C.c_int
    lib.cnf_debug_t2_layout.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.c_int]
    o = OracleCFlow(**kw)
    mapped = 0
    try:
        for c in o.coupling_specs:
            buf = (C.c_int * 512)()
            n = lib.cnf_debug_t2_layout(p, c.index, buf, 512)
            assert n >= 3
            w = list(buf[:n])
            m, cs, gc = w[:3]
            nb = len(c.branches)
            br = [w[3 + 4 * i:7 + 4 * i] for i in range(nb)]
            if not m:
                assert cs == gc and all(b[0] == b[2] and b[1] == gc for b in br)
                continue
            mapped += 1
            assert cs == gc
            q = np.array(w[3 + 4 * nb:3 + 4 * nb + 2 * (gc // 4)]).reshape(-1, 2)
            hw = c.hc * c.wc
            where = {}
            for off, pcs, out_off, cout in br:
                assert off % 4 == 0 and pcs % 4 == 0 and cout <= pcs
                for j in range(cout):
                    where[out_off + j] = (off + j, pcs)
            assert sorted(where) == list(range(gc))
            for qi in range(gc // 4):
                assert tuple(q[qi]) == where[4 * qi]
                assert all(where[4 * qi + k] == (where[4 * qi][0] + k, where[4 * qi][1]) for k in range(4))
            idx = np.concatenate([o_ + np.arange(hw) * s_ for o_, s_ in where.values()])
            assert idx.min() >= 0 and idx.max() < hw * cs and np.unique(idx).size == idx.size
    finally:
        lib.cnf_plan_destroy(p)
    assert (mapped > 0) == (name in ('cfg4', 'cfg5'))


def _schedule(lib, name, B, direction):
    lib.cnf_debug_schedule.restype = C.c_int
    lib.cnf_debug_schedule.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_char_p, C.c_int]
    kw = PRESETS[name].kwargs()
    lists = [(C.c_int * len(kw[k]))(*kw[k]) for k in ('squeeze_factor_block_list', 'ResNeXt_block_list',
                                                        'num_kernels_list', 'cardinality_list')]
    d = _lib.cnf_flow_desc(*kw['io_shape'], kw['x_d'], len(lists[0]), *lists, 100.0, 3, 1, 1, 0)
    p = C.c_void_p()
    assert lib.cnf_plan_create(C.byref(d), C.byref(p)) == 0
    try:
        buf = C.create_string_buffer(1 << 16)
        n = lib.cnf_debug_schedule(p, B, direction, buf, 1 << 16)
        assert n > 0, lib.cnf_last_error()
        names = buf.value.decode().split('\n')[:-1]
        assert len(names) == n
        return names
    finally:
        lib.cnf_plan_destroy(p)


@pytest.mark.parametrize('name', ['tiny', 'small', 'cfg2', 'cfg3', 'ref_default', 'cfg4', 'cfg5', 'narrow'])
def test_inverse_schedule_defers_like_the_forward(lib, name):
    """Host-only dry runs of the fused forward and inverse schedules (cnf_flow_forward / _inverse,
    conv_cINN_make_model.py:1723-1798): the inverse applies the deferred coupling law as the forward
    does (an LDS layer followed by an LDS layer or a block boundary launches no k_coupling), rebuilds
    each block boundary in one k_map2, and its last layer writes xy (no copy)."""
    from arl_conditional_normalizing_flows_amd.config import PRESETS as PR
    fwd = _schedule(lib, name, 3, 1)
    inv = _schedule(lib, name, 3, -1)
    assert 'copy' not in inv and 'k_map_scatter' not in inv
    nb = sum(PR[name].squeeze_factor_block_list)
    assert inv.count('k_map2') == nb and inv.count('k_map_gather') == 1
    assert fwd.count('k_map2') == nb + 1
    assert inv.count('k_net_lds') == fwd.count('k_net_lds')
    # expected k_coupling launches from the layer kinds (kind 0 coupling, 2 factor; fused_net = LDS layer):
    # a layer defers when it is an LDS layer whose successor (forward: next index; inverse: previous
    # index) is an LDS coupling or a block boundary; the forward's last layer may defer into the tail
    kw = PR[name].kwargs()
    kw.pop('group_mode')
    rc, p, keep = _plan(lib, kw)
    assert rc == 0
    info = _lib.cnf_layer_info()
    kinds = []
    try:
        for li in range(lib.cnf_plan_num_layers(p)):
            assert lib.cnf_plan_layer_info(p, li, C.byref(info)) == 0
            if info.kind != 1:   # squeezes are folded into the boundary maps
                kinds.append((info.kind, info.fused_net))
    finally:
        lib.cnf_plan_destroy(p)

    def launches(seq, tail_defers):
        n = 0
        for i, (k, lds) in enumerate(seq):
            if k != 0:
                continue
            nxt = seq[i + 1] if i + 1 < len(seq) else None
            defer = lds and ((nxt is None and tail_defers) or (nxt is not None and (nxt[0] == 2 or (nxt[0] == 0 and nxt[1]))))
            n += 0 if defer else 1
        return n
    assert fwd.count('k_coupling') == launches(kinds, True)
    assert inv.count('k_coupling') == launches(kinds[::-1], False)
