"""CPU: the oracle pinned by analytic known-answer invariants — the reference
ships no tests or golden vectors and cannot run here (TF absent), so these invariants are the
oracle's only pins ("parity unpinned" against the reference itself)."""
import numpy as np
import pytest

from oracle import cflow_np as O

TINY = dict(io_shape=[4, 4, 2], x_d=1, squeeze_factor_block_list=[0], ResNeXt_block_list=[1],
            num_kernels_list=[4], cardinality_list=[2])
TINY_SQ = dict(io_shape=[4, 4, 2], x_d=1, squeeze_factor_block_list=[1, 0], ResNeXt_block_list=[1, 1],
               num_kernels_list=[4, 4], cardinality_list=[2, 2])


def _flow(**kw):
    return O.OracleCFlow(**kw)


@pytest.mark.parametrize('kw', [TINY, TINY_SQ])
def test_roundtrip_f64(kw):
    m = _flow(**kw)
    P = m.init_params(1)
    rng = np.random.default_rng(0)
    xy = rng.standard_normal((3,) + tuple(kw['io_shape']))
    zy, ld = m.forward(xy, P)
    assert np.max(np.abs(m.inverse(zy, P) - xy)) < 1e-12


@pytest.mark.parametrize('kw', [TINY, TINY_SQ])
def test_logdet_equals_bruteforce_jacobian(kw):
    """log|det d zy / d xy| by central differences of the full map (f64) == sum of s."""
    m = _flow(**kw)
    P = m.init_params(2)
    rng = np.random.default_rng(1)
    x = rng.standard_normal((1,) + tuple(kw['io_shape']))
    n = x.size
    J = np.zeros((n, n))
    h = 1e-6
    for i in range(n):
        e = np.zeros(n)
        e[i] = h
        zp, _ = m.forward(x + e.reshape(x.shape), P)
        zm, _ = m.forward(x - e.reshape(x.shape), P)
        J[:, i] = (zp - zm).reshape(-1) / (2 * h)
    sign, logdet = np.linalg.slogdet(J)
    _, ld = m.forward(x, P)
    assert sign > 0
    assert abs(logdet - ld[0]) < 1e-6 * max(1.0, abs(logdet))


def test_zero_last_conv_is_identity():
    kw = dict(io_shape=[8, 8, 4], x_d=3, squeeze_factor_block_list=[0, 1, 0], ResNeXt_block_list=[1, 1, 1],
              num_kernels_list=[8, 8, 8], cardinality_list=[2, 2, 2])
    m = _flow(**kw)
    P = m.init_params(3, zero_last_conv=True)
    xy = np.random.default_rng(2).standard_normal((2, 8, 8, 4))
    zy, ld = m.forward(xy, P)
    assert np.array_equal(zy, xy)        # squeeze/factor/restore is the identity permutation
    assert np.all(ld == 0)


@pytest.mark.parametrize('sf', [[0, 1, 1, 0], [1, 1, 0], [0, 1], [1]])
def test_squeeze_factor_restore_is_identity_on_arange(sf):
    n = len(sf)
    kw = dict(io_shape=[16, 16, 2], x_d=1, squeeze_factor_block_list=sf, ResNeXt_block_list=[1] * n,
              num_kernels_list=[16] * n, cardinality_list=[2] * n)
    m = _flow(**kw)
    ar = np.arange(16 * 16 * 2, dtype=np.float64).reshape(1, 16, 16, 2)
    uv, zy = ar, None
    for e in m.sf_layers:
        uv, zy = (O.squeeze_forward(uv, zy) if e.kind == 'squeeze' else O.factor_forward(uv, zy))
    zy = np.concatenate([zy, uv], axis=3)
    vu = None
    for e in reversed(m.sf_layers):
        vu, zy = (O.factor_backward(vu, zy, e.num_prev_factors) if e.kind == 'factor'
                  else O.squeeze_backward(vu, zy))
    assert np.array_equal(vu, ar)
    assert sorted(np.concatenate([uv.ravel()]).tolist()) == sorted(set(uv.ravel().tolist()))


def test_space_to_depth_tf_order():
    """TF space_to_depth: out[b,i,j,(di*2+dj)*C+c] = in[b,2i+di,2j+dj,c] (!= pixel_unshuffle)."""
    x = np.arange(2 * 4 * 4 * 3).reshape(2, 4, 4, 3)
    y = O.space_to_depth(x)
    for i in range(2):
        for j in range(2):
            for di in range(2):
                for dj in range(2):
                    for c in range(3):
                        assert y[1, i, j, (di * 2 + dj) * 3 + c] == x[1, 2 * i + di, 2 * j + dj, c]
    assert np.array_equal(O.depth_to_space(y), x)


@pytest.mark.parametrize('m', [0, 1, 2, 3])
@pytest.mark.parametrize('D', [2, 3, 4])
def test_masks_partition(m, D):
    u = np.arange(2 * 4 * 6 * D, dtype=np.float64).reshape(2, 4, 6, D) + 1
    mc = {0: 1, 1: 0, 2: 3, 3: 2}[m]
    a = O.decompress(O.mask_compress(u, m), m, u.shape)
    b = O.decompress(O.mask_compress(u, mc), mc, u.shape)
    assert np.array_equal(a, O.mask_uncompressed(u, m))
    assert np.array_equal(a + b, u)
    assert np.count_nonzero(a * b) == 0


def test_group_modes_differ_only_with_cardinality():
    kw = dict(io_shape=[8, 8, 4], x_d=3, squeeze_factor_block_list=[0], ResNeXt_block_list=[1],
              num_kernels_list=[8], cardinality_list=[2])
    xy = np.random.default_rng(4).standard_normal((1, 8, 8, 4))
    r = _flow(**kw, group_mode='reference')
    i = _flow(**kw, group_mode='intended')
    P = r.init_params(5)
    assert [s for s in r.specs] == [s for s in i.specs]
    zr, _ = r.forward(xy, P)
    zi, _ = i.forward(xy, P)
    assert np.max(np.abs(zr - zi)) > 1e-6
    # closure quirk: every group reads the last slice
    c = r.coupling_specs[2]
    assert all(o == (c.card - 1) * c.branches[0].width for o in c.branches[0].in_offsets)


def test_schedule_matches_reference_comments():
    """Dilation schedule at 28x28 gives [1,2,4] (not [1,2,4,8] as conv_cINN.py:81 claims)."""
    m = _flow(io_shape=[28, 28, 2], x_d=1, squeeze_factor_block_list=[0, 1, 0, 0],
              ResNeXt_block_list=[3] * 4, num_kernels_list=[64, 64, 32, 32], cardinality_list=[8, 8, 4, 4])
    c0 = m.coupling_specs[0]
    assert c0.dilations == [1, 2, 4] and m.coupling_specs[2].dilations == [1, 2, 4]
    assert m.coupling_specs[8].H == 14 and m.coupling_specs[8].dilations == [1, 2]
    assert m.num_params() == 13113928


def test_reference_asserts():
    with pytest.raises(AssertionError, match='divisible by 2'):
        _flow(io_shape=[5, 4, 2], x_d=1, squeeze_factor_block_list=[0], ResNeXt_block_list=[1],
              num_kernels_list=[4], cardinality_list=[2])
    with pytest.raises(AssertionError, match='cardinality'):
        _flow(io_shape=[8, 8, 2], x_d=1, squeeze_factor_block_list=[0], ResNeXt_block_list=[1],
              num_kernels_list=[4], cardinality_list=[3])
    with pytest.raises(AssertionError, match='same length'):
        _flow(io_shape=[8, 8, 2], x_d=1, squeeze_factor_block_list=[0, 1], ResNeXt_block_list=[1],
              num_kernels_list=[4], cardinality_list=[2])


def test_nll_terms_definition():
    m = _flow(**TINY)
    xy = np.random.default_rng(6).standard_normal((2, 4, 4, 2))
    zy = np.random.default_rng(7).standard_normal((2, 4, 4, 2))
    llz, lly, _ = m.nll_terms(xy, zy, np.zeros(2))
    ref = [(-0.5 * zy[b, ..., :1] ** 2 - 0.5 * np.log(2 * np.pi)).sum() for b in range(2)]
    assert np.allclose(llz, ref)
    assert np.allclose(lly, [-100 * np.abs(zy[b, ..., 1:] - xy[b, ..., 1:]).sum() for b in range(2)])


def test_torch_cpu_baseline_matches_oracle():
    import torch
    from oracle.cflow_torch_cpu import TorchCPUFlow
    kw = dict(io_shape=[16, 16, 4], x_d=3, squeeze_factor_block_list=[0, 1, 0], ResNeXt_block_list=[2, 1, 1],
              num_kernels_list=[16, 16, 8], cardinality_list=[4, 4, 2])
    t = TorchCPUFlow(**kw)
    o = _flow(**kw)
    P = o.init_params(0)
    xy = O.synthetic_class_batch(2, 16, 16, 3, seed=1)
    ref = o.log_loss(xy, P)
    got = t.log_loss(torch.from_numpy(xy), {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in P.items()})
    for r, g in zip(ref, got):
        assert abs(r - float(g)) <= 1e-4 * max(1.0, abs(r))


def test_torch_cpu_float64_is_the_numpy_oracle():
    """The float64 torch-CPU restatement (the full-size parity oracle of the GPU tests) equals the
    numpy oracle: zy, per-image log-det and per-image sum|s| to float64 rounding."""
    import torch
    from oracle.cflow_torch_cpu import TorchCPUFlow
    from arl_conditional_normalizing_flows_amd.config import PRESETS
    for name in ('small', 'tiny'):
        kw = PRESETS[name].kwargs()
        o = _flow(**kw)
        P = o.init_params(2)
        H, W, D = PRESETS[name].io_shape
        xy = O.synthetic_class_batch(3, H, W, PRESETS[name].x_d, seed=4)
        zr, lr, ar = o.forward(xy, P, abs_s=True)
        t = TorchCPUFlow(**kw)
        with torch.no_grad():
            zt, st = t.forward(torch.from_numpy(xy).double(), {k: torch.from_numpy(np.asarray(v, np.float64))
                                                               for k, v in P.items()}, per_image=True)
        assert np.allclose(zt.numpy(), zr, rtol=0, atol=1e-11)
        assert np.allclose(st[0].numpy(), lr, rtol=0, atol=1e-10)
        assert np.allclose(st[1].numpy(), ar, rtol=0, atol=1e-10)
        assert np.all(ar >= np.abs(lr))


@pytest.mark.parametrize('B,H,W,x_d,seed', [(3, 8, 8, 1, 0), (5, 32, 32, 3, 7)])
def test_product_synthetic_batches_equal_the_oracle_generators(B, H, W, x_d, seed):
    """bench.py draws its inputs from the package's synthetic.py (the product never imports oracle/);
    the parity tests draw theirs from oracle/cflow_np.py. Same seeds, same bytes: the benched
    batches are exactly the distribution the parity tests cover."""
    from arl_conditional_normalizing_flows_amd import synthetic
    from oracle.cflow_np import synthetic_class_batch, synthetic_sr_batch
    assert np.array_equal(synthetic.class_batch(B, H, W, x_d, seed=seed), synthetic_class_batch(B, H, W, x_d, seed=seed))
    for p in (1, 2, 3):
        assert np.array_equal(synthetic.sr_batch(B, H, W, x_d, p, seed=seed), synthetic_sr_batch(B, H, W, x_d, p, seed=seed))


@pytest.mark.parametrize('name', ['tiny', 'small', 'cfg2'])
def test_torch_cpu_inverse_is_the_numpy_oracle(name):
    """oracle/cflow_torch_cpu.TorchCPUFlow.inverse (the CPU baseline of bench.py --mode inverse and the
    full-size inverse oracle) equals OracleCFlow.inverse in float64, and inverts the forward."""
    import torch
    from oracle.cflow_torch_cpu import TorchCPUFlow
    from arl_conditional_normalizing_flows_amd.config import PRESETS
    cfg = PRESETS[name]
    kw = cfg.kwargs()
    o, t = O.OracleCFlow(**kw), TorchCPUFlow(**kw)
    P = o.init_params(0)
    H, W, D = cfg.io_shape
    xy = O.synthetic_class_batch(2, H, W, cfg.x_d, seed=1)
    zy, _ = o.forward(xy, P)
    x1 = o.inverse(zy, P)
    x2 = t.inverse(torch.from_numpy(zy), {k: torch.from_numpy(np.asarray(v, np.float64)) for k, v in P.items()}).numpy()
    assert np.max(np.abs(x1 - x2)) <= 1e-12
    assert np.max(np.abs(x1 - xy)) <= 1e-12
