"""Golden fixtures (tests/golden/make_golden.py): the oracle reproduces them (CPU) and the HIP
path through the C ABI matches them within the north-star tolerance (GPU).

Parity note: the fixtures come from the numpy restatement; the TensorFlow reference cannot run
here and holds no vectors of its own, so parity is pinned by the oracle's
invariant KATs (tests/test_oracle.py), not by reference outputs."""
import glob
import os

import numpy as np
import pytest

from arl_conditional_normalizing_flows_amd.config import PRESETS
from oracle.cflow_np import OracleCFlow, flatten_params

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
FILES = sorted(f for f in glob.glob(os.path.join(HERE, '*.npz')) if not f.endswith('toy_cinn.npz'))
TOY = os.path.join(HERE, 'toy_cinn.npz')
RTOL = 1e-5


def _load(path):
    g = dict(np.load(path, allow_pickle=False))
    name, gm = str(g['name']), str(g['group_mode'])
    kw = PRESETS[name].kwargs()
    kw['group_mode'] = gm
    ora = OracleCFlow(**kw)
    if 'params' in g:
        flat = g['params']
    else:
        P = ora.init_params(int(g['seed']))
        flat = flatten_params({k: np.asarray(v, np.float32) for k, v in P.items()}, ora.specs).astype(np.float32)
    assert flat.size == int(g['n_params'])
    assert np.array_equal(flat[:16], g['params_head'])
    assert abs(flat.astype(np.float64).sum() - float(g['params_sum'])) <= 1e-9 * max(1.0, abs(float(g['params_sum'])))
    assert abs((flat.astype(np.float64) ** 2).sum() - float(g['params_sumsq'])) <= 1e-9 * float(g['params_sumsq'])
    P32, o = {}, 0
    for n, s in ora.specs:
        size = int(np.prod(s)) if s else 1
        P32[n] = flat[o:o + size].reshape(s)
        o += size
    return g, kw, ora, P32, flat


def test_fixtures_present():
    assert len(FILES) >= 4


@pytest.mark.parametrize('path', FILES, ids=[os.path.basename(f) for f in FILES])
def test_oracle_reproduces_golden(path):
    g, kw, ora, P32, _ = _load(path)
    zy, ld = ora.forward(g['xy'].astype(np.float64), P32)
    assert np.allclose(zy, g['zy'], rtol=0, atol=1e-10)
    assert np.allclose(ld, g['logdet'], rtol=0, atol=1e-9)
    x = ora.inverse(g['zy_in'].astype(np.float64), P32)
    assert np.allclose(x, g['x_out'], rtol=0, atol=1e-10)
    assert np.allclose(np.array(ora.log_loss(g['xy'].astype(np.float64), P32)), g['nll'], rtol=1e-12, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize('path', FILES, ids=[os.path.basename(f) for f in FILES])
def test_hip_matches_golden(gpu, path):
    import torch
    from arl_conditional_normalizing_flows_amd.make_model import cFlow
    g, kw, ora, P32, flat = _load(path)
    flow = cFlow(**kw)
    flow.set_weights(flat)
    xy = torch.from_numpy(g['xy']).to(gpu)
    zy, ld = flow(xy, 1, per_image_logdet=True)
    x = flow(torch.from_numpy(g['zy_in']).to(gpu), -1)
    nll = [t.item() for t in flow.log_loss(xy)]
    torch.cuda.synchronize()
    zr = g['zy']
    # per-image log-det bound 1e-5 * max(|ref|, sum|s|) (north star; sum|s| from the oracle on the
    # fixture's own weights and inputs)
    _, _, abs_s = ora.forward(g['xy'].astype(np.float64), P32, abs_s=True)
    tol = RTOL * np.maximum(np.abs(g['logdet']), abs_s)
    assert np.max(np.abs(zy.cpu().numpy() - zr)) <= RTOL * np.max(np.abs(zr))
    assert np.all(np.abs(ld.cpu().numpy() - g['logdet']) <= tol)
    assert np.max(np.abs(x.cpu().numpy() - g['x_out'])) <= RTOL * np.max(np.abs(g['x_out']))
    for r, v in zip(g['nll'], nll):
        assert abs(r - v) <= RTOL * max(abs(r), abs_s.mean())


def _toy():
    from oracle.toy_np import ToyCINN
    g = dict(np.load(TOY, allow_pickle=False))
    ora = ToyCINN(io_shape=3, x_d=2, num_coupling_layers=int(g['num_coupling_layers']),
                  intermediate_dims=int(g['intermediate_dims']), num_layers=int(g['num_layers']),
                  mask_indices=[int(v) for v in g['mask_indices']])
    P, o = {}, 0
    for n, s in ora.specs:
        size = int(np.prod(s))
        P[n] = g['params'][o:o + size].reshape(s)
        o += size
    assert o == g['params'].size
    return g, ora, P


def test_toy_oracle_reproduces_golden():
    g, ora, P = _toy()
    zy, ld = ora.call(g['xy'], P, -1)
    assert np.allclose(zy, g['zy'], rtol=0, atol=1e-10) and np.allclose(ld, g['logdet'], rtol=0, atol=1e-10)
    xb, _ = ora.call(g['zy'], P, 1)
    assert np.allclose(xb, g['x_back'], rtol=0, atol=1e-10)
    assert np.allclose(np.array(ora.log_loss(g['xy'], P)), g['nll'], rtol=1e-12, atol=1e-9)


@pytest.mark.gpu
def test_toy_hip_matches_golden(gpu):
    import torch
    from arl_conditional_normalizing_flows_amd.toy_model import cINN_affine
    g, ora, P = _toy()
    m = cINN_affine(3, 2, ora.L, ora.H, ora.num_layers, mask_indices=ora.mask_indices, device=gpu)
    m.set_weights(g['params'])
    zy, ld = m.call(torch.from_numpy(g['xy']).to(gpu), -1)
    torch.cuda.synchronize()
    assert np.max(np.abs(zy.cpu().numpy() - g['zy'])) <= RTOL * np.max(np.abs(g['zy']))
    # per-sample log-det at the north-star bound 1e-5 * max(|ref|, sum|A|) (sum over the 24 layers of
    # |A|, from the oracle on the fixture's weights and inputs)
    _, ld_ref, abs_a = ora.call(g['xy'], P, -1, abs_s=True)
    assert np.allclose(ld_ref, g['logdet'], rtol=0, atol=1e-10)
    tol = RTOL * np.maximum(np.abs(g['logdet']), abs_a)
    err = np.abs(ld.cpu().numpy().astype(np.float64) - g['logdet'])
    print(f'toy logdet: max abs err {err.max():.2e}, worst err/tol {np.max(err / tol):.3f}')
    assert np.all(err <= tol)
