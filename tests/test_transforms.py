"""Input transforms (conv_cINN_base_functions.py:74-318, 635-676).

CPU: known-answer tests pinning the numpy oracle (oracle/transforms_np.py). GPU: the HIP kernels
through the C ABI (base_functions.py) against the oracle; tolerance 2e-6 relative (fp32 vs
float64) for the deterministic maps, distribution moments for the Philox normals."""
import numpy as np
import pytest
import torch

from oracle import transforms_np as T


# ---------------------------------------------------------------------------------------------
# CPU: the oracle
# ---------------------------------------------------------------------------------------------

def test_down_up_known_answers():
    x = np.arange(4 * 6 * 2, dtype=np.float64).reshape(4, 6, 2)
    d = T.down(x)
    assert d.shape == (2, 3, 2)
    # block (0, 0), channel 0: pixels (0,0)=0, (0,1)=2, (1,0)=12, (1,1)=14 -> mean 7
    assert d[0, 0, 0] == 7.0 and d[1, 2, 1] == np.mean([x[2, 4, 1], x[2, 5, 1], x[3, 4, 1], x[3, 5, 1]])
    u = T.up(d)
    assert u.shape == (4, 6, 2) and np.all(u[0:2, 0:2, 0] == 7.0)
    # odd sizes are cropped (:104-107)
    assert T.down(np.zeros((5, 7, 1))).shape == (2, 3, 1)
    # batched == per element
    xb = np.random.default_rng(0).random((3, 8, 8, 2))
    assert np.allclose(T.down(xb), np.stack([T.down(e) for e in xb]))


def test_logit_map_endpoints_and_inverse():
    a = 0.01
    x = np.linspace(0.0, 1.0, 101)
    y = T.logit_preprocess(x, a)
    assert abs(y[0]) < 1e-12 and abs(y[-1] - 1.0) < 1e-12        # [0, 1] -> [0, 1] (:218-224)
    assert np.all(np.diff(y) > 0)
    assert np.allclose(T.de_logitify(y, a), x, atol=1e-12)


def test_sr_preprocess_structure():
    h = np.random.default_rng(1).random((2, 16, 16, 3))
    xy = T.sr_preprocess(h, x_down=0, y_levels=1)               # 'SR2,1'
    assert xy.shape == (2, 16, 16, 6)
    assert np.allclose(xy[..., :3] + xy[..., 3:], h)            # RESIDUAL: x + y = hires
    assert np.allclose(xy[..., 3:], T.up(T.down(h)))
    xy42 = T.sr_preprocess(h, x_down=1, y_levels=1)             # 'SR4,2'
    assert np.allclose(xy42[..., 3:], T.up(T.down(T.down(h))))
    assert np.allclose(xy42[..., :3] + xy42[..., 3:], T.down(h))
    xy4 = T.sr_preprocess(h, x_down=0, y_levels=2)              # the 4x benchmark config
    assert np.allclose(xy4[..., 3:], T.up(T.up(T.down(T.down(h)))))


def test_capi_rejects_bad_transform_arguments(lib):
    assert lib.cnf_logit(1, 1, 4, 0.7, 0, None) == -1            # a outside (0, 0.5)
    assert lib.cnf_sr_preprocess(1, 1, 1, 6, 6, 1, 0, 2, 1, None) == -1   # 6 not divisible by 4
    assert b'divisible' in lib.cnf_last_error()


# ---------------------------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------------------------

def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-30, np.max(np.abs(b))))


@pytest.mark.gpu
def test_down_up_match_oracle(gpu):
    from arl_conditional_normalizing_flows_amd import base_functions as F
    x = np.random.default_rng(2).random((3, 10, 14, 5)).astype(np.float32)
    xt = torch.from_numpy(x).to(gpu)
    assert _rel(F.down(xt).cpu().numpy(), T.down(x.astype(np.float64))) < 2e-6
    assert np.array_equal(F.up(xt).cpu().numpy(), T.up(x))
    assert F.down(xt[0]).shape == (5, 7, 5)                     # unbatched element, cropped


@pytest.mark.gpu
@pytest.mark.parametrize('a', [0.01, 0.05])
def test_logit_matches_oracle(gpu, a):
    from arl_conditional_normalizing_flows_amd import base_functions as F
    x = np.random.default_rng(3).random((4, 32, 32, 3)).astype(np.float32)
    x[0, 0, 0] = [0.0, 1.0, 0.5]
    xt = torch.from_numpy(x).to(gpu)
    y = F.preprocess_dataset_class(xt, LOGITS=True, a=a)
    ref = T.logit_preprocess(x.astype(np.float64), a)
    assert float(np.max(np.abs(y.cpu().numpy() - ref))) < 2e-6
    back = F.de_logitify(y, a).cpu().numpy()
    assert float(np.max(np.abs(back - x))) < 1e-5
    assert F.preprocess_dataset_class(xt, LOGITS=False) is not None


@pytest.mark.gpu
@pytest.mark.parametrize('model_type,y_levels,H', [('SR2,1', None, 32), ('SR4,2', None, 32), ('SR2,1', 2, 32),
                                                   ('SR2,1', 3, 64)])
def test_sr_preprocess_matches_oracle(gpu, model_type, y_levels, H):
    from arl_conditional_normalizing_flows_amd import base_functions as F
    h = np.random.default_rng(4).random((2, H, H, 3)).astype(np.float32)
    xd, yl = {'SR2,1': (0, 1), 'SR4,2': (1, 1)}[model_type]
    yl = y_levels if y_levels is not None else yl
    for residual in (True, False):
        xy = F.preprocess_dataset_SR(torch.from_numpy(h).to(gpu), model_type, residual, y_levels=y_levels)
        ref = T.sr_preprocess(h.astype(np.float64), xd, yl, residual)
        assert xy.shape == ref.shape
        assert float(np.max(np.abs(xy.cpu().numpy() - ref))) < 2e-6


@pytest.mark.gpu
def test_instance_noise_formula_and_moments(gpu):
    from arl_conditional_normalizing_flows_amd import base_functions as F
    n = 1 << 20
    x = torch.rand(n, device=gpu)
    z = F.renew_noise(x, seed=7).cpu().numpy().astype(np.float64)
    assert abs(z.mean()) < 5e-3 and abs(z.std() - 1.0) < 5e-3
    assert abs(np.mean(z ** 3)) < 1e-2 and abs(np.mean(z ** 4) - 3.0) < 3e-2     # skew 0, kurtosis 3
    # same (seed, offset) -> same normals; alpha mixes exactly as the reference formula (:652)
    y = F.instance_noise(x, 0.98, seed=7).cpu().numpy().astype(np.float64)
    ref = 0.98 * x.cpu().numpy().astype(np.float64) + 0.02 * z
    assert float(np.max(np.abs(y - ref))) < 1e-6
    assert np.array_equal(F.instance_noise(x, 1.0, seed=3).cpu().numpy(), x.cpu().numpy())
    # counter-based: a suffix starting at offset k equals the tail of the full stream
    tail = F.renew_noise(x[:1000], seed=7, offset=n - 1000).cpu().numpy().astype(np.float64)
    assert np.array_equal(tail, z[-1000:])
    assert not np.array_equal(F.renew_noise(x, seed=8).cpu().numpy()[:64], z[:64].astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize('name,B,logit_a', [('cfg2', 3, 0.0), ('cfg2', 2, 0.01), ('small', 2, 0.05), ('cfg4', 1, 0.0),
                                            ('cfg4', 1, 0.01)])
def test_noise_fused_into_the_forward(gpu, name, B, logit_a):
    """cnf_flow_forward_noise (cFlow.call(noise=...)): the input as the reference's training pipeline
    prepares it (conv_cINN.py:246-315) -- the logit map on the x channels (logit_a > 0,
    conv_cINN_base_functions.py:174-231), then the 2 % instance noise (:635-654) -- applied inside the
    first coupling layer's k_net_lds gather (cfg2, small: no pass over xy; cfg4's first layer is
    streamed: one k_prep pass first). The prepared input equals cnf_logit (x channels) followed by the
    standalone cnf_instance_noise stream bit for bit, zy / log-det equal cnf_flow_forward of it bit for
    bit, the loss is that of the prepared input, the logit map matches the numpy oracle, and zy matches
    the float64 oracle composed with the prepared input."""
    from arl_conditional_normalizing_flows_amd.base_functions import instance_noise, preprocess_dataset_class
    from arl_conditional_normalizing_flows_amd.config import PRESETS
    from arl_conditional_normalizing_flows_amd.make_model import cFlow
    from oracle.cflow_np import OracleCFlow, synthetic_class_batch
    cfg = PRESETS[name]
    kw = cfg.kwargs()
    flow = cFlow(**kw, device=gpu)
    ora = OracleCFlow(**kw)
    P = ora.init_params(2)
    flow.set_weights(P)
    H, W, _ = cfg.io_shape
    xy = synthetic_class_batch(B, H, W, cfg.x_d, seed=4)
    if logit_a:   # the logit map takes the raw images in [0, 1] (the pipeline's noise comes after it)
        xy[..., :cfg.x_d] = np.clip(xy[..., :cfg.x_d], 0.0, 1.0)
    x = torch.from_numpy(xy).to(gpu)
    noise = (0.98, 1234567, 99, logit_a)
    zy, ld, xn = flow(x, 1, per_image_logdet=True, noise=noise)
    xp = x
    if logit_a:
        xl = preprocess_dataset_class(x[..., :cfg.x_d], LOGITS=True, a=logit_a)
        xl_np = T.logit_preprocess(x[..., :cfg.x_d].cpu().double().numpy(), logit_a)
        assert np.max(np.abs(xl.cpu().numpy() - xl_np)) < 2e-6
        xp = torch.cat([xl, x[..., cfg.x_d:]], dim=-1).contiguous()
    xn_ref = instance_noise(xp, *noise[:3])
    zy_ref, ld_ref = flow(xn_ref, 1, per_image_logdet=True)
    lf = flow.log_loss(x, noise=noise)
    lr = flow.log_loss(xn_ref)
    torch.cuda.synchronize()
    assert torch.equal(xn, xn_ref)
    assert torch.equal(zy, zy_ref) and torch.equal(ld, ld_ref)
    assert all(torch.equal(a, b) for a, b in zip(lf, lr))
    assert not torch.equal(xn, x)
    z64, l64, abs_s = ora.forward(xn.cpu().double().numpy(), P, abs_s=True)
    e = np.max(np.abs(zy.cpu().numpy() - z64)) / np.max(np.abs(z64))
    assert e < 1e-5, e
    assert np.all(np.abs(ld.cpu().numpy() - l64) <= 1e-5 * np.maximum(np.abs(l64), abs_s))
