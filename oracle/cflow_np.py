"""TEST INFRASTRUCTURE ONLY — numpy restatement of the reference `cFlow` hot path.

This is the checker for the MI355X product path (parity unpinned against the
reference itself: TensorFlow is absent here, see oracle/__init__.py). It
restates, in float64 (default) or float32:

* the model schedule of `cFlow.__init__`         conv_cINN_make_model.py:1431-1695
* the compressed checkerboard / channel masks   conv_cINN_make_model.py:474-761
* the decompress scatter                         conv_cINN_make_model.py:763-1073
* the ResNeXt s,t networks                       conv_cINN_make_model.py:1076-1213,
                                                 conv_cINN_base_functions.py:330-413,501-627
* the affine coupling law + batch-mean log-det   conv_cINN_make_model.py:1215-1394
* squeeze / factor-out layers                    conv_cINN_make_model.py:130-329
* `cFlow.call` both directions                   conv_cINN_make_model.py:1723-1798
* `cFlow.log_loss` (NLL 4-tuple)                 conv_cINN_make_model.py:1800-1848

Keras/TF semantics the reference relies on but does not spell out:
LeakyReLU() alpha = 0.3; LayerNormalization() epsilon = 1e-3, biased variance,
per-element gamma/beta over the flattened axis; Conv2D HWIO kernels, cross-
correlation, bias, 'same' padding = (k-1)*d split floor/ceil; space_to_depth
order out[b,i,j,(di*2+dj)*C+c] = in[b,2i+di,2j+dj,c];
MultivariateNormalDiag(0, I).log_prob(z) = -0.5|z|^2 - (x_d/2) ln(2 pi).

The grouped-convolution closure quirk (conv_cINN_base_functions.py:402):
`Lambda(lambda z: z[..., j*_d:j*_d+_d])` binds `j` late, and a Keras functional
model re-runs each Lambda's Python function on every call, so at call time every
group of a grouped convolution reads the LAST slice [(card-1)*_d, card*_d).
`group_mode='reference'` (default) reproduces that; `group_mode='intended'`
gives the textbook grouped convolution (group j reads slice j).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

LRELU_ALPHA = 0.3          # keras.layers.LeakyReLU() default
LN_EPS = 1e-3              # keras.layers.LayerNormalization() default
LOG_2PI = math.log(2.0 * math.pi)


# ----------------------------------------------------------------------------
# schedule (conv_cINN_make_model.py:1431-1695)
# ----------------------------------------------------------------------------

@dataclass
class GroupBranch:
    dilation: int          # the (float) dilation factor, integral valued
    width: int             # _d = int((nk // d) // card)   (base_functions.py:397)
    out_off: int           # channel offset of this branch inside the concat
    in_offsets: List[int]  # per group: first input channel read


@dataclass
class CouplingSpec:
    index: int             # coupling-layer ordinal (0..n_coupling-1)
    block: int
    H: int
    W: int
    D: int
    mask: int
    mask_c: int            # complement mask
    hc: int                # compressed height / width / depth of u1c
    wc: int
    dc1: int               # uv1_d
    dc2: int               # uv2_d
    nk: int                # kernels (halved for checkerboard masks :420-423)
    card: int
    R: int
    dilations: List[int]
    branches: List[GroupBranch] = field(default_factory=list)
    gc_channels: int = 0   # concat width of the grouped stage


@dataclass
class LayerEntry:
    kind: str                      # 'coupling' | 'squeeze' | 'factor'
    coupling: Optional[CouplingSpec] = None
    num_prev_factors: int = 0      # factor layers only
    shape: Tuple[int, int, int] = (0, 0, 0)   # block io shape the layer was built for


def _dilations_for_block(h: int, w: int, ksize: int):
    """conv_cINN_make_model.py:1553-1610, float arithmetic preserved."""
    cw, cb = [], []
    min_cw = min(h, w)
    min_cb = min_cw / 2
    d = 1
    dk = ksize
    if dk > (min_cw + 1) / 2:
        cw.append(d)
        cb.append(d)
    else:
        sanity = 0
        while dk < (min_cw + 1) / 2:
            assert sanity < 10, 'dilation while loop ran unexpectedly many iterations'
            cw.append(d)
            if d < (min_cb + 1) / 2:
                cb.append(d)
            dk = (ksize - 1) * (dk - 1) + 1
            d = ((dk - ksize) / (ksize - 1)) + 1
            sanity += 1
    return cw, cb


def build_schedule(io_shape: Sequence[int], x_d: int,
                   squeeze_factor_block_list: Sequence[int],
                   ResNeXt_block_list: Sequence[int],
                   num_kernels_list: Sequence[int],
                   cardinality_list: Sequence[int],
                   ksize: int = 3, LAYER_NORM: bool = True, DILATIONS: bool = True,
                   group_mode: str = 'reference') -> List[LayerEntry]:
    """Restates cFlow.__init__ (conv_cINN_make_model.py:1431-1695)."""
    sfbl = list(squeeze_factor_block_list)
    assert len(sfbl) == len(ResNeXt_block_list) == len(num_kernels_list) == len(cardinality_list), \
        'squeeze_factor_block_list, ResNeXt_block_list, num_kernels_list, and cardinality_list must all have the same length.'
    assert not io_shape[0] % 2 and not io_shape[1] % 2, \
        'The model input and output must have spatial dimensions divisible by 2.'
    for nk in num_kernels_list:
        assert not nk % 2, 'The number of kernels in each layer must be divisible by 2.'
    for c in cardinality_list:
        assert not c % 2, 'The cardinality in each layer must be divisible by 2.'
    for s in sfbl:
        assert s in [0, 1], 'The only allowed entries in squeeze_factor_block_list are 0 and 1.'
    if group_mode not in ('reference', 'intended'):
        raise ValueError(f'unknown group_mode {group_mode!r}')

    nb = len(sfbl)
    scale_list, npf_list = [], []          # :1493-1518
    scale_flag, npf = 0, 0
    for i in range(nb):
        s = 0 if i == 0 else sfbl[i - 1]
        if not scale_flag:
            scale_list.append(1)
            scale_flag = 1
        else:
            scale_list.append(2 ** s * scale_list[-1])
        npf += s
        npf_list.append(npf)

    io_list = []                            # :1521-1536
    for i in range(nb):
        sc = scale_list[i]
        assert not io_shape[0] % (sc * 2) and not io_shape[1] % (sc * 2), \
            f'The cumulative scale must divide evenly into the i/o spatial dimensions (block {i}).'
        io_list.append((int(io_shape[0] / sc), int(io_shape[1] / sc), io_shape[2] * sc))

    dil_list = []
    if DILATIONS:
        for (h, w, _) in io_list:
            cw, cb = _dilations_for_block(h, w, ksize)
            dil_list.append({'channelwise': cw, 'checkerboard': cb})
        for i in range(nb):                 # :1613-1617
            nkc = num_kernels_list[i] / cardinality_list[i]
            for d in dil_list[i]['channelwise']:
                assert not nkc % d, \
                    f'The ratio (number of kernels / cardinality) must be evenly divisible by each dilation factor used in that coupling block. This failed in coupling block {i}.'
    else:
        # DILATIONS=False never sets self.dilations_list in the reference (it
        # would raise AttributeError at :1643). We use the undilated branch [1],
        # the only meaningful reading, and document the divergence.
        dil_list = [{'channelwise': [1], 'checkerboard': [1]} for _ in range(nb)]

    layers: List[LayerEntry] = []
    ci = 0
    for i in range(nb):
        h, w, d_ = io_list[i]
        for m in (0, 1, 2, 3):              # :1545-1550, :1639-1663
            dils = dil_list[i]['checkerboard'] if m in (0, 1) else dil_list[i]['channelwise']
            cs = _coupling_spec(ci, i, h, w, d_, m, num_kernels_list[i], cardinality_list[i],
                                ResNeXt_block_list[i], dils, group_mode)
            layers.append(LayerEntry('coupling', coupling=cs, shape=(h, w, d_)))
            ci += 1
        if sfbl[i] == 1:                    # :1666-1689
            layers.append(LayerEntry('squeeze', shape=(h, w, d_)))
            layers.append(LayerEntry('factor', num_prev_factors=npf_list[i], shape=(h, w, d_)))
    return layers


def _coupling_spec(index, block, H, W, D, mask, num_kernels, card, R, dils, group_mode):
    """coupling_layer.__init__ + get_masked_compressed_shape + coupling_function
    shapes (conv_cINN_make_model.py:355-439, 474-498, 1087-1104)."""
    assert H % 2 == 0 and W % 2 == 0, 'u/v must have spatial dimensions divisible by 2.'
    nk = int(num_kernels / 2) if mask in (0, 1) else num_kernels
    mask_c = {0: 1, 1: 0, 2: 3, 3: 2}[mask]
    if mask in (0, 1):
        hc, wc, dc1 = H // 2, W // 2, 2 * D
    else:
        hc, wc = H, W
        dc1 = int(math.ceil(D / 2)) if mask == 2 else int(math.floor(D / 2))
    if D % 2 and mask == 2:
        dc2 = dc1 - 1
    elif D % 2 and mask == 3:
        dc2 = dc1 + 1
    else:
        dc2 = dc1
    spec = CouplingSpec(index=index, block=block, H=H, W=W, D=D, mask=mask, mask_c=mask_c,
                        hc=hc, wc=wc, dc1=dc1, dc2=dc2, nk=nk, card=card, R=R,
                        dilations=[int(d) for d in dils])
    # grouped convolution geometry (base_functions.py:575-601, 364-413)
    off = 0
    for d in dils:
        nb_ch = nk // d                       # float when d is a float (2.0, 4.0 ...)
        if card == 1:
            width = int(nb_ch)
            ins = [0]
            n_out = width
        else:
            assert not nb_ch % card
            width = int(nb_ch // card)
            if width == 0:
                raise ValueError(f'zero-width group: nk={nk}, dilation={d}, cardinality={card} '
                                 f'(the reference would build a 0-filter Conv2D here)')
            if group_mode == 'reference':
                ins = [(card - 1) * width] * card   # late-bound closure: all groups read the last slice
            else:
                ins = [j * width for j in range(card)]
            n_out = card * width
        spec.branches.append(GroupBranch(dilation=int(d), width=width, out_off=off, in_offsets=ins))
        off += n_out
    spec.gc_channels = off
    return spec


# ----------------------------------------------------------------------------
# parameters (canonical Keras layouts: Conv2D kernel HWIO, LN gamma/beta (H*W*C,))
# ----------------------------------------------------------------------------

def param_specs(layers: List[LayerEntry], ksize: int = 3, LAYER_NORM: bool = True):
    """Ordered (name, shape) list. Per coupling layer: net A then net b
    (model_A, model_b of coupling_function :1208-1213); within a net the Keras
    layer creation order of coupling_function / dilated_residual_block."""
    specs = []
    k = ksize
    for e in layers:
        if e.kind != 'coupling':
            continue
        c = e.coupling
        for net in ('A', 'b'):
            p = f'c{c.index}.{net}'
            specs.append((f'{p}.conv_in.kernel', (k, k, c.dc1, c.nk)))
            specs.append((f'{p}.conv_in.bias', (c.nk,)))
            n_hw = c.hc * c.wc
            for r in range(c.R):
                q = f'{p}.rb{r}'
                if LAYER_NORM:
                    specs.append((f'{q}.ln1.gamma', (n_hw * c.nk,)))
                    specs.append((f'{q}.ln1.beta', (n_hw * c.nk,)))
                specs.append((f'{q}.conv_a.kernel', (1, 1, c.nk, c.nk)))
                specs.append((f'{q}.conv_a.bias', (c.nk,)))
                if LAYER_NORM:
                    specs.append((f'{q}.ln2.gamma', (n_hw * c.nk,)))
                    specs.append((f'{q}.ln2.beta', (n_hw * c.nk,)))
                for bi, br in enumerate(c.branches):
                    for j in range(len(br.in_offsets)):
                        specs.append((f'{q}.gc.d{bi}.g{j}.kernel', (k, k, br.width, br.width)))
                        specs.append((f'{q}.gc.d{bi}.g{j}.bias', (br.width,)))
                if LAYER_NORM:
                    specs.append((f'{q}.ln3.gamma', (n_hw * c.gc_channels,)))
                    specs.append((f'{q}.ln3.beta', (n_hw * c.gc_channels,)))
                specs.append((f'{q}.conv_b.kernel', (1, 1, c.gc_channels, c.nk)))
                specs.append((f'{q}.conv_b.bias', (c.nk,)))
            if LAYER_NORM:
                specs.append((f'{p}.ln_out.gamma', (n_hw * c.nk,)))
                specs.append((f'{p}.ln_out.beta', (n_hw * c.nk,)))
            specs.append((f'{p}.conv_out.kernel', (k, k, c.nk, c.dc2)))
            specs.append((f'{p}.conv_out.bias', (c.dc2,)))
            if net == 'A':
                specs.append((f'{p}.tanh_scale.w', ()))
    return specs


def _orthogonal(rng, shape, gain):
    """keras.initializers.Orthogonal restated (QR of a normal matrix, sign fix)."""
    n_rows = int(np.prod(shape[:-1])) if len(shape) > 1 else 1
    n_cols = shape[-1]
    flat = (max(n_cols, n_rows), min(n_cols, n_rows))
    a = rng.standard_normal(flat)
    q, r = np.linalg.qr(a)
    q = q * np.sign(np.diag(r))
    if n_rows < n_cols:
        q = q.T
    return (gain * q).reshape(shape)


def init_params(specs, seed: int = 0, kernel_gain: float = 0.1, perturb: bool = True,
                zero_last_conv: bool = False) -> Dict[str, np.ndarray]:
    """Seeded synthetic weights: conv kernels orthogonal*0.1;
    every other kind perturbed from its Keras init so that each parameter
    kind is exercised: bias~N(0,.01), gamma=1+N(0,.1), beta~N(0,.1), w=1+N(0,.1)."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in specs:
        if name.endswith('.kernel'):
            if zero_last_conv and '.conv_out.' in name:
                v = np.zeros(shape)
            else:
                v = _orthogonal(rng, shape, kernel_gain)
        elif name.endswith('.bias'):
            v = rng.normal(0, 0.01, shape) if perturb else np.zeros(shape)
            if zero_last_conv and '.conv_out.' in name:
                v = np.zeros(shape)
        elif name.endswith('.gamma'):
            v = 1.0 + rng.normal(0, 0.1, shape) if perturb else np.ones(shape)
        elif name.endswith('.beta'):
            v = rng.normal(0, 0.1, shape) if perturb else np.zeros(shape)
        elif name.endswith('.w'):
            v = np.asarray(1.0 + rng.normal(0, 0.1)) if perturb else np.asarray(1.0)
        else:
            raise KeyError(name)
        out[name] = np.asarray(v, dtype=np.float64)
    return out


def flatten_params(params: Dict[str, np.ndarray], specs) -> np.ndarray:
    return np.concatenate([np.asarray(params[n], np.float64).reshape(-1) for n, _ in specs])


# ----------------------------------------------------------------------------
# elementary ops
# ----------------------------------------------------------------------------

def leaky_relu(x):
    return np.where(x >= 0, x, LRELU_ALPHA * x)


def layer_norm_hwc(x, gamma, beta):
    """Reshape((H*W*C,)) -> LayerNormalization(axis=-1) -> Reshape
    (conv_cINN_base_functions.py:350-360): per-image stats, per-element affine."""
    B = x.shape[0]
    flat = x.reshape(B, -1)
    mu = flat.mean(axis=1, keepdims=True)
    var = ((flat - mu) ** 2).mean(axis=1, keepdims=True)
    y = (flat - mu) / np.sqrt(var + LN_EPS) * gamma.reshape(1, -1) + beta.reshape(1, -1)
    return y.reshape(x.shape)


def add_common_layers(y, ln, gamma=None, beta=None):
    """conv_cINN_base_functions.py:330-362 (dropout off)."""
    y = leaky_relu(y)
    if ln:
        y = layer_norm_hwc(y, gamma, beta)
    return y


def conv2d_same(x, kernel, bias, dilation=1):
    """Keras Conv2D(padding='same', dilation_rate=d), HWIO kernel, NHWC."""
    kh, kw, ci, co = kernel.shape
    B, H, W, C = x.shape
    assert C == ci, (C, ci)
    ph, pw = (kh - 1) * dilation, (kw - 1) * dilation
    pt, pl = ph // 2, pw // 2
    xp = np.pad(x, ((0, 0), (pt, ph - pt), (pl, pw - pl), (0, 0)))
    out = np.zeros((B, H, W, co), dtype=x.dtype)
    for i in range(kh):
        for j in range(kw):
            out += xp[:, i * dilation:i * dilation + H, j * dilation:j * dilation + W, :] @ kernel[i, j]
    return out + bias


def space_to_depth(x):
    B, H, W, C = x.shape
    return x.reshape(B, H // 2, 2, W // 2, 2, C).transpose(0, 1, 3, 2, 4, 5).reshape(B, H // 2, W // 2, 4 * C)


def depth_to_space(x):
    B, H, W, C4 = x.shape
    C = C4 // 4
    return x.reshape(B, H, W, 2, 2, C).transpose(0, 1, 3, 2, 4, 5).reshape(B, 2 * H, 2 * W, C)


_CB = {0: ((0, 0), (1, 1)), 1: ((0, 1), (1, 0))}   # (row, col) offsets of halves c0, c1


def mask_compress(u, m):
    """coupling_layer.mask(compress=True) :720-759."""
    if m in (0, 1):
        (r0, c0), (r1, c1) = _CB[m]
        return np.concatenate([u[:, r0::2, c0::2, :], u[:, r1::2, c1::2, :]], axis=-1)
    return u[..., 0::2] if m == 2 else u[..., 1::2]


def mask_uncompressed(u, m):
    """coupling_layer.mask(compress=False) :632-717 (u * M)."""
    out = np.zeros_like(u)
    if m in (0, 1):
        (r0, c0), (r1, c1) = _CB[m]
        out[:, r0::2, c0::2, :] = u[:, r0::2, c0::2, :]
        out[:, r1::2, c1::2, :] = u[:, r1::2, c1::2, :]
    elif m == 2:
        out[..., 0::2] = u[..., 0::2]
    else:
        out[..., 1::2] = u[..., 1::2]
    return out


def decompress(vc, m, out_shape):
    """coupling_layer.decompress_mask :763-1073."""
    B, H, W, D = out_shape
    out = np.zeros((vc.shape[0], H, W, D), dtype=vc.dtype)
    if m in (0, 1):
        (r0, c0), (r1, c1) = _CB[m]
        out[:, r0::2, c0::2, :] = vc[..., :D]
        out[:, r1::2, c1::2, :] = vc[..., D:]
    elif m == 2:
        out[..., 0::2] = vc
    else:
        out[..., 1::2] = vc
    return out


# ----------------------------------------------------------------------------
# s,t networks (conv_cINN_make_model.py:1076-1213)
# ----------------------------------------------------------------------------

def grouped_stage(y, c: CouplingSpec, P, q, ksize):
    """Parallel dilated grouped convolutions + concat
    (conv_cINN_base_functions.py:573-601, 364-413)."""
    outs = []
    for bi, br in enumerate(c.branches):
        for j, off in enumerate(br.in_offsets):
            xin = y[..., off:off + br.width]
            outs.append(conv2d_same(xin, P[f'{q}.gc.d{bi}.g{j}.kernel'], P[f'{q}.gc.d{bi}.g{j}.bias'],
                                    br.dilation))
    return np.concatenate(outs, axis=-1)


def st_net(u1c, c: CouplingSpec, P, net: str, ksize=3, ln=True):
    p = f'c{c.index}.{net}'
    y = conv2d_same(u1c, P[f'{p}.conv_in.kernel'], P[f'{p}.conv_in.bias'])
    for r in range(c.R):                         # dilated_residual_block :501-627
        q = f'{p}.rb{r}'
        shortcut = y
        t = add_common_layers(y, ln, P.get(f'{q}.ln1.gamma'), P.get(f'{q}.ln1.beta'))
        t = conv2d_same(t, P[f'{q}.conv_a.kernel'], P[f'{q}.conv_a.bias'])
        t = add_common_layers(t, ln, P.get(f'{q}.ln2.gamma'), P.get(f'{q}.ln2.beta'))
        t = grouped_stage(t, c, P, q, ksize)
        t = add_common_layers(t, ln, P.get(f'{q}.ln3.gamma'), P.get(f'{q}.ln3.beta'))
        t = conv2d_same(t, P[f'{q}.conv_b.kernel'], P[f'{q}.conv_b.bias'])
        y = shortcut + t
    y = add_common_layers(y, ln, P.get(f'{p}.ln_out.gamma'), P.get(f'{p}.ln_out.beta'))
    y = conv2d_same(y, P[f'{p}.conv_out.kernel'], P[f'{p}.conv_out.bias'])
    if net == 'A':
        y = np.tanh(y) * P[f'{p}.tanh_scale.w']     # :1198-1205
    return y


# ----------------------------------------------------------------------------
# layers
# ----------------------------------------------------------------------------

def coupling_forward(u, c: CouplingSpec, P, ksize=3, ln=True, with_abs=False):
    """forward_and_Jacobian :1258-1328. Returns v and the per-image sum of A(u1) (with_abs: also
    the per-image sum of |A(u1)|, the conditioning scale of that sum)."""
    u1 = mask_uncompressed(u, c.mask)
    u1c = mask_compress(u, c.mask)
    u2c = mask_compress(u, c.mask_c)
    s = st_net(u1c, c, P, 'A', ksize, ln)
    t = st_net(u1c, c, P, 'b', ksize, ln)
    v2c = np.exp(s) * u2c + t
    v = u1 + decompress(v2c, c.mask_c, u.shape)
    if with_abs:
        return v, s.reshape(s.shape[0], -1).sum(axis=1), np.abs(s).reshape(s.shape[0], -1).sum(axis=1)
    return v, s.reshape(s.shape[0], -1).sum(axis=1)


def coupling_backward(v, c: CouplingSpec, P, ksize=3, ln=True):
    """backward :1333-1394."""
    v1 = mask_uncompressed(v, c.mask)
    v1c = mask_compress(v, c.mask)
    v2c = mask_compress(v, c.mask_c)
    s = st_net(v1c, c, P, 'A', ksize, ln)
    t = st_net(v1c, c, P, 'b', ksize, ln)
    u2c = (1.0 / np.exp(s)) * (v2c - t)
    return v1 + decompress(u2c, c.mask_c, v.shape)


def squeeze_forward(u, zy):
    """squeeze_layer.forward_and_Jacobian :155-185."""
    assert u.shape[1] % 2 == 0 and u.shape[2] % 2 == 0, 'u must have spatial dimensions divisible by 2.'
    return space_to_depth(u), (space_to_depth(zy) if zy is not None else None)


def squeeze_backward(v, zy):
    """squeeze_layer.backward :191-217."""
    assert v.shape[3] % 4 == 0, 'v must have channel dimensions divisible by 4.'
    return depth_to_space(v), (depth_to_space(zy) if zy is not None else None)


def factor_forward(u, zy):
    """factor_out_zy_layer.forward_and_Jacobian :256-288."""
    split = u.shape[3] // 2
    f = u[..., :split]
    v = u[..., split:]
    zy = np.concatenate([zy, f], axis=3) if zy is not None else f
    return v, zy


def factor_backward(v, zy, num_prev_factors):
    """factor_out_zy_layer.backward :294-329."""
    if v is None:
        split = zy.shape[3] // (2 ** num_prev_factors)
    else:
        split = v.shape[3]
    re = zy[..., zy.shape[3] - split:]
    zy = zy[..., :zy.shape[3] - split]
    assert re.shape[3] == split
    u = np.concatenate([re, v], axis=3) if v is not None else re
    return u, zy


# ----------------------------------------------------------------------------
# model
# ----------------------------------------------------------------------------

class OracleCFlow:
    """cFlow restated (conv_cINN_make_model.py:1408-1904) with explicit params."""

    def __init__(self, io_shape, x_d, squeeze_factor_block_list, ResNeXt_block_list,
                 num_kernels_list, cardinality_list, lambda_y=100, ksize=3,
                 LAYER_NORM=True, DILATIONS=True, group_mode='reference'):
        self.io_shape = tuple(int(v) for v in io_shape)
        self.x_d = int(x_d)
        self.lambda_y = float(lambda_y)
        self.ksize = ksize
        self.ln = bool(LAYER_NORM)
        self.group_mode = group_mode
        self.layers = build_schedule(io_shape, x_d, squeeze_factor_block_list, ResNeXt_block_list,
                                     num_kernels_list, cardinality_list, ksize, LAYER_NORM,
                                     DILATIONS, group_mode)
        self.specs = param_specs(self.layers, ksize, LAYER_NORM)
        self.sf_layers = [e for e in self.layers if e.kind in ('squeeze', 'factor')]

    @property
    def coupling_specs(self):
        return [e.coupling for e in self.layers if e.kind == 'coupling']

    def num_params(self):
        return int(sum(int(np.prod(s)) for _, s in self.specs))

    def init_params(self, seed=0, **kw):
        return init_params(self.specs, seed, **kw)

    def _cast(self, P, dtype):
        return {k: np.asarray(v, dtype=dtype) for k, v in P.items()}

    def forward(self, xy, P, dtype=np.float64, per_layer=False, abs_s=False):
        """cFlow.call(xy, 1) :1743-1772. Returns (zy, logdet_per_image[B]);
        the reference's scalar log_detJ is logdet_per_image.mean(). abs_s: also the per-image
        sum over layers of sum|s| (the log-det's conditioning scale), appended
        to the returned tuple."""
        P = self._cast(P, dtype)
        uv = np.asarray(xy, dtype=dtype)
        zy = None
        ld = np.zeros(uv.shape[0], dtype=dtype)
        sabs = np.zeros(uv.shape[0], dtype=dtype)
        trace = []
        for e in self.layers:
            if e.kind == 'coupling':
                uv, d, a = coupling_forward(uv, e.coupling, P, self.ksize, self.ln, with_abs=True)
                ld = ld + d
                sabs = sabs + a
                if per_layer:
                    trace.append((uv.copy(), d.copy()))
            elif e.kind == 'squeeze':
                uv, zy = squeeze_forward(uv, zy)
            else:
                uv, zy = factor_forward(uv, zy)
        if not self.sf_layers:
            out = uv
        else:
            zy = np.concatenate([zy, uv], axis=3)
            vu = None
            for e in reversed(self.sf_layers):
                if e.kind == 'factor':
                    vu, zy = factor_backward(vu, zy, e.num_prev_factors)
                else:
                    vu, zy = squeeze_backward(vu, zy)
            out = vu
        res = (out, ld) + ((trace,) if per_layer else ()) + ((sabs,) if abs_s else ())
        return res

    def inverse(self, zy_in, P, dtype=np.float64):
        """cFlow.call(zy, -1) :1774-1798."""
        P = self._cast(P, dtype)
        uv = np.asarray(zy_in, dtype=dtype)
        zy = None
        for e in self.sf_layers:
            if e.kind == 'squeeze':
                uv, zy = squeeze_forward(uv, zy)
            else:
                uv, zy = factor_forward(uv, zy)
        vu = uv
        for e in reversed(self.layers):
            if e.kind == 'coupling':
                vu = coupling_backward(vu, e.coupling, P, self.ksize, self.ln)
            elif e.kind == 'squeeze':
                vu, zy = squeeze_backward(vu, zy)
            else:
                vu, zy = factor_backward(vu, zy, e.num_prev_factors)
        return vu

    def nll_terms(self, xy, zy, logdet_per_image):
        """Per-image NLL terms of log_loss :1815-1840: returns (llz[B], lly[B], ld[B])."""
        x_d = self.x_d
        y_prime = xy[..., x_d:]
        z = zy[..., :x_d]
        y = zy[..., x_d:]
        lp = -0.5 * (z * z).sum(axis=-1) - 0.5 * x_d * LOG_2PI       # MVNDiag(0,I).log_prob
        llz = lp.reshape(lp.shape[0], -1).sum(axis=1)
        lly = -self.lambda_y * np.abs(y - y_prime).reshape(y.shape[0], -1).sum(axis=1)
        return llz, lly, logdet_per_image

    def log_loss(self, xy, P, dtype=np.float64):
        """cFlow.log_loss :1800-1848 -> (loss, z_loss, y_loss, detJ_loss)."""
        xy = np.asarray(xy, dtype=dtype)
        zy, ldi = self.forward(xy, P, dtype)
        llz, lly, _ = self.nll_terms(xy, zy, ldi)
        log_detJ = ldi.mean()                       # batch-mean scalar (:1325)
        ll = (llz + lly).mean() + log_detJ
        return -ll, -llz.mean(), -lly.mean(), -log_detJ

    def sf_permutation(self, shape_hw_d=None):
        """The squeeze/factor/restore composition as an index map: for the final
        uv / factored pieces. Used by invariant tests only."""
        H, W, D = self.io_shape
        ar = np.arange(H * W * D, dtype=np.float64).reshape(1, H, W, D)
        uv, zy = ar, None
        for e in self.sf_layers:
            uv, zy = (squeeze_forward(uv, zy) if e.kind == 'squeeze' else factor_forward(uv, zy))
        return uv, zy


# ----------------------------------------------------------------------------
# synthetic inputs
# ----------------------------------------------------------------------------

def synthetic_class_batch(B, H, W, x_d=3, seed=0, noise_alpha=0.98, num_classes=10):
    """cfg2/cfg4: x~U(0,1); y-plane = k/9 for class k (conv_cINN.py:221-228,259-261);
    instance_noise(xy, 0.98) on all channels (conv_cINN.py:312-315,
    conv_cINN_base_functions.py:636-654)."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, 1, (B, H, W, x_d))
    k = rng.integers(0, num_classes, B)
    y = np.broadcast_to((k / (num_classes - 1)).reshape(B, 1, 1, 1), (B, H, W, 1))
    xy = np.concatenate([x, y], axis=-1)
    xy = noise_alpha * xy + (1 - noise_alpha) * rng.standard_normal(xy.shape)
    return xy.astype(np.float32)


def _down(img):
    """conv_cINN_base_functions.py:74-126 (2x2 mean pool)."""
    B, H, W, C = img.shape
    return img.reshape(B, H // 2, 2, W // 2, 2, C).mean(axis=(2, 4))


def _up(img):
    """conv_cINN_base_functions.py:128-164 (2x2 repeat)."""
    return img.repeat(2, axis=1).repeat(2, axis=2)


def synthetic_sr_batch(B, H, W, C=3, factor_pow=2, seed=0, noise_alpha=0.98):
    """cfg3/cfg5: hi-res h~U(0,1); y = up^p(down^p(h)); x = h - y (RESIDUAL);
    + 2% instance noise (conv_cINN_base_functions.py:233-279, conv_cINN.py:45)."""
    rng = np.random.default_rng(seed)
    h = rng.uniform(0, 1, (B, H, W, C))
    y = h
    for _ in range(factor_pow):
        y = _down(y)
    for _ in range(factor_pow):
        y = _up(y)
    xy = np.concatenate([h - y, y], axis=-1)
    xy = noise_alpha * xy + (1 - noise_alpha) * rng.standard_normal(xy.shape)
    return xy.astype(np.float32)
