"""TEST INFRASTRUCTURE ONLY — torch-CPU fp32 op-for-op restatement of the reference graph.

This is the timed CPU baseline of bench.py (`cpu_baseline.kind = "port"`): the reference's
TensorFlow CPU path cannot run here (TF is not installed), so this restates
its graph op for op on the host with the same structure TF executes: one Conv2D per group of
every grouped convolution (conv_cINN_base_functions.py:401-411), Reshape->LayerNormalization
over H*W*C (:350-360), mask / decompress via strided gathers and scatters
(conv_cINN_make_model.py:720-759, 896-1071), tanh*w, exp, the affine law, batch-mean log-det,
space_to_depth, factor-out and the final layout restoration, NLL. fp32, NHWC data,
multi-threaded oneDNN convolutions. Validated against cflow_np in tests/test_oracle.py.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from .cflow_np import (LN_EPS, LRELU_ALPHA, LOG_2PI, build_schedule, init_params, param_specs)


def _conv(x, k, b, d=1):
    """x NHWC, k HWIO -> Keras Conv2D 'same' (symmetric pad for odd k)."""
    kh = k.shape[0]
    pad = (kh - 1) * d // 2
    y = F.conv2d(x.permute(0, 3, 1, 2), k.permute(3, 2, 0, 1).contiguous(), b, padding=pad, dilation=d)
    return y.permute(0, 2, 3, 1)


def _lrelu(x):
    return F.leaky_relu(x, LRELU_ALPHA)


def _ln(x, g, b):
    B = x.shape[0]
    f = x.reshape(B, -1)
    return F.layer_norm(f, (f.shape[1],), g, b, LN_EPS).reshape(x.shape)


_CB = {0: ((0, 0), (1, 1)), 1: ((0, 1), (1, 0))}


def _compress(u, m):
    if m in (0, 1):
        (r0, c0), (r1, c1) = _CB[m]
        return torch.cat([u[:, r0::2, c0::2, :], u[:, r1::2, c1::2, :]], dim=-1)
    return u[..., 0::2] if m == 2 else u[..., 1::2]


def _masked(u, m):
    out = torch.zeros_like(u)
    if m in (0, 1):
        (r0, c0), (r1, c1) = _CB[m]
        out[:, r0::2, c0::2, :] = u[:, r0::2, c0::2, :]
        out[:, r1::2, c1::2, :] = u[:, r1::2, c1::2, :]
    elif m == 2:
        out[..., 0::2] = u[..., 0::2]
    else:
        out[..., 1::2] = u[..., 1::2]
    return out


def _decompress(vc, m, shape):
    out = torch.zeros(shape, dtype=vc.dtype)
    D = shape[3]
    if m in (0, 1):
        (r0, c0), (r1, c1) = _CB[m]
        out[:, r0::2, c0::2, :] = vc[..., :D]
        out[:, r1::2, c1::2, :] = vc[..., D:]
    elif m == 2:
        out[..., 0::2] = vc
    else:
        out[..., 1::2] = vc
    return out


def _s2d(x):
    B, H, W, C = x.shape
    return x.reshape(B, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(B, H // 2, W // 2, 4 * C)


def _d2s(x):
    B, H, W, C4 = x.shape
    C = C4 // 4
    return x.reshape(B, H, W, 2, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(B, 2 * H, 2 * W, C)


class TorchCPUFlow:
    def __init__(self, io_shape, x_d, squeeze_factor_block_list, ResNeXt_block_list, num_kernels_list,
                 cardinality_list, lambda_y=100, ksize=3, LAYER_NORM=True, DILATIONS=True, group_mode='reference'):
        self.io_shape = tuple(io_shape)
        self.x_d = x_d
        self.lambda_y = float(lambda_y)
        self.ln = LAYER_NORM
        self.layers = build_schedule(io_shape, x_d, squeeze_factor_block_list, ResNeXt_block_list,
                                     num_kernels_list, cardinality_list, ksize, LAYER_NORM, DILATIONS, group_mode)
        self.specs = param_specs(self.layers, ksize, LAYER_NORM)
        self.sf = [e for e in self.layers if e.kind != 'coupling']

    def init_params(self, seed=0):
        return {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in init_params(self.specs, seed).items()}

    def _net(self, x, c, P, net):
        p = f'c{c.index}.{net}'
        ln = self.ln
        y = _conv(x, P[f'{p}.conv_in.kernel'], P[f'{p}.conv_in.bias'])
        for r in range(c.R):
            q = f'{p}.rb{r}'
            t = _lrelu(y)
            if ln:
                t = _ln(t, P[f'{q}.ln1.gamma'], P[f'{q}.ln1.beta'])
            t = _conv(t, P[f'{q}.conv_a.kernel'], P[f'{q}.conv_a.bias'])
            t = _lrelu(t)
            if ln:
                t = _ln(t, P[f'{q}.ln2.gamma'], P[f'{q}.ln2.beta'])
            outs = []
            for bi, br in enumerate(c.branches):
                for j, off in enumerate(br.in_offsets):          # one Conv2D per group
                    outs.append(_conv(t[..., off:off + br.width], P[f'{q}.gc.d{bi}.g{j}.kernel'],
                                      P[f'{q}.gc.d{bi}.g{j}.bias'], br.dilation))
            t = torch.cat(outs, dim=-1)
            t = _lrelu(t)
            if ln:
                t = _ln(t, P[f'{q}.ln3.gamma'], P[f'{q}.ln3.beta'])
            t = _conv(t, P[f'{q}.conv_b.kernel'], P[f'{q}.conv_b.bias'])
            y = y + t
        y = _lrelu(y)
        if ln:
            y = _ln(y, P[f'{p}.ln_out.gamma'], P[f'{p}.ln_out.beta'])
        y = _conv(y, P[f'{p}.conv_out.kernel'], P[f'{p}.conv_out.bias'])
        if net == 'A':
            y = torch.tanh(y) * P[f'{p}.tanh_scale.w']
        return y

    def _coupling(self, u, c, P, direction, per_image=False):
        u1 = _masked(u, c.mask)
        u1c = _compress(u, c.mask)
        u2c = _compress(u, c.mask_c)
        s = self._net(u1c, c, P, 'A')
        t = self._net(u1c, c, P, 'b')
        if direction > 0:
            v2c = torch.exp(s) * u2c + t
            ld = s.reshape(s.shape[0], -1).sum(1)
            ld = torch.stack([ld, s.abs().reshape(s.shape[0], -1).sum(1)]) if per_image else ld.mean()
        else:
            v2c = torch.reciprocal(torch.exp(s)) * (u2c - t)
            ld = None
        return u1 + _decompress(v2c, c.mask_c, u.shape), ld

    def forward(self, xy, P, per_image=False):
        """cFlow.call(xy, 1). per_image: the log-det is returned as the [2][B] stack of the
        per-image sum of s and sum of |s| over every coupling layer (run in float64 with float64
        params and inputs this is the full-size parity oracle of tests/test_gpu_parity.py)."""
        uv, zy, ld = xy, None, 0.0
        for e in self.layers:
            if e.kind == 'coupling':
                uv, d = (self._coupling(uv, e.coupling, P, +1, True) if per_image else
                         self._coupling(uv, e.coupling, P, +1))
                ld = ld + d
            elif e.kind == 'squeeze':
                uv = _s2d(uv)
                zy = _s2d(zy) if zy is not None else None
            else:
                split = uv.shape[3] // 2
                f = uv[..., :split]
                uv = uv[..., split:]
                zy = torch.cat([zy, f], 3) if zy is not None else f
        if not self.sf:
            return uv, ld
        zy = torch.cat([zy, uv], 3)
        vu = None
        for e in reversed(self.sf):
            if e.kind == 'factor':
                split = zy.shape[3] // (2 ** e.num_prev_factors) if vu is None else vu.shape[3]
                re = zy[..., zy.shape[3] - split:]
                zy = zy[..., :zy.shape[3] - split]
                vu = torch.cat([re, vu], 3) if vu is not None else re
            else:
                vu = _d2s(vu)
                zy = _d2s(zy) if zy is not None else None
        return vu, ld

    def inverse(self, zy_in, P):
        """cFlow.call(zy, -1) (conv_cINN_make_model.py:1774-1798): the squeeze / factor layers'
        forward rebuilds the last block's layout from zy (:1782-1788), then every layer's backward
        in reverse order (:1793-1796; coupling inverse law :1235-1253, :1333-1394)."""
        uv, zy = zy_in, None
        for e in self.sf:
            if e.kind == 'squeeze':
                uv = _s2d(uv)
                zy = _s2d(zy) if zy is not None else None
            else:
                split = uv.shape[3] // 2
                f = uv[..., :split]
                uv = uv[..., split:]
                zy = torch.cat([zy, f], 3) if zy is not None else f
        vu = uv
        for e in reversed(self.layers):
            if e.kind == 'coupling':
                vu, _ = self._coupling(vu, e.coupling, P, -1)
            elif e.kind == 'squeeze':
                vu = _d2s(vu)
                zy = _d2s(zy) if zy is not None else None
            else:
                split = zy.shape[3] // (2 ** e.num_prev_factors) if vu is None else vu.shape[3]
                re = zy[..., zy.shape[3] - split:]
                zy = zy[..., :zy.shape[3] - split]
                vu = torch.cat([re, vu], 3)
        return vu

    def log_loss(self, xy, P):
        x_d = self.x_d
        zy, ld = self.forward(xy, P)
        z = zy[..., :x_d]
        y = zy[..., x_d:]
        llz = (-0.5 * (z * z).sum(-1) - 0.5 * x_d * LOG_2PI).reshape(z.shape[0], -1).sum(1)
        lly = -self.lambda_y * (y - xy[..., x_d:]).abs().reshape(y.shape[0], -1).sum(1)
        ll = (llz + lly).mean() + ld
        return -ll, -llz.mean(), -lly.mean(), -ld
