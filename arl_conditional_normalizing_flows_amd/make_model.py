"""Drop-in replacement for the reference's `conv_cINN_make_model` layer/model API on MI355X.

Same class names, constructor arguments, method names, argument order, return values and
`None` conventions as conv_cINN_make_model.py; tensors are torch tensors on the ROCm device
(NHWC, contiguous, float32) instead of TF tensors. Every computation runs in
libcnf_hip.so (hand-written gfx950 HIP kernels) through the C ABI in include/cnf.h — there is
no CPU or torch-op fallback: if the library is missing the constructor raises.

Reference map
  Layer                    conv_cINN_make_model.py:62-89
  tanh_scaling_layer       :97-122  (a scalar parameter inside net A; exposed for API parity)
  squeeze_layer            :130-217
  factor_out_zy_layer      :219-329
  coupling_layer           :337-1394
  cFlow                    :1408-1904
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr

GROUP_MODES = {'reference': 0, 'intended': 1}


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _as_input(t, what='input'):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f'{what} must be a torch.Tensor on the ROCm device')
    if not t.is_cuda:
        raise ValueError(f'{what} must live on the GPU (got {t.device}); the HIP path has no CPU fallback')
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


# ---------------------------------------------------------------------------------------------
# layers
# ---------------------------------------------------------------------------------------------

class Layer:
    """Abstract two-direction layer (conv_cINN_make_model.py:62-89)."""

    def forward_and_Jacobian(self, u, sum_log_det_J, z):
        raise NotImplementedError(str(type(self)))

    def backward(self, v, z):
        raise NotImplementedError(str(type(self)))


def _accumulate_logdet(sum_log_det_J, per_image):
    """Reference semantics: sum_log_detJ += reduce_mean(reduce_sum(A(u1))) (:1323-1326).
    If the caller passes a per-image (B,) tensor, accumulate per image instead."""
    if isinstance(sum_log_det_J, torch.Tensor) and sum_log_det_J.dim() == 1 \
            and sum_log_det_J.shape[0] == per_image.shape[0]:
        return sum_log_det_J + per_image
    return sum_log_det_J + per_image.mean()


class tanh_scaling_layer(Layer):
    """Scalar multiplier after tanh in net A (:97-122). In this implementation the scalar is
    parameter `c{i}.A.tanh_scale.w` of the owning cFlow and is applied inside k_coupling."""

    def __init__(self, flow=None, coupling_index=None):
        self._flow = flow
        self._ci = coupling_index

    @property
    def w(self):
        return self._flow.get_param(f'c{self._ci}.A.tanh_scale.w')

    def call(self, inputs):
        return self.w * inputs


class squeeze_layer(Layer):
    """space_to_depth(2) / depth_to_space(2) on u and zy (:130-217), TF channel order."""

    def forward_and_Jacobian(self, u, sum_log_det_J, zy):
        u = _as_input(u, 'u')
        assert u.shape[1] % 2 == 0 and u.shape[2] % 2 == 0, 'u must have spatial dimensions divisible by 2.'
        v = _squeeze(u, +1)
        if zy is not None:
            zy = _squeeze(_as_input(zy, 'zy'), +1)
        return v, sum_log_det_J, zy

    def backward(self, v, zy):
        v = _as_input(v, 'v')
        assert v.shape[3] % 4 == 0, 'v must have channel dimensions divisible by 4.'
        u = _squeeze(v, -1)
        if zy is not None:
            zy = _squeeze(_as_input(zy, 'zy'), -1)
        return u, zy


def _squeeze(x, direction):
    B, H, W, Cc = x.shape
    if direction > 0:
        out = torch.empty((B, H // 2, W // 2, 4 * Cc), device=x.device, dtype=torch.float32)
    else:
        out = torch.empty((B, 2 * H, 2 * W, Cc // 4), device=x.device, dtype=torch.float32)
    if x.numel() > 0:
        check(_lib.load().cnf_squeeze(ptr(x), ptr(out), B, H, W, Cc, direction, _stream()), 'cnf_squeeze')
    return out


def _channels(x, start, stop):
    """x[..., start:stop] as a new contiguous tensor (HIP channel copy)."""
    B, H, W, Cc = x.shape
    n = stop - start
    out = torch.empty((B, H, W, n), device=x.device, dtype=torch.float32)
    if n > 0 and B * H * W > 0:
        check(_lib.load().cnf_channel_copy(ptr(x), Cc, start, ptr(out), n, 0, n, B, H * W, _stream()),
              'cnf_channel_copy')
    return out


def _concat(a, b):
    """concat([a, b], axis=3) (HIP channel copies)."""
    B, H, W, ca = a.shape
    cb = b.shape[3]
    out = torch.empty((B, H, W, ca + cb), device=a.device, dtype=torch.float32)
    lib = _lib.load()
    if ca:
        check(lib.cnf_channel_copy(ptr(a), ca, 0, ptr(out), ca + cb, 0, ca, B, H * W, _stream()), 'concat')
    if cb:
        check(lib.cnf_channel_copy(ptr(b), cb, 0, ptr(out), ca + cb, ca, cb, B, H * W, _stream()), 'concat')
    return out


class factor_out_zy_layer(Layer):
    """Factor half of the channels out into zy / back in (:219-329)."""

    def __init__(self, num_prev_factors, **kwargs):
        self.num_prev_factors = int(num_prev_factors)

    def get_config(self):
        return {'num_prev_factors': self.num_prev_factors}

    def forward_and_Jacobian(self, u, sum_log_det_J, zy):
        u = _as_input(u, 'u')
        split = u.shape[3] // 2
        factored = _channels(u, 0, split)
        v = _channels(u, split, u.shape[3])
        zy = _concat(_as_input(zy, 'zy'), factored) if zy is not None else factored
        return v, sum_log_det_J, zy

    def backward(self, v, zy):
        zy = _as_input(zy, 'zy')
        if v is None:
            split = zy.shape[3] // (2 ** self.num_prev_factors)
        else:
            v = _as_input(v, 'v')
            split = v.shape[3]
        cz = zy.shape[3]
        re = _channels(zy, cz - split, cz)
        zy = _channels(zy, 0, cz - split)
        assert re.shape[3] == split
        u = _concat(re, v) if v is not None else re
        return u, zy


class coupling_layer(Layer):
    """Affine coupling layer with compressed checkerboard / channel masks and ResNeXt s,t
    networks (:337-1394). Instances are created by cFlow (they execute through the flow's
    plan and parameter buffers)."""

    def __init__(self, flow: 'cFlow', layer_index: int, info):
        self._flow = flow
        self._layer = layer_index
        self.coupling_index = info.coupling_index
        self.input_height, self.input_width, self.input_depth = info.h, info.w, info.d
        self.which_mask = info.mask
        self.which_mask_complement = {0: 1, 1: 0, 2: 3, 3: 2}[info.mask]
        self.num_res_blocks = info.num_res_blocks
        self.cardinality = info.cardinality
        self.num_kernels = info.num_kernels
        self.kernel_size = flow.ksize
        self.LAYER_NORM = flow.LAYER_NORM
        self.which_dilations = [info.dilations[i] for i in range(info.num_dilations)]
        self.compressed_height, self.compressed_width, self.compressed_depth = info.hc, info.wc, info.dc1
        self.uv2_depth = info.dc2
        self.tanh_scale = tanh_scaling_layer(flow, info.coupling_index)

    def get_config(self):
        return {'input_height': self.input_height, 'input_width': self.input_width,
                'input_depth': self.input_depth, 'which_mask': self.which_mask,
                'num_res_blocks': self.num_res_blocks, 'cardinality': self.cardinality,
                'kernel_size': self.kernel_size, 'LAYER_NORM': self.LAYER_NORM,
                'which_dilations': self.which_dilations}

    def _check(self, t, what):
        t = _as_input(t, what)
        # tf.ensure_shape(u, [None, H, W, D]) (:1276-1280, :1348-1352)
        if tuple(t.shape[1:]) != (self.input_height, self.input_width, self.input_depth):
            raise ValueError(f'{what} has shape {tuple(t.shape)}, expected [None, {self.input_height}, '
                             f'{self.input_width}, {self.input_depth}]')
        return t

    def forward_and_Jacobian(self, u, sum_log_detJ, zy):
        u = self._check(u, 'u')
        f = self._flow
        B = u.shape[0]
        v = torch.empty_like(u)
        ld = torch.zeros(B, device=u.device, dtype=torch.float32)
        ws = f._workspace(B)
        check(_lib.load().cnf_coupling_forward(f._plan, self._layer, ptr(f.params), ptr(f._aux), ptr(u), ptr(v),
                                               ptr(ld), ptr(ws), B, _stream()), 'cnf_coupling_forward')
        return v, _accumulate_logdet(sum_log_detJ, ld), zy

    def backward(self, v, zy):
        v = self._check(v, 'v')
        f = self._flow
        B = v.shape[0]
        u = torch.empty_like(v)
        ws = f._workspace(B)
        check(_lib.load().cnf_coupling_inverse(f._plan, self._layer, ptr(f.params), ptr(f._aux), ptr(v), ptr(u),
                                               ptr(ws), B, _stream()), 'cnf_coupling_inverse')
        return u, zy

    def gradients(self, u, dv, dlogdet=0.0):
        """Vector-Jacobian product of forward_and_Jacobian at u: (dL/du, dL/dparams) for
        dL/dv = dv and dL/d(per-image log-det) = dlogdet (the training backward of this layer;
        dparams is the flat canonical vector, zero outside this layer's parameters)."""
        u = self._check(u, 'u')
        dv = self._check(dv, 'dv')
        f = self._flow
        B = u.shape[0]
        du = torch.empty_like(u)
        dp = torch.empty(f.num_params, device=u.device, dtype=torch.float32)
        ws = f._train_workspace(B)
        check(_lib.load().cnf_coupling_backward(f._plan, self._layer, ptr(f.params), ptr(u), ptr(dv), ptr(du),
                                                float(dlogdet), ptr(ws), B, ptr(dp), _stream()),
              'cnf_coupling_backward')
        return du, dp


# ---------------------------------------------------------------------------------------------
# metrics (keras.metrics.Mean stand-in, :1692-1718)
# ---------------------------------------------------------------------------------------------

class Mean:
    """keras.metrics.Mean (the loss trackers of :1454-1457): the running mean of update_state values.
    Fed device tensors (train_step / test_step) it accumulates on the device in float64 — the same
    double arithmetic as a host float sum — and result() is a 0-d device tensor, as TF's train_step
    returns tensors: no host read per step (the fit loop reads the epoch's values once, at its end)."""
    def __init__(self, name):
        self.name = name
        self.reset_state()

    def reset_state(self):
        self.total = 0.0
        self.count = 0

    def update_state(self, v):
        if isinstance(v, torch.Tensor):
            v = v.detach().to(torch.float64)
        else:
            v = float(v)
        self.total = self.total + v
        self.count += 1

    def result(self):
        """Always a 0-d float64 tensor (on the device the values came from; a CPU zero before any update)."""
        if not self.count:
            return torch.zeros((), dtype=torch.float64)
        return torch.as_tensor(self.total / self.count, dtype=torch.float64)


# ---------------------------------------------------------------------------------------------
# cFlow
# ---------------------------------------------------------------------------------------------

class cFlow:
    """Conditional multi-scale RealNVP (conv_cINN_make_model.py:1408-1904) on MI355X.

    Extra keyword arguments (not in the reference): `group_mode` ('reference' reproduces the
    late-bound Lambda closure of conv_cINN_base_functions.py:402, 'intended' the textbook
    grouped convolution), `device`, `seed` (parameter init), `debug_options` (a dict or a
    "NAME=V,..." string selecting the alternative code paths the parity tests compare against:
    include/cnf.h cnf_flow_desc.debug_options; None = the defaults, which are what is benchmarked)."""

    def __init__(self, io_shape, x_d, squeeze_factor_block_list, ResNeXt_block_list, num_kernels_list,
                 cardinality_list, lambda_y=100, ksize=3, LAYER_NORM=True, DILATIONS=True, init=None,
                 group_mode='reference', device=None, seed=0, debug_options=None):
        lib = _lib.load()
        self.io_shape = [int(v) for v in io_shape]
        self.x_d = int(x_d)
        self.squeeze_factor_block_list = list(squeeze_factor_block_list)
        self.ResNeXt_block_list = list(ResNeXt_block_list)
        self.num_kernels_list = list(num_kernels_list)
        self.cardinality_list = list(cardinality_list)
        self.lambda_y = float(lambda_y)
        self.ksize = int(ksize)
        self.LAYER_NORM = bool(LAYER_NORM)
        self.DILATIONS = bool(DILATIONS)
        self.init = init
        if group_mode not in GROUP_MODES:
            raise ValueError(f'group_mode must be one of {list(GROUP_MODES)}')
        self.group_mode = group_mode
        self.device = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())

        nb = len(self.squeeze_factor_block_list)
        assert nb == len(self.ResNeXt_block_list) == len(self.num_kernels_list) == len(self.cardinality_list), \
            'squeeze_factor_block_list, ResNeXt_block_list, num_kernels_list, and cardinality_list must all have the same length.'
        arr = lambda v: (C.c_int * len(v))(*[int(x) for x in v])
        self._keep = [arr(self.squeeze_factor_block_list), arr(self.ResNeXt_block_list),
                      arr(self.num_kernels_list), arr(self.cardinality_list)]
        desc = _lib.cnf_flow_desc(self.io_shape[0], self.io_shape[1], self.io_shape[2], self.x_d, nb,
                                  self._keep[0], self._keep[1], self._keep[2], self._keep[3],
                                  self.lambda_y, self.ksize, int(self.LAYER_NORM), int(self.DILATIONS),
                                  GROUP_MODES[group_mode])
        if isinstance(debug_options, dict):
            debug_options = ','.join(f'{k}={int(v)}' for k, v in debug_options.items())
        self.debug_options = debug_options or ''
        self._opts_buf = C.create_string_buffer(self.debug_options.encode())
        desc.debug_options = C.cast(self._opts_buf, C.c_char_p)
        plan = C.c_void_p()
        check(lib.cnf_plan_create(C.byref(desc), C.byref(plan)), 'cFlow')
        self._plan = plan

        # parameter table
        self.param_specs = []
        name = C.create_string_buffer(256)
        off = C.c_int64()
        nd = C.c_int()
        shp = (C.c_int * 4)()
        for i in range(lib.cnf_plan_num_param_tensors(plan)):
            check(lib.cnf_plan_param_tensor(plan, i, name, 256, C.byref(off), C.byref(nd), shp), 'param table')
            self.param_specs.append((name.value.decode(), int(off.value), tuple(shp[j] for j in range(nd.value))))
        self._param_index = {n: (o, s) for n, o, s in self.param_specs}
        self.num_params = int(lib.cnf_plan_num_params(plan))
        self.params = torch.empty(self.num_params, device=self.device, dtype=torch.float32)
        self._aux = torch.empty(int(lib.cnf_plan_aux_floats(plan)), device=self.device, dtype=torch.float32)
        self._ws = {}

        # layers_list / squeeze_factor_layers_list (:1630-1689)
        self.layers_list: List[Layer] = []
        self.squeeze_factor_layers_list: List[Layer] = []
        info = _lib.cnf_layer_info()
        for li in range(lib.cnf_plan_num_layers(plan)):
            check(lib.cnf_plan_layer_info(plan, li, C.byref(info)), 'layer info')
            if info.kind == 0:
                self.layers_list.append(coupling_layer(self, li, info))
            elif info.kind == 1:
                L = squeeze_layer()
                self.layers_list.append(L)
                self.squeeze_factor_layers_list.append(L)
            else:
                L = factor_out_zy_layer(info.num_prev_factors)
                self.layers_list.append(L)
                self.squeeze_factor_layers_list.append(L)
        self.u1_mask_indices = [[0, 1, 2, 3] for _ in range(nb)]
        self.num_coupling_blocks = nb

        self.loss_tracker = Mean('loss')
        self.z_loss_tracker = Mean('z_loss')
        self.y_loss_tracker = Mean('y_loss')
        self.detJ_loss_tracker = Mean('detJ_loss')

        self.set_weights(self.initial_weights(seed))

    # -- lifecycle ------------------------------------------------------------------------------
    def __del__(self):
        try:
            if getattr(self, '_plan', None):
                _lib.load().cnf_plan_destroy(self._plan)
                self._plan = None
        except Exception:
            pass

    # -- parameters -----------------------------------------------------------------------------
    def initial_weights(self, seed=0) -> np.ndarray:
        """Reference initialisers: Conv2D kernels Orthogonal(gain=0.1) (:1442), biases 0,
        LayerNorm gamma 1 / beta 0, tanh scale 1 (:109-112)."""
        rng = np.random.default_rng(seed)
        flat = np.empty(self.num_params, dtype=np.float32)
        for n, o, s in self.param_specs:
            size = int(np.prod(s)) if s else 1
            if n.endswith('.kernel'):
                rows = int(np.prod(s[:-1]))
                cols = s[-1]
                a = rng.standard_normal((max(rows, cols), min(rows, cols)))
                q, r = np.linalg.qr(a)
                q = q * np.sign(np.diag(r))
                if rows < cols:
                    q = q.T
                v = 0.1 * q.reshape(-1)
            elif n.endswith('.gamma') or n.endswith('.w'):
                v = np.ones(size)
            else:
                v = np.zeros(size)
            flat[o:o + size] = v
        return flat

    def set_weights(self, weights):
        """weights: flat canonical vector (numpy/torch) or {name: array} dict."""
        if isinstance(weights, dict):
            flat = np.empty(self.num_params, dtype=np.float32)
            for n, o, s in self.param_specs:
                size = int(np.prod(s)) if s else 1
                flat[o:o + size] = np.asarray(weights[n], dtype=np.float32).reshape(-1)
            weights = flat
        if isinstance(weights, np.ndarray):
            weights = torch.from_numpy(np.ascontiguousarray(weights, dtype=np.float32))
        if weights.numel() != self.num_params:
            raise ValueError(f'expected {self.num_params} parameters, got {weights.numel()}')
        self.params.copy_(weights.reshape(-1).to(self.device, torch.float32))
        check(_lib.load().cnf_pack_params(self._plan, ptr(self.params), ptr(self._aux), _stream()), 'pack params')

    def get_weights(self) -> Dict[str, np.ndarray]:
        flat = self.params.detach().cpu().numpy()
        return {n: flat[o:o + (int(np.prod(s)) if s else 1)].reshape(s) for n, o, s in self.param_specs}

    def get_param(self, name):
        o, s = self._param_index[name]
        size = int(np.prod(s)) if s else 1
        return self.params[o:o + size].reshape(s)

    @property
    def trainable_variables(self):
        return [self.get_param(n) for n, _, _ in self.param_specs]

    def _workspace(self, B):
        ws = self._ws.get(B)
        if ws is None:
            nbytes = int(_lib.load().cnf_plan_workspace_bytes(self._plan, B))
            ws = torch.empty(max(nbytes, 256), device=self.device, dtype=torch.uint8)
            self._ws[B] = ws
        return ws

    # -- metrics --------------------------------------------------------------------------------
    @property
    def metrics(self):
        return [self.loss_tracker, self.z_loss_tracker, self.y_loss_tracker, self.detJ_loss_tracker]

    # -- the hot path ---------------------------------------------------------------------------
    def call(self, uv, direction=-1, per_image_logdet=False, layerwise=False, noise=None):
        """cFlow.call (:1723-1798). direction=+1: xy -> (zy, log_detJ) with log_detJ the batch-mean
        scalar (a (B,) tensor with per_image_logdet=True); direction=-1: zy -> xy.
        layerwise=True walks layers_list through the per-layer entry points exactly as the
        reference loop does; the default runs the whole schedule in one native call.
        noise=(alpha, seed, offset[, logit_a]) (direction=+1): the input prepared as the reference's
        training pipeline does (conv_cINN.py:246-315) -- the logit map of
        preprocess_dataset_class(LOGITS=True, a=logit_a) on the x channels when logit_a is given
        (conv_cINN_base_functions.py:174-231), then instance_noise(., alpha) (:635-654) -- inside
        the first coupling layer's gather (cnf_flow_forward_noise), returning (zy, log_detJ,
        xy_noisy); xy_noisy equals base_functions.instance_noise(xy', alpha, seed, offset) bit for
        bit (xy' = xy with its x channels through preprocess_dataset_class) and is the xy of the
        loss."""
        uv = _as_input(uv, 'uv')
        if tuple(uv.shape[1:]) != tuple(self.io_shape):
            raise ValueError(f'input shape {tuple(uv.shape)} != [None, {self.io_shape}]')
        B = uv.shape[0]
        if noise is not None:
            if direction != 1:
                raise ValueError('noise applies to the forward direction only')
            alpha, seed, offset, logit_a = (tuple(noise) + (0, 0, 0.0))[:4]
            if layerwise:
                from .base_functions import instance_noise, preprocess_dataset_class
                xp = uv
                if logit_a:
                    xp = torch.cat([preprocess_dataset_class(uv[..., :self.x_d], LOGITS=True, a=logit_a),
                                    uv[..., self.x_d:]], dim=-1).contiguous()
                xn = instance_noise(xp, alpha, seed, offset)
                zy, ld = self._call_layerwise_forward(xn)
            else:
                xn = torch.empty_like(uv)
                zy = torch.empty_like(uv)
                ld = torch.empty(B, device=uv.device, dtype=torch.float32)
                ws = self._workspace(B)
                check(_lib.load().cnf_flow_forward_noise(self._plan, ptr(self.params), ptr(self._aux), ptr(uv),
                                                         float(logit_a), float(alpha), int(seed) & (2 ** 64 - 1),
                                                         int(offset) & (2 ** 64 - 1), ptr(xn), ptr(zy), ptr(ld),
                                                         ptr(ws), B, _stream()), 'cnf_flow_forward_noise')
            return zy, (ld if per_image_logdet else ld.mean()), xn
        if direction == 1:
            if layerwise:
                zy, ld = self._call_layerwise_forward(uv)
            else:
                zy = torch.empty_like(uv)
                ld = torch.empty(B, device=uv.device, dtype=torch.float32)
                ws = self._workspace(B)
                check(_lib.load().cnf_flow_forward(self._plan, ptr(self.params), ptr(self._aux), ptr(uv), ptr(zy),
                                                   ptr(ld), ptr(ws), B, _stream()), 'cnf_flow_forward')
            return zy, (ld if per_image_logdet else ld.mean())
        elif direction == -1:
            if layerwise:
                return self._call_layerwise_inverse(uv)
            xy = torch.empty_like(uv)
            ws = self._workspace(B)
            check(_lib.load().cnf_flow_inverse(self._plan, ptr(self.params), ptr(self._aux), ptr(uv), ptr(xy),
                                               ptr(ws), B, _stream()), 'cnf_flow_inverse')
            return xy
        raise ValueError('direction must be +1 or -1')

    __call__ = call

    def _call_layerwise_forward(self, uv):
        B = uv.shape[0]
        log_detJ = torch.zeros(B, device=uv.device, dtype=torch.float32)
        zy = None
        for layer in self.layers_list:                          # :1748-1752
            uv, log_detJ, zy = layer.forward_and_Jacobian(uv, log_detJ, zy)
        if len(self.squeeze_factor_layers_list) == 0:           # :1755-1757
            return uv, log_detJ
        zy = _concat(zy, uv)                                    # :1762
        vu = None
        for layer in reversed(self.squeeze_factor_layers_list):  # :1767-1770
            vu, zy = layer.backward(vu, zy)
        return vu, log_detJ

    def _call_layerwise_inverse(self, uv):
        zy = None
        if self.squeeze_factor_layers_list:                     # :1782-1788
            for layer in self.squeeze_factor_layers_list:
                uv, _, zy = layer.forward_and_Jacobian(uv, None, zy)
        vu = uv
        for layer in reversed(self.layers_list):                # :1793-1796
            vu, zy = layer.backward(vu, zy)
        return vu

    # -- loss -----------------------------------------------------------------------------------
    def nll_sums(self, xy, zy=None, logdet_per_image=None):
        """Per-batch sums of the NLL terms on device: (sum loss_i, sum -llz_i, sum -lly_i,
        sum -logdet_i) and the per-image (llz, lly, logdet) table."""
        xy = _as_input(xy, 'xy')
        B = xy.shape[0]
        if zy is None:
            zy, logdet_per_image = self.call(xy, 1, per_image_logdet=True)
        per = torch.empty((B, 3), device=xy.device, dtype=torch.float32)
        sums = torch.empty(4, device=xy.device, dtype=torch.float32)
        check(_lib.load().cnf_nll(self._plan, ptr(xy), ptr(zy), ptr(logdet_per_image), ptr(per), ptr(sums), B,
                                  _stream()), 'cnf_nll')
        return sums, per

    def log_loss(self, xy, process_group=None, noise=None):
        """cFlow.log_loss (:1800-1848): (loss, z_loss, y_loss, detJ_loss), batch means.
        With process_group given (True = the default group) and torch.distributed initialised,
        this rank's 4 sums and its image count are all-reduced (one collective of 5 fp32,
        distributed.reduce_nll_sums) so the means are over the global batch; shards may be
        ragged. noise=(alpha, seed, offset): the loss of the instance-noised input (call(noise=...):
        the noise applied inside the forward's first kernel, y' taken from the noisy input)."""
        from .distributed import reduce_nll_sums
        xy = _as_input(xy, 'xy')
        if noise is not None:
            zy, ld, xn = self.call(xy, 1, per_image_logdet=True, noise=noise)
            sums, _ = self.nll_sums(xn, zy, ld)
        else:
            sums, _ = self.nll_sums(xy)
        grp = None if process_group is True else process_group
        return reduce_nll_sums(sums, xy.shape[0], group=grp, all_reduce=process_group is not None)

    # -- training -------------------------------------------------------------------------------
    def compile(self, optimizer=None):
        """keras Model.compile(optimizer=Adam(...)) (conv_cINN.py:567-569)."""
        from .optimizers import Adam
        self.optimizer = optimizer if optimizer is not None else Adam()

    def _train_workspace(self, B):
        key = ('train', B)
        ws = self._ws.get(key)
        if ws is None:
            nbytes = int(_lib.load().cnf_plan_train_workspace_bytes(self._plan, B))
            if nbytes <= 0:
                raise RuntimeError(_lib.load().cnf_last_error().decode())
            ws = torch.empty(nbytes, device=self.device, dtype=torch.uint8)
            self._ws[key] = ws
        return ws

    def _coupling_param_ranges(self):
        """{coupling index: (lo, hi)} of its parameters (names 'c<i>.*') in the flat canonical vector."""
        r = getattr(self, '_cranges', None)
        if r is None:
            r = {}
            for n, o, s in self.param_specs:
                ci = int(n.split('.', 1)[0][1:])
                size = int(np.prod(s)) if s else 1
                lo, hi = r.get(ci, (o, o))
                if o != hi:
                    raise RuntimeError(f'parameters of coupling {ci} are not contiguous')
                r[ci] = (lo, o + size)
            self._cranges = r
        return r

    def gradients(self, xy, process_group=None, overlap=None):
        """tape.gradient(loss, trainable_variables) of train_step (:1863-1869) as one flat
        vector in the canonical parameter order, plus the 4 loss terms (batch means, device
        scalars). With process_group (True = default group) the loss sums and the gradient are
        all-reduced, so both are those of the global batch: the 5-float loss all-reduce runs
        between forward and backward with no host read of its result (the backward takes the
        global image count from the device buffer), and each coupling layer's gradient range is
        all-reduced asynchronously as soon as that layer's backward is enqueued, overlapping the
        backward of the layers before it (the default on RCCL; overlap=False / True forces it off / on)."""
        from .distributed import allreduce_grads, pack_nll_sums
        xy = _as_input(xy, 'xy')
        if tuple(xy.shape[1:]) != tuple(self.io_shape):
            raise ValueError(f'input shape {tuple(xy.shape)} != [None, {self.io_shape}]')
        lib = _lib.load()
        B = xy.shape[0]
        ws = self._train_workspace(B)
        zy = torch.empty_like(xy)
        ld = torch.empty(B, device=xy.device, dtype=torch.float32)
        check(lib.cnf_flow_forward_train(self._plan, ptr(self.params), ptr(self._aux), ptr(xy), ptr(zy), ptr(ld),
                                         ptr(ws), B, _stream()), 'cnf_flow_forward_train')
        sums, _ = self.nll_sums(xy, zy, ld)
        buf = pack_nll_sums(sums, B)
        grp = None if process_group is True else process_group
        dist = None
        if process_group is not None:
            import torch.distributed as tdist
            if tdist.is_available() and tdist.is_initialized():
                dist = tdist
        if dist is not None:
            dist.all_reduce(buf, group=grp)
        if getattr(self, '_grads', None) is None or self._grads.numel() != self.num_params:
            self._grads = torch.empty(self.num_params, device=self.device, dtype=torch.float32)
        # the per-layer asynchronous all-reduce overlaps on RCCL (stream-ordered); gloo copies every range
        # through the host with a device sync per call, which the measured 1-GPU 2-rank rehearsal ran 33x
        # slower than one all-reduce after the backward: overlap by default on 'nccl' only
        if overlap is None:
            overlap = dist is not None and dist.get_backend(grp) == 'nccl'
        overlap = bool(overlap) and dist is not None
        works = []
        errors = []
        reported = []
        if overlap:
            ranges = self._coupling_param_ranges()
            grads = self._grads

            def done(_user, ci):
                # an exception must not escape into C (ctypes would print it and return, and this rank
                # would silently skip the layer's all-reduce while the other ranks pair it with the next)
                try:
                    reported.append(ci)
                    lo, hi = ranges[ci]
                    works.append(dist.all_reduce(grads[lo:hi], group=grp, async_op=True))
                except BaseException as e:   # noqa: BLE001 -- re-raised below
                    errors.append(e)
            cb = _lib.LAYER_DONE_FN(done)
        else:
            cb = _lib.LAYER_DONE_FN()
        check(lib.cnf_flow_backward_ex(self._plan, ptr(self.params), ptr(xy), ptr(zy), ptr(ws), B, ptr(buf) + 16,
                                       ptr(self._grads), cb, None, _stream()), 'cnf_flow_backward_ex')
        if overlap and not errors and sorted(reported) != sorted(self._coupling_param_ranges()):
            errors.append(RuntimeError(f'layer_done reported couplings {sorted(reported)}, expected each of '
                                       f'{sorted(self._coupling_param_ranges())} once'))
        if errors:
            # this rank's collective sequence no longer matches the other ranks': raised before any wait
            # (a wait could hang); the caller decides whether to abort the process group
            raise RuntimeError('per-layer gradient all-reduce failed') from errors[0]
        for w in works:
            w.wait()
        if dist is not None and not overlap:
            allreduce_grads(self._grads, group=grp)
        m = buf[:4] / buf[4]
        return self._grads, (m[0], m[1], m[2], m[3])

    def train_step(self, xy, process_group=None, overlap=None):
        """cFlow.train_step (:1850-1880): NLL gradient (GradientTape), optimizer.apply_gradients,
        Mean trackers; returns {'loss', 'z_loss', 'y_loss', 'detJ_loss'} as 0-d device tensors (TF
        returns tensors too; float() reads one). Data-parallel with process_group: the loss sums and
        the gradient are all-reduced over the global batch."""
        if getattr(self, 'optimizer', None) is None:
            self.compile()
        grads, terms = self.gradients(xy, process_group, overlap)
        self.optimizer.apply_flat(self.params, grads)
        check(_lib.load().cnf_pack_params(self._plan, ptr(self.params), ptr(self._aux), _stream()), 'pack params')
        for t, v in zip(self.metrics, terms):   # device scalars: no host sync (the trackers stay on the device)
            t.update_state(v)
        return {t.name: t.result() for t in self.metrics}

    def test_step(self, xy, process_group=None):
        """:1882-1904 — loss without a weight update; updates the Mean trackers. With
        process_group the loss terms are global-batch means (log_loss), the same on every rank."""
        loss, lz, ly, ld = self.log_loss(xy, process_group=process_group)
        for t, v in zip(self.metrics, (loss, lz, ly, ld)):
            t.update_state(v)
        return {t.name: t.result() for t in self.metrics}
