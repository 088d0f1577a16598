"""Drop-in replacement for the reference's `TOYcINN_make_model.cINN_affine` (BASELINE configs[0]).

Same constructor arguments, `call(u, direction=-1)` / `log_loss` / `test_step` / `metrics`
semantics as TOYcINN_make_model.py:105-506, on torch tensors [B, 3] fp32 on the ROCm device; the
flow runs in libcnf_hip.so (k_toy) through the C ABI. Note the toy's direction convention is the
reverse of cFlow's: -1 maps xy' -> zy (training direction, returns the per-sample log-det),
+1 maps zy -> xy'.

Parameters: per coupling network j (mask type j % 6), the b net then the A net, each Dense as
kernel [in][out] then bias [out] (oracle.toy_np.net_specs order / names `t{j}.{b|A}.d{k}.*`).
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Dict, Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr
from .make_model import Mean, _as_input, _stream

MASK_U1 = {0: [0], 1: [1], 2: [2], 3: [0, 1], 4: [0, 2], 5: [1, 2]}


def _default_mask_indices(n: int, seed: int):
    """arange(n) shuffled within consecutive groups of 6 (:192-205; seeded here)."""
    rng = np.random.default_rng(seed)
    out = []
    for g in range(n // 6):
        blk = np.arange(6 * g, 6 * (g + 1))
        rng.shuffle(blk)
        out.extend(int(v) for v in blk)
    out.extend(range(6 * (n // 6), n))
    return out


class cINN_affine:
    """TOYcINN_make_model.cINN_affine (:105-506)."""

    def __init__(self, io_shape, x_d, num_coupling_layers, intermediate_dims, num_layers, init=None,
                 mask_indices: Optional[Sequence[int]] = None, device=None, seed: int = 0):
        self.io_shape = int(io_shape)
        self.x_d = int(x_d)
        self.num_coupling_layers = int(num_coupling_layers)
        self.intermediate_dims = int(intermediate_dims)
        self.num_layers = int(num_layers)
        self.init = init   # stored, unused — as in the reference (:138)
        self.lambda_y = 100
        self.device = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        self.mask_indices = list(mask_indices) if mask_indices else _default_mask_indices(num_coupling_layers, seed)
        self._order = (C.c_int * len(self.mask_indices))(*self.mask_indices)
        self._desc = _lib.cnf_toy_desc(self.io_shape, self.x_d, self.num_coupling_layers, self.intermediate_dims,
                                       self.num_layers, self._order, float(self.lambda_y))
        lib = _lib.load()
        n = lib.cnf_toy_num_params(C.byref(self._desc))
        if n < 0:
            raise AssertionError(lib.cnf_last_error().decode())
        self.num_params = int(n)
        self.params = torch.empty(self.num_params, device=self.device, dtype=torch.float32)
        self._init_weights(seed)
        self.loss_tracker = Mean('loss')
        self.z_loss_tracker = Mean('z_loss')
        self.y_loss_tracker = Mean('y_loss')
        self.detJ_loss_tracker = Mean('detJ_loss')

    # -- parameters ----------------------------------------------------------------------------
    def param_specs(self):
        specs = []
        H, L = self.intermediate_dims, self.num_layers
        for j in range(self.num_coupling_layers):
            u1 = len(MASK_U1[j % 6])
            u2 = self.io_shape - u1
            for blk in ('b', 'A'):
                dims = [u1] + [H] * (L + 1) + [u2]
                for k in range(L + 2):
                    specs.append((f't{j}.{blk}.d{k}.kernel', (dims[k], dims[k + 1])))
                    specs.append((f't{j}.{blk}.d{k}.bias', (dims[k + 1],)))
        return specs

    def _init_weights(self, seed):
        """glorot_uniform kernels, zero biases (Keras Dense defaults)."""
        rng = np.random.default_rng(seed)
        flat = []
        for n, s in self.param_specs():
            if n.endswith('.kernel'):
                lim = math.sqrt(6.0 / (s[0] + s[1]))
                flat.append(rng.uniform(-lim, lim, s).reshape(-1))
            else:
                flat.append(np.zeros(s).reshape(-1))
        self.set_weights(np.concatenate(flat))

    def set_weights(self, weights):
        if isinstance(weights, dict):
            weights = np.concatenate([np.asarray(weights[n], np.float32).reshape(-1) for n, _ in self.param_specs()])
        w = torch.as_tensor(np.ascontiguousarray(weights, dtype=np.float32)) if isinstance(weights, np.ndarray) \
            else weights
        if w.numel() != self.num_params:
            raise ValueError(f'expected {self.num_params} parameters, got {w.numel()}')
        self.params.copy_(w.reshape(-1).to(self.device, torch.float32))

    def get_weights(self) -> Dict[str, np.ndarray]:
        flat = self.params.detach().cpu().numpy()
        out, o = {}, 0
        for n, s in self.param_specs():
            size = int(np.prod(s))
            out[n] = flat[o:o + size].reshape(s)
            o += size
        return out

    @property
    def metrics(self):
        return [self.loss_tracker, self.z_loss_tracker, self.y_loss_tracker, self.detJ_loss_tracker]

    # -- the flow --------------------------------------------------------------------------------
    def _run(self, u, direction, want_terms=False):
        u = _as_input(u, 'u')
        if u.dim() != 2 or u.shape[1] != self.io_shape:
            raise AssertionError(f'u must have shape (batch, {self.io_shape})')
        B = u.shape[0]
        v = torch.empty_like(u)
        ld = torch.empty(B, device=u.device, dtype=torch.float32) if direction == -1 else None
        per = torch.empty((B, 3), device=u.device, dtype=torch.float32) if want_terms else None
        check(_lib.load().cnf_toy_call(C.byref(self._desc), ptr(self.params), ptr(u), ptr(v),
                                       ptr(ld) if ld is not None else None,
                                       ptr(per) if per is not None else None, B, direction, _stream()),
              'cnf_toy_call')
        return v, ld, per

    def call(self, u, direction=-1):
        """(:237-417) direction -1: xy' -> (zy, log_detJ[B]); +1: zy -> (xy', 0)."""
        if direction not in (-1, 1):
            raise AssertionError('direction must be -1 or +1')
        v, ld, _ = self._run(u, direction)
        return v, (ld if direction == -1 else 0)

    __call__ = call

    def log_loss(self, xy, process_group=None):
        """(:419-451) -> (loss, -mean llz, -mean lly, -mean log_detJ); with process_group the 4 sums
        and the sample count are all-reduced (one 5-float collective)."""
        from .distributed import reduce_nll_sums
        xy = _as_input(xy, 'xy')
        _, _, per = self._run(xy, -1, want_terms=True)
        sums = torch.empty(4, device=xy.device, dtype=torch.float32)
        check(_lib.load().cnf_toy_nll_sums(ptr(per), ptr(sums), xy.shape[0], _stream()), 'cnf_toy_nll_sums')
        grp = None if process_group is True else process_group
        return reduce_nll_sums(sums, xy.shape[0], group=grp, all_reduce=process_group is not None)

    def train_step(self, xy):
        raise NotImplementedError('the NLL training step (backward kernels + Adam) is the next milestone; '
                                  'see DESIGN.md')

    def test_step(self, xy):
        """(:483-506) loss without a weight update; updates the Mean trackers."""
        vals = [t.item() for t in self.log_loss(xy)]
        for tr, v in zip(self.metrics, vals):
            tr.update_state(v)
        return {tr.name: tr.result() for tr in self.metrics}
