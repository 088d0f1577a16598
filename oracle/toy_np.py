"""TEST INFRASTRUCTURE ONLY — float64 numpy restatement of the reference's TOYcINN model
(BASELINE configs[0]): `TOYcINN_make_model.cINN_affine` and its dense
`coupling_layer`, plus the crescents data of `TOYcINN_make_datasets.make_moons_dataset`.

Reference semantics reproduced (file:line in TOYcINN_make_model.py unless stated):
  * coupling_layer(u1, u2, H, L) :29-97 — two dense nets on u1: b = Dense(H)+LReLU, L x
    [Dense(H)+LReLU], Dense(u2) (linear); A = same stack, Dense(u2), then tanh (no learned scale,
    :90-95). LeakyReLU alpha = 0.3 (Keras default). Kernel init glorot_uniform, bias 0 (the `init`
    argument is stored but never used, :138).
  * masks :149-190 — mask type t = j % 6: u1 = {[0], [1], [2], [0,1], [0,2], [1,2]}[t],
    u2 = the complement; network j and mask j travel together (coupling_layers_list[j]).
  * mask_indices :192-205 — arange(L) shuffled within consecutive groups of 6 when not given
    (the reference uses the unseeded global numpy RNG; here an explicit seed).
  * call(u, direction=-1) :237-417 — direction -1 is the TRAINING direction xy' -> zy, layers in
    reverse index order, v2 = exp(A(u1)) u2 + b(u1), log_detJ += sum(A) PER SAMPLE (:386-387);
    direction +1 is zy -> xy', layers in index order, u2 = (v2 - b) / exp(A).
  * log_loss :419-451 — -(mean(log N(z; 0, I_xd) + (-lambda_y sum|y - y'|) + log_detJ)), lambda_y 100;
    returns (loss, -mean llz, -mean lly, -mean log_detJ).

Parity unpinned against TensorFlow for the same reason as oracle/cflow_np.py (TF absent, no
reference vectors); pinned by the invariant tests in tests/test_toy.py (exact inverse, brute-force
log|det J|, per-layer volume change).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

LRELU_ALPHA = 0.3
LOG_2PI = math.log(2.0 * math.pi)

MASK_U1 = {0: [0], 1: [1], 2: [2], 3: [0, 1], 4: [0, 2], 5: [1, 2]}   # :149-155
MASK_U2 = {0: [1, 2], 1: [0, 2], 2: [0, 1], 3: [2], 4: [1], 5: [0]}   # :157-163


def default_mask_indices(num_coupling_layers: int, seed: int = 0) -> List[int]:
    """arange(L) shuffled within groups of 6 (:192-205); a remainder beyond the last full group
    keeps its order (the reference drops it from the shuffle array)."""
    rng = np.random.default_rng(seed)
    idx = np.arange(num_coupling_layers, dtype=np.int64)
    out = []
    for g in range(num_coupling_layers // 6):
        blk = idx[6 * g:6 * (g + 1)].copy()
        rng.shuffle(blk)
        out.extend(int(v) for v in blk)
    out.extend(int(v) for v in idx[6 * (num_coupling_layers // 6):])
    return out


def net_specs(j: int, io_shape: int, H: int, L: int) -> List[Tuple[str, Tuple[int, ...]]]:
    """Parameters of coupling network j in construction order (:48-94): b-block then A-block;
    each Dense(in -> out) is (kernel [in][out], bias [out])."""
    t = j % 6
    u1, u2 = len(MASK_U1[t]), len(MASK_U2[t])
    specs = []
    for blk in ('b', 'A'):
        dims = [u1] + [H] * (L + 1) + [u2]
        for k in range(L + 2):
            specs.append((f't{j}.{blk}.d{k}.kernel', (dims[k], dims[k + 1])))
            specs.append((f't{j}.{blk}.d{k}.bias', (dims[k + 1],)))
    return specs


def lrelu(x):
    return np.where(x >= 0, x, LRELU_ALPHA * x)


def dense_net(u1, P, j, blk, L):
    h = u1
    for k in range(L + 1):
        h = lrelu(h @ P[f't{j}.{blk}.d{k}.kernel'] + P[f't{j}.{blk}.d{k}.bias'])
    return h @ P[f't{j}.{blk}.d{L + 1}.kernel'] + P[f't{j}.{blk}.d{L + 1}.bias']


class ToyCINN:
    """cINN_affine (:105-506) with explicit parameters."""

    def __init__(self, io_shape: int = 3, x_d: int = 2, num_coupling_layers: int = 24,
                 intermediate_dims: int = 32, num_layers: int = 6, mask_indices: Optional[Sequence[int]] = None,
                 lambda_y: float = 100.0, mask_seed: int = 0):
        if io_shape != 3:
            raise AssertionError('the reference masks are defined for 3-dimensional xy only (:149-163)')
        self.io_shape = io_shape
        self.x_d = x_d
        self.L = num_coupling_layers
        self.H = intermediate_dims
        self.num_layers = num_layers
        self.lambda_y = float(lambda_y)
        self.mask_indices = list(mask_indices) if mask_indices else default_mask_indices(self.L, mask_seed)
        if sorted(self.mask_indices) != list(range(self.L)):
            raise AssertionError('mask_indices must be a permutation of range(num_coupling_layers)')
        self.specs = []
        for j in range(self.L):
            self.specs += net_specs(j, io_shape, self.H, self.num_layers)

    def num_params(self):
        return int(sum(int(np.prod(s)) for _, s in self.specs))

    def init_params(self, seed: int = 0, bias_std: float = 0.01) -> Dict[str, np.ndarray]:
        """glorot_uniform kernels (Keras Dense default); biases ~N(0, bias_std) instead of 0 so
        that every parameter is exercised by the tests."""
        rng = np.random.default_rng(seed)
        P = {}
        for n, s in self.specs:
            if n.endswith('.kernel'):
                lim = math.sqrt(6.0 / (s[0] + s[1]))
                P[n] = rng.uniform(-lim, lim, s)
            else:
                P[n] = rng.normal(0.0, bias_std, s)
        return P

    def coupling(self, u, P, j, direction, with_abs=False):
        t = j % 6
        i1, i2 = MASK_U1[t], MASK_U2[t]
        u1, u2 = u[:, i1], u[:, i2]
        b = dense_net(u1, P, j, 'b', self.num_layers)
        A = np.tanh(dense_net(u1, P, j, 'A', self.num_layers))
        v = u.copy()
        if direction == -1:
            v[:, i2] = np.exp(A) * u2 + b
            if with_abs:
                return v, A.sum(axis=1), np.abs(A).sum(axis=1)
            return v, A.sum(axis=1)
        v[:, i2] = (u2 - b) / np.exp(A)
        return (v, None, None) if with_abs else (v, None)

    def call(self, u, P, direction=-1, abs_s=False):
        """(:237-417) returns (v, log_detJ[B]) for direction -1 and (v, None) for +1. abs_s=True
        (direction -1) also returns the per-sample sum over layers of |A| (the log-det's
        conditioning scale, the Sum|s| of the north-star bound)."""
        u = np.asarray(u, np.float64)
        P = {k: np.asarray(v, np.float64) for k, v in P.items()}
        ld = np.zeros(u.shape[0])
        sa = np.zeros(u.shape[0])
        for i in list(range(self.L))[::direction]:
            u, d, a = self.coupling(u, P, self.mask_indices[i], direction, with_abs=True)
            if d is not None:
                ld = ld + d
                sa = sa + a
        if abs_s:
            return u, (ld if direction == -1 else None), (sa if direction == -1 else None)
        return u, (ld if direction == -1 else None)

    def log_loss(self, xy, P):
        xy = np.asarray(xy, np.float64)
        zy, ld = self.call(xy, P, -1)
        x_d = self.x_d
        z, y, yp = zy[:, :x_d], zy[:, x_d:], xy[:, x_d:]
        llz = -0.5 * (z * z).sum(axis=1) - 0.5 * x_d * LOG_2PI
        lly = -self.lambda_y * np.abs(y - yp).sum(axis=1)
        loss = -(llz + lly + ld).mean()
        return loss, -llz.mean(), -lly.mean(), -ld.mean()


def flatten(P: Dict[str, np.ndarray], specs) -> np.ndarray:
    return np.concatenate([np.asarray(P[n], np.float64).reshape(-1) for n, _ in specs])


def my_make_moons(n_per: int, noise: float, overlapping: bool, rng) -> Tuple[np.ndarray, np.ndarray]:
    """TOYcINN_make_datasets.py:36-103 (sklearn.make_moons adaptation)."""
    t = np.linspace(0, math.pi, n_per)
    x = np.concatenate([np.cos(t), 1 - np.cos(t)])
    y2 = 1 - np.sin(t) + (0.25 if overlapping else -0.5)
    yv = np.concatenate([np.sin(t), y2])
    X = np.stack([x, yv], axis=1)
    Y = np.concatenate([np.zeros(n_per), (2.0 if overlapping else 1.0) * np.ones(n_per)])
    X = X + rng.normal(0.0, noise, X.shape)
    return X, Y


def moons_batch(batch: int, cls: int, noise: float = 0.05, overlapping: bool = False, seed: int = 0) -> np.ndarray:
    """One single-class batch [batch, 3] of standardised crescent points (:105-270): mean/std from
    a 10^4-per-crescent reference cloud, angle ~U(0, pi), Gaussian noise on both coordinates."""
    rng = np.random.default_rng(seed)
    Xr, Yr = my_make_moons(10 ** 4, noise, overlapping, rng)
    xy_ref = np.concatenate([Xr, Yr[:, None]], axis=1)
    mean = xy_ref.mean(axis=0).astype(np.float32)
    std = xy_ref.std(axis=0).astype(np.float32)
    ang = rng.uniform(0.0, math.pi, batch)
    if cls == 0:
        x0, x1 = np.cos(ang), np.sin(ang)
    else:
        x0, x1 = 1 - np.cos(ang), 1 - np.sin(ang) + (0.25 if overlapping else -0.5)
    x0 = x0 + rng.normal(0.0, noise, batch)
    x1 = x1 + rng.normal(0.0, noise, batch)
    yl = np.full(batch, float(cls if cls == 0 else (2 if overlapping else 1)))
    xy = np.stack([x0, x1, yl], axis=1)
    return ((xy - mean) / std).astype(np.float32)
