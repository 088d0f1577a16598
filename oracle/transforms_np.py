"""TEST INFRASTRUCTURE ONLY — numpy restatement of the reference's input transforms
(conv_cINN_base_functions.py), the checker for cnf_logit / cnf_sr_preprocess / cnf_down / cnf_up /
cnf_instance_noise. Pinned by known-answer tests in tests/test_transforms.py (exact block means
on arange inputs, the logit map's endpoints, logit o de_logitify = identity); the TF originals
cannot run here, so parity against TF itself is unpinned.
"""
from __future__ import annotations

import numpy as np


def down(img):
    """2x2 average pool (conv_cINN_base_functions.py:74-125): crops to even H, W; accepts HxWxD or
    BxHxWxD."""
    img = np.asarray(img)
    batch = img.ndim == 4
    if not batch:
        img = img[None]
    B, M, N, D = img.shape
    MK, NL = M // 2, N // 2
    x = img[:, :MK * 2, :NL * 2, :].reshape(B, MK, 2, NL, 2, D)
    out = x.mean(axis=(2, 4))
    return out if batch else out[0]


def up(img):
    """2x2 repeat in H and W (:127-160)."""
    img = np.asarray(img)
    batch = img.ndim == 4
    if not batch:
        img = img[None]
    out = np.repeat(np.repeat(img, 2, axis=1), 2, axis=2)
    return out if batch else out[0]


def _logit(x):
    return np.log(x / (1 - x))


def logit_preprocess(x, a=0.01):
    """preprocess_dataset_class(LOGITS=True) element map (:174-231)."""
    b = (1 - 2 * a) / (1 - a)
    lo, hi = _logit(a), _logit(1 - a)
    return (_logit(a + (1 - a) * b * np.asarray(x, np.float64)) - lo) / (hi - lo)


def de_logitify(x, a=0.01):
    """:287-318."""
    lo, hi = _logit(a), _logit(1 - a)
    b = (1 - 2 * a) / (1 - a)
    z = np.asarray(x, np.float64) * (hi - lo) + lo
    return (1 / (1 + np.exp(-z)) - a) / (b * (1 - a))


def sr_preprocess(hires, x_down=0, y_levels=1, residual=True):
    """preprocess_dataset_SR (:233-279) generalised to y_levels nested downsamplings:
    x0 = down^x_down(h), y = up^y_levels(down^y_levels(x0)), x = x0 - y (RESIDUAL), xy = concat."""
    x0 = np.asarray(hires, np.float64)
    for _ in range(x_down):
        x0 = down(x0)
    y = x0
    for _ in range(y_levels):
        y = down(y)
    for _ in range(y_levels):
        y = up(y)
    x = x0 - y if residual else x0
    return np.concatenate([x, y], axis=-1)
