"""Synthetic inputs of the BASELINE shapes (there is no dataset access). Distributions follow
the reference's data pipelines:

class  x ~ U(0,1); y-plane = k/9 for a class k ~ U{0..9} (conv_cINN.py:221-228, 259-261);
       xy <- 0.98 xy + 0.02 N(0,1) on all channels (conv_cINN.py:312-315).
sr     hi-res h ~ U(0,1); y = up^p(down^p(h)) (conv_cINN_base_functions.py:74-164);
       x = h - y (RESIDUAL, conv_cINN.py:45); + 2% instance noise.
"""
from __future__ import annotations

import numpy as np


def class_batch(B, H, W, x_d=3, seed=0, noise_alpha=0.98, num_classes=10):
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, 1, (B, H, W, x_d))
    k = rng.integers(0, num_classes, B)
    y = np.broadcast_to((k / (num_classes - 1)).reshape(B, 1, 1, 1), (B, H, W, 1))
    xy = np.concatenate([x, y], axis=-1)
    xy = noise_alpha * xy + (1 - noise_alpha) * rng.standard_normal(xy.shape)
    return xy.astype(np.float32)


def _down(img):
    B, H, W, C = img.shape
    return img.reshape(B, H // 2, 2, W // 2, 2, C).mean(axis=(2, 4))


def _up(img):
    return img.repeat(2, axis=1).repeat(2, axis=2)


def sr_batch(B, H, W, C=3, factor_pow=2, seed=0, noise_alpha=0.98):
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
