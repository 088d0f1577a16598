"""GPU input transforms mirroring conv_cINN_base_functions.py (the step before the flow).

Same names and argument meaning as the reference; tensors are torch tensors on the ROCm device
(NHWC fp32), the work runs in libcnf_hip.so (cnf_transforms.hip) through the C ABI. The
reference applies these per tf.data element (`dataset.map`); here they take whole batches.

  down / up                   conv_cINN_base_functions.py:74-160
  preprocess_dataset_class    :174-231  (LOGITS=True logit map; identity otherwise)
  preprocess_dataset_SR       :233-279  (model_type 'SR4,2' / 'SR2,1'; y_levels generalises it)
  de_logitify                 :287-318
  instance_noise / renew_noise :635-676 (Philox4x32-10 normals: reproducible, not TF's stream)
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import check, ptr


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _dev(t, what):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f'{what} must be a torch tensor on the ROCm device (no CPU fallback)')
    return t.float().contiguous()


def _batched(img):
    img = _dev(img, 'img')
    if img.dim() == 3:
        return img[None], False
    if img.dim() != 4:
        raise ValueError('expected HxWxD or BxHxWxD')
    return img, True


def down(img):
    """2x2 average-pooled downsampling (:74-125); odd trailing rows/columns are cropped."""
    x, batch = _batched(img)
    B, H, W, C = x.shape
    out = torch.empty((B, H // 2, W // 2, C), device=x.device, dtype=torch.float32)
    check(_lib.load().cnf_down(ptr(x), ptr(out), B, H, W, C, _stream()), 'cnf_down')
    return out if batch else out[0]


def up(img):
    """2x2-repeated upscaling (:127-160)."""
    x, batch = _batched(img)
    B, H, W, C = x.shape
    out = torch.empty((B, 2 * H, 2 * W, C), device=x.device, dtype=torch.float32)
    check(_lib.load().cnf_up(ptr(x), ptr(out), B, H, W, C, _stream()), 'cnf_up')
    return out if batch else out[0]


def preprocess_dataset_class(x, LOGITS=False, a=0.01):
    """x in [0, 1] -> logit(a + (1-a) b x) rescaled to [0, 1] when LOGITS (:174-231), else x."""
    x = _dev(x, 'x')
    if not LOGITS:
        return x
    out = torch.empty_like(x)
    check(_lib.load().cnf_logit(ptr(x), ptr(out), x.numel(), float(a), 0, _stream()), 'cnf_logit')
    return out


def de_logitify(x, a=0.01):
    """Inverse of the logit preprocessing (:287-318)."""
    x = _dev(x, 'x')
    out = torch.empty_like(x)
    check(_lib.load().cnf_logit(ptr(x), ptr(out), x.numel(), float(a), 1, _stream()), 'cnf_logit')
    return out


_SR_TYPES = {'SR4,2': (1, 1), 'SR2,1': (0, 1)}


def preprocess_dataset_SR(x_hires, model_type='SR2,1', RESIDUAL=True, y_levels=None):
    """Hi-res batch [B,H,W,C] -> xy = concat(x, y) (:233-279). model_type 'SR4,2' / 'SR2,1' as in
    the reference; y_levels overrides the number of 2x2 levels in y (the 4x / 8x configs: 2 / 3)."""
    h, batch = _batched(x_hires)
    if model_type not in _SR_TYPES:
        raise ValueError(f"model_type must be one of {sorted(_SR_TYPES)}")
    xd, yl = _SR_TYPES[model_type]
    if y_levels is not None:
        yl = int(y_levels)
    B, H, W, C = h.shape
    xy = torch.empty((B, H >> xd, W >> xd, 2 * C), device=h.device, dtype=torch.float32)
    check(_lib.load().cnf_sr_preprocess(ptr(h), ptr(xy), B, H, W, C, xd, yl, int(bool(RESIDUAL)), _stream()),
          'cnf_sr_preprocess')
    return xy if batch else xy[0]


def instance_noise(x_element, alpha, seed=0, offset=0):
    """alpha x + (1 - alpha) N(0, 1) (:635-654)."""
    x = _dev(x_element, 'x_element')
    out = torch.empty_like(x)
    check(_lib.load().cnf_instance_noise(ptr(x), ptr(out), x.numel(), float(alpha), int(seed) & (2 ** 64 - 1),
                                         int(offset), _stream()), 'cnf_instance_noise')
    return out


def renew_noise(element, seed=0, offset=0):
    """A fresh N(0, 1) tensor of the element's shape (:660-676)."""
    e = _dev(element, 'element')
    out = torch.empty_like(e)
    check(_lib.load().cnf_instance_noise(None, ptr(out), out.numel(), 0.0, int(seed) & (2 ** 64 - 1), int(offset),
                                         _stream()), 'cnf_instance_noise')
    return out
