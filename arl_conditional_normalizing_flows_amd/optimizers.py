"""Keras-compatible Adam for the training step (conv_cINN.py:567-569
`model.compile(optimizer=tf.keras.optimizers.Adam(learning_rate=...))`).

The update runs on the device (k_adam through `cnf_adam_step`) over the flat canonical parameter
vector, with the moment buffers kept as two more flat fp32 vectors of the same size (288 GB of HBM
holds them next to every activation of the largest BASELINE configuration). Keras semantics:
    m += (g - m)(1 - beta_1);  v += (g^2 - v)(1 - beta_2)
    p -= lr sqrt(1 - beta_2^t) / (1 - beta_1^t) * m / (sqrt(v) + epsilon)
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import check, ptr


class Adam:
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.learning_rate = float(learning_rate)
        self.beta_1 = float(beta_1)
        self.beta_2 = float(beta_2)
        self.epsilon = float(epsilon)
        self.iterations = 0
        self._m = None
        self._v = None

    def _slots(self, params: torch.Tensor):
        if self._m is None or self._m.numel() != params.numel() or self._m.device != params.device:
            self._m = torch.zeros_like(params)
            self._v = torch.zeros_like(params)
        return self._m, self._v

    def apply_flat(self, params: torch.Tensor, grads: torch.Tensor):
        """One Adam step on the flat parameter vector (in place)."""
        m, v = self._slots(params)
        self.iterations += 1
        check(_lib.load().cnf_adam_step(ptr(params), ptr(grads), ptr(m), ptr(v), params.numel(), self.learning_rate,
                                        self.beta_1, self.beta_2, self.epsilon, self.iterations,
                                        torch.cuda.current_stream().cuda_stream), 'cnf_adam_step')
