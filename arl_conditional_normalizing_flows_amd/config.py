"""Model configurations: a frozen mirror of the cFlow constructor arguments
(conv_cINN_make_model.py:1431-1442) plus the named BASELINE.json presets
(architectures per SURVEY.md §8; the reference itself ships only the 28x28 MNIST one,
conv_cINN.py:56-65)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Tuple


@dataclass(frozen=True)
class FlowConfig:
    io_shape: Tuple[int, int, int]
    x_d: int
    squeeze_factor_block_list: Tuple[int, ...]
    ResNeXt_block_list: Tuple[int, ...]
    num_kernels_list: Tuple[int, ...]
    cardinality_list: Tuple[int, ...]
    lambda_y: float = 100.0
    ksize: int = 3
    LAYER_NORM: bool = True
    DILATIONS: bool = True
    group_mode: str = 'reference'
    batch: int = 1
    data: str = 'class'          # synthetic input family: 'class' or 'sr'
    sr_pow: int = 2              # SR: y = up^p(down^p(h))
    name: str = ''

    def kwargs(self):
        return dict(io_shape=list(self.io_shape), x_d=self.x_d,
                    squeeze_factor_block_list=list(self.squeeze_factor_block_list),
                    ResNeXt_block_list=list(self.ResNeXt_block_list),
                    num_kernels_list=list(self.num_kernels_list),
                    cardinality_list=list(self.cardinality_list),
                    lambda_y=self.lambda_y, ksize=self.ksize, LAYER_NORM=self.LAYER_NORM,
                    DILATIONS=self.DILATIONS, group_mode=self.group_mode)


PRESETS = {
    # reference default architecture (conv_cINN.py:56-65), 28x28 fMNIST SR2,1 -> xy 28x28x2
    'ref_default': FlowConfig((28, 28, 2), 1, (0, 1, 0, 0), (3, 3, 3, 3), (64, 64, 32, 32), (8, 8, 4, 4),
                              batch=32, data='sr', sr_pow=1, name='ref_default'),
    # BASELINE configs[1]: 32x32x3 class-conditioned, 3-scale, batch 64 (the headline metric)
    'cfg2': FlowConfig((32, 32, 4), 3, (0, 1, 1, 0), (3, 3, 3, 3), (64, 64, 32, 16), (8, 8, 4, 2),
                       batch=64, data='class', name='cfg2'),
    # configs[2]: 32x32 4x super-resolution (8x8 content in y), batch 128
    'cfg3': FlowConfig((32, 32, 6), 3, (0, 1, 1, 0), (3, 3, 3, 3), (64, 64, 32, 16), (8, 8, 4, 2),
                       batch=128, data='sr', sr_pow=2, name='cfg3'),
    # configs[3]: 64x64x3 class-conditioned, 4-scale, batch 256 global
    'cfg4': FlowConfig((64, 64, 4), 3, (0, 1, 1, 1, 0), (3, 3, 3, 3, 3), (64, 64, 32, 16, 8), (4, 4, 2, 2, 2),
                       batch=256, data='class', name='cfg4'),
    # configs[4]: 128x128 8x SR, 5-scale, batch 512 global
    'cfg5': FlowConfig((128, 128, 6), 3, (0, 1, 1, 1, 1, 0), (3, 3, 3, 3, 3, 3), (64, 64, 32, 16, 8, 8),
                       (2, 2, 2, 2, 2, 2), batch=512, data='sr', sr_pow=3, name='cfg5'),
    # small architectures for tests
    'tiny': FlowConfig((8, 8, 2), 1, (0, 1), (1, 1), (8, 8), (2, 2), batch=2, name='tiny'),
    'small': FlowConfig((16, 16, 4), 3, (0, 1, 0), (2, 1, 1), (16, 16, 8), (4, 4, 2), batch=3, name='small'),
    # squeezes down to 2x2 blocks: checkerboard couplings 2 and 1 pixels wide (a shape the reference
    # accepts; the training path's narrow-width weight-gradient fallback)
    'narrow': FlowConfig((8, 8, 4), 3, (1, 1, 0), (1, 1, 1), (8, 8, 8), (2, 2, 2), batch=2, name='narrow'),
}
