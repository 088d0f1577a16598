"""Diagnostic (not a test): per-phase timing of k_net_lds from barrier-free shader-clock stamps
(wave 0 of workgroup (0, 0)). Run on a GPU box: CNF_STAMPS=1 python profiles/diag/diag_stamps.py"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arl_conditional_normalizing_flows_amd import _lib  # noqa: E402
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402

RB = ['LN1.final', 'LN1.apply', 'W.ca', 'bar+pf', 'conv_a', 'bar', 'LN2.final', 'LN2.apply', 'tables', 'W.br',
      'bar+pf', 'branches', 'bar', 'LN3.final', 'LN3.apply', 'W.cb', 'bar+pf', 'conv_b', 'bar']

lib = _lib.load()
lib.cnf_debug_read_stamps.restype = C.c_int
lib.cnf_debug_read_stamps.argtypes = [C.c_void_p, C.c_int]
lib.cnf_debug_read_cycles.restype = C.c_int
lib.cnf_debug_read_cycles.argtypes = [C.c_void_p, C.c_int]
cfg = PRESETS[os.environ.get('CNF_DIAG_CFG', 'cfg2')]
flow = cFlow(**cfg.kwargs())
buf = np.zeros(256, dtype=np.int64)
cyc = np.zeros(256, dtype=np.int64)
prev = None
for li, layer in enumerate(flow.layers_list):
    if not hasattr(layer, 'which_mask'):
        continue
    u = torch.randn((64, layer.input_height, layer.input_width, layer.input_depth), device='cuda')
    for _ in range(3):
        layer.forward_and_Jacobian(u, 0.0, None)
    torch.cuda.synchronize()
    lib.cnf_debug_read_stamps(buf.ctypes.data, 256)
    lib.cnf_debug_read_cycles(cyc.ctypes.data, 256)
    n = int(buf[255])
    if n == 0 or (prev is not None and np.array_equal(prev, buf)):
        continue   # streamed layer: no k_net_lds launch (the stamps are the previous layer's)
    prev = buf.copy()
    c = cyc[:n].astype(np.float64)
    rt_us = (buf[1] - buf[0]) * 10.0 / 1000.0
    ghz = (c[-1] - c[0]) / max(rt_us, 1e-9) / 1e3
    d = np.diff(c) / (ghz * 1e3)   # us
    print(f'layer {li} mask {layer.which_mask} {layer.compressed_height}x{layer.compressed_width}: '
          f'{rt_us:.1f} us, {ghz:.2f} GHz')
    labels = ['prologue', 'conv_in+bar']
    R = (n - 5) // len(RB)
    for r in range(R):
        labels += [f'{x}' for x in RB]
    labels += ['LN_out', 'co.W+bar', 'co.gemm', 'co.bar', 'co.sum+end'] if n - 5 - R * len(RB) == 3 else ['LN_out', 'conv_out']
    print('   ' + '  '.join(f'{lab}={v:.2f}' for lab, v in zip(labels, d)))
