"""Diagnostic (not a test): per-phase timing of k_net_lds via s_memrealtime stamps.
Run on a GPU box: CNF_STAMPS=1 python tests/diag_stamps.py"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arl_conditional_normalizing_flows_amd import _lib  # noqa: E402
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402
from arl_conditional_normalizing_flows_amd.synthetic import class_batch  # noqa: E402

lib = _lib.load()
lib.cnf_debug_read_stamps.restype = C.c_int
lib.cnf_debug_read_stamps.argtypes = [C.c_void_p, C.c_int]
lib.cnf_debug_read_cycles.restype = C.c_int
lib.cnf_debug_read_cycles.argtypes = [C.c_void_p, C.c_int]
cfg = PRESETS['cfg2']
flow = cFlow(**cfg.kwargs())
xy = torch.from_numpy(class_batch(64, 32, 32, 3, seed=1)).cuda()
buf = np.zeros(256, dtype=np.int64)
for li, layer in enumerate(flow.layers_list):
    if not hasattr(layer, 'which_mask'):
        continue
    if li not in (0, 10, 12, 16, 18):
        continue
    u = torch.randn((64, layer.input_height, layer.input_width, layer.input_depth), device='cuda')
    for _ in range(3):
        layer.forward_and_Jacobian(u, 0.0, None)
    torch.cuda.synchronize()
    lib.cnf_debug_read_stamps(buf.ctypes.data, 256)
    n = int(buf[255])
    t = buf[:n].astype(np.float64) * 10.0 / 1000.0   # 100 MHz ticks -> us
    print(f'layer {li} mask {layer.which_mask} {layer.compressed_height}x{layer.compressed_width}: total {t[-1]-t[0]:.1f} us')
    print('  phase deltas (us):', ' '.join(f'{d:.1f}' for d in np.diff(t)))
    cyc = np.zeros(256, dtype=np.int64)
    lib.cnf_debug_read_cycles(cyc.ctypes.data, 256)
    c = cyc[:n].astype(np.float64)
    print(f'  shader clock over the launch: {(c[-1] - c[0]) / (t[-1] - t[0]) / 1e3:.2f} GHz')
