"""Diagnostic (not a test): per-phase clock stamps of the fused LDS backward (k_lds_bwd) of the last
launched LDS layer (coupling 0 of cfg2) at the bench batch. Run on a GPU box:
    CNF_LDSBWD_STAMPS=1 python profiles/diag/diag_bwd_stamps.py"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arl_conditional_normalizing_flows_amd import _lib  # noqa: E402
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402
from arl_conditional_normalizing_flows_amd.synthetic import class_batch  # noqa: E402

lib = _lib.load()
lib.cnf_debug_read_bwd_stamps.restype = C.c_int
lib.cnf_debug_read_bwd_stamps.argtypes = [C.c_void_p, C.c_int]
cfg = PRESETS['cfg2']
flow = cFlow(**cfg.kwargs())
xy = torch.from_numpy(class_batch(int(os.environ.get('B', '64')), 32, 32, 3, seed=1)).cuda()
for _ in range(3):
    flow.gradients(xy)
torch.cuda.synchronize()
buf = np.zeros(128, dtype=np.int64)
lib.cnf_debug_read_bwd_stamps(buf.ctypes.data, 128)
n = int(buf[0])
t = buf[1:1 + n]
d = np.diff(t)
print(f'{n} stamps, total {t[-1] - t[0]} cycles (s_memtime, 100 MHz: {(t[-1] - t[0]) / 100:.1f} us)')
print(' '.join(f'{int(v)}' for v in d))
