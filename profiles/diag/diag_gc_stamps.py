"""Diagnostic (not a test): phase stamps of workgroup (0, 0) of every k_gc launch of one forward
(s_memrealtime, 100 MHz), from a CNF_EXTRA_FLAGS=-DCNF_GC_STAMPS build loaded through CNF_LIB.
Run on a GPU box: CNF_LIB=.../var_gcst.so python profiles/diag/diag_gc_stamps.py [config] [batch]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arl_conditional_normalizing_flows_amd import _lib  # noqa: E402
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'cfg5'
cfg = PRESETS[name]
B = int(sys.argv[2]) if len(sys.argv) > 2 else cfg.batch
lib = _lib.load()
lib.cnf_debug_read_gc_stamps.restype = C.c_int
lib.cnf_debug_read_gc_stamps.argtypes = [C.c_void_p, C.c_int]
flow = cFlow(**cfg.kwargs())
x = torch.rand((B,) + tuple(cfg.io_shape), device='cuda')
flow(x, 1)
torch.cuda.synchronize()
plan = flow._plan
n = lib.cnf_plan_num_recorded_launches(plan)
nm = C.create_string_buffer(256)
fl, by = C.c_double(), C.c_double()
buf = np.zeros(64, dtype=np.int64)
seen = set()
for i in range(n):
    _lib.check(lib.cnf_plan_recorded_launch_info(plan, i, nm, 256, C.byref(fl), C.byref(by)), 'info')
    if not nm.value.startswith(b'k_gc') or (fl.value, by.value) in seen:
        continue
    seen.add((fl.value, by.value))
    for _ in range(2):
        _lib.check(lib.cnf_plan_relaunch(plan, i, None), 'relaunch')
    torch.cuda.synchronize()
    lib.cnf_debug_read_gc_stamps(buf.ctypes.data, 64)
    k = int(buf[63])
    d = np.diff(buf[:k]).astype(np.float64) / 100.0   # us
    print(f'launch {i} ({fl.value / 1e9:.2f} GFLOP, {by.value / 1e6:.1f} MB): stamps {k}, '
          f'total {(buf[k - 1] - buf[0]) / 100.0:.1f} us')
    print('   ' + ' '.join(f'{v:.2f}' for v in d[:24]) + (' ...' if len(d) > 24 else ''))
