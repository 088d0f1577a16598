"""Diagnostic (not a test): per-workgroup timeline of one streamed kernel from a stamps build
(CNF_EXTRA_FLAGS=-DCNF_PW_STAMPS=SID for a k_pw instantiation, or -DCNF_GC_WGSTAMPS for k_gc),
loaded through CNF_LIB. Runs eager cfg2 forwards; the stamps of the last launch of that kernel
are summarised: dispatch spread of the workgroups' starts, prologue, per-image times, ends (us).
usage: CNF_LIB=.../var_X.so python profiles/diag/diag_wg_stamps.py [config] [batch]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arl_conditional_normalizing_flows_amd import _lib  # noqa: E402
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'cfg2'
cfg = PRESETS[name]
B = int(sys.argv[2]) if len(sys.argv) > 2 else cfg.batch
lib = _lib.load()
lib.cnf_debug_read_pw_stamps.restype = C.c_int
lib.cnf_debug_read_pw_stamps.argtypes = [C.c_void_p]
flow = cFlow(**cfg.kwargs())
x = torch.rand((B,) + tuple(cfg.io_shape), device='cuda')
for _ in range(5):
    flow(x, 1)
torch.cuda.synchronize()
buf = np.zeros((2048, 12), dtype=np.int64)
_lib.check(lib.cnf_debug_read_pw_stamps(buf.ctypes.data), 'read stamps')
rows = buf[buf[:, 0] > 0]
last = rows[:, 0].max()
rows = rows[rows[:, 0] > last - 20000]          # the last launch (100 MHz ticks: within 200 us)
t0 = rows[:, 0].min()
T = (rows - t0) / 100.0                           # us from the first workgroup's start
T[rows == 0] = np.nan
q = lambda v: ' '.join(f'{np.nanpercentile(v, p):6.2f}' for p in (0, 10, 50, 90, 100))
print(f'{name} B={B}: {len(rows)} workgroups (percentiles 0/10/50/90/100, us)')
print('  start          ', q(T[:, 0]))
ncol = int(np.max(np.sum(rows > 0, axis=1)))
for c in range(1, ncol):
    print(f'  stamp {c:2d} - {c - 1:2d}  ', q(T[:, c] - T[:, c - 1]))
end = np.nanmax(T, axis=1)
print('  end            ', q(end))
print(f'  kernel span {np.nanmax(end):.2f} us')
