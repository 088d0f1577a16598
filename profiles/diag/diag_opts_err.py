"""zy / log-det error against the float64 oracle for one preset under several debug option sets
(localises a parity failure to a kernel path). usage: python profiles/diag/diag_opts_err.py cfg5 1"""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402
from oracle.cflow_np import OracleCFlow, synthetic_class_batch, synthetic_sr_batch  # noqa: E402

name, B = sys.argv[1], int(sys.argv[2])
sets = sys.argv[3:] or ['', 'GENERIC=1', 'LAYOUT=3', 'GC=0', 'NETLDS=0', 'LAYOUT=3,GENERIC=1']
cfg = PRESETS[name]
kw = cfg.kwargs()
ora = OracleCFlow(**kw)
P = ora.init_params(0)
H, W, D = cfg.io_shape
xy = synthetic_class_batch(B, H, W, cfg.x_d, seed=1) if cfg.data == 'class' else \
    synthetic_sr_batch(B, H, W, cfg.x_d, cfg.sr_pow, seed=1)
zr, lr, _ = ora.forward(xy, P, abs_s=True)
for opt in sets:
    try:
        f = cFlow(**kw, debug_options=opt)
        f.set_weights(P)
        zy, ld = f(torch.from_numpy(xy).cuda(), 1, per_image_logdet=True)
        torch.cuda.synchronize()
        e = float(np.max(np.abs(zy.cpu().numpy() - zr)) / np.max(np.abs(zr)))
        el = float(np.max(np.abs(ld.cpu().numpy() - lr)))
        print(f'{name} B={B} [{opt}]: zy rel err {e:.3e}, logdet abs err {el:.3e}', flush=True)
    except Exception as ex:   # noqa: BLE001
        print(f'{name} [{opt}]: {ex}', flush=True)
