"""Run-to-run nondeterminism and oracle error of one preset under several debug option sets: each
set runs the forward three times on the same input; prints the max relative difference between the
runs and the error against the float64 oracle (localises a race to a kernel path).
usage: python profiles/diag/diag_nondet.py cfg5 2 '' GC=0 LAYOUT=3"""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402
from oracle.cflow_np import OracleCFlow, synthetic_class_batch, synthetic_sr_batch  # noqa: E402

name, B = sys.argv[1], int(sys.argv[2])
sets = sys.argv[3:] or ['']
cfg = PRESETS[name]
kw = cfg.kwargs()
ora = OracleCFlow(**kw)
P = ora.init_params(0)
H, W, D = cfg.io_shape
xy = synthetic_class_batch(B, H, W, cfg.x_d, seed=1) if cfg.data == 'class' else \
    synthetic_sr_batch(B, H, W, cfg.x_d, cfg.sr_pow, seed=1)
zr, lr, _ = ora.forward(xy, P, abs_s=True)
u = torch.from_numpy(xy).cuda()
for opt in sets:
    try:
        f = cFlow(**kw, debug_options=opt)
        f.set_weights(P)
        outs = []
        for _ in range(3):
            zy, _ = f(u, 1, per_image_logdet=True)
            torch.cuda.synchronize()
            outs.append(zy.cpu().numpy())
        sc = float(np.max(np.abs(zr)))
        d = [float(np.max(np.abs(outs[i] - outs[j]))) / sc for i, j in ((0, 1), (0, 2), (1, 2))]
        e = [float(np.max(np.abs(o - zr))) / sc for o in outs]
        print(f'{name} B={B} [{opt}]: run pairs 01 02 12 ' + ' '.join(f'{x:.2e}' for x in d) +
              ', oracle err per run ' + ' '.join(f'{x:.2e}' for x in e), flush=True)
    except Exception as ex:   # noqa: BLE001
        print(f'{name} [{opt}]: {ex}', flush=True)
