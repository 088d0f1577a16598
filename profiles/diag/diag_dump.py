"""Forward zy / per-image log-det of one preset saved to an .npz (bitwise A/B of two library builds:
run once per CNF_LIB, then compare the files). usage: diag_dump.py cfg5 4 out.npz"""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402
from oracle.cflow_np import OracleCFlow, synthetic_class_batch, synthetic_sr_batch  # noqa: E402

name, B, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
cfg = PRESETS[name]
kw = cfg.kwargs()
P = OracleCFlow(**kw).init_params(0)
H, W, D = cfg.io_shape
xy = synthetic_class_batch(B, H, W, cfg.x_d, seed=1) if cfg.data == 'class' else \
    synthetic_sr_batch(B, H, W, cfg.x_d, cfg.sr_pow, seed=1)
f = cFlow(**kw)
f.set_weights(P)
zy, ld = f(torch.from_numpy(xy).cuda(), 1, per_image_logdet=True)
xi = f(zy, -1)
torch.cuda.synchronize()
np.savez(out, zy=zy.cpu().numpy(), ld=ld.cpu().numpy(), xi=xi.cpu().numpy())
print(name, B, 'saved', out)
