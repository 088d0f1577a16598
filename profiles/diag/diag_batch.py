"""Batch-invariance bisection (round-5 verdict item 3): the same images in one large batch and in
batches of 5 must give the same bits. Prints, per configuration and knob, how many images differ
bitwise (forward zy, per-image log-det, inverse) and the largest relative difference.
usage: python profiles/diag/diag_batch.py CFG B [KNOB=VAL ...]   (knobs are set before the plan)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
for kv in sys.argv[3:]:
    k, v = kv.split('=', 1)
    os.environ[k] = v

import numpy as np  # noqa: E402
import torch  # noqa: E402

from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402
from oracle.cflow_np import OracleCFlow, synthetic_class_batch, synthetic_sr_batch  # noqa: E402

name, B = sys.argv[1], int(sys.argv[2])
dev = torch.device('cuda', 0)
cfg = PRESETS[name]
kw = cfg.kwargs()
flow = cFlow(**kw, device=dev)
flow.set_weights(OracleCFlow(**kw).init_params(0))
H, W, _ = cfg.io_shape
xy = (synthetic_class_batch(B, H, W, cfg.x_d, seed=5) if cfg.data == 'class'
      else synthetic_sr_batch(B, H, W, cfg.x_d, cfg.sr_pow, seed=5))
x = torch.from_numpy(xy).to(dev)


def run(layerwise):
    zy, ld = flow(x, 1, per_image_logdet=True, layerwise=layerwise)
    xi = flow(zy, -1, layerwise=layerwise)
    zs, ls, xs = [], [], []
    for s in range(0, B, 5):
        a, b = flow(x[s:s + 5], 1, per_image_logdet=True, layerwise=layerwise)
        zs.append(a)
        ls.append(b)
        xs.append(flow(zy[s:s + 5], -1, layerwise=layerwise))
    torch.cuda.synchronize()
    out = []
    for big, small in ((zy, torch.cat(zs)), (ld, torch.cat(ls)), (xi, torch.cat(xs))):
        d = (big - small).reshape(B, -1)
        nd = int((d != 0).any(dim=1).sum().item())
        rel = (d.abs().max() / big.abs().max()).item()
        first = int(torch.nonzero((d != 0).any(dim=1))[0].item()) if nd else -1
        out.append(f'{nd:3d} imgs differ (first {first:3d}) rel {rel:.2e}')
    return out


for lw in (False, True):
    r = run(lw)
    print(f'{name} B={B} {" ".join(sys.argv[3:]) or "default"} {"layerwise" if lw else "fused"}: '
          f'zy [{r[0]}] ld [{r[1]}] inv [{r[2]}]', flush=True)
