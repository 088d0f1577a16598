"""Layer-by-layer comparison of two debug-option sets on one preset: every layer of flow b gets
flow a's input of that layer, and the max relative output difference is printed per layer
(localises a kernel difference to a layer). usage: diag_layerwise.py cfg5 1 GENERIC=2 ''"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402
from oracle.cflow_np import OracleCFlow, synthetic_class_batch, synthetic_sr_batch  # noqa: E402

name, B, oa, ob = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
cfg = PRESETS[name]
kw = cfg.kwargs()
P = OracleCFlow(**kw).init_params(0)
H, W, D = cfg.io_shape
xy = synthetic_class_batch(B, H, W, cfg.x_d, seed=1) if cfg.data == 'class' else \
    synthetic_sr_batch(B, H, W, cfg.x_d, cfg.sr_pow, seed=1)
fa, fb = cFlow(**kw, debug_options=oa), cFlow(**kw, debug_options=ob)
fa.set_weights(P)
fb.set_weights(P)
u = torch.from_numpy(xy).cuda()
ld = torch.zeros(B, device='cuda')
z = None
for i, (la, lb) in enumerate(zip(fa.layers_list, fb.layers_list)):
    va, lda, za = la.forward_and_Jacobian(u, ld, z)
    vb, ldb, zb = lb.forward_and_Jacobian(u, ld, z)
    torch.cuda.synchronize()
    e = ((va - vb).abs().max() / va.abs().max()).item()
    print(f'layer {i} {type(la).__name__} {tuple(u.shape)}: rel diff {e:.3e}', flush=True)
    u, ld, z = va, lda, za
