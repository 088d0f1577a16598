"""Where one layer's output differs between two debug-option sets (same input): max |diff| per
64-pixel tile row block and per channel. usage: diag_layer_map.py cfg5 1 LAYER OPT_A OPT_B"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402
from oracle.cflow_np import OracleCFlow, synthetic_class_batch, synthetic_sr_batch  # noqa: E402

name, B, L, oa, ob = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
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
for i, la in enumerate(fa.layers_list):
    if i == L:
        break
    u, ld, z = la.forward_and_Jacobian(u, ld, z)
for rep in range(3):
    va = fa.layers_list[L].forward_and_Jacobian(u, ld, z)[0]
    vb = fb.layers_list[L].forward_and_Jacobian(u, ld, z)[0]
    torch.cuda.synchronize()
    d = (va - vb).abs()
    print(f'rep {rep}: max {d.max().item():.3e}; per image {[round(x, 4) for x in d.amax(dim=(1, 2, 3)).tolist()]}')
    hh, ww = d.shape[1], d.shape[2]
    rows = d.amax(dim=(0, 2, 3)).reshape(-1)
    print('  per row (max over 8-row blocks):', [round(rows[r:r + 8].max().item(), 4) for r in range(0, hh, 8)])
    cols = d.amax(dim=(0, 1, 3)).reshape(-1)
    print('  per col (8-col blocks):', [round(cols[c:c + 8].max().item(), 4) for c in range(0, ww, 8)])
    print('  per channel:', [round(x, 4) for x in d.amax(dim=(0, 1, 2)).tolist()])
    nz = (d > 1e-3).nonzero()
    print('  pixels > 1e-3:', nz.shape[0], nz[:10].tolist())
