"""Diagnostic: host time of each part of cFlow.gradients in steady-state stepping (no pre-sleep), against
the GPU time of the step: is the backward's enqueue throttled by the GPU (host-bound chains)?"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from arl_conditional_normalizing_flows_amd import _lib  # noqa: E402
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow, check, ptr, _stream  # noqa: E402
from arl_conditional_normalizing_flows_amd.synthetic import class_batch  # noqa: E402

cfg = PRESETS['cfg2']
B = 64
flow = cFlow(**cfg.kwargs(), device=torch.device('cuda', 0))
H, W, _ = cfg.io_shape
xy = torch.from_numpy(class_batch(B, H, W, cfg.x_d, seed=1)).cuda()
lib = _lib.load()
for _ in range(3):
    flow.gradients(xy)
torch.cuda.synchronize()
ws = flow._train_workspace(B)
zy = torch.empty_like(xy)
ld = torch.empty(B, device=xy.device, dtype=torch.float32)
buf = torch.zeros(8, device=xy.device, dtype=torch.float32)
buf[4] = B
for rep in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    check(lib.cnf_flow_forward_train(flow._plan, ptr(flow.params), ptr(flow._aux), ptr(xy), ptr(zy), ptr(ld),
                                     ptr(ws), B, _stream()), 'fwd')
    t1 = time.perf_counter()
    check(lib.cnf_flow_backward_ex(flow._plan, ptr(flow.params), ptr(xy), ptr(zy), ptr(ws), B, ptr(buf) + 16,
                                   ptr(flow._grads), _lib.LAYER_DONE_FN(), None, _stream()), 'bwd')
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print(f'forward_train enqueue {1e3 * (t1 - t0):.2f} ms, backward enqueue {1e3 * (t2 - t1):.2f} ms, '
          f'then GPU done after {1e3 * (t3 - t2):.2f} ms (step {1e3 * (t3 - t0):.2f} ms)', flush=True)
