#!/usr/bin/env python3
"""Is the training step host-bound? Host enqueue time of cFlow.gradients (forward_train + NLL +
backward launches, no sync inside) against the GPU completion time of the same step."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402
from arl_conditional_normalizing_flows_amd.synthetic import class_batch  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'cfg2'
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
cfg = PRESETS[name]
flow = cFlow(**cfg.kwargs(), device=torch.device('cuda', 0))
H, W, _ = cfg.io_shape
xy = torch.from_numpy(class_batch(B, H, W, cfg.x_d, seed=1)).cuda()
for _ in range(3):
    flow.gradients(xy)
torch.cuda.synchronize()
for rep in range(5):
    torch.cuda._sleep(100_000_000)   # keep the GPU busy so the enqueue is not throttled by completion
    t0 = time.perf_counter()
    flow.gradients(xy)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'{name} B={B}: host enqueue {1e3 * (t1 - t0):.2f} ms, enqueue->done {1e3 * (t2 - t1):.2f} ms')
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    flow.gradients(xy)
    torch.cuda.synchronize()
    print(f'{name} B={B}: step (no pre-sleep) {1e3 * (time.perf_counter() - t0):.2f} ms')
