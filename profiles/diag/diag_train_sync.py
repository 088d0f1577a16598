"""Diagnostic (not a test): the training step's per-step host sync. cFlow.train_step reads the 4 loss
terms back for the Mean trackers (one host sync per step, as Keras's progress bar does); the same
work without that read (gradients + Adam + pack, the terms left on the device) lets the host enqueue
the next step while the GPU still runs this one.  usage: python profiles/diag/diag_train_sync.py [cfg] [B]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arl_conditional_normalizing_flows_amd import _lib  # noqa: E402
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd._lib import ptr  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow, _stream  # noqa: E402
from arl_conditional_normalizing_flows_amd.optimizers import Adam  # noqa: E402
from arl_conditional_normalizing_flows_amd.synthetic import class_batch  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'cfg2'
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
cfg = PRESETS[name]
dev = torch.device('cuda', 0)
flow = cFlow(**cfg.kwargs(), device=dev, seed=0)
flow.compile(Adam(3e-4))
H, W, _ = cfg.io_shape
xy = torch.from_numpy(class_batch(B, H, W, cfg.x_d, seed=1)).to(dev)
lib = _lib.load()


def nosync():
    grads, terms = flow.gradients(xy)
    flow.optimizer.apply_flat(flow.params, grads)
    _lib.check(lib.cnf_pack_params(flow._plan, ptr(flow.params), ptr(flow._aux), _stream()), 'pack')
    return terms


for label, fn in (('train_step', lambda: flow.train_step(xy)), ('no sync', nosync)) * 2:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    print(f'{name} B={B} {label}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms/step', flush=True)
