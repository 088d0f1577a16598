"""Diagnostic (not a test): bench.serving_inflight on a fresh flow, then again after bench's in-stream
kernel timing (measure_in_stream), to find what serialises the lanes inside bench.py."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from arl_conditional_normalizing_flows_amd import _lib  # noqa: E402
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402

cfg = PRESETS['cfg2']
dev = torch.device('cuda', 0)
flow = cFlow(**cfg.kwargs(), device=dev, seed=0)
lib = _lib.load()
B = 64
xy = torch.from_numpy(bench.synth(cfg, B, 1000)).to(dev)
print('fresh', bench.serving_inflight(flow, lib, xy, B, 2, 100, dev), flush=True)
zy = torch.empty_like(xy)
ld = torch.empty(B, device=dev)
ws = flow._workspace(B)


def local_step():
    st = torch.cuda.current_stream().cuda_stream
    _lib.check(lib.cnf_flow_forward(flow._plan, flow.params.data_ptr(), flow._aux.data_ptr(), xy.data_ptr(),
                                    zy.data_ptr(), ld.data_ptr(), ws.data_ptr(), B, st), 'forward')


bench.measure_in_stream(flow, local_step)
print('after measure_in_stream', bench.serving_inflight(flow, lib, xy, B, 2, 100, dev), flush=True)
