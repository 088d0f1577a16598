"""Diagnostic (not a test): throughput of cfg2 forward + NLL steps with two batches in flight on
two HIP streams (each its own workspace, input and captured graph) against one stream, to see
whether one batch's k_net_lds layers (128 workgroups: half the CUs) overlap the other's streamed
layers. usage: python profiles/diag/diag_two_streams.py [config] [batch] [iters]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arl_conditional_normalizing_flows_amd import _lib  # noqa: E402
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402
from arl_conditional_normalizing_flows_amd.make_model import cFlow  # noqa: E402
from arl_conditional_normalizing_flows_amd.synthetic import class_batch, sr_batch  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'cfg2'
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
K = int(sys.argv[3]) if len(sys.argv) > 3 else 200
cfg = PRESETS[name]
dev = torch.device('cuda', 0)
flow = cFlow(**cfg.kwargs(), device=dev, seed=0)
lib = _lib.load()
H, W, D = cfg.io_shape


def make_lane(seed):
    xy = torch.from_numpy(class_batch(B, H, W, cfg.x_d, seed=seed) if cfg.data == 'class'
                          else sr_batch(B, H, W, cfg.x_d, cfg.sr_pow, seed=seed)).to(dev)
    assert tuple(xy.shape[1:]) == tuple(cfg.io_shape), (xy.shape, cfg.io_shape)   # raw pointers below
    ws = torch.empty(int(lib.cnf_plan_workspace_bytes(flow._plan, B)), device=dev, dtype=torch.uint8)
    zy = torch.empty_like(xy)
    ld = torch.empty(B, device=dev)
    per = torch.empty((B, 3), device=dev)
    sums = torch.empty(4, device=dev)

    def step():
        st = torch.cuda.current_stream().cuda_stream
        _lib.check(lib.cnf_flow_forward(flow._plan, flow.params.data_ptr(), flow._aux.data_ptr(), xy.data_ptr(),
                                        zy.data_ptr(), ld.data_ptr(), ws.data_ptr(), B, st), 'fwd')
        _lib.check(lib.cnf_nll(flow._plan, xy.data_ptr(), zy.data_ptr(), ld.data_ptr(), per.data_ptr(),
                               sums.data_ptr(), B, st), 'nll')
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        step()
    torch.cuda.synchronize()
    return g, s, step


# CNF_DIAG_DUMMY_STREAMS=n: create n streams first (HIP maps streams onto GPU_MAX_HW_QUEUES hardware
# queues: lanes that share a queue serialise)
_dummy = [torch.cuda.Stream(device=dev) for _ in range(int(os.environ.get('CNF_DIAG_DUMMY_STREAMS', '0')))]
lanes = [make_lane(1000 + i) for i in range(3)]


def run(nl, iters, offset_us=0):
    """a round = every lane's step; lane i > 0 starts offset_us * i later (a GPU sleep on its stream,
    ordered after the round's start by an event), and the round ends when all lanes are done"""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        ev = torch.cuda.Event()
        ev.record(lanes[0][1])
        for i, (g, s, _) in enumerate(lanes[:nl]):
            with torch.cuda.stream(s):
                if i > 0 and offset_us > 0:
                    s.wait_event(ev)
                    torch.cuda._sleep(int(offset_us * i * 2000))   # ~2000 cycles per us
                g.replay()
        for g, s, _ in lanes[1:nl]:
            lanes[0][1].wait_stream(s)   # round barrier: one batch (nl * B images) per round
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def round_graph(nl):
    """one captured graph of a whole round: the capture stream forks to the nl lane streams and
    joins them (does graph replay keep the branches concurrent?)"""
    s0 = torch.cuda.Stream(device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s0):
        for _, s, step in lanes[:nl]:
            s.wait_stream(s0)
            with torch.cuda.stream(s):
                step()
        for _, s, _ in lanes[:nl]:
            s0.wait_stream(s)
    torch.cuda.synchronize()
    return g, s0


if os.environ.get('CNF_DIAG_ROUND_GRAPH') == '1':
    for nl in (1, 2, 3):
        g, s0 = round_graph(nl)
        for it in (10, K):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with torch.cuda.stream(s0):
                for _ in range(it):
                    g.replay()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        print(f'{name} B={B}: round graph of {nl} lane(s): {nl * B * K / el:9.1f} images/s, '
              f'{el / K * 1e3:.3f} ms per round', flush=True)
    sys.exit(0)

offsets = [int(v) for v in os.environ.get('CNF_DIAG_OFFSETS', '0').split(',')]
for nl in (1, 2, 3):
    for off in (offsets if nl > 1 else [0]):
        run(nl, 10, off)
        el = run(nl, K, off)
        print(f'{name} B={B}: {nl} stream(s), offset {off} us: {nl * B * K / el:9.1f} images/s, '
              f'{el / K * 1e3:.3f} ms per round of {nl} batches', flush=True)
