"""The path's exchange step with the HIP-produced NLL sums.

* gloo, world size 2 (both ranks on cuda:0): every rank runs the HIP forward + cnf_nll on its
  shard of the global batch, and the single 5-float all-reduce of its sums (distributed.py) must
  reproduce the float64 oracle's log_loss over the global batch
  (conv_cINN_make_model.py:1800-1848), ragged shards included.
* The C-ABI communicator (cnf_comm_* / cnf_nll_allreduce, RCCL) for a non-torch caller: one rank
  (RCCL refuses two ranks on one device, and the box has one GPU); the 8-GPU path is the
  driver's scaling run.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from arl_conditional_normalizing_flows_amd import _lib
from arl_conditional_normalizing_flows_amd.config import PRESETS
from arl_conditional_normalizing_flows_amd.distributed import shard_range
from oracle.cflow_np import OracleCFlow, synthetic_class_batch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _hip_worker(rank, world, port, G, out_dir):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from arl_conditional_normalizing_flows_amd.make_model import cFlow
        from arl_conditional_normalizing_flows_amd.distributed import reduce_nll_sums
        dev = torch.device('cuda', 0)
        cfg = PRESETS['small']
        kw = cfg.kwargs()
        flow = cFlow(**kw, device=dev)
        flow.set_weights(OracleCFlow(**kw).init_params(0))
        H, W, _ = cfg.io_shape
        xy = synthetic_class_batch(G, H, W, cfg.x_d, seed=7)
        lo, hi = shard_range(G, rank, world)
        x = torch.from_numpy(xy[lo:hi]).to(dev)
        lib = _lib.load()
        zy, ld = flow(x, 1, per_image_logdet=True)
        per = torch.empty((hi - lo, 3), device=dev)
        sums = torch.empty(4, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        _lib.check(lib.cnf_nll(flow._plan, x.data_ptr(), zy.data_ptr(), ld.data_ptr(), per.data_ptr(),
                               sums.data_ptr(), hi - lo, st), 'nll')
        torch.cuda.synchronize()
        got = torch.stack(reduce_nll_sums(sums.cpu(), hi - lo)).numpy()   # the gloo all-reduce
        np.save(os.path.join(out_dir, f'r{rank}.npy'), got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('G', [6, 7])
def test_gloo_world2_hip_nll_sums_match_global_batch(gpu, tmp_path, G):
    world = 2
    mp.spawn(_hip_worker, args=(world, _free_port(), G, str(tmp_path)), nprocs=world, join=True)
    cfg = PRESETS['small']
    kw = cfg.kwargs()
    ora = OracleCFlow(**kw)
    P = ora.init_params(0)
    H, W, _ = cfg.io_shape
    xy = synthetic_class_batch(G, H, W, cfg.x_d, seed=7).astype(np.float64)
    ref = np.array(ora.log_loss(xy, P))
    _, _, abs_s = ora.forward(xy, P, abs_s=True)
    r0 = np.load(tmp_path / 'r0.npy')
    r1 = np.load(tmp_path / 'r1.npy')
    print('global means', r0, 'oracle', ref)
    assert np.array_equal(r0, r1)          # every rank sees the same global means
    assert np.all(np.abs(r0 - ref) <= 1e-5 * np.maximum(np.abs(ref), abs_s.mean()))


def test_capi_comm_one_rank(gpu):
    """cnf_comm_unique_id -> cnf_comm_init -> cnf_nll_allreduce / cnf_allreduce_sum_f32 on one rank:
    the packed payload is (the 4 cnf_nll sums, B) and a sum over one rank is the identity."""
    lib = _lib.load()
    uid = C.create_string_buffer(128)
    _lib.check(lib.cnf_comm_unique_id(uid), 'unique id')
    comm = C.c_void_p()
    _lib.check(lib.cnf_comm_init(0, 1, uid, C.byref(comm)), 'comm init')
    try:
        dev = torch.device('cuda', 0)
        st = torch.cuda.current_stream().cuda_stream
        sums = torch.tensor([1.5, -2.0, 3.25, 4.0], device=dev)
        red = torch.full((5,), 7.0, device=dev)
        _lib.check(lib.cnf_nll_allreduce(comm, sums.data_ptr(), 13, red.data_ptr(), st), 'nll allreduce')
        x = torch.arange(1000, dtype=torch.float32, device=dev)
        _lib.check(lib.cnf_allreduce_sum_f32(comm, x.data_ptr(), 1000, st), 'allreduce')
        torch.cuda.synchronize()
        assert red.cpu().tolist() == [1.5, -2.0, 3.25, 4.0, 13.0]
        assert torch.equal(x.cpu(), torch.arange(1000, dtype=torch.float32))
        # the no-communicator form packs only
        _lib.check(lib.cnf_nll_allreduce(None, sums.data_ptr(), 2, red.data_ptr(), st), 'pack')
        torch.cuda.synchronize()
        assert red.cpu().tolist() == [1.5, -2.0, 3.25, 4.0, 2.0]
    finally:
        lib.cnf_comm_destroy(comm)
    assert lib.cnf_comm_init(1, 1, uid, C.byref(comm)) == -1      # rank out of range


def test_capi_comm_rejects_bad_arguments(gpu):
    lib = _lib.load()
    comm = C.c_void_p()
    assert lib.cnf_comm_init(0, 0, b'\0' * 128, C.byref(comm)) == -1
    assert lib.cnf_allreduce_sum_f32(None, None, 4, None) == -1


def _grad_worker(rank, world, port, G, out_dir, overlap):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from arl_conditional_normalizing_flows_amd.make_model import cFlow
        dev = torch.device('cuda', 0)
        cfg = PRESETS['small']
        kw = cfg.kwargs()
        flow = cFlow(**kw, device=dev)
        flow.set_weights(OracleCFlow(**kw).init_params(3))
        H, W, _ = cfg.io_shape
        xy = synthetic_class_batch(G, H, W, cfg.x_d, seed=9)
        lo, hi = shard_range(G, rank, world)
        g, terms = flow.gradients(torch.from_numpy(xy[lo:hi]).to(dev), process_group=True, overlap=overlap)
        torch.cuda.synchronize()
        np.save(os.path.join(out_dir, f'g{rank}_{int(overlap)}.npy'), g.cpu().numpy())
        np.save(os.path.join(out_dir, f't{rank}_{int(overlap)}.npy'), torch.stack(terms).cpu().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('G', [6, 7])
def test_gloo_world2_overlapped_gradient_allreduce(gpu, tmp_path, G):
    """cFlow.gradients(process_group=...): each coupling layer's gradient range all-reduced
    asynchronously as its backward is enqueued (cnf_flow_backward_ex layer callbacks), the global image
    count read on the device (no host sync) — bitwise the non-overlapped path (one all-reduce after
    the backward, overlap=False), the same on every rank, and equal (to fp32 summation order) to
    one process's gradient of the whole global batch."""
    world = 2
    for overlap in (True, False):
        mp.spawn(_grad_worker, args=(world, _free_port(), G, str(tmp_path), overlap), nprocs=world, join=True)
    g = {(r, o): np.load(tmp_path / f'g{r}_{o}.npy') for r in (0, 1) for o in (0, 1)}
    t = {(r, o): np.load(tmp_path / f't{r}_{o}.npy') for r in (0, 1) for o in (0, 1)}
    assert np.array_equal(g[0, 1], g[0, 0]) and np.array_equal(g[1, 1], g[1, 0])
    assert np.array_equal(g[0, 1], g[1, 1]) and np.array_equal(t[0, 1], t[1, 1])
    from arl_conditional_normalizing_flows_amd.make_model import cFlow
    cfg = PRESETS['small']
    kw = cfg.kwargs()
    flow = cFlow(**kw, device=gpu)
    flow.set_weights(OracleCFlow(**kw).init_params(3))
    H, W, _ = cfg.io_shape
    xy = synthetic_class_batch(G, H, W, cfg.x_d, seed=9)
    g1, t1 = flow.gradients(torch.from_numpy(xy).to(gpu))
    g1 = g1.cpu().numpy()
    err = np.max(np.abs(g[0, 1] - g1))
    print(f'G={G}: sharded vs whole-batch gradient max abs diff {err:.2e} (max |g| {np.max(np.abs(g1)):.2e})')
    assert err <= 1e-5 * np.max(np.abs(g1))
    assert np.allclose(t[0, 1], torch.stack(t1).cpu().numpy(), rtol=1e-5, atol=1e-4)


def test_layer_done_orders_every_gradient_write(gpu):
    """cnf_flow_backward_ex's layer_done contract (include/cnf.h): when coupling c is reported,
    every kernel writing c's gradient range is ordered on the caller's stream before that point.
    The callback records an event on the caller's stream and, on a side stream ordered ONLY by
    that event, snapshots the range and then poisons it with NaN. If a kernel writing the range
    were still unordered, its result would be missing from the snapshot (snapshot != the plain
    backward's gradient) or would land after the poison (a non-NaN left in the range). This is the
    ordering the RCCL overlap (cFlow.gradients on 'nccl') relies on; one GPU suffices. cfg2 B=8
    covers the streamed layers (four streams), the split LDS backward (weight gradients on a side
    stream, reported two layers late) and the LDS layers."""
    from arl_conditional_normalizing_flows_amd.make_model import cFlow, _stream
    from arl_conditional_normalizing_flows_amd.distributed import pack_nll_sums
    cfg = PRESETS['cfg2']
    kw = cfg.kwargs()
    flow = cFlow(**kw, device=gpu)
    flow.set_weights(OracleCFlow(**kw).init_params(4))
    H, W, _ = cfg.io_shape
    B = 8
    x = torch.from_numpy(synthetic_class_batch(B, H, W, cfg.x_d, seed=12)).to(gpu)
    g_ref = flow.gradients(x)[0].clone()
    torch.cuda.synchronize()

    lib = _lib.load()
    ranges = flow._coupling_param_ranges()
    ws = flow._train_workspace(B)
    zy = torch.empty_like(x)
    ld = torch.empty(B, device=gpu, dtype=torch.float32)
    main = torch.cuda.current_stream()
    side = torch.cuda.Stream(device=gpu)
    _lib.check(lib.cnf_flow_forward_train(flow._plan, flow.params.data_ptr(), flow._aux.data_ptr(), x.data_ptr(),
                                          zy.data_ptr(), ld.data_ptr(), ws.data_ptr(), B, _stream()), 'forward_train')
    sums, _ = flow.nll_sums(x, zy, ld)
    buf = pack_nll_sums(sums, B)
    grads = torch.full((flow.num_params,), 7.0, device=gpu)
    snap = torch.full_like(grads, 3.0)
    reported, errors, events = [], [], []

    def done(_user, ci):
        try:
            reported.append(ci)
            lo, hi = ranges[ci]
            ev = torch.cuda.Event()
            ev.record(main)
            events.append(ev)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                snap[lo:hi].copy_(grads[lo:hi])
                grads[lo:hi].fill_(float('nan'))
        except BaseException as e:   # noqa: BLE001
            errors.append(e)
    cb = _lib.LAYER_DONE_FN(done)
    _lib.check(lib.cnf_flow_backward_ex(flow._plan, flow.params.data_ptr(), x.data_ptr(), zy.data_ptr(),
                                        ws.data_ptr(), B, buf.data_ptr() + 16, grads.data_ptr(), cb, None,
                                        _stream()), 'backward_ex')
    torch.cuda.synchronize()
    assert not errors, errors
    assert sorted(reported) == sorted(ranges), reported
    assert torch.equal(snap, g_ref), 'a gradient write was not ordered before its layer_done'
    assert torch.isnan(grads).all(), 'a gradient write landed after its layer_done'
