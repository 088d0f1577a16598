#!/usr/bin/env python3
"""Benchmark: images/sec of fwd + log-det (+ NLL sums) of the conditional RealNVP hot path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2] [--global-batch G]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one cFlow.call(xy, +1) (zy + per-image log-det) + the NLL 4-sum over one batch of
synthetic inputs already resident in HBM; with N>1 every rank processes its own batch
(weak scaling, BASELINE configs[1] batch 64 per GPU; --global-batch G instead shards a fixed
global batch of G images: strong scaling, BASELINE configs[3]/[4]) and the 4 NLL sums are
all-reduced (the path's only exchange step, one RCCL all-reduce of 5 fp32: the 4 sums + the image
count). value = images processed by all ranks / max-over-ranks wall time of the K timed steps.

Extra fields of the JSON line (rank 0):
  roofline        the dominant kernel (largest GPU time per step, by kernel symbol): algorithmic
                  FLOPs or bytes per launch / its average duration measured IN THE STREAM (an eager
                  forward with a HIP event pair around every launch, the queue pre-filled so the
                  kernels run back to back as in the graph); `per_kernel` gives every symbol.
                  `traffic` = HBM bytes per launch from the committed rocprofv3 PMC summary.
  step_roofline   the whole step against the path's roofline: SURVEY.md §8(d) algorithmic FLOPs
                  and bytes per image x images, the bound the slower of the two roofs sets.
  bits_per_dim    of the GPU's NLL on the bench batch; cpu_baseline.bits_per_dim_ref is the float64
                  oracle's on the same batch and weights (computed in the CPU leg).
  step_ms_median  median of per-step HIP-event times over >= 100 extra graph replays (BASELINE.md's
                  protocol); `value` / `ms_per_step` are the K-step wall-clock means.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import platform
import sys
import time

import numpy as np

# kernel arguments in device memory for eager launches too (set before HIP initialises): graph replay
# already reads them from device memory, so the eager in-stream timing pass (per_kernel / roofline)
# then times the same kernels the timed graph runs (with host-memory kernargs the large argument
# blocks of k_net_lds / k_gc cost 3-4 us per launch there: profiles/sessions/r5_kernarg.sh)
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from arl_conditional_normalizing_flows_amd import _lib  # noqa: E402
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_16x16x4_f32) dense peak


def synth(cfg, B, seed, noise_alpha=0.98):
    """noise_alpha=1: the clean batch (--noise applies the pipeline's noise inside the forward)"""
    from arl_conditional_normalizing_flows_amd.synthetic import class_batch, sr_batch
    H, W, D = cfg.io_shape
    if cfg.data == 'class':
        return class_batch(B, H, W, cfg.x_d, seed=seed, noise_alpha=noise_alpha)
    return sr_batch(B, H, W, cfg.x_d, cfg.sr_pow, seed=seed, noise_alpha=noise_alpha)


def kernel_symbol(name):
    """recorded launch name -> kernel symbol (k_pw<4,8,conv_b> -> k_pw), the granularity of the
    rocprofv3 summary once its template instantiations are summed."""
    return name.split('<', 1)[0]


def measure_in_stream(flow, forward, reps=20):
    """Per-launch GPU durations of the forward in its place in the stream: with
    cnf_plan_set_launch_timing on, every kernel is dispatched with hipExtLaunchKernelGGL start/stop
    events that receive its own begin / end timestamps (no packets in between, the numbers
    rocprofv3's kernel trace reads); a GPU-side sleep before each rep lets the host enqueue the
    whole forward ahead of the GPU, so the kernels run back to back as in the graph.
    Returns [(name, flops, bytes, mean ms)] in launch order."""
    import ctypes as C
    lib = _lib.load()
    plan = flow._plan
    _lib.check(lib.cnf_plan_set_launch_timing(plan, 1), 'timing on')
    acc = None
    try:
        for _ in range(reps):
            torch.cuda._sleep(20_000_000)
            forward()
            torch.cuda.synchronize()
            n = lib.cnf_plan_num_recorded_launches(plan)
            ms = C.c_float()
            t = []
            for i in range(n):
                _lib.check(lib.cnf_plan_launch_time_ms(plan, i, C.byref(ms)), 'launch time')
                t.append(ms.value)
            acc = t if acc is None else [a + b for a, b in zip(acc, t)]
    finally:
        _lib.check(lib.cnf_plan_set_launch_timing(plan, 0), 'timing off')
    name = C.create_string_buffer(256)
    fl, by = C.c_double(), C.c_double()
    out = []
    for i, tot in enumerate(acc):
        _lib.check(lib.cnf_plan_recorded_launch_info(plan, i, name, 256, C.byref(fl), C.byref(by)), 'info')
        out.append((name.value.decode(), fl.value, by.value, tot / reps))
    return out


def roofline_of(flops, nbytes, ms):
    t = ms / 1e3
    ai = flops / max(nbytes, 1.0)
    ridge = FP32_MFMA_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)
    if ai >= ridge:
        a = flops / t / 1e12
        return {'bound': 'mfma', 'achieved': round(a, 3), 'peak': FP32_MFMA_TFLOPS, 'unit': 'TFLOP/s',
                'frac': round(a / FP32_MFMA_TFLOPS, 4)}
    a = nbytes / t / 1e9
    return {'bound': 'hbm', 'achieved': round(a, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(a / HBM_PEAK_GBS, 4)}


def roofline_for(launches):
    per = {}
    for nm, fl, by, ms in launches:
        if not nm.startswith('k_'):
            continue
        d = per.setdefault(kernel_symbol(nm), {'ms': 0.0, 'flops': 0.0, 'bytes': 0.0, 'launches': 0})
        d['ms'] += ms
        d['flops'] += fl
        d['bytes'] += by
        d['launches'] += 1
    name, d = max(per.items(), key=lambda kv: kv[1]['ms'])
    rf = roofline_of(d['flops'], d['bytes'], d['ms'])
    rf.update({'kernel': name, 'launches_per_step': d['launches'],
               'avg_launch_us': round(d['ms'] * 1e3 / d['launches'], 3),
               'alg_flops_per_launch': d['flops'] / d['launches'],
               'alg_bytes_per_launch': d['bytes'] / d['launches'],
               'timing': 'in-stream kernel timestamps (hipExtLaunchKernelGGL start/stop events, eager forward, queue pre-filled)'})
    rf.update(pmc_traffic(name))
    rf['per_kernel'] = {
        k: dict(roofline_of(v['flops'], v['bytes'], v['ms']), ms_per_step=round(v['ms'], 4), launches=v['launches'],
                avg_launch_us=round(v['ms'] * 1e3 / v['launches'], 3))
        for k, v in sorted(per.items(), key=lambda kv: -kv[1]['ms'])}
    # the same by launch name (kernel + role, e.g. k_pw<4,4,conv_a>): the ResNeXt stages of one symbol apart
    roles = {}
    for nm, fl, by, ms in launches:
        if nm.startswith('k_'):
            d = roles.setdefault(nm, [0.0, 0])
            d[0] += ms
            d[1] += 1
    rf['per_role'] = {k: {'ms_per_step': round(v[0], 4), 'launches': v[1], 'avg_launch_us': round(v[0] * 1e3 / v[1], 3)}
                      for k, v in sorted(roles.items(), key=lambda kv: -kv[1][0])}
    return rf, per


def pmc_traffic(kernel):
    """HBM traffic per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/<round>_summary.json, written by profiles/pmc_summary.py from separate FETCH_SIZE /
    WRITE_SIZE passes of this bench command, gfx950 FETCH_SIZE x2 correction applied there)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, 'profiles', '*_summary.json')))
    for f in reversed(files):
        try:
            with open(f) as fh:
                ks = json.load(fh).get('kernels', {})
        except (OSError, ValueError):
            continue
        # every instantiation of the symbol (shape-specialised ones included), weighted by dispatches
        tot = n = 0.0
        for k, e in ks.items():
            sym = k.split('::')[-1]
            h = e.get('hbm')
            if h and (sym.startswith(kernel + '<') or sym.split('(')[0] == kernel):
                d = float(h.get('dispatches', 1))
                tot += h['traffic_bytes'] * d
                n += d
        if n > 0:
            return {'traffic': round(tot / n, 1), 'traffic_unit': 'bytes/launch',
                    'traffic_source': os.path.relpath(f, ROOT)}
    return {'traffic': None}


def algorithmic_per_image(flow, B):
    """FLOPs = 2 x conv MACs (grouped convs at the reference's group widths);
    bytes = 4*2*H*W*D (xy in, zy out) + 8*N_LN (every LN input written once and read once) +
    4*P_LN/B (LN gamma/beta read once per batch). From the plan's parameter table."""
    import ctypes as C
    lib = _lib.load()
    hw = {}
    info = _lib.cnf_layer_info()
    for li in range(lib.cnf_plan_num_layers(flow._plan)):
        _lib.check(lib.cnf_plan_layer_info(flow._plan, li, C.byref(info)), 'layer info')
        if info.kind == 0:
            hw[info.coupling_index] = info.hc * info.wc
    flops = 0.0
    n_ln = 0
    for n, _o, s in flow.param_specs:
        if n.endswith('.kernel'):
            ci = int(n.split('.', 1)[0][1:])
            flops += 2.0 * hw[ci] * float(np.prod(s))
        elif n.endswith('.gamma'):
            n_ln += int(np.prod(s))
    H, W, D = flow.io_shape
    nbytes = 4.0 * 2 * H * W * D + 8.0 * n_ln + 4.0 * 2 * n_ln / B
    return flops, nbytes, n_ln


def cpu_threads():
    """The host cores this process may use: its affinity set, capped by a cgroup CPU quota when
    one is set (on the GPU box os.cpu_count() reports every core of the machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    quota = None
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, per = f.read().split()
            if q != 'max':
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as f:
                q = int(f.read())
            with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None:
        n = min(n, max(1, int(math.ceil(quota))))
    return n


def cpu_baseline(cfg, flow, xy_np, B, budget_s=20.0):
    """The oracle's torch-CPU fp32 op-for-op restatement of the reference graph, timed on this
    host on a bounded sample of the same workload (rank 0, N=1 only): whole batches of the config's
    B images, median per-batch time. Also the float64 oracle's bits/dim on the bench batch and
    weights (the `bits/dim vs ref` half of the metric)."""
    try:
        from oracle.cflow_torch_cpu import TorchCPUFlow
    except Exception as e:  # pragma: no cover
        return {'value': None, 'unit': 'images/s', 'cores': 0, 'kind': 'port', 'sample': f'unavailable: {e}'}
    threads = cpu_threads()
    torch.set_num_threads(threads)
    tf = TorchCPUFlow(**cfg.kwargs())
    W = flow.get_weights()
    P32 = {k: torch.from_numpy(np.ascontiguousarray(v, np.float32)) for k, v in W.items()}
    xy = torch.from_numpy(np.ascontiguousarray(xy_np, np.float32))
    times = []
    with torch.no_grad():
        tf.log_loss(xy, P32)          # warm-up
        t_all = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            tf.log_loss(xy, P32)
            times.append(time.perf_counter() - t0)
            if time.perf_counter() - t_all > budget_s and len(times) >= 3:
                break
        # bits/dim of the float64 oracle on the same batch and weights
        P64 = {k: v.double() for k, v in P32.items()}
        loss64 = float(tf.log_loss(xy.double(), P64)[0])
    med = float(np.median(times))
    model = platform.processor() or platform.machine()
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    H, Wd, _ = cfg.io_shape
    return {'value': round(B / med, 3), 'unit': 'images/s', 'cores': threads, 'kind': 'port',
            'sample': f'{len(times)} batches of {B} images of {cfg.name} fwd+logdet+NLL (the bench batch and weights), '
                      f'median {med * 1e3:.1f} ms/batch over {sum(times):.1f}s, torch-CPU fp32 restatement '
                      f'(oracle/cflow_torch_cpu.py), {threads} threads, {model}',
            'loss_ref_f64': loss64,
            'bits_per_dim_ref': loss64 / (math.log(2) * H * Wd * cfg.x_d)}


def cpu_baseline_inverse(cfg, flow, zy_np, B, budget_s=20.0):
    """The torch-CPU fp32 restatement's inverse (oracle/cflow_torch_cpu.py TorchCPUFlow.inverse,
    conv_cINN_make_model.py:1774-1798) on the bench's zy batch and weights, whole batches of B for
    about budget_s, median per batch (rank 0, N=1 only)."""
    try:
        from oracle.cflow_torch_cpu import TorchCPUFlow
    except Exception as e:  # pragma: no cover
        return {'value': None, 'unit': 'images/s', 'cores': 0, 'kind': 'port', 'sample': f'unavailable: {e}'}
    threads = cpu_threads()
    torch.set_num_threads(threads)
    tf = TorchCPUFlow(**cfg.kwargs())
    P32 = {k: torch.from_numpy(np.ascontiguousarray(v, np.float32)) for k, v in flow.get_weights().items()}
    zy = torch.from_numpy(np.ascontiguousarray(zy_np, np.float32))
    times = []
    with torch.no_grad():
        tf.inverse(zy, P32)           # warm-up
        t_all = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            tf.inverse(zy, P32)
            times.append(time.perf_counter() - t0)
            if time.perf_counter() - t_all > budget_s and len(times) >= 3:
                break
    med = float(np.median(times))
    return {'value': round(B / med, 3), 'unit': 'images/s', 'cores': threads, 'kind': 'port',
            'sample': f'{len(times)} batches of {B} images of {cfg.name} inverse (the bench zy and weights), '
                      f'median {med * 1e3:.1f} ms/batch over {sum(times):.1f}s, torch-CPU fp32 restatement '
                      f'(oracle/cflow_torch_cpu.py), {threads} threads'}


def cpu_baseline_train(cfg, flow, xy_np, B, budget_s=20.0):
    """The torch-CPU fp32 restatement's training step (oracle/cflow_torch_cpu.py: log_loss, autograd
    backward, torch Adam at the reference's lr 3e-4 / Keras eps 1e-7) on the bench batch and weights,
    whole batches of B for about budget_s, median per step (rank 0, N=1 only)."""
    try:
        from oracle.cflow_torch_cpu import TorchCPUFlow
    except Exception as e:  # pragma: no cover
        return {'value': None, 'unit': 'images/s', 'cores': 0, 'kind': 'port', 'sample': f'unavailable: {e}'}
    threads = cpu_threads()
    torch.set_num_threads(threads)
    tf = TorchCPUFlow(**cfg.kwargs())
    P = {k: torch.tensor(np.ascontiguousarray(v, np.float32), requires_grad=True) for k, v in flow.get_weights().items()}
    opt = torch.optim.Adam(list(P.values()), lr=3e-4, eps=1e-7)
    xy = torch.from_numpy(np.ascontiguousarray(xy_np, np.float32))

    def step():
        opt.zero_grad(set_to_none=True)
        tf.log_loss(xy, P)[0].backward()
        opt.step()

    step()   # warm-up
    times = []
    t_all = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_all > budget_s and len(times) >= 3:
            break
    med = float(np.median(times))
    return {'value': round(B / med, 3), 'unit': 'images/s', 'cores': threads, 'kind': 'port',
            'sample': f'{len(times)} training steps of {B} images of {cfg.name} (log_loss + autograd backward + '
                      f'Adam, the bench batch and weights), median {med * 1e3:.1f} ms/step over {sum(times):.1f}s, '
                      f'torch-CPU fp32 restatement (oracle/cflow_torch_cpu.py), {threads} threads'}


def train_bench(args, cfg, flow, xy, B, G, world, rank, dist, dev, scaling):
    """images/s of cFlow.train_step (conv_cINN_make_model.py:1850-1880) on the bench batch: every
    step = cnf_flow_forward_train + cnf_nll + the 5-float loss all-reduce + cnf_flow_backward + the
    gradient all-reduce (N>1) + Keras Adam + cnf_pack_params, eager; the loss trackers stay on the
    device (no host read per step; the last step's logs are read after the timed region)."""
    from arl_conditional_normalizing_flows_amd.optimizers import Adam
    flow.compile(Adam(3e-4))                       # conv_cINN.py:567
    pg = True if dist is not None else None
    for _ in range(args.warmup):
        logs = flow.train_step(xy, process_group=pg)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        logs = flow.train_step(xy, process_group=pg)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    if rank == 0:
        fl_img, _by, _n = algorithmic_per_image(flow, B)
        ms = el / args.steps * 1e3
        # forward_train (1x the forward convs, activations saved) + the backward's data and weight
        # gradients (2x): 3x the forward FLOPs
        tf = 3.0 * fl_img * G / (ms / 1e3) / 1e12 / world
        # the step against the FP32 MFMA roof (the training step is MFMA-bound: 3 GFLOP per cfg2 image over
        # ~0.2 GB of activation saves and gradients); the per-kernel breakdown of the same command is the
        # committed rocprofv3 summary named in kernel_stats
        import glob
        stats = sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*_train_kernel_stats.csv')))
        roof = {'bound': 'mfma', 'achieved': round(tf, 3), 'peak': FP32_MFMA_TFLOPS, 'unit': 'TFLOP/s',
                'frac': round(tf / FP32_MFMA_TFLOPS, 4), 'kernel': 'whole training step (every kernel)',
                'alg_flops_per_step': 3.0 * fl_img * B,
                'alg_note': '3x the forward conv FLOPs (SURVEY 8(d)): the forward with saves, the data and the '
                            'weight gradients', 'traffic': None,
                'kernel_stats': os.path.relpath(stats[-1], ROOT) if stats else None}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline_train(cfg, flow, xy.cpu().numpy(), B)
        out = {'metric': f'images/sec NLL train step (fwd + bwd + Adam), {cfg.name}',
               'value': round(G * args.steps / el, 2), 'unit': 'images/s', 'n_gpus': world, 'steps': args.steps,
               'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True, 'scaling': scaling,
               'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic', 'config': {
                   'workload': f'{cfg.name}: cFlow.train_step(xy), xy {list(cfg.io_shape)}, {B} images per GPU',
                   'model': f'cFlow {cfg.name}', 'global_batch': G, 'per_gpu_batch': B, 'seq_len': None,
                   'parallelism': f'dp{world} (batch shards, gradient all-reduce)'},
               'alg_tflops_per_gpu': round(tf, 3), 'mfma_frac': round(tf / FP32_MFMA_TFLOPS, 4),
               'roofline': roof, 'cpu_baseline': cpu,
               'loss': float(logs['loss'])}
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def serving_inflight(flow, lib, xy, B, nl, steps, dev, noise=None, logit=0.0):
    """Serving throughput with nl batches in flight: nl lanes (own workspace, input copy, outputs,
    HIP stream and captured graph of one step: forward + log-det + NLL sums of B images), steps
    issued round-robin over the lanes, K steps timed between two synchronisations. One batch's
    k_net_lds layers (128 workgroups at B=64: half the CUs) and kernel prologues / tails then overlap
    another batch's kernels. Per-batch latency: the median event time of one lane's step while the
    other lanes run."""
    lanes = []
    for i in range(nl):
        L = {'xy': xy.clone(), 'zy': torch.empty_like(xy), 'ld': torch.empty(B, device=dev),
             'per': torch.empty((B, 3), device=dev), 'sums': torch.empty(4, device=dev),
             'ws': torch.empty(int(lib.cnf_plan_workspace_bytes(flow._plan, B)), device=dev, dtype=torch.uint8),
             's': torch.cuda.Stream(device=dev)}
        L['xn'] = torch.empty_like(xy) if noise is not None else L['xy']

        def step(L=L):
            st = torch.cuda.current_stream().cuda_stream
            if noise is not None:
                _lib.check(lib.cnf_flow_forward_noise(flow._plan, flow.params.data_ptr(), flow._aux.data_ptr(),
                                                      L['xy'].data_ptr(), float(logit), float(noise), 2000 + i, 0,
                                                      L['xn'].data_ptr(), L['zy'].data_ptr(), L['ld'].data_ptr(),
                                                      L['ws'].data_ptr(), B, st), 'forward')
            else:
                _lib.check(lib.cnf_flow_forward(flow._plan, flow.params.data_ptr(), flow._aux.data_ptr(),
                                                L['xy'].data_ptr(), L['zy'].data_ptr(), L['ld'].data_ptr(),
                                                L['ws'].data_ptr(), B, st), 'forward')
            _lib.check(lib.cnf_nll(flow._plan, L['xn'].data_ptr(), L['zy'].data_ptr(), L['ld'].data_ptr(),
                                   L['per'].data_ptr(), L['sums'].data_ptr(), B, st), 'nll')
        with torch.cuda.stream(L['s']):
            step()
        torch.cuda.synchronize()
        L['g'] = torch.cuda.CUDAGraph()
        with torch.cuda.graph(L['g'], stream=L['s']):
            step()
        lanes.append(L)
    torch.cuda.synchronize()

    def issue(k):
        L = lanes[k % nl]
        with torch.cuda.stream(L['s']):
            L['g'].replay()
    for k in range(4 * nl):
        issue(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        issue(k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # latency of one batch with the others in flight: events around lane 0's steps
    evs = []
    for k in range(nl * 20):
        L = lanes[k % nl]
        with torch.cuda.stream(L['s']):
            if k % nl == 0:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                L['g'].replay()
                b.record()
                evs.append((a, b))
            else:
                L['g'].replay()
    torch.cuda.synchronize()
    lat = float(np.median([a.elapsed_time(b) for a, b in evs]))
    # (with --noise every lane draws its own noise: no comparison runs, and the field says so)
    ok = all(torch.equal(L['sums'], lanes[0]['sums']) for L in lanes[1:]) if noise is None else None
    return {'batches_in_flight': nl, 'value': round(B * steps / el, 2), 'unit': 'images/s', 'steps': steps,
            'ms_per_step': round(el / steps * 1e3, 4), 'batch_latency_ms_median': round(lat, 4),
            'lanes_bitwise_equal': ok,
            'note': 'each step = one batch of B images (fwd + log-det + NLL sums), steps round-robin over '
                    'nl HIP streams with their own workspaces and captured graphs'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--config', default='cfg2')
    ap.add_argument('--batch', type=int, default=0, help='per-GPU batch (default: the config batch)')
    ap.add_argument('--global-batch', type=int, default=0,
                    help='strong scaling: shard this many images over the ranks (default: weak scaling, '
                         'the per-GPU batch on every rank)')
    ap.add_argument('--mode', choices=['forward', 'inverse', 'train'], default='forward',
                    help='train: the NLL training step (cFlow.train_step: forward with saved layer inputs, '
                         'backward, gradient all-reduce when N>1, Keras Adam, weight repack) instead of the '
                         'fwd+logdet metric step; prints its own JSON line. inverse: sampling, '
                         'cFlow.call(zy, -1) (conv_cINN_make_model.py:1774-1798) on the forward\'s zy of the '
                         'bench batch (no collective: the inverse has no cross-image term)')
    ap.add_argument('--noise', type=float, default=None, metavar='ALPHA',
                    help='forward mode: the training pipeline\'s instance noise alpha xy + (1 - alpha) N(0,1) '
                         '(conv_cINN.py:312-315, e.g. 0.98) applied inside the first coupling kernel '
                         '(cnf_flow_forward_noise), the NLL taken on the noisy input')
    ap.add_argument('--logit', type=float, default=0.0, metavar='A',
                    help='with --noise: the logit preprocess (preprocess_dataset_class(LOGITS=True, a=A), '
                         'conv_cINN_base_functions.py:174-231) on the x channels first, fused likewise')
    ap.add_argument('--inflight', type=int, default=2,
                    help='also measure serving throughput with this many batches (of the same size) in flight on '
                         'as many HIP streams, each its own captured step (reported as "serving"; `value` is one '
                         'batch in flight); 1: skip')
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--debug-options', default='', metavar='NAME=V,...',
                    help='plan debug options (A/B of alternative code paths; the default is what is reported)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-roofline', action='store_true')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # rehearsal knobs (one-GPU boxes): CNF_BENCH_DEVICE pins every rank to one device,
    # CNF_BENCH_BACKEND=gloo replaces RCCL; the driver's multi-GPU runs use neither
    if os.environ.get('CNF_BENCH_DEVICE') is not None:
        local = int(os.environ['CNF_BENCH_DEVICE'])
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get('CNF_BENCH_BACKEND', 'nccl')
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(backend)

    cfg = PRESETS[args.config]
    from arl_conditional_normalizing_flows_amd.distributed import shard_range, pack_nll_sums
    if args.global_batch:
        G = args.global_batch
        lo, hi = shard_range(G, rank, world)
        scaling = 'strong'
    else:
        Bp = args.batch or cfg.batch
        G = Bp * world
        lo, hi = shard_range(G, rank, world)
        scaling = 'weak'
    B = hi - lo
    if B <= 0:
        raise SystemExit(f'rank {rank}: empty shard of a global batch of {G}')
    from arl_conditional_normalizing_flows_amd.make_model import cFlow
    flow = cFlow(**cfg.kwargs(), device=dev, seed=0, debug_options=args.debug_options or None)
    # one seeded global batch, sliced per rank
    xy_np = synth(cfg, G, 1000, 1.0 if (args.noise is not None and args.mode == 'forward') else 0.98)[lo:hi].copy()
    xy = torch.from_numpy(xy_np).to(dev)
    if args.mode == 'train':
        return train_bench(args, cfg, flow, xy, B, G, world, rank, dist, dev, scaling)
    red = torch.empty(5, device=dev)
    zy = torch.empty_like(xy)
    ld = torch.empty(B, device=dev)
    per = torch.empty((B, 3), device=dev)
    sums = torch.empty(4, device=dev)
    ws = flow._workspace(B)
    lib = _lib.load()

    inverse = args.mode == 'inverse'
    noisy = args.noise is not None and not inverse
    xn = torch.empty_like(xy) if noisy else xy   # the noisy input (cnf_flow_forward_noise writes it)
    if inverse:
        # sampling input: the forward's zy of the bench batch (a valid latent of this flow)
        zy_in, _ = flow(xy, 1)
        x_out = torch.empty_like(xy)
        torch.cuda.synchronize()

    def local_step():
        st = torch.cuda.current_stream().cuda_stream
        if inverse:
            _lib.check(lib.cnf_flow_inverse(flow._plan, flow.params.data_ptr(), flow._aux.data_ptr(),
                                            zy_in.data_ptr(), x_out.data_ptr(), ws.data_ptr(), B, st), 'inverse')
            return
        if noisy:
            _lib.check(lib.cnf_flow_forward_noise(flow._plan, flow.params.data_ptr(), flow._aux.data_ptr(),
                                                  xy.data_ptr(), float(args.logit), float(args.noise), 1000 + rank, 0,
                                                  xn.data_ptr(),
                                                  zy.data_ptr(), ld.data_ptr(), ws.data_ptr(), B, st), 'forward')
        else:
            _lib.check(lib.cnf_flow_forward(flow._plan, flow.params.data_ptr(), flow._aux.data_ptr(),
                                            xy.data_ptr(), zy.data_ptr(), ld.data_ptr(), ws.data_ptr(), B, st),
                       'forward')
        _lib.check(lib.cnf_nll(flow._plan, xn.data_ptr(), zy.data_ptr(), ld.data_ptr(), per.data_ptr(),
                               sums.data_ptr(), B, st), 'nll')

    def exchange():
        # the path's one exchange step, issued eagerly after the (graph-replayed) local work: RCCL
        # collectives are never captured into the graph (the inverse has none)
        if dist is not None and not inverse:
            pack_nll_sums(sums, B, red)
            dist.all_reduce(red)

    def step():
        local_step()
        exchange()

    def note(msg):
        if os.environ.get('CNF_BENCH_VERBOSE'):
            print(f'# rank {rank}: {msg}', file=sys.stderr, flush=True)

    serving = None
    if world == 1 and not inverse and args.inflight > 1:
        # first, on a fresh runtime: after hipExtLaunchKernelGGL with events (measure_in_stream), or
        # once the step graph has run on the default stream, the runtime serialises the lanes'
        # streams (measured in profiles/diag/diag_serving.py: 59.1k -> 43.3k images/s)
        serving = serving_inflight(flow, lib, xy, B, args.inflight, max(args.steps, 50), dev, args.noise, args.logit)
    note('first step')
    step()
    note('first step done')
    torch.cuda.synchronize()
    noise_pass = None
    if noisy:   # is the noise applied by a launch of its own (first layer streamed) or inside k_net_lds?
        nm = C.create_string_buffer(256)
        fl, by = C.c_double(), C.c_double()
        names = []
        for i in range(lib.cnf_plan_num_recorded_launches(flow._plan)):
            _lib.check(lib.cnf_plan_recorded_launch_info(flow._plan, i, nm, 256, C.byref(fl), C.byref(by)), 'info')
            names.append(nm.value.decode())
        noise_pass = 'k_prep' in names
    graph = None
    if not args.no_graph:
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                local_step()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                local_step()
            torch.cuda.synchronize()
        except Exception as e:  # pragma: no cover
            print(f'# graph capture failed, eager: {e}', file=sys.stderr)
            graph = None

    def replay():
        graph.replay()
        exchange()
    run = replay if graph is not None else step
    note(f'graph {graph is not None}; warmup')

    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    note('timed steps done')
    if dist is not None:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    ms = el / args.steps * 1e3
    total_imgs = G * args.steps
    value = total_imgs / el

    # results of the timed steps
    ld_mean = ld.mean().item() if not inverse else None
    loss_mean = ((red[0] / red[4]).item() if dist is not None else sums[0].item() / B) if not inverse else None
    rt_err = ((x_out - xy).abs().max() / xy.abs().max()).item() if inverse else None
    out = None
    if rank == 0:
        # per-step times for the median (BASELINE.md protocol): local work only, rank 0
        st_ms = []
        if graph is not None:
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(100)]
            for a, b in evs:
                a.record()
                graph.replay()
                b.record()
            torch.cuda.synchronize()
            st_ms = [a.elapsed_time(b) for a, b in evs]
        roof = None
        step_roof = None
        fl_img, by_img, n_ln = algorithmic_per_image(flow, B)
        if not args.no_roofline:
            launches = measure_in_stream(flow, local_step)
            roof, per_k = roofline_for(launches)
            tot = sum(d['ms'] for d in per_k.values())
            print(f'# per-kernel (in-stream kernel timestamps): total {tot:.3f} ms/step', file=sys.stderr)
            for nm, fl, by, t_ms in launches:
                print(f'#  {nm:34s} {t_ms * 1e3:8.2f} us  {fl / max(t_ms, 1e-9) / 1e9:7.2f} TF/s '
                      f'{by / max(t_ms, 1e-9) / 1e6:8.1f} GB/s', file=sys.stderr)
        t_mfma = fl_img * B / (FP32_MFMA_TFLOPS * 1e12) * 1e3
        t_hbm = by_img * B / (HBM_PEAK_GBS * 1e9) * 1e3
        step_ms = float(np.median(st_ms)) if st_ms else ms
        step_roof = {'bound': 'mfma' if t_mfma >= t_hbm else 'hbm', 'alg_gflop_per_image': round(fl_img / 1e9, 4),
                     'alg_mb_per_image': round(by_img / 1e6, 3), 'ln_elems_per_image': n_ln,
                     'roof_ms': round(max(t_mfma, t_hbm), 4), 'mfma_ms': round(t_mfma, 4), 'hbm_ms': round(t_hbm, 4),
                     'step_ms': round(step_ms, 4), 'frac': round(max(t_mfma, t_hbm) / step_ms, 4),
                     'achieved_tflops': round(fl_img * B / (step_ms / 1e3) / 1e12, 3),
                     'achieved_gbs': round(by_img * B / (step_ms / 1e3) / 1e9, 1)}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = (cpu_baseline_inverse(cfg, flow, zy_in.cpu().numpy(), B) if inverse
                   else cpu_baseline(cfg, flow, xn.cpu().numpy() if noisy else xy_np, B))
        H, W, _ = cfg.io_shape
        bpd = float(loss_mean / (np.log(2) * H * W * cfg.x_d)) if not inverse else None
        if inverse:
            metric = f'images/sec inverse (sampling, zy -> xy), {args.config}'
        elif args.config == 'cfg2':
            metric = 'images/sec fwd+logdet, 32x32x3 3-scale flow @1/2/4/8 GPU; bits/dim vs ref'
        else:
            metric = f'images/sec fwd+logdet ({args.config})'
        out = {
            'metric': metric,
            'value': round(value, 2), 'unit': 'images/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms, 4), 'higher_is_better': True, 'scaling': scaling,
            'vs_baseline': None, 'dtype': 'f32',
            'data': ('synthetic (seeded class-conditional batch, ' if cfg.data == 'class' else
                     'synthetic (seeded SR batch: residual x, down/up y, ')
                    + ('clean; logit + 2% noise applied in the forward' if noisy and args.logit else
                       'clean; 2% noise applied in the forward' if noisy else '2% noise')
                    + '), seeded orthogonal-init weights',
            'config': {'workload': (f'{cfg.name}: cFlow.call(zy,-1), zy {list(cfg.io_shape)}, ' if inverse else
                                    f'{cfg.name}: cFlow.call(xy,+1) + log-det + NLL sums, xy {list(cfg.io_shape)}, ')
                                   + (f'{G} images global over {world} GPUs' if scaling == 'strong'
                                      else f'{B} images per GPU'),
                       'model': f'cFlow {cfg.name}', 'global_batch': G,
                       'per_gpu_batch': B, 'seq_len': None, 'parallelism': f'dp{world} (batch shards, '
                                                                          f'1 all-reduce of 5 fp32)',
                       'graph': graph is not None,
                       'input_noise': ({'alpha': args.noise, 'logit_a': args.logit or None,
                                        'separate_noise_pass': noise_pass}
                                       if noisy else None)},
            'step_ms_median': round(float(np.median(st_ms)), 4) if st_ms else None,
            'bits_per_dim': round(bpd, 6) if bpd is not None else None,
            'logdet_mean': ld_mean,
            'roundtrip_rel_err': rt_err,
            'roofline': roof,
            'step_roofline': step_roof,
            'cpu_baseline': cpu,
            'serving': serving,
        }
        if cpu and cpu.get('bits_per_dim_ref') is not None and world == 1:
            out['bits_per_dim_ref'] = round(cpu['bits_per_dim_ref'], 6)
            out['bits_per_dim_abs_err'] = abs(bpd - cpu['bits_per_dim_ref'])
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
