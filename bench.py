#!/usr/bin/env python3
"""Benchmark: images/sec of fwd + log-det (+ NLL sums) of the conditional RealNVP hot path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one cFlow.call(xy, +1) (zy + per-image log-det) + the NLL 4-sum over one batch of
synthetic inputs already resident in HBM; with N>1 every rank processes its own batch
(weak scaling, BASELINE configs[1] batch 64 per GPU) and the 4 NLL sums are all-reduced
(the path's only exchange step, one RCCL all-reduce of 5 fp32: the 4 sums + the image count). value = images processed by
all ranks / max-over-ranks wall time of the K timed steps.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from arl_conditional_normalizing_flows_amd import _lib  # noqa: E402
from arl_conditional_normalizing_flows_amd.config import PRESETS  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_16x16x4_f32) dense peak


def synth(cfg, B, seed):
    from arl_conditional_normalizing_flows_amd.synthetic import class_batch, sr_batch
    H, W, D = cfg.io_shape
    if cfg.data == 'class':
        return class_batch(B, H, W, cfg.x_d, seed=seed)
    return sr_batch(B, H, W, cfg.x_d, cfg.sr_pow, seed=seed)


def measure_dominant_kernel(flow, stream, reps=50):
    """Re-launch every recorded launch of the last forward with HIP events on the launch
    stream; aggregate per kernel symbol; return the symbol with the largest total time."""
    lib = _lib.load()
    plan = flow._plan
    n = lib.cnf_plan_num_recorded_launches(plan)
    import ctypes as C
    name = C.create_string_buffer(256)
    fl = C.c_double()
    by = C.c_double()
    per = {}
    s = torch.cuda.current_stream()
    for i in range(n):
        _lib.check(lib.cnf_plan_recorded_launch_info(plan, i, name, 256, C.byref(fl), C.byref(by)), 'info')
        nm = name.value.decode()
        if not nm.startswith('k_'):
            continue
        # warm
        for _ in range(3):
            _lib.check(lib.cnf_plan_relaunch(plan, i, stream), 'relaunch')
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            _lib.check(lib.cnf_plan_relaunch(plan, i, stream), 'relaunch')
        e1.record(s)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        d = per.setdefault(nm, {'ms': 0.0, 'flops': 0.0, 'bytes': 0.0, 'launches': 0})
        d['ms'] += ms
        d['flops'] += fl.value
        d['bytes'] += by.value
        d['launches'] += 1
    return per


def roofline_for(per):
    name, d = max(per.items(), key=lambda kv: kv[1]['ms'])
    t = d['ms'] / 1e3
    tflops = d['flops'] / t / 1e12
    gbs = d['bytes'] / t / 1e9
    # bound = the roof the kernel's algorithmic intensity runs into first
    ai = d['flops'] / max(d['bytes'], 1.0)
    ridge = FP32_MFMA_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)
    if ai >= ridge:
        rf = {'bound': 'mfma', 'achieved': round(tflops, 3), 'peak': FP32_MFMA_TFLOPS, 'unit': 'TFLOP/s',
              'frac': round(tflops / FP32_MFMA_TFLOPS, 4)}
    else:
        rf = {'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
              'frac': round(gbs / HBM_PEAK_GBS, 4)}
    rf.update({'kernel': name, 'launches_per_step': d['launches'],
               'avg_launch_us': round(d['ms'] * 1e3 / d['launches'], 3),
               'alg_flops_per_launch': d['flops'] / d['launches'],
               'alg_bytes_per_launch': d['bytes'] / d['launches']})
    rf.update(pmc_traffic(name))
    return rf


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
            if h and (sym.startswith(kernel + '<') or sym == kernel):
                d = float(h.get('dispatches', 1))
                tot += h['traffic_bytes'] * d
                n += d
        if n > 0:
            return {'traffic': round(tot / n, 1), 'traffic_unit': 'bytes/launch',
                    'traffic_source': os.path.relpath(f, ROOT)}
    return {'traffic': None}


def cpu_baseline(cfg, budget_s=12.0):
    """The oracle's torch-CPU fp32 op-for-op restatement of the reference graph, timed on this
    host on a bounded sample of the same workload (rank 0, N=1 only)."""
    try:
        from oracle.cflow_torch_cpu import TorchCPUFlow
    except Exception as e:  # pragma: no cover
        return {'value': None, 'unit': 'images/s', 'cores': 0, 'kind': 'port', 'sample': f'unavailable: {e}'}
    # the host's CPU share, not the machine's: os.cpu_count() on the GPU box reports every core
    try:
        threads = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        threads = os.cpu_count() or 1
    threads = max(1, min(threads, int(os.environ.get('OMP_NUM_THREADS', '16') or 16), 16))
    torch.set_num_threads(threads)
    flow = TorchCPUFlow(**cfg.kwargs())
    P = flow.init_params(0)
    B = 8
    xy = torch.from_numpy(synth(cfg, B, 123))
    with torch.no_grad():
        flow.log_loss(xy, P)          # warm-up
        n_img, t0 = 0, time.perf_counter()
        while True:
            flow.log_loss(xy, P)
            n_img += B
            el = time.perf_counter() - t0
            if el > budget_s:
                break
    model = platform.processor() or platform.machine()
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    return {'value': round(n_img / el, 3), 'unit': 'images/s', 'cores': threads, 'kind': 'port',
            'sample': f'{n_img} images ({n_img // B} batches of {B}) of {cfg.name} fwd+logdet+NLL, '
                      f'{el:.1f}s, torch-CPU fp32 restatement (oracle/cflow_torch_cpu.py), {model}'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--config', default='cfg2')
    ap.add_argument('--batch', type=int, default=0, help='per-GPU batch (default: the config batch)')
    ap.add_argument('--no-graph', action='store_true')
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
    B = args.batch or cfg.batch
    from arl_conditional_normalizing_flows_amd.make_model import cFlow
    flow = cFlow(**cfg.kwargs(), device=dev, seed=0)
    # one seeded global batch, sliced per rank (weak scaling: B images per rank)
    from arl_conditional_normalizing_flows_amd.distributed import shard_range, pack_nll_sums
    lo, hi = shard_range(B * world, rank, world)
    xy = torch.from_numpy(synth(cfg, B * world, 1000)[lo:hi].copy()).to(dev)
    red = torch.empty(5, device=dev)
    zy = torch.empty_like(xy)
    ld = torch.empty(B, device=dev)
    per = torch.empty((B, 3), device=dev)
    sums = torch.empty(4, device=dev)
    ws = flow._workspace(B)
    lib = _lib.load()

    def local_step():
        st = torch.cuda.current_stream().cuda_stream
        _lib.check(lib.cnf_flow_forward(flow._plan, flow.params.data_ptr(), flow._aux.data_ptr(), xy.data_ptr(),
                                        zy.data_ptr(), ld.data_ptr(), ws.data_ptr(), B, st), 'forward')
        _lib.check(lib.cnf_nll(flow._plan, xy.data_ptr(), zy.data_ptr(), ld.data_ptr(), per.data_ptr(),
                               sums.data_ptr(), B, st), 'nll')

    def exchange():
        # the path's one exchange step, issued eagerly after the (graph-replayed) local work: RCCL
        # collectives are never captured into the graph
        if dist is not None:
            pack_nll_sums(sums, B, red)
            dist.all_reduce(red)

    def step():
        local_step()
        exchange()

    def note(msg):
        if os.environ.get('CNF_BENCH_VERBOSE'):
            print(f'# rank {rank}: {msg}', file=sys.stderr, flush=True)

    note('first step')
    step()
    note('first step done')
    torch.cuda.synchronize()
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
    total_imgs = B * world * args.steps
    value = total_imgs / el

    # results of the timed steps, read before the roofline re-launches below overwrite the
    # workspace (kernels re-run out of order, e.g. conv_b's in-place residual accumulates)
    ld_mean = ld.mean().item()
    out = None
    if rank == 0:
        roof = None
        if not args.no_roofline:
            local_step()   # eager forward records its launches (no collective: rank 0 only)
            torch.cuda.synchronize()
            per_k = measure_dominant_kernel(flow, torch.cuda.current_stream().cuda_stream)
            roof = roofline_for(per_k)
            tot = sum(d['ms'] for d in per_k.values())
            print(f'# per-kernel (re-launched in isolation): total {tot:.3f} ms/step', file=sys.stderr)
            for nm, d in sorted(per_k.items(), key=lambda kv: -kv[1]['ms']):
                t = d['ms'] / 1e3
                print(f'#  {nm:34s} {d["ms"]:8.3f} ms  x{d["launches"]:3d}  {d["flops"] / t / 1e12:7.2f} TF/s '
                      f'{d["bytes"] / t / 1e9:8.1f} GB/s', file=sys.stderr)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(cfg)
        # global batch-mean NLL (nats/image): the all-reduced sums when sharded
        loss_mean = (red[0] / red[4]).item() if dist is not None else sums[0].item() / B
        out = {
            'metric': 'images/sec fwd+logdet, 32x32x3 3-scale flow @1/2/4/8 GPU; bits/dim vs ref'
            if args.config == 'cfg2' else f'images/sec fwd+logdet ({args.config})',
            'value': round(value, 2), 'unit': 'images/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms, 4), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic (seeded class-conditional batch, 2% noise), '
                                                        'seeded orthogonal-init weights',
            'config': {'workload': f'{cfg.name}: cFlow.call(xy,+1) + log-det + NLL sums, xy {list(cfg.io_shape)}, '
                                   f'{B} images per GPU', 'model': f'cFlow {cfg.name}', 'global_batch': B * world,
                       'per_gpu_batch': B, 'seq_len': None, 'parallelism': f'dp{world} (batch shards, '
                                                                          f'1 all-reduce of 5 fp32)',
                       'graph': graph is not None},
            'bits_per_dim': round(float(loss_mean / (np.log(2) * cfg.io_shape[0] * cfg.io_shape[1] * cfg.x_d)), 6),
            'logdet_mean': ld_mean,
            'roofline': roof,
            'cpu_baseline': cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
