"""bench.py's N > 1 path rehearsed on one GPU: two ranks over gloo pinned to cuda:0
(CNF_BENCH_DEVICE / CNF_BENCH_BACKEND). Covers the sharded batch, the eager exchange step after the
graph replay, the max-over-ranks timing and rank 0's roofline measurement (which must not issue
a collective the other ranks never join)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_gloo_rehearsal(gpu):
    env = dict(os.environ, CNF_BENCH_DEVICE='0', CNF_BENCH_BACKEND='gloo')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2', '--master-addr',
           '127.0.0.1', '--master-port', '29541', os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--steps', '2',
           '--warmup', '1', '--no-cpu-baseline']
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1                       # rank 0 only
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2 and out['config']['global_batch'] == 2 * out['config']['per_gpu_batch']
    assert out['value'] > 0 and out['roofline'] is not None
