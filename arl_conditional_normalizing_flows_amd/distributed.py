"""Batch sharding of the flow across ranks (one process per GPU) and the path's single exchange
step: the batch-mean NLL terms of cFlow.log_loss (conv_cINN_make_model.py:1800-1848) and the
batch-mean log-det (:1323-1326) are the only cross-image quantities, so each rank computes the
sums of its own images and one all-reduce (RCCL over xGMI on the GPU box, gloo in the CPU tests)
of 5 fp32 — [sum loss_i, sum -llz_i, sum -lly_i, sum -logdet_i, n_images] — yields the global
means. Shards may be ragged; the image count travels with the sums."""
from __future__ import annotations

from typing import Optional, Tuple

import torch


def shard_range(global_batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Images [lo, hi) of rank `rank`: contiguous, sizes differ by at most one."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f'bad rank {rank} / world {world}')
    if global_batch < 0:
        raise ValueError('negative batch')
    q, r = divmod(global_batch, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def pack_nll_sums(sums: torch.Tensor, n_local: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[4 sums] + [n_local] -> one contiguous 5-float buffer (the all-reduce payload)."""
    if out is None:
        out = torch.empty(5, device=sums.device, dtype=torch.float32)
    out[:4].copy_(sums.reshape(4))
    out[4].fill_(float(n_local))
    return out


def reduce_nll_sums(sums: torch.Tensor, n_local: int, group=None, all_reduce: bool = True):
    """Global (loss, z_loss, y_loss, detJ_loss) batch means from this rank's 4 sums: one
    all-reduce of 5 fp32 when torch.distributed is initialised (and all_reduce is True)."""
    buf = pack_nll_sums(sums, n_local)
    if all_reduce:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(buf, group=group)
    n = buf[4]
    m = buf[:4] / n
    return m[0], m[1], m[2], m[3]


def allreduce_grads(grads: torch.Tensor, group=None, bucket_floats: int = 1 << 24) -> torch.Tensor:
    """Sum the flat gradient over ranks (the training step's exchange, cFlow.train_step on a
    data-parallel batch). Buckets of up to 64 MiB: large enough to run each ring collective at
    the xGMI link rate, small enough to bound the staging memory."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return grads
    flat = grads.reshape(-1)
    for lo in range(0, flat.numel(), bucket_floats):
        dist.all_reduce(flat[lo:lo + bucket_floats], group=group)
    return grads
