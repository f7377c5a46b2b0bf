"""Clip sharding across the GPUs of one node (one process per GPU).

Replaces the reference's single-process ``torch.nn.DataParallel`` (per-call
replicate + scatter + gather; pytorch/predict.py:239, pytorch/main_strong.py:541).
Clips are independent, so each rank loads the weights once, runs its
contiguous slice of clips, and the only collective is one gather of the
framewise (+ clipwise) outputs to rank 0 over RCCL (torch ``nccl`` backend on
ROCm) — xGMI point-to-point, no reduction.
"""
import os

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get('WORLD_SIZE', '1')), int(os.environ.get('RANK', '0')), \
        int(os.environ.get('LOCAL_RANK', '0'))


def init(backend=None):
    """Initialise the process group from torchrun env vars (no-op at world 1)."""
    world, rank, local = env_world()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = 'nccl' if torch.cuda.is_available() else 'gloo'
        if backend == 'nccl':
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return world, rank, local


def shard_range(n_items, rank, world):
    """Contiguous shard [lo, hi) of n_items for ``rank``."""
    base, rem = divmod(n_items, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def gather_to_rank0(t, world, rank):
    """Gather equally-shaped per-rank tensors to rank 0 (concatenated on dim 0);
    returns the full tensor on rank 0 and None elsewhere."""
    if world == 1:
        return t
    t = t.contiguous()
    if rank == 0:
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.gather(t, gather_list=parts, dst=0)
        return torch.cat(parts, dim=0)
    dist.gather(t, dst=0)
    return None


def gather_ragged_to_rank0(t, world, rank):
    """Gather per-rank tensors whose dim 0 differs (uneven shards)."""
    if world == 1:
        return t
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[:t.shape[0]] = t
    full = gather_to_rank0(pad, world, rank)
    if rank != 0:
        return None
    return torch.cat([full[i * mx:i * mx + s] for i, s in enumerate(sizes)], dim=0)
