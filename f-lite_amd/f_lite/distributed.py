"""Multi-GPU sampling: independent images sharded one per GPU (replica data parallelism).

The reference has no multi-GPU inference; its torch.distributed use is training-only
(f_lite/distributed.py:71-80, NCCL). Here every rank holds a full copy of the weights (22 GB of bf16 for the
10B model, far below the 288 GB of HBM) and generates its own images; the only collective is one broadcast of
the shared text embedding from rank 0 (RCCL over xGMI with the "nccl" backend), before the denoise loop.
No per-step communication. With APG enabled the reference's batch-global reductions (pipeline.py:281-285)
couple images; sharded APG is per image (documented in DESIGN.md).
"""
from __future__ import annotations

import os
from typing import List

import torch


def world() -> "tuple[int, int, int]":
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


def image_indices(n_images: int, rank: int, world_size: int) -> List[int]:
    """Global image indices owned by `rank`: image i -> rank i mod world_size."""
    return list(range(rank, n_images, world_size))


def broadcast_context(ctx: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    """The one collective of the path: the shared text embedding from rank `src` to every rank (in place)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(ctx, src=src, group=group)
    return ctx


def max_over_ranks(seconds: float, device=None, group=None) -> float:
    """Job wall time = the slowest rank's time (bench.py contract)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
