"""Data-parallel frame sharding.

Inference over video frames is embarrassingly parallel (seg_video_old_no_plot.py:157-166
processes frames independently): one process per GPU takes a contiguous range of frames
and runs the HIP engine on it; no collective touches the data path.  The only exchanges
are host-side bookkeeping: the max-over-ranks of a timed region (bench.py) and, for
evaluation, the sum of per-rank confusion matrices (semantic_seg.py:455-457 accumulates
fast_hist over the whole val set).

The reference's multi-GPU drivers use torch.distributed over NCCL (semantic_seg_multigpu.py
:467-468, rmbsnn_main.py:169); here the same API maps to RCCL ("nccl" backend on ROCm) on
the GPU box and to gloo in the CPU tests.
"""
from __future__ import annotations

import os


def world():
    """(rank, world_size, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(total: int, rank: int, world_size: int) -> range:
    """Contiguous, balanced frame range of `rank` (sizes differ by at most one)."""
    if world_size <= 0 or not 0 <= rank < world_size:
        raise ValueError("bad rank/world_size")
    base, extra = divmod(total, world_size)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def max_over_ranks(value: float, device=None) -> float:
    """Max of a host scalar over all ranks (timing: the slowest rank defines the job)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(tensor):
    """In-place sum of a (small) tensor over ranks, e.g. the 19x19 int64 confusion matrix."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(tensor, op=dist.ReduceOp.SUM)
    return tensor
