"""Sequence sharding across GPUs: one process per GPU, sequence i on rank i % world.

The reference maps sequences to GPUs by Pool worker id (``worker_id % num_gpu``,
RGBT_workspace/test_rgbt_mgpus.py:80-86; ViPT/lib/test/evaluation/running.py:104-113). Tracking
has no cross-sequence exchange, so the only collectives are a barrier and the max-reduction of a
timed region (bench.py) -- none on the data path.
"""
from __future__ import annotations

import os


def rank_world():
    """(rank, world) from torch.distributed when initialised, else from the torchrun env."""
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
    except Exception:
        pass
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def shard_indices(n: int, rank: int, world: int):
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    return list(range(rank, n, world))


def shard(items, rank: int, world: int):
    return [items[i] for i in shard_indices(len(items), rank, world)]


def max_over_ranks(value: float) -> float:
    """Max of a host float over all ranks (gloo or nccl); identity when not distributed."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    dev = "cpu" if dist.get_backend() == "gloo" else torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    dev = "cpu" if dist.get_backend() == "gloo" else torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
