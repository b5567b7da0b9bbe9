"""Multi-GPU plumbing: one process per GPU, tasks sharded round-robin, ONE collective per
meta-step (sum of the flat [meta-gradient | query-loss scalar] buffer), replicated outer update.

Backend "nccl" is RCCL over xGMI on ROCm; "gloo" runs the same logic on CPU for tests.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_from_env(backend: str = "nccl", device: Optional[torch.device] = None):
    rank, world, _ = env_rank()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": device} if (device is not None and backend == "nccl") else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return rank, world


def active():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def shard_tasks(n_tasks: int, rank: int, world: int) -> List[int]:
    """Round-robin task -> rank assignment (15 tasks on 8 ranks: {2,2,2,2,2,2,2,1})."""
    return [j for j in range(n_tasks) if j % world == rank]


def reduce_meta(buf: torch.Tensor, group=None):
    """In place: buf <- sum over ranks. ``buf`` is the flat [meta-gradient | query-loss sum]
    buffer of MetaLearner (one collective per meta-step; just the scalar in reference mode)."""
    if not active():
        return
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)


def max_over_ranks(x: float, device) -> float:
    if not active():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def min_over_ranks(x: float, device) -> float:
    if not active():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())
