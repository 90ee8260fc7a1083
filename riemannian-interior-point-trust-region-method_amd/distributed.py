"""Instance sharding across GPUs: one process per GPU, torch.distributed over RCCL ("nccl").

The reference runs its Hydra multi-run axis (problem_instance x problem_initialpoint,
``src/NonnegPCA/config_simulation.yaml:38-42``) one solve after another.  Instances share no
state during a solve, so the path partitions with no data-path collective: global instance
``b`` is owned by rank ``b % world`` (interleaving balances instances whose cost differs), each
rank solves its shard with its own ``NonnegPCABatch``, and the only communication is the final
gather of per-instance results (x, y, stats) and the timing max.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist


def shard_ids(total: int, world: int, rank: int) -> List[int]:
    """Global instance ids owned by ``rank``: rank, rank + world, ..."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    return list(range(rank, total, world))


def gather_rows(local: torch.Tensor, total: int, world: int, rank: int, group=None) -> torch.Tensor:
    """All-gather per-instance rows (shape (len(shard_ids), ...)) into global instance order.

    Shards differ in length by at most one row; each rank pads to the longest shard so a single
    ``all_gather`` (RCCL on GPU tensors, gloo on CPU) moves everything at once."""
    per = (total + world - 1) // world
    pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    out = torch.empty((total,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    for r in range(world):
        ids = shard_ids(total, world, r)
        out[ids] = bufs[r][: len(ids)]
    return out


def max_over_ranks(value: float, device, group=None) -> float:
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def solve_sharded(problems: Sequence, option, log_capacity: int = 8192) -> Tuple[List, List[int]]:
    """Each rank solves its shard of ``problems`` (same n) on its GPU with the drop-in RIPTRM
    and returns (its Outputs, their global ids).  Call ``gather_rows`` on what must be shared."""
    from RIPTRM import RIPTRM
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    ids = shard_ids(len(problems), world, rank)
    outs = RIPTRM(option).run_batch([problems[i] for i in ids], log_capacity=log_capacity) if ids else []
    return outs, ids
