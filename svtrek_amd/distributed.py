"""Multi-GPU sharding of SV loci: one process per GPU, one gather of refined calls.

SURVEY.md §8(e): records are independent (reference thread_func keeps no cross-record
state, audit.c:50-248), so rank g refines the contiguous row range
[g*ceil(N/G), (g+1)*ceil(N/G)) and the only collective is ONE gather of the fixed-size
results to rank 0 (RCCL over xGMI with the nccl backend; gloo on CPU for tests).
Results travel as uint32 pairs padded to ceil(N/G) rows with 0xFFFFFFFF.
"""
from __future__ import annotations

from typing import Callable

import numpy as np

from ._lib import RESULT_DTYPE, SVT_NA


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    per = (n + world - 1) // world if world > 0 else n
    b0 = min(n, per * rank)
    return b0, min(n, b0 + per)


def gather_results(local: np.ndarray, n_total: int, device=None, group=None) -> np.ndarray | None:
    """Gather every rank's RESULT_DTYPE rows to rank 0 (rows in rank order)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    per = (n_total + world - 1) // world
    buf = np.full((per, 2), SVT_NA, dtype=np.uint32)
    if len(local):
        buf[:len(local), 0] = local["start"]
        buf[:len(local), 1] = local["end"]
    t = torch.from_numpy(buf.view(np.int32).copy())
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, parts, dst=0, group=group)
    if rank != 0:
        return None
    allrows = np.concatenate([p.cpu().numpy().view(np.uint32) for p in parts])[:n_total]
    out = np.empty(n_total, dtype=RESULT_DTYPE)
    out["start"] = allrows[:, 0]
    out["end"] = allrows[:, 1]
    return out


def run_sharded(loci: np.ndarray, refine: Callable[[np.ndarray], np.ndarray], device=None,
                group=None) -> np.ndarray | None:
    """Refine this rank's shard with `refine` and gather all results to rank 0."""
    import torch.distributed as dist

    b0, b1 = shard_bounds(len(loci), dist.get_world_size(group), dist.get_rank(group))
    local = refine(loci[b0:b1]) if b1 > b0 else np.zeros(0, dtype=RESULT_DTYPE)
    return gather_results(local, len(loci), device=device, group=group)
