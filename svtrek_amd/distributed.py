"""Multi-GPU sharding of SV loci: one process per GPU, one gather of refined calls.

SURVEY.md §8(e): records are independent (reference thread_func keeps no cross-record
state, audit.c:50-248).  Loci are put in genomic order (tid, pos) keeping their VCF row
index, rank g refines the contiguous range [g*ceil(N/G), (g+1)*ceil(N/G)) of that order
against only the reads its queries can reach (pileup.halo_slice), and the only collective
is ONE gather to rank 0 of fixed-size {uint32 vcf_index, start, end, pad} records (RCCL
over xGMI with the nccl backend; gloo on CPU for tests), padded to ceil(N/G) rows with
vcf_index 0xFFFFFFFF.  Rank 0 scatters the records back into VCF order.
"""
from __future__ import annotations

from typing import Callable

import numpy as np

from ._lib import RESULT_DTYPE, SVT_NA

PAD_INDEX = 0xFFFFFFFF


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    per = (n + world - 1) // world if world > 0 else n
    b0 = min(n, per * rank)
    return b0, min(n, b0 + per)


def genomic_order(loci: np.ndarray) -> np.ndarray:
    """VCF row indices sorted by (chrom, pos), stable (ties keep VCF order)."""
    return np.lexsort((loci["pos"], loci["chrom"])).astype(np.int64)


def shard_rows(loci: np.ndarray, world: int, rank: int) -> np.ndarray:
    """The VCF row indices rank `rank` refines: a contiguous slice of the genomic order."""
    b0, b1 = shard_bounds(len(loci), world, rank)
    return genomic_order(loci)[b0:b1]


def padded_rows(n_total: int, world: int) -> int:
    """Rows per rank in the gather (every rank sends the same count)."""
    return max(1, (n_total + world - 1) // world)


def shard_workload(loci: np.ndarray, pileup, params, world: int, rank: int):
    """(rows, shard loci in genomic order, the reads their queries can reach) of rank `rank`.

    params: anything with wider_interval / median_interval / narrow_interval (Params)."""
    from .pileup import halo_slice
    rows = shard_rows(loci, world, rank)
    sl = loci[rows]
    if world == 1:
        return rows, sl, pileup
    return rows, sl, halo_slice(pileup, sl, params.wider_interval, params.median_interval, params.narrow_interval)


def pack_records(rows: np.ndarray, local: np.ndarray, per: int) -> np.ndarray:
    """{vcf_index, start, end, pad} uint32 records, padded to `per` rows."""
    if len(rows) > per:
        raise ValueError(f"shard of {len(rows)} rows exceeds the padded size {per}")
    buf = np.full((per, 4), SVT_NA, dtype=np.uint32)
    buf[:, 0] = PAD_INDEX
    buf[:len(rows), 0] = rows
    buf[:len(rows), 1] = local["start"]
    buf[:len(rows), 2] = local["end"]
    buf[:, 3] = 0
    return buf


def unpack_records(recs: np.ndarray, n_total: int) -> np.ndarray:
    """Scatter gathered records into VCF order; every row must arrive exactly once."""
    recs = recs.reshape(-1, 4)
    real = recs[recs[:, 0] != PAD_INDEX]
    idx = real[:, 0].astype(np.int64)
    if len(idx) != n_total or (n_total and (idx.max() >= n_total or np.bincount(idx, minlength=n_total).max() != 1)):
        raise RuntimeError("gathered records do not cover every VCF row exactly once")
    out = np.empty(n_total, dtype=RESULT_DTYPE)
    out["start"][idx] = real[:, 1]
    out["end"][idx] = real[:, 2]
    return out


class PipelinedGather:
    """Multi-buffered gather of per-step record buffers to rank 0 (bench.py's N > 1 step).

    `buffer(i)` hands out step i's buffer, i % nbuf (waiting -- as a stream dependency on GPU
    backends -- for the gather that last read it), `submit(i)` starts its asynchronous gather, so
    the gather of step i overlaps the refinement launches of the next steps.  nbuf >= the steps
    in flight: no two steps in flight write one buffer."""

    def __init__(self, make_buf, world: int, rank: int, enabled: bool = True, group=None, nbuf: int = 2,
                 host_stage: bool = False):
        import torch
        self.n = max(2, int(nbuf))
        self.bufs = [make_buf() for _ in range(self.n)]
        # host_stage (gloo with device buffers, the one-device emulation): each submit copies its
        # buffer to host memory (waiting for the step) and gathers the host copy
        self.host = host_stage and self.bufs[0].device.type != "cpu"
        self.send = [torch.empty(b.shape, dtype=b.dtype) for b in self.bufs] if self.host else self.bufs
        self.lists = [[torch.empty_like(b) for _ in range(world)] if rank == 0 else None for b in self.send]
        self.handles = [None] * self.n
        self.enabled = enabled and world > 1
        self.group = group

    def buffer(self, i: int):
        b = i % self.n
        if self.handles[b] is not None:
            self.handles[b].wait()
            self.handles[b] = None
        return self.bufs[b]

    def submit(self, i: int) -> None:
        if self.enabled:
            import torch.distributed as dist
            b = i % self.n
            if self.host:
                self.send[b].copy_(self.bufs[b])
            self.handles[b] = dist.gather(self.send[b], self.lists[b], dst=0, group=self.group, async_op=True)

    def drain(self) -> None:
        for b in range(self.n):
            if self.handles[b] is not None:
                self.handles[b].wait()
                self.handles[b] = None

    def gathered(self, i: int):
        """Rank 0: the buffers every rank sent at step i (after drain()); else None."""
        if not self.enabled:
            return [self.bufs[i % self.n]]
        return self.lists[i % self.n]


def gather_results(rows: np.ndarray, local: np.ndarray, n_total: int, device=None,
                   group=None) -> np.ndarray | None:
    """Gather every rank's (rows, results) to rank 0 and return all results in VCF order."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    per = max(1, (n_total + world - 1) // world)
    t = torch.from_numpy(pack_records(rows, local, per).view(np.int32).copy())
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, parts, dst=0, group=group)
    if rank != 0:
        return None
    allrecs = np.concatenate([p.cpu().numpy().view(np.uint32) for p in parts])
    return unpack_records(allrecs, n_total)


def run_sharded(loci: np.ndarray, refine: Callable[[np.ndarray], np.ndarray], device=None,
                group=None) -> np.ndarray | None:
    """Refine this rank's genomic shard with `refine(loci_subset)` and gather to rank 0.

    `refine` sees the shard's loci in genomic order; callers that hold a pileup give it
    `pileup.halo_slice(full, shard_loci, ...)` first (see audt_dist)."""
    import torch.distributed as dist

    rows = shard_rows(loci, dist.get_world_size(group), dist.get_rank(group))
    local = refine(loci[rows]) if len(rows) else np.zeros(0, dtype=RESULT_DTYPE)
    return gather_results(rows, local, len(loci), device=device, group=group)
