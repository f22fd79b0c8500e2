"""Multi-GPU `audt`: one process per GPU, VCF-row shards, one RCCL gather to rank 0.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m svtrek_amd.audt_dist -b sample.bam -v calls.vcf [--wider-interval N ...]

Every rank parses the VCF (svth_vcf_parse, multithreaded), takes the contiguous slice
[r*ceil(N/G), (r+1)*ceil(N/G)) of the loci in genomic order and reads from the BAM only what
that slice's queries can reach: the records from the BAI's linear-index offset of the
slice's first query to its last query's end (svth_bam_read_region; the whole file when there
is no BAI), trimmed to the queries' hull (pileup.halo_slice).  It refines them on its own GPU
(svtrek_amd.Engine, HIP); the ranks agree on success with one all-reduce of a status flag
(a rank that failed makes every rank exit non-zero instead of leaving the others blocked in
the gather), then rank 0 gathers the 16-byte {vcf_index, start, end, pad} records
(torch.distributed nccl = RCCL over xGMI) and prints the reference's stdout (A11) in VCF
order.  Single-node `svtrek audt --gpus N` does the same sharding with host threads.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np


def parse_vcf(path: str, threads: int = 4):
    """A1 over every data line (audit.c:301-338) via the C++ batch parser: (loci, stderr text)."""
    from . import host
    with open(path, "rb") as f:
        data = f.read()
    return host.parse_vcf_text(data, threads=threads)


def shard_region(loci: np.ndarray, wider: int, median: int, narrow: int):
    """(tid0, beg0, tid1, end1) spanning every query of `loci` (one genomic-order shard), or
    None when they issue none: the part of a sorted BAM svth_bam_read_region has to read."""
    from .pileup import query_spans
    if len(loci) == 0:
        return None
    nt = int(max(1, int(loci["chrom"].max())))
    sp = query_spans(loci, wider, median, narrow, nt)
    live = np.nonzero(sp[:, 1] > sp[:, 0])[0]
    if len(live) == 0:
        return None
    t0, t1 = int(live[0]), int(live[-1])
    return t0, int(sp[t0, 0]), t1, int(sp[t1, 1])


def load_shard(bam: str, loci: np.ndarray, prm, threads: int):
    """The reads the shard's queries can yield: a BAI region read + halo trim (or, without a
    BAI, the whole file + halo trim)."""
    from . import host
    from .pileup import halo_slice
    reg = shard_region(loci, prm.wider_interval, prm.median_interval, prm.narrow_interval)
    if reg is None:
        reg = (0, 0, 0, 0)
    if os.path.exists(bam + ".bai"):
        pl, info = host.read_bam(bam, threads=threads, region=reg)
    else:
        sys.stderr.write(f"[svtrek_amd] no {bam}.bai: reading the whole BAM\n")
        pl, info = host.read_bam(bam, threads=threads)
    return halo_slice(pl, loci, prm.wider_interval, prm.median_interval, prm.narrow_interval), info


def run_rank(bam: str, loci, prm, threads: int, refine, world: int, rank: int, device=None):
    """One rank's whole job: shard, region load, refine (refine(pileup, loci) -> results),
    status agreement, gather.  Returns every result in VCF order on rank 0, None elsewhere.

    `loci` may be the parsed array or a zero-argument callable that parses the VCF; every step
    that can fail on one rank -- parsing, the engine (built lazily by `refine`), the BAM read,
    the refinement, packing the gather records -- runs before the status all-reduce, so a
    failing rank makes every rank raise instead of leaving the others blocked in a collective."""
    import torch
    import torch.distributed as dist

    from ._lib import RESULT_DTYPE
    from .distributed import pack_records, padded_rows, shard_rows, unpack_records
    err = None
    rows = np.zeros(0, dtype=np.int64)
    local = np.zeros(0, dtype=RESULT_DTYPE)
    payload = None
    n_total = 0
    try:
        if callable(loci):
            loci = loci()
        n_total = len(loci)
        rows = shard_rows(loci, world, rank)
        mine = loci[rows]
        if len(rows):
            pl, _ = load_shard(bam, mine, prm, threads)
            local = refine(pl, mine)
        if world > 1:
            payload = pack_records(rows, local, padded_rows(n_total, world))
    except Exception as e:   # noqa: BLE001 -- reported, then every rank stops together
        err = f"rank {rank}: {type(e).__name__}: {e}"
    if world > 1:
        flag = torch.tensor([1 if err else 0], dtype=torch.int32, device=device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if int(flag.item()):
            raise RuntimeError(err or f"rank {rank}: another rank failed")
        t = torch.from_numpy(payload.view(np.int32).copy())
        if device is not None:
            t = t.to(device)
        parts = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
        dist.gather(t, parts, dst=0)
        if rank != 0:
            return None
        return unpack_records(np.concatenate([p.cpu().numpy().view(np.uint32) for p in parts]), n_total)
    if err:
        raise RuntimeError(err)
    out = np.empty(n_total, dtype=RESULT_DTYPE)
    out[rows] = local
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-b", "--bam", required=True)
    ap.add_argument("-v", "--vcf", required=True)
    ap.add_argument("-t", type=int, default=4)
    ap.add_argument("--wider-interval", type=int, default=20000)
    ap.add_argument("--median-interval", type=int, default=10000)
    ap.add_argument("--narrow-interval", type=int, default=2000)
    ap.add_argument("--consensus-interval-range", type=int, default=500)
    ap.add_argument("--consensus-interval", type=int, default=5)
    ap.add_argument("--consensus-min-count", type=int, default=3)
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    from . import Engine, Params, host

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank (RCCL); with fewer GPUs than ranks the ranks share them round-robin and the
    # status all-reduce and gather go through host memory (gloo): the one-device emulation
    ndev = torch.cuda.device_count()
    gpu = local % max(ndev, 1)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    emulated = world > 1 and ndev < world
    if world > 1:
        if emulated:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    if rank == 0:
        sys.stdout.write("[INFO] Started processing variation file.\n")
        sys.stdout.flush()
    prm = Params(a.wider_interval, a.median_interval, a.narrow_interval, a.consensus_interval_range,
                 a.consensus_interval, a.consensus_min_count)
    state = {}

    def load_loci():   # parsed inside run_rank's guarded region (a bad VCF stops every rank)
        loci, msgs = parse_vcf(a.vcf, threads=max(1, a.t))
        state["loci"] = loci
        if rank == 0 and msgs:
            sys.stderr.write(msgs)
        return loci

    def refine(pl, mine):   # the engine is built on first use, inside the guarded region too
        if "eng" not in state:
            state["eng"] = Engine(prm, device=gpu)
        state["eng"].load_pileup(pl)
        return state["eng"].refine(mine)

    rc = 0
    try:
        res = run_rank(a.bam, load_loci, prm, max(1, a.t), refine, world, rank, device=None if emulated else dev)
    except RuntimeError as e:
        sys.stderr.write(f"[ERROR] {e}\n")
        res, rc = None, 1
    finally:
        if "eng" in state:
            state["eng"].close()
    if rank == 0 and rc == 0:
        sys.stdout.write(host.format_batch(state["loci"], res, threads=max(1, a.t)))
        sys.stdout.write("[INFO] Ended processing variation file\n")
        sys.stdout.flush()
    if world > 1:
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
