"""Multi-GPU `audt`: one process per GPU, VCF-row shards, one RCCL gather to rank 0.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m svtrek_amd.audt_dist -b sample.bam -v calls.vcf [--wider-interval N ...]

Every rank reads the BAM into a columnar pileup, takes the contiguous slice
[r*ceil(N/G), (r+1)*ceil(N/G)) of the loci in genomic order, uploads only the reads its
queries can reach (pileup.halo_slice) and refines them on its own GPU
(svtrek_amd.Engine, HIP); rank 0 gathers the 16-byte {vcf_index, start, end, pad}
records (torch.distributed nccl = RCCL over xGMI) and prints the reference's stdout
(A11) in VCF order.  Single-node `svtrek audt --gpus N` does the
same sharding with host threads instead of processes.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np


def parse_vcf(path: str):
    """A1 over every data line (audit.c:301-338) via the C++ parser; returns (loci, stderr lines)."""
    from . import host
    from ._lib import LOCUS_DTYPE
    rows, errs = [], []
    with open(path, "rb") as f:
        data = f.read().decode("latin-1")
    i = 0
    while i < len(data):
        j = data.find("\n", i)
        line = data[i:] if j < 0 else data[i:j + 1]
        i += len(line)
        if len(line) < 2 or line[0] == "#":
            continue
        if line.endswith("\n"):
            line = line[:-1]
        act, rec, err = host.parse_line(line)
        if act == 2:
            errs.append(err)
        if act == 1:
            if rec[0] not in (1, 2, 3):
                errs.append("[ERROR] Unkown type.\n")
            rows.append(rec)
    loci = np.zeros(len(rows), dtype=LOCUS_DTYPE)
    for k, r in enumerate(rows):
        loci[k] = r
    return loci, errs


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
    from .distributed import gather_results, shard_rows
    from .pileup import halo_slice

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    if rank == 0:
        sys.stdout.write("[INFO] Started processing variation file.\n")
    loci, errs = parse_vcf(a.vcf)
    if rank == 0:
        for e in errs:
            sys.stderr.write(e)
    pileup, _ = host.read_bam(a.bam, threads=max(1, a.t))
    prm = Params(a.wider_interval, a.median_interval, a.narrow_interval, a.consensus_interval_range,
                 a.consensus_interval, a.consensus_min_count)
    with Engine(prm, device=local) as eng:
        if world > 1:
            rows = shard_rows(loci, world, rank)
            mine = loci[rows]
            eng.load_pileup(halo_slice(pileup, mine, a.wider_interval, a.median_interval, a.narrow_interval))
            del pileup
            local_res = eng.refine(mine)
            res = gather_results(rows, local_res, len(loci), device=dev)
        else:
            eng.load_pileup(pileup)
            res = eng.refine(loci)
    if rank == 0:
        out = [host.format_result(loci[k], res[k]) for k in range(len(loci))]
        sys.stdout.write("".join(out))
        sys.stdout.write("[INFO] Ended processing variation file\n")
        sys.stdout.flush()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
