"""TEST INFRASTRUCTURE (bench.py's cpu_baseline leg only): the reference-shaped CPU baseline
of SURVEY.md §8(d) on a bounded sample of the bench workload.

The sample: the first K loci (genomic order) of contig 1 of the workload.  Their reads -- every
record overlapping the union of their windows -- are written as a coordinate-sorted BAM with
random SEQ/QUAL (the reference's bam_read1 copies them) and a BAI (sim.write_bam(region=...)),
so every one of their region queries yields exactly the reads it yields on the full genome.
oracle/bgzf_ref.c then runs them the way the reference's tpool path does (T workers, each with
its own BAM handle and BAI; per query a linear-index seek, BGZF inflate, record decode; the
oracle's CIGAR walks and vote), at T threads and at 1 thread, and its results are checked
against the in-memory oracle on the same loci.
"""
from __future__ import annotations

import os
import shutil
import tempfile
import time

import numpy as np

import oracle_ffi as O


def _sample(res, loci: np.ndarray, params, k: int):
    """(sample loci in genomic order, (tid, beg, end) region covering all their windows)."""
    c1 = loci[loci["chrom"] == 1]
    c1 = c1[np.argsort(c1["pos"], kind="stable")][:k]
    if len(c1) == 0:
        return c1, None
    w = max(params.wider_interval, params.median_interval, params.narrow_interval)
    beg = max(0, int(c1["pos"].min()) - w - 1)
    end = int(max(int(c1["pos"].max()), int(c1["end"].max()))) + w + 1
    return c1, (0, beg, end)


def run(res, loci: np.ndarray, n_threads: int, budget_s: float = 24.0, params=None, k: int = 1000,
        level: int = 1) -> dict:
    from svtrek_amd import Params, sim
    params = params or Params()
    sl, region = _sample(res, loci, params, k)
    if region is None or res.handle is None:
        return {}
    d = tempfile.mkdtemp(prefix="svt_bgzf_")
    try:
        bam = os.path.join(d, "sample.bam")
        t0 = time.perf_counter()
        sim.write_bam(res, bam, with_seq=True, level=level, bai=True, region=region)
        write_s = time.perf_counter() - t0
        want = O.refine_batch(res.pileup, sl, params)

        def timed(n: int, threads: int, min_s: float):
            done, t = 0, time.perf_counter()
            stats = None
            while True:
                got, stats = O.bgzf_refine_batch(bam, sl[:n], params, threads=threads, with_stats=True)
                if not (np.array_equal(got["start"], want["start"][:n]) and np.array_equal(got["end"], want["end"][:n])):
                    raise RuntimeError("BGZF baseline disagrees with the in-memory oracle")
                done += n
                dt = time.perf_counter() - t
                if dt >= min_s:
                    return done / dt, done, stats

        # 1 thread on a prefix sized to ~1/3 of the budget, then T threads on the whole sample
        t = time.perf_counter()
        O.bgzf_refine_batch(bam, sl[:20], params, threads=1)
        per = max(time.perf_counter() - t, 1e-6) / min(20, len(sl))
        n1 = int(min(len(sl), max(20, budget_s / 3 / per)))
        v1, d1, _ = timed(n1, 1, budget_s / 3)
        vt, dt, st = timed(len(sl), n_threads, budget_s * 2 / 3)
        bam_mb = os.path.getsize(bam) / 1e6
        return {
            "value_bgzf": round(vt, 1),
            "value_bgzf_1thread": round(v1, 1),
            "bgzf_sample": (f"first {len(sl)} loci of contig 1 (genomic order; BAM of their {region[2] - region[1]} bp "
                            f"region: {bam_mb:.0f} MB, random SEQ/QUAL, zlib level {level}, + BAI), repeated for "
                            f">= {budget_s * 2 / 3:.0f} s ({dt} loci) on {n_threads} worker threads, each with its own "
                            f"BAM handle and BAI; per query a linear-index seek + BGZF inflate + record decode "
                            f"(oracle/bgzf_ref.c); 1 thread: {d1} loci; results equal the in-memory oracle's"),
            "bgzf_inflated_bytes_per_locus": round(st["bytes_inflated"] / max(1, len(sl)), 1),
            "bgzf_write_s": round(write_s, 2),
        }
    finally:
        shutil.rmtree(d, ignore_errors=True)
