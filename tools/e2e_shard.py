"""End-to-end `svtrek audt` on one rank's slice of the headline workload.

The 8-GPU path (bench.py, audt_dist.py) gives rank r of N the contiguous genomic slice of the
VCF rows and only the reads its queries can reach.  This writes exactly that input for the
chosen ranks -- the slice's loci as a VCF and the records overlapping its windows (every contig
the slice spans, with SEQ/QUAL, level-1 BGZF, + BAI) as a BAM -- and times the drop-in CLI on
it on one GPU, so that each rank's ingest / load / refine / print split is measured on real
bytes.  The ranks of a node run side by side on their own GPUs, so the implied whole-node rate
is all loci / the slowest rank's wall time (host cores, disk and PCIe shared by 8 ranks are not
modelled; the note says so).  One JSON line per rank, then a summary line.

    python tools/e2e_shard.py [--world 8] [--ranks 0,3,7] [--workload cfg4_1m_delins_30x_hifi] [-t 16]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def shard_regions(loci, prm) -> list[tuple[int, int, int]]:
    """(tid, beg, end) per contig of the slice: every window [s - 1, e - 1) of its loci inside."""
    import numpy as np
    w = max(prm.wider_interval, prm.median_interval, prm.narrow_interval)
    out = []
    for c in np.unique(loci["chrom"]):
        m = loci[loci["chrom"] == c]
        hi = max(int(m["pos"].max()), int(m["end"].max()))
        out.append((int(c) - 1, max(0, int(m["pos"].min()) - w - 1), hi + w + 1))
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg4_1m_delins_30x_hifi")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", default="0,3,7")
    ap.add_argument("-t", type=int, default=16)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()

    from svtrek_amd import Params, sim
    from svtrek_amd.distributed import shard_rows

    stop = threading.Event()

    def ticker():   # a line a while: long BAM writes are not mistaken for a hang
        t0 = time.time()
        while not stop.wait(20):
            print(f"[e2e_shard] ... {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=ticker, daemon=True).start()

    t = time.perf_counter()
    r = sim.generate(sim.WORKLOADS[a.workload], keep_handle=True)
    gen_s = time.perf_counter() - t
    prm = Params()
    cli = os.path.join(ROOT, "svtrek_amd", "svtrek")
    rows_all = []
    for rank in (int(x) for x in a.ranks.split(",")):
        d = tempfile.mkdtemp(prefix=f"svt_shard{rank}_", dir=a.dir)
        try:
            rows = shard_rows(r.loci, a.world, rank)
            loci = r.loci[rows]
            regions = shard_regions(loci, prm)
            bam, vcf = os.path.join(d, "s.bam"), os.path.join(d, "s.vcf")
            t = time.perf_counter()
            sim.write_bam_regions(r, bam, regions, with_seq=True, level=1)
            sim.write_vcf(loci, vcf)
            write_s = time.perf_counter() - t
            times, stages, lines = [], None, None
            for _ in range(a.reps):
                t = time.perf_counter()
                p = subprocess.run([cli, "audt", "-b", bam, "-v", vcf, "-t", str(a.t), "--verbose", "--inflate", "gpu"],
                                   stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=900)
                times.append(time.perf_counter() - t)
                if p.returncode != 0:
                    print(p.stderr.decode(errors="replace")[-2000:], file=sys.stderr)
                    return p.returncode
                lines = p.stdout.count(b"\n") - 2
                st = [ln for ln in p.stderr.decode(errors="replace").splitlines() if ln.startswith("[svtrek_amd]")]
                stages = st[-1] if st else None
            # the CLI prints INS rows and DEL / INV rows longer than 50 bp (audit.c's print, as
            # vcf_audit.cpp's svth_format)
            import numpy as np
            from svtrek_amd import SVT_DEL, SVT_INS, SVT_INV
            span = (loci["end"].astype(np.uint32) - loci["pos"].astype(np.uint32)).astype(np.uint32)
            want = int(((loci["type"] == SVT_INS) | (np.isin(loci["type"], (SVT_DEL, SVT_INV)) & (span > 50))).sum())
            if lines != want:
                print(f"rank {rank}: printed {lines} records, expected {want} of {len(loci)} loci", file=sys.stderr)
                return 1
            best = min(times)
            row = {"metric": "end-to-end svtrek audt on one rank's slice", "workload": a.workload, "world": a.world,
                   "rank": rank, "loci": int(len(loci)), "printed_records": int(lines), "regions": regions, "bam_bytes": os.path.getsize(bam),
                   "with_seq": True, "host_threads": a.t, "seconds_best": round(best, 3),
                   "seconds_all": [round(x, 3) for x in times], "loci_per_s": round(len(loci) / best, 1),
                   "write_seconds": round(write_s, 1), "stages_last_run": stages}
            rows_all.append(row)
            print(json.dumps(row), flush=True)
        finally:
            shutil.rmtree(d, ignore_errors=True)
    stop.set()
    slow = max(rows_all, key=lambda x: x["seconds_best"])
    print(json.dumps({
        "metric": "implied whole-node end-to-end loci/s (8 ranks side by side)", "workload": a.workload,
        "loci_total": int(len(r.loci)), "ranks_measured": [x["rank"] for x in rows_all],
        "slowest_rank": slow["rank"], "slowest_seconds": slow["seconds_best"],
        "value": round(len(r.loci) / slow["seconds_best"], 1), "north_star": ">= 100000 loci/s on 8 x MI355X",
        "generate_seconds": round(gen_s, 1),
        "note": "each rank measured alone on one GPU with the box's host cores; 8 ranks on one node share "
                "host cores, page cache and disk bandwidth, which this does not model"}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
