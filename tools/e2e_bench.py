"""End-to-end `svtrek audt` timing (reported separately from bench.py's kernel metric).

Writes the workload's BAM (+ plain VCF) once, then times the drop-in CLI
(`svtrek_amd/svtrek audt`): BGZF inflate + columnar pileup + H2D + batched refinement
+ printing.  Prints one JSON line.

    python tools/e2e_bench.py [--workload cfg2_10kdel_30x_ont] [--with-seq] [-t 16] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2_10kdel_30x_ont")
    ap.add_argument("--with-seq", action="store_true", help="store random SEQ/QUAL (realistic BAM size)")
    ap.add_argument("-t", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--level", type=int, default=1, help="BGZF deflate level for the written BAM")
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()

    from svtrek_amd import sim
    d = a.dir or tempfile.mkdtemp(prefix="svt_e2e_")
    bam, vcf = os.path.join(d, "w.bam"), os.path.join(d, "w.vcf")
    t = time.perf_counter()
    r = sim.generate(sim.WORKLOADS[a.workload], keep_handle=True)
    sim.write_bam(r, bam, with_seq=a.with_seq, level=a.level)
    sim.write_vcf(r.loci, vcf)
    prep = time.perf_counter() - t
    cli = os.path.join(ROOT, "svtrek_amd", "svtrek")
    times = []
    for _ in range(a.reps):
        t = time.perf_counter()
        p = subprocess.run([cli, "audt", "-b", bam, "-v", vcf, "-t", str(a.t), "--verbose"], stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, timeout=1800)
        times.append(time.perf_counter() - t)
        if p.returncode != 0:
            print(p.stderr.decode()[-2000:], file=sys.stderr)
            return p.returncode
    lines = p.stdout.count(b"\n") - 2
    stages = [l for l in p.stderr.decode(errors="replace").splitlines() if l.startswith("[svtrek_amd]")]
    best = min(times)
    print(json.dumps({
        "metric": "end-to-end svtrek audt (BAM ingest + H2D + refine + print)", "workload": a.workload,
        "loci": int(len(r.loci)), "printed_records": int(lines), "bam_bytes": os.path.getsize(bam),
        "with_seq": a.with_seq, "inflate_threads": a.t, "seconds_best": round(best, 3),
        "seconds_all": [round(x, 3) for x in times], "loci_per_s": round(len(r.loci) / best, 1),
        "prep_seconds": round(prep, 1), "stages_last_run": stages[-1] if stages else None}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
