"""End-to-end `svtrek audt` timing (reported separately from bench.py's kernel metric).

Writes the workload's BAM (+ plain VCF) once, then times the drop-in CLI
(`svtrek_amd/svtrek audt`): BGZF inflate + columnar pileup + H2D + batched refinement
+ printing.  Prints one JSON line.

    python tools/e2e_bench.py [--workload cfg2_10kdel_30x_ont] [--with-seq] [-t 16] [--reps 3]
    python tools/e2e_bench.py --workload cfg4_1m_delins_30x_hifi --region-sample 1000   # cpu_baseline's bytes
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
    ap.add_argument("--inflate", default="gpu,gpuhost,cpu",
                    help="ingest modes to time, comma-separated: gpu (BGZF inflate + record decode on the device, "
                         "svt_bam_dec_*), gpuhost (device inflate, host record parse: SVTREK_HOSTPARSE=1), cpu (host "
                         "threads); gpu:MB / gpuhost:MB set the batch (SVTREK_INFLATE_BATCH_MB)")
    ap.add_argument("--region-sample", type=int, default=0, metavar="K",
                    help="the CPU baseline's sample instead of the whole workload: the first K loci of contig 1 "
                         "(genomic order) and the BAM of their region, with SEQ/QUAL -- the same bytes bench.py's "
                         "cpu_baseline BGZF leg times (oracle/bgzf_baseline.py)")
    ap.add_argument("--libs", default="tree",
                    help="engine builds to time on the same files, comma-separated: 'tree' the in-tree libsvtrek_hip.so, "
                         "else a directory holding a variant libsvtrek_hip.so (LD_LIBRARY_PATH); reps alternate between them")
    a = ap.parse_args()

    import numpy as np

    from svtrek_amd import Params, sim
    d = a.dir or tempfile.mkdtemp(prefix="svt_e2e_")
    bam, vcf = os.path.join(d, "w.bam"), os.path.join(d, "w.vcf")
    t = time.perf_counter()
    r = sim.generate(sim.WORKLOADS[a.workload], keep_handle=True)
    loci, region = r.loci, None
    if a.region_sample:   # the cpu_baseline sample: same loci, same region, same writer settings
        prm = Params()
        c1 = r.loci[r.loci["chrom"] == 1]
        loci = c1[np.argsort(c1["pos"], kind="stable")][:a.region_sample]
        w = max(prm.wider_interval, prm.median_interval, prm.narrow_interval)
        region = (0, max(0, int(loci["pos"].min()) - w - 1), int(max(int(loci["pos"].max()), int(loci["end"].max()))) + w + 1)
    st = os.statvfs(d)
    free_gb = st.f_bavail * st.f_frsize / 1e9
    sim.write_bam(r, bam, with_seq=a.with_seq or bool(a.region_sample), level=a.level, region=region)
    sim.write_vcf(loci, vcf)
    prep = time.perf_counter() - t
    cli = os.path.join(ROOT, "svtrek_amd", "svtrek")
    outs = {}
    libs = a.libs.split(",")
    for mode in a.inflate.split(","):
        times = {lb: [] for lb in libs}
        stages = {}
        for _ in range(a.reps):
            for lb in libs:
                env = dict(os.environ)
                if lb != "tree":
                    env["LD_LIBRARY_PATH"] = os.path.abspath(lb)
                if ":" in mode:
                    env["SVTREK_INFLATE_BATCH_MB"] = mode.split(":")[1]
                base = mode.split(":")[0]
                if base == "gpuhost":
                    env["SVTREK_HOSTPARSE"] = "1"
                t = time.perf_counter()
                p = subprocess.run([cli, "audt", "-b", bam, "-v", vcf, "-t", str(a.t), "--verbose", "--inflate",
                                    "gpu" if base == "gpuhost" else base], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                   timeout=1800, env=env)
                times[lb].append(time.perf_counter() - t)
                if p.returncode != 0:
                    print(p.stderr.decode()[-2000:], file=sys.stderr)
                    return p.returncode
                outs[(mode, lb)] = p.stdout
                st = [l for l in p.stderr.decode(errors="replace").splitlines() if l.startswith("[svtrek_amd]")]
                stages[lb] = st[-1] if st else None
        for lb in libs:
            lines = outs[(mode, lb)].count(b"\n") - 2
            best = min(times[lb])
            print(json.dumps({
                "metric": "end-to-end svtrek audt (BAM ingest + H2D + refine + print)", "workload": a.workload,
                "inflate": mode, "engine": "in-tree" if lb == "tree" else lb, "loci": int(len(loci)),
                "printed_records": int(lines), "bam_bytes": os.path.getsize(bam),
                "with_seq": a.with_seq or bool(a.region_sample), "host_threads": a.t, "seconds_best": round(best, 3),
                "seconds_all": [round(x, 3) for x in times[lb]], "loci_per_s": round(len(loci) / best, 1),
                "region_sample": {"loci": a.region_sample, "region": region} if a.region_sample else None,
                "disk_free_gb_before": round(free_gb, 1),
                "prep_seconds": round(prep, 1), "stages_last_run": stages[lb]}), flush=True)
    if len(outs) > 1 and len(set(outs.values())) != 1:
        print("stdout differs between inflate modes / engine builds", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
