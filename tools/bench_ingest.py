"""BAM ingest timing with SEQ/QUAL: host-thread inflate vs the device inflater at several batch
sizes, pinned or pageable buffers (host.read_bam -> svth_bam_read[_ex]), stage split of the
device path.  One JSON line per configuration.

    python tools/bench_ingest.py [--workload cfg2_10kdel_30x_ont] [--scale 0.2] [-t 16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2_10kdel_30x_ont")
    ap.add_argument("--scale", type=float, default=0.2)
    ap.add_argument("-t", type=int, default=16)
    ap.add_argument("--batches", default="256,1024,4096", help="device batch sizes, MiB")
    a = ap.parse_args()
    from dataclasses import replace

    from svtrek_amd import Engine, Params, host, sim
    cfg = sim.WORKLOADS[a.workload]
    cfg = replace(cfg, n_loci=max(1, int(cfg.n_loci * a.scale)))
    d = tempfile.mkdtemp(prefix="svt_ing_")
    path = os.path.join(d, "w.bam")
    r = sim.generate(cfg, keep_handle=True)
    sim.write_bam(r, path, with_seq=True, level=1)
    del r
    size = os.path.getsize(path)
    runs = [("host", 0, True)] + [(f"device_{m}M", m << 20, True) for m in map(int, a.batches.split(","))] + \
           [(f"device_{int(a.batches.split(',')[1])}M_pageable", int(a.batches.split(",")[1]) << 20, False)]
    ref = None
    with Engine(Params(), device=0) as eng:
        for name, batch, pinned in runs:
            t = time.perf_counter()
            pl, info = host.read_bam(path, threads=a.t, inflate=None if name == "host" else eng, batch_bytes=batch,
                                     pinned=pinned)
            dt = time.perf_counter() - t
            same = None
            if ref is None:
                ref = pl
            else:
                same = all((getattr(ref, k) == getattr(pl, k)).all() for k in ("pos", "endpos", "cig_off", "cigar"))
            print(json.dumps({"metric": "BAM ingest (s)", "config": name, "bam_bytes": size, "records": info["records"],
                              "seconds": round(dt, 3), "stage_s": info["stage_s"], "same_as_host": same}), flush=True)
            del pl
    return 0


if __name__ == "__main__":
    sys.exit(main())
