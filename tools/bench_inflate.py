"""BGZF inflate throughput: the device kernel (svt_bgzf_inflate, one wave per block) vs the
host (zlib on T threads, the same per-block inflate the host ingest runs), on a BAM with
SEQ/QUAL written by the simulator.  Prints one JSON line.

    python tools/bench_inflate.py [--workload cfg2_10kdel_30x_ont] [--scale 0.1] [-t 16] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2_10kdel_30x_ont")
    ap.add_argument("--scale", type=float, default=0.1)
    ap.add_argument("-t", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--phase", action="store_true", help="read a -DSVT_PHASE_PROF=1 build's counters")
    ap.add_argument("--level", type=int, default=1)
    a = ap.parse_args()
    from dataclasses import replace

    import numpy as np

    from svtrek_amd import Engine, Params, sim
    from svtrek_amd.bgzf import block_table
    cfg = sim.WORKLOADS[a.workload]
    cfg = replace(cfg, n_loci=max(1, int(cfg.n_loci * a.scale)))
    d = tempfile.mkdtemp(prefix="svt_inf_")
    path = os.path.join(d, "w.bam")
    t = time.perf_counter()
    r = sim.generate(cfg, keep_handle=True)
    sim.write_bam(r, path, with_seq=True, level=a.level)
    prep = time.perf_counter() - t
    comp = np.fromfile(path, dtype=np.uint8)
    blocks = block_table(comp)
    out_bytes = int(blocks["uoff"][-1]) + int(blocks["ulen"][-1])
    prof = None
    with Engine(Params(), device=0) as eng:
        eng.bgzf_inflate(comp, blocks, out_bytes)   # warm-up (buffers, code object)
        if a.phase:   # a -DSVT_PHASE_PROF=1 build (SVTREK_ENGINE_LIB): clear, then read after the reps
            import ctypes as C
            buf = (C.c_ulonglong * 16)()
            eng.lib.svt_diag_phase(buf)
        kms, api = [], []
        for _ in range(a.reps):
            t = time.perf_counter()
            out = eng.bgzf_inflate(comp, blocks, out_bytes)
            api.append(time.perf_counter() - t)
            kms.append(eng.last_inflate_ms())
        if a.phase:
            eng.lib.svt_diag_phase(buf)
            v = [int(x) / a.reps for x in buf]
            names = ["hdr_ticks", "codes_ticks", "deflate_blocks", "dynamic", "stored_bytes", "literals", "matches",
                     "match_bytes", "far_matches", "bgzf_blocks", "bgzf_ticks"]
            prof = dict(zip(names, v))
    # host: zlib per block on T threads (zlib releases the GIL)
    cb = comp.tobytes()

    def part(lo_hi):
        lo, hi = lo_hi
        return b"".join(zlib.decompress(cb[int(b["coff"]):int(b["coff"]) + int(b["clen"])], -15) for b in blocks[lo:hi])
    T = a.t
    cuts = [(len(blocks) * i // T, len(blocks) * (i + 1) // T) for i in range(T)]
    t = time.perf_counter()
    with ThreadPoolExecutor(T) as ex:
        host = b"".join(ex.map(part, cuts))
    host_s = time.perf_counter() - t
    ok = host == out.tobytes()
    k = min(kms)
    print(json.dumps({
        "metric": "BGZF inflate throughput (output GB/s)", "workload": a.workload, "scale": a.scale,
        "bam_bytes": int(comp.nbytes), "blocks": int(len(blocks)), "out_bytes": out_bytes, "level": a.level,
        "kernel_ms": round(k, 3), "kernel_gbs": round(out_bytes / (k * 1e-3) / 1e9, 2),
        "api_s": round(min(api), 4), "api_gbs": round(out_bytes / min(api) / 1e9, 2),
        "host_zlib_threads": T, "host_s": round(host_s, 3), "host_gbs": round(out_bytes / host_s / 1e9, 3),
        "identical_to_zlib": ok, "prep_s": round(prep, 1), **({"phase": prof} if prof else {})}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
