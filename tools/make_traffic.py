"""Turn a tools/gpu_profile.sh run into the committed profile + profiles/traffic.json.

    python tools/make_traffic.py gpurun_out/prof_TAG profiles/TAG [--workload cfg2_10kdel_30x_ont]

Copies the kernel stats / PMC CSVs and bench logs into profiles/TAG and writes
profiles/traffic.json for the dominant kernel (refine_kernel<false, true>): HBM bytes per
launch = 2 x FETCH_SIZE (gfx950 reports half the bytes of 16-B-per-lane streaming loads,
MI355X_MICROARCH.md HBM section) + WRITE_SIZE, median over the profiled launches.  bench.py
reports it as roofline.traffic when the engine version and workload match.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
import statistics

KERNEL = "refine_kernel<false, true>"


def counter_values(path: str, name: str) -> list[float]:
    with open(path) as f:
        return [float(r["Counter_Value"]) for r in csv.DictReader(f)
                if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == name]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--workload", default="cfg2_10kdel_30x_ont")
    a = ap.parse_args()
    os.makedirs(a.dst, exist_ok=True)
    copies = {"trace/run_kernel_stats.csv": "kernel_stats.csv", "pmc_fetch/run_counter_collection.csv":
              "pmc_fetch_size.csv", "pmc_write/run_counter_collection.csv": "pmc_write_size.csv",
              "trace.log": "bench_under_rocprof.log"}
    for s, d in copies.items():
        if os.path.exists(os.path.join(a.src, s)):
            shutil.copy(os.path.join(a.src, s), os.path.join(a.dst, d))
    fetch = counter_values(os.path.join(a.src, "pmc_fetch/run_counter_collection.csv"), "FETCH_SIZE")
    write = counter_values(os.path.join(a.src, "pmc_write/run_counter_collection.csv"), "WRITE_SIZE")
    ver = None
    with open(os.path.join(a.src, "trace.log")) as f:
        for line in f:
            if line.startswith("{"):
                d = json.loads(line)
                ver = d.get("engine_version", ver)
    if ver is None:   # bench logs before engine_version was printed: the in-tree build's
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from svtrek_amd import version
        ver = version()
    fk, wk = statistics.median(fetch), statistics.median(write)
    out = {
        "kernel": KERNEL,
        "workload": a.workload,
        "engine_version": ver,
        "launches": len(fetch),
        "fetch_size_kb_raw": fk,
        "write_size_kb_raw": wk,
        "hbm_bytes_per_launch": int(round(2 * fk * 1024 + wk * 1024)),
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (tools/gpu_profile.sh); "
                  "FETCH_SIZE x2 for 16-B-per-lane streaming loads on gfx950 (MI355X_MICROARCH.md, HBM section), "
                  "WRITE_SIZE as read; median over the profiled launches",
        "source": f"{a.dst}/pmc_fetch_size.csv, {a.dst}/pmc_write_size.csv",
    }
    with open(os.path.join(os.path.dirname(a.dst.rstrip("/")), "traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
