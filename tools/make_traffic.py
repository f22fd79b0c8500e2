"""Turn a tools/gpu_profile.sh run into the committed profile + profiles/traffic.json.

    python tools/make_traffic.py gpurun_out/prof_TAG profiles/TAG [--workload W]

Copies the kernel stats / PMC CSVs and bench logs into profiles/TAG and writes
profiles/traffic.json entries for every kernel of bench.py's step and for the step itself
(their sum): HBM bytes per launch =
read bytes from the L2 fabric read requests by size class (TCC_EA0_RDREQ_{32B,64B,128B}:
32/64/128 B each; cross-checked against 2 x FETCH_SIZE, which gfx950 tallies at 64 B per
128-B request, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, median over the profiled
launches.  bench.py reports the step entry as roofline.traffic when engine version and
workload match.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
import statistics


def counter_values(path: str, kernel: str, name: str) -> list[float]:
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return [float(r["Counter_Value"]) for r in csv.DictReader(f)
                if kernel in r["Kernel_Name"] and r["Counter_Name"] == name]


def med(v: list[float]) -> float | None:
    return statistics.median(v) if v else None


STEP = {   # the kernels of one bench.py step (label -> substring of rocprofv3's kernel name); the
           # index build is either the lane-per-read pair (short reads) or the stream walk (long reads)
    "ix2_census_kernel": "ix2_census_kernel",
    "ix2_emit_kernel": "ix2_emit_kernel",
    "ix_scan_blocks_kernel": "ix_scan_blocks_kernel",
    "index_kernel": "(anonymous namespace)::index_kernel(",
    "ix_copy_kernel": "ix_copy_kernel",
    "ixb_lane_kernel": "ixb_lane_kernel<false>",   # value buckets: the short-read filing pass
    "ixb_copy_kernel": "ixb_copy_kernel",          # ... the long reads' stage filed
    "refine_lane_kernel": "refine_lane_kernel",
    "refine_span_kernel": "refine_span_kernel",   # (the engine's pick below 64K windows: cfg1, cfg2)
    "refine_redo_kernel": "refine_redo_kernel",
}


def kernel_avg_ns(src: str, kernel: str) -> float | None:
    """Average duration of the kernel in the run's rocprofv3 --stats summary: the one-step-in-flight
    trace (trace1/: no other step's kernels beside it) when the run has one, else trace/."""
    path = os.path.join(src, "trace1", "run_kernel_stats.csv")
    if not os.path.exists(path):
        path = os.path.join(src, "trace", "run_kernel_stats.csv")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Name"]:
                return float(r["AverageNs"])
    return None


def kernel_calls(src: str, kernel: str) -> int | None:
    """Launches of the kernel in the traced run (trace/run_kernel_stats.csv)."""
    path = os.path.join(src, "trace", "run_kernel_stats.csv")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Name"]:
                return int(r["Calls"])
    return None


def kernel_bytes(src: str, kernel: str) -> dict | None:
    j = lambda sub: os.path.join(src, sub, "run_counter_collection.csv")  # noqa: E731
    fetch = med(counter_values(j("pmc_fetch"), kernel, "FETCH_SIZE"))
    write = med(counter_values(j("pmc_write"), kernel, "WRITE_SIZE"))
    n32 = med(counter_values(j("pmc_rdreq"), kernel, "TCC_EA0_RDREQ_32B_sum"))
    n64 = med(counter_values(j("pmc_rdreq"), kernel, "TCC_EA0_RDREQ_64B_sum"))
    n128 = med(counter_values(j("pmc_rdreq"), kernel, "TCC_EA0_RDREQ_128B_sum"))
    dram32 = med(counter_values(j("pmc_dram"), kernel, "TCC_EA0_RDREQ_DRAM_32B_sum"))
    if n128 is None and fetch is None:
        return None
    if n128 is not None:
        rd = 32 * (n32 or 0) + 64 * (n64 or 0) + 128 * n128
        method_rd = "TCC_EA0_RDREQ_{32B,64B,128B}_sum x {32,64,128} B"
    else:
        rd = 2 * fetch * 1024
        method_rd = "2 x FETCH_SIZE"
    return {
        "read_bytes_per_launch": int(round(rd)),
        "write_bytes_per_launch": int(round((write or 0) * 1024)),
        "hbm_bytes_per_launch": int(round(rd + (write or 0) * 1024)),
        "fetch_size_kb_raw": fetch,
        "write_size_kb_raw": write,
        "rdreq": {"32B": n32, "64B": n64, "128B": n128},
        "dram_rdreq_32B_units": dram32,
        "method": f"rocprofv3 --pmc passes of tools/gpu_profile.sh, one counter group per pass; reads: {method_rd} "
                  "(2 x FETCH_SIZE agrees: gfx950 tallies a 128-B request at 64 B); writes: WRITE_SIZE; "
                  "median over the profiled launches",
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--workload", default="cfg4_1m_delins_30x_hifi")
    a = ap.parse_args()
    os.makedirs(a.dst, exist_ok=True)
    copies = {"trace/run_kernel_stats.csv": "kernel_stats.csv", "trace1/run_kernel_stats.csv": "kernel_stats_inflight1.csv",
              "trace1.log": "bench_under_rocprof_inflight1.log", "pmc_fetch/run_counter_collection.csv":
              "pmc_fetch_size.csv", "pmc_write/run_counter_collection.csv": "pmc_write_size.csv",
              "pmc_rdreq/run_counter_collection.csv": "pmc_rdreq.csv",
              "pmc_dram/run_counter_collection.csv": "pmc_dram.csv", "pmc_sq/run_counter_collection.csv": "pmc_sq.csv",
              "trace.log": "bench_under_rocprof.log"}
    for s_, d in copies.items():
        sp = os.path.join(a.src, s_)
        if not os.path.exists(sp):
            continue
        if s_.startswith("pmc_"):   # the engine's kernels only (the run's torch / runtime copies dropped)
            with open(sp) as f, open(os.path.join(a.dst, d), "w", newline="") as g:
                rd = csv.reader(f)
                wr = csv.writer(g)
                hdr = next(rd)
                wr.writerow(hdr)
                kn = hdr.index("Kernel_Name")
                wr.writerows(r for r in rd if "anonymous namespace" in r[kn])
        else:
            shutil.copy(sp, os.path.join(a.dst, d))
    ver = None
    with open(os.path.join(a.src, "trace.log")) as f:
        for line in f:
            if line.startswith("{"):
                ver = json.loads(line).get("engine_version", ver)
    new = []
    step = {"read_bytes_per_launch": 0, "write_bytes_per_launch": 0, "hbm_bytes_per_launch": 0}
    calls = {label: kernel_calls(a.src, sub) for label, sub in STEP.items()}
    per_step = max([calls.get("refine_lane_kernel") or 0, calls.get("refine_span_kernel") or 0])
    for label, sub in STEP.items():
        kb = kernel_bytes(a.src, sub)
        if kb is None:
            continue
        if per_step and (calls.get(label) or 0) * 2 < per_step:
            continue   # a load-time kernel (e.g. the span lists built once beside the value buckets)
        ns = kernel_avg_ns(a.src, sub)
        e = {"kernel": label, "records": True, "workload": a.workload, "engine_version": ver, **kb,
             "avg_ns": ns, "source": f"{a.dst}/pmc_*.csv, {a.dst}/kernel_stats.csv"}
        new.append(e)
        for k in step:
            step[k] += kb[k]
    if new:
        new.append({"kernel": "step", "records": True, "workload": a.workload, "engine_version": ver, **step,
                    "kernels": [e["kernel"] for e in new],
                    "method": "sum over the step's kernels of each kernel's median bytes per launch (one launch "
                              "of each per bench.py step)", "source": f"{a.dst}/pmc_*.csv"})
    # profiles/traffic.json: one entry per (engine version, workload, kernel, records)
    # profiles/traffic.json: the profiles/ directory above dst (dst may be nested: profiles/TAG/cfg)
    d = os.path.abspath(a.dst)
    while os.path.basename(d) != "profiles" and os.path.dirname(d) != d:
        d = os.path.dirname(d)
    tpath = os.path.join(d if os.path.basename(d) == "profiles" else os.path.dirname(os.path.abspath(a.dst)), "traffic.json")
    try:
        with open(tpath) as f:
            old = json.load(f)
        old = old if isinstance(old, list) else [old]
    except (OSError, ValueError):
        old = []
    key = lambda e: (e.get("engine_version"), e.get("workload"), e.get("kernel"), bool(e.get("records")))  # noqa
    keys = {key(e) for e in new}
    entries = [e for e in old if key(e) not in keys] + new
    with open(tpath, "w") as f:
        json.dump(entries, f, indent=1)
    for e in new:
        print(json.dumps({k: e[k] for k in ("kernel", "read_bytes_per_launch", "write_bytes_per_launch",
                                            "hbm_bytes_per_launch")}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
