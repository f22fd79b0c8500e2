"""Shrink a tools/gpu_profile.sh output directory in place (on the GPU box, before gpurun copies
gpurun_out/ back under its size cap): drop the per-dispatch kernel traces and keep only the
engine's kernels in the PMC CSVs.   python tools/trim_prof.py gpurun_out/prof_TAG"""
import csv
import glob
import os
import sys

d = sys.argv[1]
for p in glob.glob(os.path.join(d, "trace*", "run_kernel_trace.csv")):
    os.unlink(p)
for p in glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv")):
    with open(p) as f:
        rows = list(csv.reader(f))
    kn = rows[0].index("Kernel_Name")
    with open(p, "w", newline="") as f:
        csv.writer(f).writerows([rows[0]] + [r for r in rows[1:] if "anonymous namespace" in r[kn]])
