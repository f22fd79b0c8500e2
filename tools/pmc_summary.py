"""Median per-launch PMC values of one kernel from rocprofv3 --pmc CSV directories.

    python tools/pmc_summary.py KERNEL DIR [DIR ...]
"""
import collections
import csv
import glob
import statistics
import sys


def summary(kernel: str, d: str) -> dict:
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel in r["Kernel_Name"]:
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


if __name__ == "__main__":
    k = sys.argv[1]
    rows = [(d, summary(k, d)) for d in sys.argv[2:]]
    names = sorted({n for _, s in rows for n in s})
    print("dir".ljust(36) + "".join(n[:18].rjust(20) for n in names))
    for d, s in rows:
        print(d[-36:].ljust(36) + "".join(f"{s.get(n, float('nan')):20.4g}" for n in names))
