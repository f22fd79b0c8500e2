"""Host read bandwidth of the ingest's batch reads, all ranks of a node at once (no GPU).

    python tools/pread_bench.py --files 8 --gib 2 [--dir DIR] [--batch-mib 256] [--keep]

The CLI's device ingest (`svtrek audt`, svth_bam_read_device) reads its BAM in 256 MiB batches
with pread into host buffers; an 8-GPU node runs 8 such readers at once, one per rank slice.
This writes --files files of --gib GiB each (random bytes, like compressed BGZF), then reads
them all concurrently, one thread per file, in --batch-mib batches:
  * buffered: pread through the page cache (the files were just written, so this is the
    warm-cache rate the round-5 end-to-end runs saw);
  * direct: O_DIRECT preads into aligned buffers (the page cache bypassed: the storage's own
    rate, what a cold BAM on this host reads at).
Prints one JSON line: aggregate GB/s per mode and the implied time for 8 rank slices of
--slice-gb GB each (cfg4's rank slice with SEQ/QUAL: 15 GB).  Not root: nothing is dropped
from the page cache; the direct mode is the cold figure.
"""
from __future__ import annotations

import argparse
import json
import mmap
import os
import tempfile
import threading
import time


def write_files(d: str, n: int, size: int, chunk: int) -> list[str]:
    paths = []
    buf = os.urandom(chunk)
    for i in range(n):
        p = os.path.join(d, f"slice{i}.bin")
        with open(p, "wb") as f:
            left = size
            while left > 0:
                k = min(left, chunk)
                f.write(buf[:k])
                left -= k
            f.flush()
            os.fsync(f.fileno())
        paths.append(p)
    return paths


def read_all(paths: list[str], batch: int, direct: bool) -> tuple[float, int]:
    total = [0] * len(paths)
    errs: list[str] = []

    def reader(i: int, p: str) -> None:
        flags = os.O_RDONLY | (os.O_DIRECT if direct else 0)
        try:
            fd = os.open(p, flags)
        except OSError as e:
            errs.append(f"{p}: {e}")
            return
        buf = mmap.mmap(-1, batch)   # page-aligned: O_DIRECT's alignment
        off = 0
        try:
            while True:
                k = os.preadv(fd, [buf], off)
                if k <= 0:
                    break
                off += k
                total[i] += k
                if k < batch:
                    break
        except OSError as e:
            errs.append(f"{p}: {e}")
        finally:
            os.close(fd)
            buf.close()

    ts = [threading.Thread(target=reader, args=(i, p)) for i, p in enumerate(paths)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    if errs:
        raise OSError("; ".join(errs))
    return dt, sum(total)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--batch-mib", type=int, default=256)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--slice-gb", type=float, default=15.0)
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args()
    d = a.dir or tempfile.mkdtemp(prefix="pread_bench_", dir=os.environ.get("TMPDIR", "/tmp"))
    os.makedirs(d, exist_ok=True)
    size = int(a.gib * (1 << 30))
    batch = a.batch_mib << 20
    t0 = time.perf_counter()
    paths = write_files(d, a.files, size, min(batch, 64 << 20))
    t_write = time.perf_counter() - t0
    out = {"files": a.files, "bytes_per_file": size, "batch_bytes": batch, "dir": d,
           "write_s": round(t_write, 3), "write_gbs": round(a.files * size / t_write / 1e9, 2)}
    try:
        for mode, direct in (("buffered", False), ("direct", True)):
            try:
                dt, n = read_all(paths, batch, direct)
                out[mode] = {"s": round(dt, 3), "bytes": n, "gbs": round(n / dt / 1e9, 2),
                             "node_8_slices_s": round(8 * a.slice_gb * 1e9 / (n / dt), 2)}
            except OSError as e:
                out[mode] = {"error": str(e)}
    finally:
        if not a.keep:
            for p in paths:
                os.unlink(p)
            if a.dir is None:
                os.rmdir(d)
    out["note"] = ("aggregate pread rate of all files read at once, one thread each; node_8_slices_s = the time "
                   f"8 rank slices of {a.slice_gb} GB take at that rate (the host-read bound of the node's ingest)")
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
