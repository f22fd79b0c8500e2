"""ctypes bindings of libsvtrek_host.so: BAM ingest, VCF record parsing, result printing."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import LOCUS_DTYPE, PKG, SvtPileupView
from .pileup import Pileup

_host = None


def load_host() -> C.CDLL:
    global _host
    if _host is None:
        path = os.path.join(PKG, "libsvtrek_host.so")
        if not os.path.exists(path):
            raise RuntimeError(f"host library not built: {path}")
        L = C.CDLL(path)
        P = C.c_void_p
        L.svth_bam_read.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_size_t]
        L.svth_bam_read.restype = P
        L.svth_bam_read_region.argtypes = [C.c_char_p, C.c_int, C.c_int32, C.c_int64, C.c_int32, C.c_int64,
                                           C.c_char_p, C.c_size_t]
        L.svth_bam_read_region.restype = P
        L.svth_bam_read_ex.argtypes = [C.c_char_p, C.c_int, C.c_int32, C.c_int64, C.c_int32, C.c_int64, P,
                                       C.c_char_p, C.c_size_t]
        L.svth_bam_read_ex.restype = P
        L.svth_bam_read_device.argtypes = [C.c_char_p, C.c_int, P, P, P, C.c_char_p, C.c_size_t]
        L.svth_bam_read_device.restype = C.c_int
        L.svth_vcf_parse.argtypes = [C.c_char_p, C.c_size_t, C.c_int]
        L.svth_vcf_parse.restype = P
        L.svth_vcf_count.argtypes = [P]
        L.svth_vcf_count.restype = C.c_size_t
        L.svth_vcf_loci.argtypes = [P]
        L.svth_vcf_loci.restype = P
        L.svth_vcf_messages.argtypes = [P, C.POINTER(C.c_size_t)]
        L.svth_vcf_messages.restype = P
        L.svth_vcf_free.argtypes = [P]
        L.svth_vcf_free.restype = None
        L.svth_format_batch.argtypes = [P, P, C.c_size_t, C.c_int, C.POINTER(C.c_size_t)]
        L.svth_format_batch.restype = P
        L.svth_free.argtypes = [P]
        L.svth_free.restype = None
        L.svth_bam_free.argtypes = [P]
        L.svth_bam_free.restype = None
        L.svth_bam_view.argtypes = [P, C.POINTER(SvtPileupView)]
        L.svth_bam_view.restype = None
        L.svth_bam_n_targets.argtypes = [P]
        L.svth_bam_n_targets.restype = C.c_int32
        L.svth_bam_target_name.argtypes = [P, C.c_int32]
        L.svth_bam_target_name.restype = C.c_char_p
        L.svth_bam_n_records.argtypes = [P]
        L.svth_bam_n_records.restype = C.c_int64
        L.svth_bam_n_cg_restored.argtypes = [P]
        L.svth_bam_n_cg_restored.restype = C.c_int64
        L.svth_bam_stage_seconds.argtypes = [P, P]
        L.svth_bam_stage_seconds.restype = None
        L.svth_parse_line.argtypes = [C.c_char_p, P, C.c_char_p, C.c_size_t]
        L.svth_parse_line.restype = C.c_int
        L.svth_format.argtypes = [P, P, C.c_char_p, C.c_size_t]
        L.svth_format.restype = C.c_int
        L.svth_is_unknown_type.argtypes = [P]
        L.svth_is_unknown_type.restype = C.c_int
        _host = L
    return _host


INFLATE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                         C.c_void_p, C.c_size_t)
ALLOC_FN = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.c_size_t)
RELEASE_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p)


class SvthInflater(C.Structure):
    _fields_ = [("inflate", C.c_void_p), ("alloc", C.c_void_p), ("release", C.c_void_p), ("user", C.c_void_p),
                ("batch_bytes", C.c_size_t)]


BEGIN_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int32, C.c_void_p, C.c_size_t)
FEED_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_uint64, C.c_void_p,
                      C.c_size_t)


class SvthDevSink(C.Structure):
    _fields_ = [("begin", C.c_void_p), ("feed", C.c_void_p), ("alloc", C.c_void_p), ("release", C.c_void_p),
                ("user", C.c_void_p), ("batch_bytes", C.c_size_t)]


def load_bam_device(engine, path: str, threads: int = 4, batch_bytes: int = 0, pinned: bool = True) -> dict:
    """The BAM decoded on the engine's device (svth_bam_read_device feeding svt_bam_dec_*: BGZF
    inflate + record decode there) and loaded as the engine's pileup; returns the decoder's
    stats and the reader's stage times.  The same as engine.load_pileup(read_bam(path)[0])."""
    from ._lib import SvtBamDecStats
    L = load_host()
    lib, ctx = engine.lib, engine._h
    dec = C.c_void_p()
    err = C.create_string_buffer(512)

    def put(e, ecap, m: bytes) -> None:
        m = m[:max(int(ecap) - 1, 0)]
        C.memmove(e, m + b"\0", len(m) + 1)

    def begin(_u, nt, e, ecap):
        rc = lib.svt_bam_dec_open(ctx, nt, C.byref(dec))
        if rc:
            put(e, ecap, lib.svt_last_error(ctx))
        return 1 if rc else 0

    def feed(_u, comp, cb, blocks, n, skip, e, ecap):
        rc = lib.svt_bam_dec_feed(dec, comp, cb, blocks, n, skip)
        if rc:
            put(e, ecap, lib.svt_last_error(ctx))
        return 1 if rc else 0
    fb, ff = BEGIN_FN(begin), FEED_FN(feed)
    fa = ALLOC_FN(lambda _u, n: lib.svt_host_alloc(ctx, n))
    fr = RELEASE_FN(lambda _u, p: lib.svt_host_free(ctx, p))
    sink = SvthDevSink(C.cast(fb, C.c_void_p), C.cast(ff, C.c_void_p), C.cast(fa, C.c_void_p) if pinned else None,
                       C.cast(fr, C.c_void_p) if pinned else None, None, batch_bytes)
    st4 = (C.c_double * 4)()
    try:
        if L.svth_bam_read_device(path.encode(), threads, C.byref(sink), None, st4, err, 512) != 0:
            raise OSError(err.value.decode())
        engine._check(lib.svt_bam_dec_load(dec))
        st = SvtBamDecStats()
        engine._check(lib.svt_bam_dec_stats_get(dec, C.byref(st)))
    finally:
        lib.svt_bam_dec_close(dec)
    out = {k: getattr(st, k) for k, _ in SvtBamDecStats._fields_}
    out["stage_s"] = dict(zip(("read", "feed", "wait", "total"), (round(x, 4) for x in st4)))
    return out


def read_bam(path: str, threads: int = 4, region: tuple[int, int, int, int] | None = None,
             inflate=None, batch_bytes: int = 0, pinned: bool = True) -> tuple[Pileup, dict]:
    """The BAM as a columnar pileup.  region = (tid0, beg0, tid1, end1): only the records from
    the BAI's linear-index offset of (tid0, beg0) up to the first at or past (tid1, end1)
    (svth_bam_read_region; needs `path`.bai) -- what one shard's queries can yield.
    inflate = an Engine: the BGZF blocks are inflated by its svt_bgzf_inflate (the device, in
    ~1 GiB batches overlapped with the record parse) instead of host threads."""
    L = load_host()
    err = C.create_string_buffer(512)
    t0, b0, t1, e1 = (int(x) for x in region) if region is not None else (-1, 0, -1, 0)
    if inflate is None:
        h = L.svth_bam_read_region(path.encode(), threads, t0, b0, t1, e1, err, 512)
    else:
        lib, ctx = inflate.lib, inflate._h

        def cb(_user, comp, cbytes, blocks, n, out, obytes, e, ecap):
            rc = lib.svt_bgzf_inflate(ctx, comp, cbytes, blocks, n, out, obytes)
            if rc:
                m = lib.svt_last_error(ctx)[:max(int(ecap) - 1, 0)]
                C.memmove(e, m + b"\0", len(m) + 1)
            return rc
        fn = INFLATE_FN(cb)
        fa = ALLOC_FN(lambda _u, n: lib.svt_host_alloc(ctx, n))
        fr = RELEASE_FN(lambda _u, p: lib.svt_host_free(ctx, p))
        inf = SvthInflater(C.cast(fn, C.c_void_p), C.cast(fa, C.c_void_p) if pinned else None,
                           C.cast(fr, C.c_void_p) if pinned else None, None, batch_bytes)
        h = L.svth_bam_read_ex(path.encode(), threads, t0, b0, t1, e1, C.byref(inf), err, 512)
    if not h:
        raise OSError(err.value.decode())
    try:
        v = SvtPileupView()
        L.svth_bam_view(h, C.byref(v))
        nt = v.n_targets

        def arr(p, dtype, n):
            if n == 0 or not p:
                return np.zeros(0, dtype=dtype)
            return np.frombuffer((C.c_char * (n * np.dtype(dtype).itemsize)).from_address(p), dtype=dtype).copy()

        tid_off = arr(v.tid_off, np.int64, nt + 1)
        if nt == 0:
            tid_off = np.zeros(1, dtype=np.int64)
        nr = int(tid_off[-1])
        cig_off = arr(v.cig_off, np.uint64, nr + 1)
        if len(cig_off) == 0:
            cig_off = np.zeros(1, dtype=np.uint64)
        pl = Pileup(tid_off=tid_off, pos=arr(v.pos, np.int32, nr), endpos=arr(v.endpos, np.int32, nr),
                    cig_off=cig_off, cigar=arr(v.cigar, np.uint32, int(cig_off[-1])),
                    clip=arr(v.clip, np.uint8, nr))
        st = (C.c_double * 6)()
        L.svth_bam_stage_seconds(h, st)
        info = {"names": [L.svth_bam_target_name(h, t).decode() for t in range(nt)],
                "records": int(L.svth_bam_n_records(h)), "cg_restored": int(L.svth_bam_n_cg_restored(h)),
                "stage_s": dict(zip(("read", "scan", "alloc", "inflate", "wait", "total"), (round(x, 4) for x in st)))}
        return pl, info
    finally:
        L.svth_bam_free(h)


def parse_line(line: str):
    """-> (action, (type, chrom, pos, end) | None, stderr_text)"""
    L = load_host()
    buf = C.create_string_buffer(line.encode("latin-1"))
    loc = np.zeros(1, dtype=LOCUS_DTYPE)
    err = C.create_string_buffer(1024)
    act = L.svth_parse_line(buf, loc.ctypes.data, err, 1024)
    rec = tuple(int(x) for x in loc[0]) if act == 1 else None
    return act, rec, err.value.decode("latin-1")


def parse_vcf_text(data: bytes, threads: int = 4) -> tuple[np.ndarray, str]:
    """A1 over a whole VCF (svth_vcf_parse, multithreaded): (loci in file order, the stderr
    text the reference's workers print for skipped / unknown records, in file order)."""
    L = load_host()
    h = L.svth_vcf_parse(data, len(data), threads)
    if not h:
        raise MemoryError("svth_vcf_parse failed")
    try:
        n = int(L.svth_vcf_count(h))
        loci = np.zeros(n, dtype=LOCUS_DTYPE)
        if n:
            C.memmove(loci.ctypes.data, L.svth_vcf_loci(h), n * LOCUS_DTYPE.itemsize)
        ml = C.c_size_t(0)
        mp = L.svth_vcf_messages(h, C.byref(ml))
        msgs = C.string_at(mp, ml.value).decode("latin-1") if ml.value else ""
        return loci, msgs
    finally:
        L.svth_vcf_free(h)


def format_batch(loci: np.ndarray, res: np.ndarray, threads: int = 4) -> str:
    """A11 of every record, in order (svth_format_batch, multithreaded)."""
    L = load_host()
    loci = np.ascontiguousarray(loci)
    res = np.ascontiguousarray(res)
    n = C.c_size_t(0)
    p = L.svth_format_batch(loci.ctypes.data, res.ctypes.data, len(loci), threads, C.byref(n))
    if not p:
        raise MemoryError("svth_format_batch failed")
    try:
        return C.string_at(p, n.value).decode("latin-1")
    finally:
        L.svth_free(p)


def format_result(locus: np.void, result: np.void) -> str:
    from ._lib import RESULT_DTYPE
    L = load_host()
    lo = np.array([locus], dtype=LOCUS_DTYPE)
    r = np.array([result], dtype=RESULT_DTYPE)
    buf = C.create_string_buffer(512)
    n = L.svth_format(lo.ctypes.data, r.ctypes.data, buf, 512)
    return buf.raw[:n].decode("latin-1")


def format_sw_lines(queries: np.ndarray, off: np.ndarray, sub: np.ndarray, window_size: int) -> str:
    """The stdout lines sliding_window_ins prints (sliding_window.c:86-87) for the
    sub-windows of `queries`, in order: one per sub-window whose bestCandidate != -1."""
    out = []
    for i, q in enumerate(queries):
        s0, e0 = int(q["start"]), int(q["end"])
        for k in range(int(off[i]), int(off[i + 1])):
            ss = (s0 + (k - int(off[i])) * window_size) & 0xFFFFFFFF
            se = min(ss + window_size, e0)
            c, sp = int(sub[k]["candidate"]), int(sub[k]["support"])
            if c != -1:
                i32 = lambda x: x - (1 << 32) if x >= (1 << 31) else x   # noqa: E731  (%d of uint32)
                out.append(f"INS Discovery in window [{i32(ss)}, {i32(se)}] at position {c} with support {sp}\n")
    return "".join(out)
