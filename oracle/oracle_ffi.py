"""TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/liboracle.so (the CPU parity oracle).

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


class OrcParams(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("wider_interval", "median_interval", "narrow_interval",
                                          "consensus_interval_range", "consensus_interval",
                                          "consensus_min_count")]


class OrcPileup(C.Structure):
    _fields_ = [("n_targets", C.c_int32), ("tid_off", C.c_void_p), ("pos", C.c_void_p),
                ("endpos", C.c_void_p), ("cig_off", C.c_void_p), ("cigar", C.c_void_p), ("clip", C.c_void_p)]


class OrcWork(C.Structure):
    _fields_ = [("windows", C.c_uint64), ("reads", C.c_uint64), ("ops_walked", C.c_uint64),
                ("candidates", C.c_uint64)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: {path}")
        L = C.CDLL(path)
        P = C.c_void_p
        L.orc_consensus_pos.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_consensus_pos.restype = C.c_int
        L.orc_lower_bound.argtypes = [P, C.c_int, C.c_int]
        L.orc_upper_bound.argtypes = [P, C.c_int, C.c_int]
        for fn in ("orc_refine_start", "orc_refine_end", "orc_refine_point"):
            getattr(L, fn).argtypes = [P, C.c_int, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, P, P]
            getattr(L, fn).restype = C.c_int
        L.orc_refine_ins.argtypes = [P, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, P, P]
        L.orc_refine_ins.restype = C.c_int
        L.orc_refine_batch.argtypes = [P, P, P, C.c_size_t, P, C.c_int, P]
        L.orc_refine_batch.restype = C.c_int
        L.orc_bgzf_refine_batch.argtypes = [C.c_char_p, P, P, C.c_size_t, P, C.c_int, P, C.c_char_p, C.c_size_t]
        L.orc_bgzf_refine_batch.restype = C.c_int
        L.orc_parse_line.argtypes = [C.c_char_p, P, C.c_char_p, C.c_size_t]
        L.orc_parse_line.restype = C.c_int
        L.orc_format_result.argtypes = [P, P, C.c_char_p, C.c_size_t]
        L.orc_format_result.restype = C.c_int
        L.orc_audit_text.argtypes = [C.c_char_p, C.c_size_t, P, P, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        L.orc_audit_text.restype = C.c_int
        L.orc_free.argtypes = [P]
        L.orc_sliding_window_ins.argtypes = [P, C.c_int, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_int, P, P]
        L.orc_sliding_window_ins.restype = C.c_int
        _lib = L
    return _lib


def params(p=None) -> OrcParams:
    if p is None:
        return OrcParams(20000, 10000, 2000, 500, 5, 3)
    return OrcParams(p.wider_interval, p.median_interval, p.narrow_interval, p.consensus_interval_range,
                     p.consensus_interval, p.consensus_min_count)


def pileup(pl) -> tuple[OrcPileup, list]:
    keep = [pl.tid_off, pl.pos, pl.endpos, pl.cig_off, pl.cigar, pl.clip]
    v = OrcPileup(pl.n_targets, pl.tid_off.ctypes.data, pl.pos.ctypes.data, pl.endpos.ctypes.data,
                  pl.cig_off.ctypes.data, pl.cigar.ctypes.data,
                  pl.clip.ctypes.data if pl.clip is not None else None)
    return v, keep


def consensus_pos(locs, pos: int, min_count: int = 3, ci: int = 5, rng: int = 500) -> int:
    a = np.ascontiguousarray(np.array(locs, dtype=np.int32))
    return lib().orc_consensus_pos(a.ctypes.data if len(a) else None, len(a), pos, min_count, ci, rng)


def refine_batch(pl, loci: np.ndarray, prm=None, threads: int = 1, with_work: bool = False):
    from svtrek_amd._lib import RESULT_DTYPE
    v, keep = pileup(pl)
    pr = params(prm)
    loci = np.ascontiguousarray(loci)
    out = np.empty(len(loci), dtype=RESULT_DTYPE)
    w = OrcWork()
    rc = lib().orc_refine_batch(C.byref(v), C.byref(pr), loci.ctypes.data, len(loci), out.ctypes.data,
                                threads, C.byref(w))
    if rc != 0:
        raise RuntimeError("orc_refine_batch failed")
    del keep
    if with_work:
        return out, {f: int(getattr(w, f)) for f, _ in OrcWork._fields_}
    return out


def bgzf_refine_batch(bam_path: str, loci: np.ndarray, prm=None, threads: int = 1, with_stats: bool = False):
    """The reference-shaped baseline (bgzf_ref.c): per-thread BAM handle + BAI, per-query
    linear-index seek, BGZF inflate and record decode.  Needs `bam_path`.bai."""
    from svtrek_amd._lib import RESULT_DTYPE
    pr = params(prm)
    loci = np.ascontiguousarray(loci)
    out = np.empty(len(loci), dtype=RESULT_DTYPE)
    st = (C.c_uint64 * 3)()
    err = C.create_string_buffer(512)
    rc = lib().orc_bgzf_refine_batch(bam_path.encode(), C.byref(pr), loci.ctypes.data, len(loci), out.ctypes.data,
                                     threads, st, err, 512)
    if rc != 0:
        raise RuntimeError(err.value.decode() or "orc_bgzf_refine_batch failed")
    if with_stats:
        return out, {"blocks_inflated": int(st[0]), "bytes_inflated": int(st[1]), "records_decoded": int(st[2])}
    return out


def parse_line(line: str):
    """-> (action, (type, chrom, pos, end) or None, err)"""
    from svtrek_amd._lib import LOCUS_DTYPE
    buf = C.create_string_buffer(line.encode("latin-1"))
    loc = np.zeros(1, dtype=LOCUS_DTYPE)
    err = C.create_string_buffer(512)
    act = lib().orc_parse_line(buf, loc.ctypes.data, err, 512)
    rec = tuple(int(x) for x in loc[0]) if act == 1 else None
    return act, rec, err.value.decode("latin-1")


def audit_text(vcf_text: str, pl, prm=None) -> str:
    v, keep = pileup(pl)
    pr = params(prm)
    data = vcf_text.encode("latin-1")
    out = C.c_void_p()
    n = C.c_size_t()
    rc = lib().orc_audit_text(data, len(data), C.byref(v), C.byref(pr), C.byref(out), C.byref(n))
    if rc != 0:
        raise RuntimeError("orc_audit_text failed")
    s = C.string_at(out, n.value).decode("latin-1")
    lib().orc_free(out)
    del keep
    return s


def sliding_window_ins(pl, chrom: int, start: int, end: int, window_size: int, slide_size: int,
                       min_count: int = 3):
    """-> (bestCandidateOverall, int32 candidate per sub-window, int32 support per sub-window)"""
    v, keep = pileup(pl)
    ws = max(int(window_size), 1)
    nsub = max(0, (int(end) - int(start) + ws - 1) // ws)
    cand = np.empty(nsub, dtype=np.int32)
    sup = np.empty(nsub, dtype=np.int32)
    best = lib().orc_sliding_window_ins(C.byref(v), chrom, start & 0xFFFFFFFF, end & 0xFFFFFFFF, window_size,
                                        slide_size, min_count, cand.ctypes.data, sup.ctypes.data)
    del keep
    return best, cand, sup


# ---------------------------------------------------------------- allele consensus (POA)
POA_FIELDS = ("match", "mismatch", "gap_open", "gap_ext", "band_b", "band_f_permille", "max_seqs", "max_len",
              "max_nodes", "support_radius", "max_support")
POA_DEFAULTS = dict(match=2, mismatch=4, gap_open=4, gap_ext=2, band_b=10, band_f_permille=10, max_seqs=32,
                    max_len=4000, max_nodes=32768, support_radius=20, max_support=64)


class OrcPoaParams(C.Structure):
    _fields_ = [(n, C.c_int32) for n in POA_FIELDS]


def poa_params(**kw) -> OrcPoaParams:
    d = dict(POA_DEFAULTS)
    d.update(kw)
    return OrcPoaParams(*(d[n] for n in POA_FIELDS))


def _poa_lib():
    L = lib()
    if not getattr(L, "_poa_bound", False):
        P = C.c_void_p
        L.orc_poa_consensus.argtypes = [P, P, C.c_int, P, P, C.c_int, P]
        L.orc_poa_consensus.restype = C.c_int
        L.orc_poa_support.argtypes = [P, P, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, P, P, C.c_int]
        L.orc_poa_support.restype = C.c_int
        L._poa_bound = True
    return L


def poa_consensus(seqs, cap: int = 1 << 16, **kw) -> tuple[np.ndarray, int]:
    """Consensus (nt4 uint8 array) of the sequences, in order, and how many were fused."""
    L = _poa_lib()
    off = np.zeros(len(seqs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(s) for s in seqs])
    bases = np.concatenate([np.asarray(s, dtype=np.uint8) for s in seqs]) if seqs else np.zeros(1, np.uint8)
    out = np.zeros(cap, dtype=np.uint8)
    used = C.c_int32(0)
    pp = poa_params(**kw)
    n = L.orc_poa_consensus(bases.ctypes.data, off.ctypes.data, len(seqs), C.byref(pp), out.ctypes.data, cap,
                            C.byref(used))
    if n < 0:
        raise MemoryError("orc_poa_consensus")
    return out[:min(n, cap)].copy(), int(used.value)


def poa_support(pl, ins_base: np.ndarray, chrom: int, s: int, e: int, refined: int, cap: int = 64, **kw) -> np.ndarray:
    L = _poa_lib()
    v, keep = pileup(pl)
    ib = np.ascontiguousarray(ins_base, dtype=np.uint64)
    idx = np.zeros(cap, dtype=np.int64)
    pp = poa_params(**kw)
    n = L.orc_poa_support(C.byref(v), ib.ctypes.data, chrom, s & 0xFFFFFFFF, e & 0xFFFFFFFF, refined & 0xFFFFFFFF,
                          C.byref(pp), idx.ctypes.data, cap)
    del keep
    return idx[:min(n, cap)].copy()
