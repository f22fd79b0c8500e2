"""ctypes bindings of the product libraries (C ABI in include/svtrek_gpu.h).

The engine library must exist: there is no CPU fallback anywhere in the product
path -- a missing or unloadable libsvtrek_hip.so raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))

SVT_OK = 0
SVT_EINVAL = -1
SVT_EDEVICE = -2
SVT_ENOMEM = -3
SVT_ESTATE = -4
SVT_EOVERFLOW = -5
STATUS_NAMES = {0: "OK", -1: "EINVAL", -2: "EDEVICE", -3: "ENOMEM", -4: "ESTATE", -5: "EOVERFLOW"}

SVT_UNKNOWN, SVT_INS, SVT_DEL, SVT_INV, SVT_DUP, SVT_TRA, SVT_BND = range(7)
SVT_NA = 0xFFFFFFFF
SVT_LDS_CANDS = 256

LOCUS_DTYPE = np.dtype([("type", "<i4"), ("chrom", "<i4"), ("pos", "<u4"), ("end", "<u4")])
RESULT_DTYPE = np.dtype([("start", "<u4"), ("end", "<u4")])
SW_QUERY_DTYPE = np.dtype([("chrom", "<i4"), ("start", "<u4"), ("end", "<u4")])     # svt_sw_query
SW_WINDOW_DTYPE = np.dtype([("candidate", "<i4"), ("support", "<i4")])               # svt_sw_window
BGZF_BLOCK_DTYPE = np.dtype([("coff", "<u8"), ("uoff", "<u8"), ("clen", "<u4"), ("ulen", "<u4")])   # svt_bgzf_block
RECORD_DTYPE = np.dtype([("index", "<u4"), ("start", "<u4"), ("end", "<u4"), ("pad", "<u4")])   # svt_record


class SvtParams(C.Structure):
    _fields_ = [
        ("wider_interval", C.c_int32),
        ("median_interval", C.c_int32),
        ("narrow_interval", C.c_int32),
        ("consensus_interval_range", C.c_int32),
        ("consensus_interval", C.c_int32),
        ("consensus_min_count", C.c_int32),
        ("spill_bytes", C.c_uint64),
    ]


class SvtPileupView(C.Structure):
    _fields_ = [
        ("n_targets", C.c_int32),
        ("tid_off", C.c_void_p),
        ("pos", C.c_void_p),
        ("endpos", C.c_void_p),
        ("cig_off", C.c_void_p),
        ("cigar", C.c_void_p),
        ("clip", C.c_void_p),
    ]


class SvtPoaParams(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("match", "mismatch", "gap_open", "gap_ext", "band_b", "band_f_permille",
                                          "max_seqs", "max_len", "max_nodes", "support_radius", "max_support")]


class SvtInsseqView(C.Structure):
    _fields_ = [("n_ins", C.c_uint64), ("off", C.c_void_p), ("bases", C.c_void_p)]


POA_RESULT_DTYPE = np.dtype([("len", "<i4"), ("n_support", "<i4"), ("n_used", "<i4"), ("status", "<i4")])


class SvtWork(C.Structure):
    _fields_ = [
        ("windows", C.c_uint64),
        ("reads", C.c_uint64),
        ("ops_walked", C.c_uint64),
        ("candidates", C.c_uint64),
        ("spilled_windows", C.c_uint64),
        ("queries", C.c_uint64),
        ("probe_entries", C.c_uint64),
        ("range_reads", C.c_uint64),
        ("list_reads", C.c_uint64),
        ("list_entries", C.c_uint64),
        ("stop_searches", C.c_uint64),
        ("stop_chunk_words", C.c_uint64),
        ("span_bounds", C.c_uint64),
        ("span_events", C.c_uint64),
        ("event_bytes", C.c_uint64),
        ("bucket_queries", C.c_uint64),
        ("bucket_events", C.c_uint64),
    ]


class SvtLoadStats(C.Structure):
    _fields_ = [
        ("host_ms", C.c_double),
        ("upload_ms", C.c_double),
        ("index_ms", C.c_double),
        ("total_ms", C.c_double),
        ("index_bytes", C.c_uint64),
        ("span_events", C.c_uint64),
        ("lead_blocks", C.c_uint64),
        ("slow_reads", C.c_uint64),
        ("index_kind", C.c_uint64),
        ("bucket_index", C.c_uint64),
        ("buckets", C.c_uint64),
        ("bucket_events", C.c_uint64),
        ("bucket_bytes", C.c_uint64),
    ]


class SvtBamDecStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("records", "reads", "cigar_ops", "cg_restored", "batches", "rechained",
                                          "inflated_bytes")] + [("feed_ms", C.c_double), ("rechained_chunks", C.c_uint64)]


# every symbol include/svtrek_gpu.h declares
ENGINE_SYMBOLS = (
    "svt_open", "svt_load_pileup", "svt_refine_batch", "svt_refine_device", "svt_sync",
    "svt_count_work", "svt_pileup_device_bytes", "svt_last_error", "svt_close", "svt_version",
    "svt_sw_subwindows", "svt_sliding_window_ins",
    "svt_poa_default_params", "svt_pileup_ins_count", "svt_load_insseq", "svt_poa_consensus",
    "svt_poa_deferred", "svt_last_load_stats", "svt_open_multi", "svt_device_count",
    "svt_refine_device_records", "svt_reindex",
    "svt_bgzf_inflate", "svt_bgzf_inflate_device", "svt_bgzf_inflate_status", "svt_bgzf_last_inflate_ms",
    "svt_host_alloc", "svt_host_free",
    "svt_bam_dec_open", "svt_bam_dec_feed", "svt_bam_dec_load", "svt_bam_dec_stats_get", "svt_bam_dec_close",
)

_engine = None


def engine_path() -> str:
    """The in-tree engine; SVTREK_ENGINE_LIB may name a variant build (A/B benchmarking)."""
    return os.environ.get("SVTREK_ENGINE_LIB") or os.path.join(PKG, "libsvtrek_hip.so")


def load_engine() -> C.CDLL:
    """Load libsvtrek_hip.so (raises if it is missing: no fallback path exists)."""
    global _engine
    if _engine is not None:
        return _engine
    path = engine_path()
    if not os.path.exists(path):
        raise RuntimeError(f"svtrek_amd HIP engine not built: {path} (run __graft_entry__.build())")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7 and the
    # engine's dependency on that soname binds to whichever copy is loaded first.  When the
    # engine comes first, a later torch (device buffers, streams, RCCL) runs on the system
    # copy and finds no GPUs, so torch -- where installed -- is loaded before the engine.
    if os.environ.get("SVTREK_NO_TORCH_FIRST") is None:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    _engine = bind_abi(C.CDLL(path))
    return _engine


def bind_abi(lib: C.CDLL) -> C.CDLL:
    """Declare include/svtrek_gpu.h's entry points on a loaded library (the HIP engine; the
    tests also bind oracle/libsvtrek_cpu.so, the CPU restatement behind the same header)."""
    P = C.c_void_p
    lib.svt_open.argtypes = [C.POINTER(SvtParams), C.c_int, C.POINTER(P)]
    lib.svt_open_multi.argtypes = [C.POINTER(SvtParams), C.c_int, P, C.POINTER(P)]
    lib.svt_device_count.argtypes = [P]
    lib.svt_device_count.restype = C.c_int
    lib.svt_refine_device_records.argtypes = [P, P, C.c_size_t, P, C.c_uint32, P, P]
    lib.svt_load_pileup.argtypes = [P, C.POINTER(SvtPileupView)]
    lib.svt_refine_batch.argtypes = [P, P, C.c_size_t, P]
    lib.svt_refine_device.argtypes = [P, P, C.c_size_t, P, P]
    lib.svt_sync.argtypes = [P, P]
    lib.svt_reindex.argtypes = [P, P]
    lib.svt_count_work.argtypes = [P, P, C.c_size_t, C.POINTER(SvtWork)]
    lib.svt_pileup_device_bytes.argtypes = [P]
    lib.svt_pileup_device_bytes.restype = C.c_uint64
    lib.svt_last_error.argtypes = [P]
    lib.svt_last_error.restype = C.c_char_p
    lib.svt_close.argtypes = [P]
    lib.svt_close.restype = None
    lib.svt_version.restype = C.c_char_p
    lib.svt_last_load_stats.argtypes = [P, C.POINTER(SvtLoadStats)]
    lib.svt_sw_subwindows.argtypes = [P, C.c_int32]
    lib.svt_sw_subwindows.restype = C.c_uint64
    lib.svt_sliding_window_ins.argtypes = [P, P, C.c_size_t, C.c_int32, C.c_int32, P, P]
    lib.svt_poa_default_params.argtypes = [C.POINTER(SvtPoaParams)]
    lib.svt_poa_default_params.restype = None
    lib.svt_pileup_ins_count.argtypes = [P]
    lib.svt_pileup_ins_count.restype = C.c_uint64
    lib.svt_load_insseq.argtypes = [P, C.POINTER(SvtInsseqView)]
    lib.svt_poa_consensus.argtypes = [P, C.POINTER(SvtPoaParams), P, P, C.c_size_t, C.c_int32, P, P]
    lib.svt_poa_deferred.argtypes = [P]
    lib.svt_poa_deferred.restype = C.c_uint64
    lib.svt_bgzf_inflate.argtypes = [P, P, C.c_size_t, P, C.c_size_t, P, C.c_size_t]
    lib.svt_bgzf_inflate_device.argtypes = [P, P, P, C.c_size_t, P, P]
    lib.svt_bgzf_inflate_status.argtypes = [P, P, C.POINTER(C.c_uint32)]
    lib.svt_bgzf_last_inflate_ms.argtypes = [P]
    lib.svt_bgzf_last_inflate_ms.restype = C.c_double
    lib.svt_host_alloc.argtypes = [P, C.c_size_t]
    lib.svt_host_alloc.restype = P
    lib.svt_host_free.argtypes = [P, P]
    lib.svt_host_free.restype = None
    lib.svt_bam_dec_open.argtypes = [P, C.c_int32, C.POINTER(P)]
    lib.svt_bam_dec_feed.argtypes = [P, P, C.c_size_t, P, C.c_size_t, C.c_uint64]
    lib.svt_bam_dec_load.argtypes = [P]
    lib.svt_bam_dec_stats_get.argtypes = [P, C.POINTER(SvtBamDecStats)]
    lib.svt_bam_dec_close.argtypes = [P]
    lib.svt_bam_dec_close.restype = None
    for name in ("svt_bam_dec_open", "svt_bam_dec_feed", "svt_bam_dec_load", "svt_bam_dec_stats_get"):
        getattr(lib, name).restype = C.c_int32
    for name in ("svt_bgzf_inflate", "svt_bgzf_inflate_device", "svt_bgzf_inflate_status",
                 "svt_open", "svt_open_multi", "svt_refine_device_records", "svt_load_pileup", "svt_refine_batch", "svt_refine_device", "svt_sync",
                 "svt_reindex", "svt_count_work", "svt_sliding_window_ins", "svt_load_insseq", "svt_poa_consensus"):
        getattr(lib, name).restype = C.c_int32
    return lib


_sim = None


def load_sim() -> C.CDLL:
    global _sim
    if _sim is not None:
        return _sim
    path = os.path.join(PKG, "libsvtrek_sim.so")
    if not os.path.exists(path):
        raise RuntimeError(f"simulator not built: {path} (run __graft_entry__.build())")
    lib = C.CDLL(path)
    P = C.c_void_p
    lib.sim_generate.argtypes = [P]
    lib.sim_generate.restype = P
    lib.sim_free.argtypes = [P]
    lib.sim_free.restype = None
    for name, rt in (("sim_n_targets", C.c_int32), ("sim_n_reads", C.c_int64), ("sim_n_ops", C.c_uint64),
                     ("sim_n_loci", C.c_int32)):
        getattr(lib, name).argtypes = [P]
        getattr(lib, name).restype = rt
    lib.sim_contig_len.argtypes = [P, C.c_int32]
    lib.sim_contig_len.restype = C.c_int32
    for name in ("sim_tid_off", "sim_pos", "sim_endpos", "sim_cig_off", "sim_cigar", "sim_flag", "sim_loci",
                 "sim_truth"):
        getattr(lib, name).argtypes = [P]
        getattr(lib, name).restype = P
    lib.sim_write_bam.argtypes = [P, C.c_char_p, C.c_int, C.c_int]
    lib.sim_write_bam.restype = C.c_int
    lib.sim_write_bam_region.argtypes = [P, C.c_char_p, C.c_int, C.c_int, C.c_int32, C.c_int64, C.c_int64, C.c_int]
    lib.sim_write_bam_region.restype = C.c_int
    lib.sim_write_bam_regions.argtypes = [P, C.c_char_p, C.c_int, C.c_int, C.c_int, P, P, P, C.c_int]
    lib.sim_write_bam_regions.restype = C.c_int
    lib.sim_insseq.argtypes = [P, C.c_uint64, C.c_int32, C.c_int32, C.POINTER(C.c_uint64), C.POINTER(P),
                               C.POINTER(P)]
    lib.sim_insseq.restype = C.c_int
    lib.sim_free_buf.argtypes = [P]
    lib.sim_free_buf.restype = None
    _sim = lib
    return lib


def ptr(a: np.ndarray | None) -> int | None:
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays passed over the C ABI must be C-contiguous"
    return a.ctypes.data
