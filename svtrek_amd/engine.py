"""Python host mirror of the reference's per-record refinement calls, over the C ABI.

`Engine.refine(loci)` is the batched form of what thread_func (reference
audit.c:175-232) does per record through deletion()/insertion()/inversion()
(refinement.c:327-339): same parameters (t_arg's six refinement fields,
params.h:81-87, defaults params.h:27-32), same result encoding (0xFFFFFFFF = the
reference's -1 "not refined").  Every call runs the HIP engine; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import (LOCUS_DTYPE, POA_RESULT_DTYPE, RESULT_DTYPE, STATUS_NAMES, SW_QUERY_DTYPE, SW_WINDOW_DTYPE,
                   SvtInsseqView, SvtLoadStats, SvtParams, SvtPoaParams, SvtWork, load_engine, ptr)
from .pileup import Pileup

# params.h:27-32
WIDER_INTERVAL = 20000
MEDIAN_INTERVAL = 10000
NARROW_INTERVAL = 2000
CONSENSUS_INTERVAL_RANGE = 500
CONSENSUS_INTERVAL = 5
CONSENSUS_MIN_COUNT = 3


@dataclass
class Params:
    wider_interval: int = WIDER_INTERVAL
    median_interval: int = MEDIAN_INTERVAL
    narrow_interval: int = NARROW_INTERVAL
    consensus_interval_range: int = CONSENSUS_INTERVAL_RANGE
    consensus_interval: int = CONSENSUS_INTERVAL
    consensus_min_count: int = CONSENSUS_MIN_COUNT
    spill_bytes: int = 0

    def to_c(self) -> SvtParams:
        return SvtParams(self.wider_interval, self.median_interval, self.narrow_interval,
                         self.consensus_interval_range, self.consensus_interval, self.consensus_min_count,
                         self.spill_bytes)


class SvtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"svt error {code} ({STATUS_NAMES.get(code, '?')}): {msg}")
        self.code = code


class Engine:
    """One GPU context (svt_ctx).  Use one Engine per process/GPU."""

    def __init__(self, params: Params | None = None, device: int = -1, devices: list[int] | None = None,
                 lib: C.CDLL | None = None):
        """One context on `device` (-1 = current), or -- with `devices` -- one context over
        several GPUs (svt_open_multi: the pileup is replicated, host batches are split).
        lib: another library implementing include/svtrek_gpu.h, bound with _lib.bind_abi --
        only the tests pass one (oracle/libsvtrek_cpu.so, the CPU restatement, to run the
        same calls on both backends); by default the HIP engine, which must be built."""
        self.lib = lib if lib is not None else load_engine()
        self.params = params or Params()
        self._cp = self.params.to_c()
        h = C.c_void_p()
        if devices is not None:
            dv = (C.c_int * len(devices))(*devices)
            rc = self.lib.svt_open_multi(C.byref(self._cp), len(devices), dv, C.byref(h))
        else:
            rc = self.lib.svt_open(C.byref(self._cp), int(device), C.byref(h))
        if rc != 0:
            raise SvtError(rc, "svt_open failed (no HIP device, or consensus_min_count < 1)")
        self._h = h
        self._pileup = None

    @property
    def n_devices(self) -> int:
        return int(self.lib.svt_device_count(self._h))

    def _check(self, rc: int) -> None:
        if rc != 0:
            raise SvtError(rc, self.lib.svt_last_error(self._h).decode(errors="replace"))

    def load_pileup(self, pileup: Pileup) -> None:
        view = pileup.view()
        self._check(self.lib.svt_load_pileup(self._h, C.byref(view)))
        self._pileup = pileup

    def refine(self, loci: np.ndarray) -> np.ndarray:
        loci = np.ascontiguousarray(loci, dtype=LOCUS_DTYPE)
        out = np.empty(len(loci), dtype=RESULT_DTYPE)
        if len(loci):
            self._check(self.lib.svt_refine_batch(self._h, ptr(loci), len(loci), ptr(out)))
        return out

    def refine_device(self, d_loci: int, n: int, d_out: int, stream: int | None = None) -> None:
        """Device pointers (e.g. torch tensor .data_ptr()) on a hipStream_t handle (int)."""
        self._check(self.lib.svt_refine_device(self._h, C.c_void_p(d_loci), n, C.c_void_p(d_out),
                                               C.c_void_p(stream or 0)))

    def refine_device_records(self, d_loci: int, n: int, d_rec: int, d_index: int | None = None,
                              index_base: int = 0, stream: int | None = None) -> None:
        """As refine_device, writing RECORD_DTYPE gather records {index, start, end, 0}."""
        self._check(self.lib.svt_refine_device_records(self._h, C.c_void_p(d_loci), n, C.c_void_p(d_index or 0),
                                                       int(index_base), C.c_void_p(d_rec), C.c_void_p(stream or 0)))

    def reindex(self, stream: int | None = None) -> None:
        """Rebuild the device index of the loaded pileup on a hipStream_t handle (svt_reindex:
        asynchronous, no host work, results unchanged)."""
        self._check(self.lib.svt_reindex(self._h, C.c_void_p(stream or 0)))

    def bgzf_inflate(self, comp, blocks: np.ndarray, out_bytes: int | None = None) -> np.ndarray:
        """Inflate BGZF blocks on the device (svt_bgzf_inflate): comp = the compressed bytes,
        blocks = BGZF_BLOCK_DTYPE rows {coff, uoff, clen, ulen}; returns the uint8 output."""
        from ._lib import BGZF_BLOCK_DTYPE
        c = np.ascontiguousarray(np.frombuffer(comp, dtype=np.uint8) if isinstance(comp, (bytes, bytearray)) else comp,
                                 dtype=np.uint8)
        b = np.ascontiguousarray(blocks, dtype=BGZF_BLOCK_DTYPE)
        if out_bytes is None:
            out_bytes = int((b["uoff"].astype(np.uint64) + b["ulen"]).max()) if len(b) else 0
        out = np.empty(max(out_bytes, 1), dtype=np.uint8)
        self._check(self.lib.svt_bgzf_inflate(self._h, c.ctypes.data, c.nbytes, b.ctypes.data, len(b),
                                              out.ctypes.data, out_bytes))
        return out[:out_bytes]

    def last_inflate_ms(self) -> float:
        return float(self.lib.svt_bgzf_last_inflate_ms(self._h))

    def sync(self, stream: int | None = None) -> None:
        self._check(self.lib.svt_sync(self._h, C.c_void_p(stream or 0)))

    def count_work(self, loci: np.ndarray) -> dict:
        loci = np.ascontiguousarray(loci, dtype=LOCUS_DTYPE)
        w = SvtWork()
        self._check(self.lib.svt_count_work(self._h, ptr(loci), len(loci), C.byref(w)))
        return {f: int(getattr(w, f)) for f, _ in SvtWork._fields_}

    def sliding_window_ins(self, queries: np.ndarray, window_size: int, slide_size: int,
                           with_subwindows: bool = False):
        """sliding_window_ins (reference sliding_window.c:8-97) for every query
        {chrom, start, end} (SW_QUERY_DTYPE): int32 bestCandidateOverall per query (-1 = none),
        plus, with `with_subwindows`, (offsets, SW_WINDOW_DTYPE per sub-window in order).
        Uses this engine's consensus_min_count."""
        q = np.ascontiguousarray(queries, dtype=SW_QUERY_DTYPE)
        best = np.empty(len(q), dtype=np.int32)
        sub = None
        off = None
        if with_subwindows:
            off = np.zeros(len(q) + 1, dtype=np.int64)
            ws = max(int(window_size), 1)
            span = q["end"].astype(np.int64) - q["start"].astype(np.int64)
            off[1:] = np.cumsum(np.where(span > 0, (span + ws - 1) // ws, 0))
            sub = np.empty(int(off[-1]), dtype=SW_WINDOW_DTYPE)
        self._check(self.lib.svt_sliding_window_ins(self._h, ptr(q), len(q), int(window_size), int(slide_size),
                                                    ptr(best), ptr(sub)))
        return (best, off, sub) if with_subwindows else best

    # ---- allele consensus (POA) of refined INS calls: no reference behaviour (the reference
    # never calls abPOA); parity against oracle/poa_oracle.c only.  See include/svtrek_gpu.h.
    @property
    def ins_count(self) -> int:
        """I >= 50 ops in the loaded pileup: the sequence count load_insseq expects."""
        return int(self.lib.svt_pileup_ins_count(self._h))

    def load_insseq(self, off: np.ndarray, bases: np.ndarray) -> None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        bases = np.ascontiguousarray(bases, dtype=np.uint8)
        v = SvtInsseqView(len(off) - 1, ptr(off), ptr(bases) if len(bases) else None)
        self._check(self.lib.svt_load_insseq(self._h, C.byref(v)))
        self._insseq = (off, bases)

    @staticmethod
    def poa_params(**kw) -> SvtPoaParams:
        p = SvtPoaParams()
        load_engine().svt_poa_default_params(C.byref(p))
        for k, v in kw.items():
            setattr(p, k, int(v))
        return p

    def poa_consensus(self, loci: np.ndarray, refined: np.ndarray, cap: int = 4096, **kw):
        """(POA_RESULT_DTYPE per locus, uint8 [n, cap] nt4 consensus bases)."""
        loci = np.ascontiguousarray(loci, dtype=LOCUS_DTYPE)
        refined = np.ascontiguousarray(refined, dtype=RESULT_DTYPE)
        res = np.zeros(len(loci), dtype=POA_RESULT_DTYPE)
        out = np.zeros((len(loci), cap), dtype=np.uint8)
        p = self.poa_params(**kw)
        if len(loci):
            self._check(self.lib.svt_poa_consensus(self._h, C.byref(p), ptr(loci), ptr(refined), len(loci), cap,
                                                   ptr(out), ptr(res)))
        return res, out

    @property
    def poa_deferred(self) -> int:
        """Loci the last poa_consensus call reran on full-size scratch slots."""
        return int(self.lib.svt_poa_deferred(self._h))

    @property
    def device_bytes(self) -> int:
        return int(self.lib.svt_pileup_device_bytes(self._h))

    def load_stats(self) -> dict:
        """Timings (ms) of the last load_pileup: host pass, H2D copies, device index build."""
        st = SvtLoadStats()
        self._check(self.lib.svt_last_load_stats(self._h, C.byref(st)))
        return {k: (round(v, 3) if isinstance(v, float) else int(v))
                for k, v in ((k, getattr(st, k)) for k, _ in SvtLoadStats._fields_)}

    def close(self) -> None:
        if getattr(self, "_h", None):
            self.lib.svt_close(self._h)
            self._h = None
        self._pileup = None   # the host arrays (a large pileup's memory) are no longer pinned here

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def version() -> str:
    return load_engine().svt_version().decode()
