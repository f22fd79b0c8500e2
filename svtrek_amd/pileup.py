"""Columnar pileup: the reads an htslib region iterator can yield, laid out for HBM.

Field meaning is the svt_pileup_view of include/svtrek_gpu.h: per contig (tid),
reads sorted by pos; pos/endpos as htslib's bam1_core_t.pos and bam_endpos();
CIGARs packed BAM-style (len << 4 | op) in one arena indexed by cig_off.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from ._lib import SvtPileupView, ptr

OP_M, OP_I, OP_D, OP_N, OP_S, OP_H, OP_P, OP_EQ, OP_X = range(9)
CIGAR_CHARS = "MIDNSHP=X"


@dataclass
class Pileup:
    tid_off: np.ndarray            # int64 [n_targets+1]
    pos: np.ndarray                # int32 [n_reads]
    endpos: np.ndarray             # int32 [n_reads]
    cig_off: np.ndarray            # uint64 [n_reads+1]
    cigar: np.ndarray              # uint32 [n_ops]
    clip: np.ndarray | None = None  # uint8 [n_reads] SVT_CLIP_* bits (None: derive from cigar)
    contig_len: np.ndarray | None = None
    flag: np.ndarray | None = None
    _keepalive: list = field(default_factory=list, repr=False)

    @property
    def n_targets(self) -> int:
        return int(len(self.tid_off) - 1)

    @property
    def n_reads(self) -> int:
        return int(self.tid_off[-1])

    @property
    def n_ops(self) -> int:
        return int(self.cig_off[-1])

    def view(self) -> SvtPileupView:
        """C view (the arrays must outlive the view)."""
        for name in ("tid_off", "pos", "endpos", "cig_off", "cigar"):
            a = getattr(self, name)
            assert a.flags["C_CONTIGUOUS"], name
        assert self.tid_off.dtype == np.int64 and self.pos.dtype == np.int32
        assert self.endpos.dtype == np.int32 and self.cig_off.dtype == np.uint64
        assert self.cigar.dtype == np.uint32
        if self.clip is not None:
            assert self.clip.dtype == np.uint8 and len(self.clip) == self.n_reads
        return SvtPileupView(self.n_targets, ptr(self.tid_off), ptr(self.pos), ptr(self.endpos),
                             ptr(self.cig_off), ptr(self.cigar), ptr(self.clip))

    def read_cigar(self, r: int) -> np.ndarray:
        return self.cigar[int(self.cig_off[r]):int(self.cig_off[r + 1])]

    def cigar_string(self, r: int) -> str:
        return "".join(f"{int(w) >> 4}{CIGAR_CHARS[int(w) & 15] if (int(w) & 15) < 9 else '?'}"
                       for w in self.read_cigar(r))


def endpos_of(pos: int, ops: np.ndarray, unmapped: bool = False) -> int:
    """htslib bam_endpos(): pos + Σ len(M/D/N/=/X), or +1 when that is 0 / unmapped."""
    rl = 0
    if not unmapped:
        for w in ops:
            op = int(w) & 15
            if op in (OP_M, OP_D, OP_N, OP_EQ, OP_X):
                rl += int(w) >> 4
    return pos + (rl if rl > 0 else 1)


def from_reads(n_targets: int, reads: list[tuple[int, int, list[tuple[int, int]]]],
               clip: dict[int, int] | None = None) -> Pileup:
    """Build a pileup from [(tid, pos, [(op, len), ...]), ...] (any order)."""
    by_tid: list[list[tuple[int, int, list[tuple[int, int]]]]] = [[] for _ in range(n_targets)]
    for i, (tid, pos, ops) in enumerate(reads):
        by_tid[tid].append((pos, i, ops))
    tid_off = [0]
    pos_l, end_l, off_l, cig_l, clip_l = [], [], [0], [], []
    for t in range(n_targets):
        for pos, i, ops in sorted(by_tid[t], key=lambda x: (x[0], x[1])):
            words = np.array([(ln << 4) | op for op, ln in ops], dtype=np.uint32)
            pos_l.append(pos)
            end_l.append(endpos_of(pos, words))
            cig_l.extend(int(w) for w in words)
            off_l.append(len(cig_l))
            if clip is not None:
                if i in clip:
                    clip_l.append(clip[i])
                else:
                    c = 0
                    if len(ops) and ops[-1][0] == OP_S:
                        c |= 1
                    if len(ops) and ops[0][0] == OP_S:
                        c |= 2
                    clip_l.append(c)
        tid_off.append(len(pos_l))
    return Pileup(
        tid_off=np.array(tid_off, dtype=np.int64),
        pos=np.array(pos_l, dtype=np.int32),
        endpos=np.array(end_l, dtype=np.int32),
        cig_off=np.array(off_l, dtype=np.uint64),
        cigar=np.array(cig_l, dtype=np.uint32),
        clip=np.array(clip_l, dtype=np.uint8) if clip is not None else None,
    )


def make_loci(rows) -> np.ndarray:
    """[(type, chrom, pos, end), ...] -> LOCUS_DTYPE array."""
    from ._lib import LOCUS_DTYPE
    a = np.zeros(len(rows), dtype=LOCUS_DTYPE)
    for i, (t, c, p, e) in enumerate(rows):
        a[i] = (t, c, p & 0xFFFFFFFF, e & 0xFFFFFFFF)
    return a


def query_spans(loci: np.ndarray, wider: int, median: int, narrow: int, n_targets: int) -> np.ndarray:
    """Per contig, the [beg, end) hull of every htslib query the loci issue (int64 [n_targets, 2];
    beg > end when the contig has none).

    Windows are A2 (audit.c:178 INS, :191-192 DEL) in uint32 with wrap-around and the query
    bounds are sam_itr_queryi(start-1, end-1) (refinement.c:114); an empty query (end <= beg)
    or a tid outside the header yields nothing.  INV never collects (A7), so it adds no span.
    """
    M = np.uint64(0xFFFFFFFF)
    t = loci["type"]
    pos = loci["pos"].astype(np.uint64)
    end = loci["end"].astype(np.uint64)
    tid = loci["chrom"].astype(np.int64) - 1
    wins = []
    ins, dl = t == 1, t == 2
    wins.append((ins, pos - np.uint64(median), pos + np.uint64(median)))
    wins.append((dl, pos - np.uint64(wider), pos + np.uint64(narrow)))
    wins.append((dl, end - np.uint64(narrow), end + np.uint64(narrow)))
    out = np.empty((n_targets, 2), dtype=np.int64)
    out[:, 0] = np.iinfo(np.int64).max
    out[:, 1] = np.iinfo(np.int64).min
    for sel, s, e in wins:
        beg = ((s & M) - np.uint64(1)) & M
        qend = ((e & M) - np.uint64(1)) & M
        ok = sel & (qend > beg) & (tid >= 0) & (tid < n_targets)
        if ok.any():
            np.minimum.at(out[:, 0], tid[ok], beg[ok].astype(np.int64))
            np.maximum.at(out[:, 1], tid[ok], qend[ok].astype(np.int64))
    return out


def halo_slice(pl: Pileup, loci: np.ndarray, wider: int, median: int, narrow: int) -> Pileup:
    """The reads any query of `loci` can yield (a rank ingests only its shard's
    genomic span plus the halo of query windows and read spans).  Keeps per-contig order
    and tids, so refining `loci` against the slice is bit-identical to the full pileup:
    every read with pos < q.end and endpos > q.beg for some query q is kept."""
    span = query_spans(loci, wider, median, narrow, pl.n_targets)
    keep = np.zeros(pl.n_reads, dtype=bool)
    tid_off = np.zeros(pl.n_targets + 1, dtype=np.int64)
    for t in range(pl.n_targets):
        a, b = int(pl.tid_off[t]), int(pl.tid_off[t + 1])
        lo, hi = span[t]
        if b > a and hi > lo:
            cut = a + int(np.searchsorted(pl.pos[a:b], hi, side="left"))   # pos < hi
            keep[a:cut] = pl.endpos[a:cut].astype(np.int64) > lo
        tid_off[t + 1] = tid_off[t] + int(keep[a:b].sum())
    idx = np.nonzero(keep)[0]
    starts = pl.cig_off[:-1][idx].astype(np.int64)
    lens = (pl.cig_off[1:][idx] - pl.cig_off[:-1][idx]).astype(np.int64)
    cig_off = np.zeros(len(idx) + 1, dtype=np.uint64)
    np.cumsum(lens, out=cig_off[1:])
    if len(idx):
        gather = np.repeat(starts - cig_off[:-1].astype(np.int64), lens) + np.arange(int(cig_off[-1]))
        cigar = np.ascontiguousarray(pl.cigar[gather])
    else:
        cigar = np.zeros(0, dtype=np.uint32)
    return Pileup(tid_off=tid_off, pos=np.ascontiguousarray(pl.pos[idx]),
                  endpos=np.ascontiguousarray(pl.endpos[idx]), cig_off=cig_off, cigar=cigar,
                  clip=None if pl.clip is None else np.ascontiguousarray(pl.clip[idx]),
                  contig_len=pl.contig_len, flag=None if pl.flag is None else pl.flag[idx])
