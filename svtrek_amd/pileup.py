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
