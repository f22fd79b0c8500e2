"""Adversarial pileups/loci for parity tests (seeded numpy; small sizes).

Covers the quirks of SURVEY.md §8 A3-A10: every CIGAR op code 0..15 (H, P, N and
9..15 advance the walk, refinement.c:141), D/I lengths straddling 50 (>50 for D,
>=50 for I), leading/trailing soft clips (both soft-clip candidate rules), reads that
start long before a window, reads with endpos == query beg (excluded) and
pos == query end - 1 (included), windows that wrap in uint32, contigs out of range,
clusters tied at the consensus interval, and candidate counts straddling min_count.
"""
from __future__ import annotations

import numpy as np

from svtrek_amd.pileup import Pileup, endpos_of, make_loci

LEN_CHOICES = np.array([1, 2, 3, 5, 9, 20, 49, 50, 51, 52, 60, 100, 300, 1000, 2500], dtype=np.int64)


def random_pileup(rng: np.random.Generator, n_targets: int = 2, contig_len: int = 60000,
                  n_reads: int = 400, max_ops: int = 150, hot: list[int] | None = None,
                  p_exotic: float = 0.1, with_clip_quirks: bool = True) -> Pileup:
    """Random reads; `hot` positions attract D/I ops so windows see real clusters."""
    hot = hot or []
    rows = []
    for _ in range(n_reads):
        tid = int(rng.integers(0, n_targets))
        if hot and rng.random() < 0.7:
            h = int(rng.choice(hot))
            pos = max(0, h - int(rng.integers(0, 8000)))
        else:
            pos = int(rng.integers(0, contig_len))
        nops = int(rng.integers(1, max_ops + 1))
        ops = []
        rp = pos
        for k in range(nops):
            u = rng.random()
            if u < p_exotic:
                op = int(rng.choice([3, 5, 6, 9, 10, 11, 12, 13, 14, 15]))
            elif u < 0.45:
                op = 0
            elif u < 0.6:
                op = int(rng.choice([7, 8]))
            elif u < 0.75:
                op = 2
            elif u < 0.9:
                op = 1
            else:
                op = 4
            ln = int(rng.choice(LEN_CHOICES))
            if hot and op in (1, 2) and rng.random() < 0.3:
                # steer a big indel onto a hot breakpoint (+- small jitter)
                h = int(rng.choice(hot))
                if h > rp:
                    ops.append((0, h - rp + int(rng.integers(-3, 4)) if h - rp > 5 else h - rp + 3))
                    rp += ops[-1][1]
                ln = int(rng.choice([49, 50, 51, 80, 500, 1500]))
            ops.append((op, ln))
            if op not in (1, 4):
                rp += ln
        rows.append((tid, pos, ops))
    # build columnar
    by_tid = [[] for _ in range(n_targets)]
    for i, (tid, pos, ops) in enumerate(rows):
        by_tid[tid].append((pos, i, ops))
    tid_off = [0]
    pos_l, end_l, off_l, cig_l, clip_l = [], [], [0], [], []
    for t in range(n_targets):
        for pos, i, ops in sorted(by_tid[t], key=lambda x: (x[0], x[1])):
            words = [(ln << 4) | op for op, ln in ops]
            pos_l.append(pos)
            end_l.append(endpos_of(pos, np.array(words, dtype=np.uint32)))
            cig_l.extend(words)
            off_l.append(len(cig_l))
            c = (1 if ops[-1][0] == 4 else 0) | (2 if ops[0][0] == 4 else 0)
            if with_clip_quirks and rng.random() < 0.05:
                c = int(rng.integers(0, 4))   # bytes the reference reads past a 0-op CIGAR
            clip_l.append(c)
        tid_off.append(len(pos_l))
    return Pileup(tid_off=np.array(tid_off, dtype=np.int64), pos=np.array(pos_l, dtype=np.int32),
                  endpos=np.array(end_l, dtype=np.int32), cig_off=np.array(off_l, dtype=np.uint64),
                  cigar=np.array(cig_l, dtype=np.uint32), clip=np.array(clip_l, dtype=np.uint8))


def random_loci(rng: np.random.Generator, n: int, n_targets: int, contig_len: int,
                hot: list[int] | None = None) -> np.ndarray:
    hot = hot or []
    rows = []
    for _ in range(n):
        t = int(rng.choice([1, 2, 2, 2, 3, 0, 4]))
        chrom = int(rng.choice([1, 1, 1, 2, 2, 0, n_targets + 1, -1])) if n_targets >= 2 else 1
        if hot and rng.random() < 0.8:
            pos = int(rng.choice(hot)) + int(rng.integers(-60, 61))
        else:
            pos = int(rng.integers(0, contig_len))
        if rng.random() < 0.05:
            pos = int(rng.integers(0, 100))          # windows that wrap in uint32
        ln = int(rng.choice([50, 51, 120, 3000, 20000]))
        end = pos + ln
        if hot and rng.random() < 0.5:
            end = int(rng.choice(hot)) + int(rng.integers(-60, 61))
        if rng.random() < 0.03:
            end = (pos - 40) & 0xFFFFFFFF             # CIEND-quirk style huge END
        rows.append((t, chrom, pos, end))
    return make_loci(rows)


def cluster_pileup(values: list[int], tid: int = 0, n_targets: int = 1, kind: str = "del_start",
                   read_len: int = 5000) -> Pileup:
    """One read per candidate value so that a DEL-start (or INS) window sees exactly `values`."""
    rows = []
    for v in values:
        lead = 1000
        pos = v - lead
        if kind == "ins":
            ops = [(0, lead), (1, 80), (0, read_len)]
        else:
            ops = [(0, lead), (2, 200), (0, read_len)]
        rows.append((tid, pos, ops))
    from svtrek_amd.pileup import from_reads
    return from_reads(n_targets, rows, clip={})
