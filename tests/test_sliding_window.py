"""sliding_window_ins (reference sliding_window.c:8-97), the optional INS-discovery mode.

The reference never calls it, so no reference run or fixture pins it: PARITY UNPINNED by
the reference.  The C oracle (oracle/svtrek_oracle.c orc_sliding_window_ins) is
cross-checked here against a second, independent pure-Python restatement on small
pileups, including the reference's 32-bit `int` sum wrap-around (sliding_window.c:78-82);
the GPU engine is checked against the oracle in test_gpu_sliding_window.py.
"""
import os
import random
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

import oracle_ffi as O  # noqa: E402

from svtrek_amd import from_reads  # noqa: E402
from svtrek_amd.pileup import endpos_of  # noqa: E402

M32 = 0xFFFFFFFF


def i32(x):
    x &= M32
    return x - (1 << 32) if x >> 31 else x


def c_div(a, b):   # C integer division: truncation toward zero
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def py_sliding_window_ins(reads, chrom, start, end, ws, slide, min_count):
    """Literal restatement over [(tid, pos, [(op, len), ...])]."""
    best_overall, max_overall = -1, 0
    subs = []
    ss = start
    while ss < end:
        se = min((ss + ws) & M32, end)
        beg, qend = (ss - 1) & M32, (se - 1) & M32
        locs = []
        if qend > beg:
            for tid, pos, ops in reads:
                words = np.array([(ln << 4) | op for op, ln in ops], dtype=np.uint32)
                if tid != chrom - 1 or not (pos < qend and endpos_of(pos, words) > beg):
                    continue
                rp = pos & M32
                for op, ln in ops:
                    if op == 1 and ln >= 50:
                        locs.append(i32(rp))
                    if op not in (1, 4):
                        rp = (rp + ln) & M32
                    if rp > se:
                        break
        best, max_sup = -1, 0
        locs.sort()
        for i in range(0, len(locs), slide):
            e = i
            while e < len(locs) and locs[e] - locs[i] <= ws:
                e += 1
            sup = e - i
            if sup >= min_count and sup > max_sup:
                max_sup = sup
                tot = i32(sum(locs[i:e]))
                best = c_div(i32(tot + sup // 2), sup)
        subs.append((best, max_sup))
        if best != -1 and max_sup > max_overall:
            max_overall, best_overall = max_sup, best
        ss = (ss + ws) & M32
    return best_overall, subs


def random_reads(rng, n_reads, base, span, ins_sites, n_targets=2):
    reads = []
    for _ in range(n_reads):
        tid = rng.randrange(n_targets)
        pos = base + rng.randrange(span)
        ops = []
        if rng.random() < 0.2:
            ops.append((rng.choice([4, 5]), rng.randrange(1, 300)))
        for _ in range(rng.randrange(1, 12)):
            r = rng.random()
            if r < 0.35:
                ops.append((1, rng.choice([10, 49, 50, 51, 300])))
            elif r < 0.45:
                ops.append((rng.choice([2, 3, 5, 6, 7, 8]), rng.randrange(1, 400)))
            else:
                ops.append((0, rng.randrange(1, 2000)))
        if rng.random() < 0.5 and ins_sites:
            site = rng.choice(ins_sites)
            pos = max(0, site - rng.randrange(0, 3000))
            ops = [(0, site - pos + rng.randrange(-20, 21) if site - pos > 20 else 1), (1, 120), (0, 2500)]
        reads.append((tid, pos, ops))
    return reads


@pytest.mark.parametrize("seed", range(6))
def test_oracle_matches_python_restatement(seed):
    rng = random.Random(seed)
    base = rng.choice([0, 1000, 90_000_000, 200_000_000])   # large bases overflow the int sum
    sites = [base + rng.randrange(0, 20000) for _ in range(4)]
    reads = random_reads(rng, 160, base, 20000, sites)
    pl = from_reads(2, reads)
    for _ in range(12):
        chrom = rng.choice([1, 1, 2, 3, 0])
        start = base + rng.randrange(-500, 15000) if base else rng.randrange(0, 15000)
        start = max(start, 0)
        length = rng.choice([0, 1, 999, 5000, 12000])
        ws = rng.choice([1, 50, 500, 1000, 4000])
        slide = rng.choice([1, 2, 3, 7])
        mc = rng.choice([1, 2, 3, 5])
        want_best, want_subs = py_sliding_window_ins(reads, chrom, start, start + length, ws, slide, mc)
        got_best, cand, sup = O.sliding_window_ins(pl, chrom, start, start + length, ws, slide, mc)
        assert got_best == want_best
        assert list(zip(cand.tolist(), sup.tolist())) == want_subs


def test_int_sum_wraps_like_the_reference():
    """30 insertions at ~2e8: the int sum exceeds 2^31, the reference's wrapped mean differs
    from the true mean; both restatements reproduce the wrapped value."""
    site = 200_000_000
    reads = [(0, site - 1000 + k, [(0, 1000 - k), (1, 80), (0, 3000)]) for k in range(30)]
    pl = from_reads(1, reads)
    best, cand, sup = O.sliding_window_ins(pl, 1, site - 500, site + 500, 1000, 1, 3)
    want, subs = py_sliding_window_ins(reads, 1, site - 500, site + 500, 1000, 1, 3)
    assert (best, list(zip(cand.tolist(), sup.tolist()))) == (want, subs)
    assert sup[0] == 30 and best != site     # wrapped: not the true mean
