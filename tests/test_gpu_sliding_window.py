"""GPU sliding_window_ins mode (svt_sliding_window_ins) vs the CPU oracle, bit-exact per
sub-window (candidate, support) and per query (bestCandidateOverall).  Parity unpinned by
the reference (dead code there, no caller); see test_sliding_window.py."""
import os
import random
import sys
from dataclasses import replace

import numpy as np
import oracle_ffi as O
import pytest

from svtrek_amd import Params, SvtError, from_reads, sim
from svtrek_amd._lib import SW_QUERY_DTYPE
from svtrek_amd.host import format_sw_lines

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_sliding_window import random_reads  # noqa: E402

pytestmark = pytest.mark.gpu


def queries(rows):
    q = np.zeros(len(rows), dtype=SW_QUERY_DTYPE)
    for i, (c, s, e) in enumerate(rows):
        q[i] = (c, s & 0xFFFFFFFF, e & 0xFFFFFFFF)
    return q


def check(eng, pl, q, ws, slide, mc):
    best, off, sub = eng.sliding_window_ins(q, ws, slide, with_subwindows=True)
    for i, r in enumerate(q):
        wb, wc, wsup = O.sliding_window_ins(pl, int(r["chrom"]), int(r["start"]), int(r["end"]), ws, slide, mc)
        got = sub[off[i]:off[i + 1]]
        assert np.array_equal(got["candidate"], wc) and np.array_equal(got["support"], wsup), \
            f"query {i} {r} ws={ws} slide={slide}"
        assert best[i] == wb
    return best, off, sub


def test_sim_ins_loci(engine_factory):
    cfg = replace(sim.WORKLOADS["cfg3_50k_delins_30x_ont"], n_loci=400, n_targets=2)
    r = sim.generate(cfg)
    ins = r.loci[r.loci["type"] == 1]
    rows = [(int(l["chrom"]), int(l["pos"]) - 10000, int(l["pos"]) + 10000) for l in ins[:150]]
    q = queries(rows)
    for ws, slide, mc in ((1000, 1, 3), (500, 3, 3), (4000, 2, 5)):
        eng = engine_factory(Params(consensus_min_count=mc))
        eng.load_pileup(r.pileup)
        best, _, _ = check(eng, r.pileup, q, ws, slide, mc)
    assert (best != -1).mean() > 0.5


@pytest.mark.parametrize("seed", range(4))
def test_random_reads(engine_factory, seed):
    rng = random.Random(seed)
    base = rng.choice([0, 1000, 90_000_000, 200_000_000])
    sites = [base + rng.randrange(0, 20000) for _ in range(4)]
    pl = from_reads(2, random_reads(rng, 300, base, 20000, sites))
    rows = []
    for _ in range(40):
        start = max(0, base + rng.randrange(-500, 15000))
        rows.append((rng.choice([1, 1, 2, 3, 0]), start, start + rng.choice([0, 1, 999, 5000, 12000])))
    q = queries(rows)
    for ws, slide, mc in ((1, 1, 1), (50, 2, 2), (1000, 1, 3), (4000, 7, 3)):
        eng = engine_factory(Params(consensus_min_count=mc))
        eng.load_pileup(pl)
        check(eng, pl, q, ws, slide, mc)


def test_spill_deep_subwindow(engine_factory):
    """700 insertions in one sub-window: past the 256 LDS candidates, exact via the spill pool."""
    site = 150_000_000
    reads = [(0, site - 2000 + (k % 97), [(0, 2000 - (k % 97) + (k % 13)), (1, 60), (0, 4000)]) for k in range(700)]
    pl = from_reads(1, reads)
    eng = engine_factory(Params())
    eng.load_pileup(pl)
    best, off, sub = check(eng, pl, queries([(1, site - 3000, site + 3000)]), 2000, 1, 3)
    assert sub["support"].max() > 256


def test_errors_and_empty(engine_factory):
    pl = from_reads(1, [(0, 100, [(0, 500), (1, 70), (0, 500)])] * 4)
    eng = engine_factory(Params())
    eng.load_pileup(pl)
    best, off, sub = eng.sliding_window_ins(queries([(1, 500, 500), (1, 900, 100)]), 100, 1, with_subwindows=True)
    assert best.tolist() == [-1, -1] and len(sub) == 0
    for ws, slide, row in ((0, 1, (1, 0, 10)), (10, 0, (1, 0, 10)), (16, 1, (1, 0, 0xFFFFFFF8))):
        with pytest.raises(SvtError):
            eng.sliding_window_ins(queries([row]), ws, slide)
    best, off, sub = eng.sliding_window_ins(queries([(1, 1, 1200)]), 1000, 1, with_subwindows=True)
    assert best.tolist() == [600] and sub.tolist() == [(600, 4), (600, 4)]
    assert format_sw_lines(queries([(1, 1, 1200)]), off, sub, 1000) == \
        ("INS Discovery in window [1, 1001] at position 600 with support 4\n"
         "INS Discovery in window [1001, 1200] at position 600 with support 4\n")
