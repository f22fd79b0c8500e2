"""BASELINE.json configs 3-5 read models at parity-test sizes: every locus bit-exact vs the
oracle, and the device work counters equal the oracle's (the roofline's algorithmic bytes)."""
from dataclasses import replace

import numpy as np
import oracle_ffi as O
import pytest

from svtrek_amd import sim

pytestmark = pytest.mark.gpu


def _check(engine_factory, cfg, threads=16):
    r = sim.generate(cfg)
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    got = eng.refine(r.loci)
    want, ow = O.refine_batch(r.pileup, r.loci, threads=threads, with_work=True)
    bad = np.nonzero((got["start"] != want["start"]) | (got["end"] != want["end"]))[0]
    assert len(bad) == 0, f"{len(bad)} loci differ, first {r.loci[bad[0]]}: gpu {got[bad[0]]} oracle {want[bad[0]]}"
    w = eng.count_work(r.loci)
    assert (w["reads"], w["ops_walked"], w["candidates"]) == (ow["reads"], ow["ops_walked"], ow["candidates"])
    return r, got


def test_cfg3_del_ins_mix_subset(engine_factory):
    cfg = replace(sim.WORKLOADS["cfg3_50k_delins_30x_ont"], n_loci=3000, n_targets=2)
    r, got = _check(engine_factory, cfg)
    ins = r.loci["type"] == 1
    assert ins.any() and (~ins).any()
    assert (got["start"][ins] != 0xFFFFFFFF).mean() > 0.5          # INS refined
    assert (got["end"][ins] == 0xFFFFFFFF).all()                   # INS has no end window


def test_cfg4_hifi_dense_subset(engine_factory):
    """HiFi-like (15 kb, ~30 ops/read) with loci every ~3 kb: windows overlap heavily."""
    cfg = replace(sim.WORKLOADS["cfg4_1m_delins_30x_hifi"], n_loci=20000, n_targets=2)
    _check(engine_factory, cfg)


def test_cfg5_ultralong_subset(engine_factory):
    """60x ultra-long (50 kb, ~2000 ops/read): deep pileups, reads crossing several tiles."""
    cfg = replace(sim.WORKLOADS["cfg5_100k_60x_ul_ont"], n_loci=400, n_targets=1)
    _check(engine_factory, cfg)


def test_cfg3_full_parity(engine_factory):
    """BASELINE config 3 at full size: all 50k DEL+INS loci (16 oracle threads)."""
    r, got = _check(engine_factory, sim.WORKLOADS["cfg3_50k_delins_30x_ont"])
    assert len(got) == 50000


def test_cfg4_full_parity(engine_factory):
    """BASELINE config 4 at full size -- the bench's workload: all 1M loci over 22 contigs,
    including the windows that spill past the LDS candidate buffer."""
    cfg = sim.WORKLOADS["cfg4_1m_delins_30x_hifi"]
    r = sim.generate(cfg)
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    got = eng.refine(r.loci)
    want, ow = O.refine_batch(r.pileup, r.loci, threads=16, with_work=True)
    bad = np.nonzero((got["start"] != want["start"]) | (got["end"] != want["end"]))[0]
    assert len(bad) == 0, f"{len(bad)} loci differ, first {r.loci[bad[0]]}: gpu {got[bad[0]]} oracle {want[bad[0]]}"
    w = eng.count_work(r.loci)
    assert (w["windows"], w["reads"], w["ops_walked"], w["candidates"]) == \
        (ow["windows"], ow["reads"], ow["ops_walked"], ow["candidates"])
    assert w["spilled_windows"] > 0          # the spill path ran at scale, and agreed
    assert len(got) == 1_000_000


@pytest.mark.timeout(900)
def test_cfg5_full_parity(engine_factory):
    """BASELINE config 5 at full size: 100k DEL+INS loci over 8 contigs of 60x ultra-long
    (50 kb, ~2000 ops/read) reads -- 9 G CIGAR ops (36 GB), generated zero-copy and walked by
    the device index build; every locus, the work counters and the spilled windows vs the
    oracle (16 threads)."""
    import sys
    import time
    cfg = sim.WORKLOADS["cfg5_100k_60x_ul_ont"]
    t0 = time.time()
    r = sim.generate(cfg, keep_handle=True)
    print(f"cfg5: {r.pileup.n_reads} reads, {r.pileup.n_ops} ops, generated in {time.time() - t0:.1f} s",
          file=sys.stderr, flush=True)
    eng = engine_factory()
    try:
        eng.load_pileup(r.pileup)
        st = eng.load_stats()
        print(f"cfg5: load {st}", file=sys.stderr, flush=True)
        assert st["span_events"] > 0 and st["index_kind"] == 2   # long reads: the stream walk
        got = eng.refine(r.loci)
        want, ow = O.refine_batch(r.pileup, r.loci, threads=16, with_work=True)
        bad = np.nonzero((got["start"] != want["start"]) | (got["end"] != want["end"]))[0]
        assert len(bad) == 0, f"{len(bad)} loci differ, first {r.loci[bad[0]]}: gpu {got[bad[0]]} oracle {want[bad[0]]}"
        w = eng.count_work(r.loci)
        assert (w["windows"], w["reads"], w["ops_walked"], w["candidates"]) == \
            (ow["windows"], ow["reads"], ow["ops_walked"], ow["candidates"])
        print(f"cfg5: work {w}", file=sys.stderr, flush=True)
        eng.reindex()
        got2 = eng.refine(r.loci)
        assert (got2 == got).all()
        assert len(got) == 100_000
    finally:
        eng.close()
