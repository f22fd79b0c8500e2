"""GPU allele-consensus (POA) mode vs the CPU oracle (oracle/poa_oracle.c), bit-exact per
locus: supporting sequences, sequences fused, consensus bases.  The reference never calls
abPOA, so this mode is parity-unpinned by the reference (see test_poa_oracle.py)."""
import os
import subprocess
import sys

import numpy as np
import oracle_ffi as O
import pytest

from svtrek_amd import SVT_NA, Params, SvtError, from_reads, make_loci, sim

pytestmark = pytest.mark.gpu


def ins_base_of(pl) -> np.ndarray:
    """Per read: index of its first I >= 50 op in the pileup-wide (read, op) order."""
    ins = ((pl.cigar & 15) == 1) & ((pl.cigar >> 4) >= 50)
    c = np.concatenate([[0], np.cumsum(ins, dtype=np.int64)])
    return c[pl.cig_off[:-1].astype(np.int64)].astype(np.uint64)


def check(eng, pl, loci, off, bases, cap=4096, **kw):
    refined = eng.refine(loci)
    res, out = eng.poa_consensus(loci, refined, cap=cap, **kw)
    ib = ins_base_of(pl)
    prm = eng.params
    pp = dict(O.POA_DEFAULTS)
    pp.update(kw)
    n_checked = 0
    for i, l in enumerate(loci):
        R = int(refined["start"][i])
        if int(l["type"]) != 1 or R == SVT_NA:
            assert res["len"][i] == -1
            continue
        s = (int(l["pos"]) - prm.median_interval) & 0xFFFFFFFF
        e = (int(l["pos"]) + prm.median_interval) & 0xFFFFFFFF
        idx = O.poa_support(pl, ib, int(l["chrom"]), s, e, R, cap=pp["max_support"], **kw)
        seqs = [bases[off[k]:off[k + 1]] for k in idx]
        want, used = O.poa_consensus(seqs, **kw)     # full length; the GPU writes min(len, cap)
        assert res["n_used"][i] == used, (i, res[i], used)
        assert res["len"][i] == len(want), (i, res[i], len(want))
        assert np.array_equal(out[i, :min(len(want), cap)], want[:cap]), i
        n_checked += 1
    return n_checked, res


def noisy_sub(rng, a, p):
    s = a.copy()
    m = rng.random(len(s)) < p
    s[m] = (s[m] + rng.integers(1, 4, int(m.sum()))) & 3
    return s


def test_direct_clusters(engine_factory):
    """INS clusters with known alleles: reads carry noisy copies (plus unrelated I >= 50 ops)."""
    rng = np.random.default_rng(1)
    rows, seqrows = [], []
    loci_rows = []
    for k in range(12):
        c = 100000 + 40000 * k
        L = int(rng.choice([50, 80, 300, 1200]))
        allele = rng.integers(0, 4, L).astype(np.uint8)
        for _ in range(int(rng.integers(3, 14))):
            lead = 2000 + int(rng.integers(-500, 500))
            pos = c + int(rng.integers(-3, 4)) - lead
            s = noisy_sub(rng, allele, 0.05) if rng.random() < 0.85 else rng.integers(0, 4, L).astype(np.uint8)
            ops = [(0, lead), (1, len(s)), (0, 3000)]
            sq = [s]
            if rng.random() < 0.2:   # an unrelated insertion later in the read
                x = rng.integers(0, 4, 60).astype(np.uint8)
                ops += [(1, 60), (0, 500)]
                sq.append(x)
            rows.append((0, pos, ops))
            seqrows.append(sq)
        loci_rows.append((1, 1, c + int(rng.integers(-30, 30)), c + 1))
    order = sorted(range(len(rows)), key=lambda i: (rows[i][1], i))
    rows = [rows[i] for i in order]
    seqrows = [seqrows[i] for i in order]
    pl = from_reads(1, rows)
    flat = [s for sq in seqrows for s in sq]
    off = np.concatenate([[0], np.cumsum([len(s) for s in flat])]).astype(np.uint64)
    bases = np.concatenate(flat).astype(np.uint8)
    eng = engine_factory(Params(consensus_min_count=2))
    eng.load_pileup(pl)
    assert eng.ins_count == len(flat)
    eng.load_insseq(off, bases)
    n, res = check(eng, pl, make_loci(loci_rows), off, bases)
    assert n >= 8 and (res["n_used"] > 0).sum() >= 8


def test_sim_workload(engine_factory):
    cfg = sim.SimConfig(seed=21, n_targets=2, n_loci=60, del_frac=0.3, coverage=15, sv_max_len=1500,
                        p_noise_sv=0.2)
    r = sim.generate(cfg, keep_handle=True)
    off, bases = sim.insertion_sequences(r, cfg, err_permille=60)
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    eng.load_insseq(off, bases)
    n, res = check(eng, r.pileup, r.loci, off, bases)
    assert n >= 20


def test_small_caps_and_params(engine_factory):
    cfg = sim.SimConfig(seed=22, n_targets=1, n_loci=30, del_frac=0.0, coverage=20, sv_max_len=900)
    r = sim.generate(cfg, keep_handle=True)
    off, bases = sim.insertion_sequences(r, cfg, err_permille=80)
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    eng.load_insseq(off, bases)
    check(eng, r.pileup, r.loci, off, bases, cap=100, max_seqs=5, max_support=8, band_b=6, band_f_permille=20,
          support_radius=8, max_nodes=1500, max_len=900)


def test_insseq_validation(engine_factory):
    cfg = sim.SimConfig(seed=23, n_targets=1, n_loci=5, del_frac=0.0, coverage=5)
    r = sim.generate(cfg, keep_handle=True)
    off, bases = sim.insertion_sequences(r, cfg)
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    with pytest.raises(SvtError):   # before svt_load_insseq
        eng.poa_consensus(r.loci, eng.refine(r.loci))
    with pytest.raises(SvtError):   # wrong count
        eng.load_insseq(off[:-1], bases)
    eng.load_insseq(off, bases)
    with pytest.raises(SvtError):   # band wider than 63
        eng.poa_consensus(r.loci, eng.refine(r.loci), band_b=60)


def test_deferred_loci_rerun_on_full_slots(engine_factory, monkeypatch):
    """Graphs that outgrow the small scratch slots rerun on full-size ones; results unchanged."""
    cfg = sim.SimConfig(seed=24, n_targets=1, n_loci=40, del_frac=0.0, coverage=15, sv_min_len=200,
                        sv_max_len=1500)
    r = sim.generate(cfg, keep_handle=True)
    off, bases = sim.insertion_sequences(r, cfg, err_permille=60)
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    eng.load_insseq(off, bases)
    monkeypatch.setenv("SVTREK_POA_SMALL_NODES", "1")    # budget = max_len + 2 nodes
    n, res = check(eng, r.pileup, r.loci, off, bases, max_len=1500)
    assert n >= 10
    assert eng.poa_deferred >= 5
    assert (res["status"] == 0).all()
    monkeypatch.delenv("SVTREK_POA_SMALL_NODES")
    res2, _ = eng.poa_consensus(r.loci, eng.refine(r.loci), max_len=1500)
    if not os.environ.get("SVTREK_POA_SUBRUN"):   # the ring-2 build also defers on spill overflow
        assert eng.poa_deferred == 0
    assert np.array_equal(res, res2)


def test_spill_rows_ring2_build():
    """The POA parity tests above, rerun on the engine built with a 2-row LDS ring
    (svtrek_amd/variants/libsvtrek_hip_ring2.so): nearly every predecessor row then comes from
    a spill row, and small slots defer on spill overflow.  One child process."""
    if os.environ.get("SVTREK_POA_SUBRUN"):
        pytest.skip("already the ring-2 run")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "svtrek_amd", "variants", "libsvtrek_hip_ring2.so")
    assert os.path.exists(lib), "ring-2 test engine not built (python svtrek_amd/build.py)"
    env = dict(os.environ, SVTREK_ENGINE_LIB=lib, SVTREK_POA_SUBRUN="1")
    r = subprocess.run([sys.executable, "-m", "pytest", os.path.abspath(__file__), "-x", "-q", "-m", "gpu",
                        "-p", "no:cacheprovider", "--timeout", "240", "--timeout-method", "thread"],
                       env=env, cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]


def test_long_alleles_two_cells_per_lane(engine_factory):
    """Alleles over 2100 bp: the band (2w + 1 columns) exceeds the wave, two cells per lane."""
    cfg = sim.SimConfig(seed=25, n_targets=1, n_loci=12, del_frac=0.0, coverage=10, sv_min_len=2300,
                        sv_max_len=3800)
    r = sim.generate(cfg, keep_handle=True)
    off, bases = sim.insertion_sequences(r, cfg, err_permille=50)
    eng = engine_factory()
    eng.load_pileup(r.pileup)
    eng.load_insseq(off, bases)
    n, res = check(eng, r.pileup, r.loci, off, bases)
    assert n >= 5
    assert (res["len"][res["len"] > 0] > 2100).sum() >= 5


def test_edge_cases(engine_factory):
    """N bases (code 4 never matches), one-sequence loci (consensus = the sequence), loci
    whose supports all exceed max_len (n_used 0), cap 0, max_seqs 1."""
    rng = np.random.default_rng(7)
    rows, seqs, loci_rows = [], [], []
    for k in range(10):
        c = 200000 + 50000 * k
        L = [60, 120, 700, 1000, 90, 400, 75, 2000, 55, 300][k]
        allele = rng.integers(0, 5, L).astype(np.uint8)          # includes N (4)
        n = 1 if k in (1, 4) else int(rng.integers(2, 9))
        for _ in range(n):
            lead = 1500 + int(rng.integers(-200, 200))
            s = noisy_sub(rng, allele, 0.04)
            s[rng.random(L) < 0.02] = 4
            rows.append((0, c - lead + int(rng.integers(-2, 3)), [(0, lead), (1, L), (0, 2500)]))
            seqs.append(s)
        loci_rows.append((1, 1, c + int(rng.integers(-20, 20)), c + 1))
    order = sorted(range(len(rows)), key=lambda i: (rows[i][1], i))
    rows = [rows[i] for i in order]
    seqs = [seqs[i] for i in order]
    pl = from_reads(1, rows)
    off = np.concatenate([[0], np.cumsum([len(s) for s in seqs])]).astype(np.uint64)
    bases = np.concatenate(seqs).astype(np.uint8)
    eng = engine_factory(Params(consensus_min_count=1))
    eng.load_pileup(pl)
    eng.load_insseq(off, bases)
    loci = make_loci(loci_rows)
    n, res = check(eng, pl, loci, off, bases)
    assert n >= 8 and (res["n_used"] == 1).sum() >= 1
    n, res = check(eng, pl, loci, off, bases, max_len=500)        # long alleles: no support
    assert (res["len"] == 0).sum() >= 1
    check(eng, pl, loci, off, bases, cap=0)
    n, res = check(eng, pl, loci, off, bases, max_seqs=1)
    assert res["n_used"].max() <= 1


@pytest.mark.timeout(900)
def test_poa_cfg3_workload(engine_factory):
    """BASELINE config 3's "abPOA consensus path enabled" at size: the allele consensus of every
    refined INS call of the full 50k-locus cfg3 workload on the GPU, checked against the oracle
    on the first 12k loci (over 5k INS calls; 16 checker threads).  Parity unpinned: the
    reference never calls abPOA (Makefile:16)."""
    from concurrent.futures import ThreadPoolExecutor
    cfg = sim.WORKLOADS["cfg3_50k_delins_30x_ont"]
    r = sim.generate(cfg, keep_handle=True)
    off, bases = sim.insertion_sequences(r, cfg, err_permille=50)
    eng = engine_factory()
    try:
        eng.load_pileup(r.pileup)
        eng.load_insseq(off, bases)
        refined = eng.refine(r.loci)
        res, out = eng.poa_consensus(r.loci, refined, cap=4096)
        ins = r.loci["type"] == 1
        done = (res["len"] >= 0)
        assert (done == (ins & (refined["start"] != SVT_NA))).all()   # every refined INS call, nothing else
        ib = ins_base_of(r.pileup)
        prm, pp = eng.params, dict(O.POA_DEFAULTS)
        sub = [i for i in range(min(12000, len(r.loci))) if done[i]]

        def one(i):
            l, R = r.loci[i], int(refined["start"][i])
            s = (int(l["pos"]) - prm.median_interval) & 0xFFFFFFFF
            e = (int(l["pos"]) + prm.median_interval) & 0xFFFFFFFF
            idx = O.poa_support(r.pileup, ib, int(l["chrom"]), s, e, R, cap=pp["max_support"])
            want, used = O.poa_consensus([bases[off[k]:off[k + 1]] for k in idx])
            ok = (res["n_used"][i] == used and res["len"][i] == len(want) and
                  np.array_equal(out[i, :min(len(want), 4096)], want[:4096]))
            return i, ok

        with ThreadPoolExecutor(16) as ex:
            bad = [i for i, ok in ex.map(one, sub) if not ok]
        assert not bad, f"{len(bad)} of {len(sub)} INS consensus differ, first locus {bad[0]}"
        assert len(sub) >= 5000
        print(f"cfg3 POA: {int(done.sum())} INS consensus on the GPU, {len(sub)} checked", file=sys.stderr)
    finally:
        eng.close()
