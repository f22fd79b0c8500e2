"""CPU checks of the allele-consensus (POA) oracle and its test data.

The reference never calls abPOA (Makefile:16; abPOA is an empty submodule), so the POA mode
has no reference behaviour: these tests pin the oracle's own properties (the GPU kernel is
checked against it in test_gpu_poa.py).  Parity unpinned by the reference.
"""
import difflib

import numpy as np
import oracle_ffi as O
import pytest

from svtrek_amd import sim


def noisy(rng, a, p):
    out = []
    for b in a:
        u = rng.random()
        if u < p / 3:
            continue
        if u < 2 * p / 3:
            out.append(int(rng.integers(0, 4)))
            out.append(int(b))
            continue
        if u < p:
            out.append(int((b + 1 + rng.integers(0, 3)) % 4))
            continue
        out.append(int(b))
    return np.array(out, np.uint8)


def identity(a, b):
    sm = difflib.SequenceMatcher(None, a.tolist(), b.tolist(), autojunk=False)
    return sum(t.size for t in sm.get_matching_blocks()) / max(len(a), len(b), 1)


def test_single_and_identical_sequences():
    rng = np.random.default_rng(0)
    a = rng.integers(0, 4, 137).astype(np.uint8)
    c, used = O.poa_consensus([a])
    assert used == 1 and np.array_equal(c, a)
    c, used = O.poa_consensus([a, a, a, a])
    assert used == 4 and np.array_equal(c, a)
    c, used = O.poa_consensus([])
    assert used == 0 and len(c) == 0


@pytest.mark.parametrize("length,err,n", [(60, 0.05, 9), (400, 0.08, 20), (1500, 0.06, 30)])
def test_noisy_copies_recover_the_allele(length, err, n):
    rng = np.random.default_rng(length)
    a = rng.integers(0, 4, length).astype(np.uint8)
    seqs = [noisy(rng, a, err) for _ in range(n)]
    c, used = O.poa_consensus(seqs)
    assert used >= n - 2
    assert identity(c, a) >= 0.995
    assert identity(c, a) > max(identity(s, a) for s in seqs[:5])


def test_max_seqs_and_node_cap():
    rng = np.random.default_rng(3)
    a = rng.integers(0, 4, 300).astype(np.uint8)
    seqs = [noisy(rng, a, 0.05) for _ in range(12)]
    _, used = O.poa_consensus(seqs, max_seqs=5)
    assert used == 5
    # a sequence that would exceed max_nodes is skipped (the first one always fits)
    _, used = O.poa_consensus(seqs, max_nodes=600)
    assert 1 <= used < 12


def test_sim_insertion_sequences_follow_the_cigars():
    cfg = sim.SimConfig(seed=5, n_targets=2, n_loci=40, del_frac=0.0, coverage=12, sv_max_len=800)
    r = sim.generate(cfg, keep_handle=True)
    off, bases = sim.insertion_sequences(r, cfg, err_permille=40)
    pl = r.pileup
    ops = pl.cigar & 15
    lens = pl.cigar >> 4
    ins = (ops == 1) & (lens >= 50)
    assert len(off) - 1 == int(ins.sum())
    assert np.array_equal(np.diff(off), lens[ins].astype(np.uint64))
    assert bases.max() <= 3
    # reads carrying the same INS allele agree closely (substitutions only)
    first = {}
    same = 0
    for k in range(len(off) - 1):
        s = bases[off[k]:off[k + 1]]
        key = len(s)
        if key in first and len(first[key]) == len(s):
            if np.mean(first[key] == s) > 0.85:
                same += 1
        else:
            first[key] = s
    assert same > 0


@pytest.mark.parametrize("seed", range(6))
def test_oracle_matches_python_restatement(seed):
    """The C oracle and tests/poa_ref.py (written independently from the same spec) agree
    bit-exactly, including the graph order rule (aligned groups kept contiguous)."""
    from poa_ref import poa_consensus as ref
    rng = np.random.default_rng(100 + seed)
    length = int(rng.choice([40, 90, 200]))
    a = rng.integers(0, 4, length).astype(np.uint8)
    seqs = [noisy(rng, a, float(rng.choice([0.05, 0.12, 0.25]))) for _ in range(int(rng.integers(2, 9)))]
    kw = dict(band_b=int(rng.choice([6, 10, 20])))
    c, used = O.poa_consensus(seqs, **kw)
    want, wused = ref([s.tolist() for s in seqs], **kw)
    assert used == wused
    assert c.tolist() == want
