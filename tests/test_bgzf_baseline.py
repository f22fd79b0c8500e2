"""The reference-shaped CPU baseline (oracle/bgzf_ref.c: per-thread BAM handle + BAI,
per-query linear-index seek + BGZF inflate + record decode) gives the in-memory oracle's
results, and the BAI written by the synthetic BAM writer is a valid linear index."""
import struct

import numpy as np
import oracle_ffi as O
import pytest

from svtrek_amd import Params, sim


def _bai_linear(path):
    b = open(path, "rb").read()
    assert b[:4] == b"BAI\x01"
    (n_ref,) = struct.unpack_from("<i", b, 4)
    o, lin = 8, []
    for _ in range(n_ref):
        (n_bin,) = struct.unpack_from("<i", b, o)
        o += 4
        for _ in range(n_bin):
            _, n_chunk = struct.unpack_from("<Ii", b, o)
            o += 8 + 16 * n_chunk
        (n_intv,) = struct.unpack_from("<i", b, o)
        o += 4
        lin.append(struct.unpack_from(f"<{n_intv}Q", b, o))
        o += 8 * n_intv
    return lin


@pytest.mark.parametrize("with_seq,threads", [(False, 1), (True, 3)])
def test_bgzf_leg_matches_oracle(tmp_path, with_seq, threads):
    cfg = sim.SimConfig(seed=21, n_targets=3, n_loci=240, del_frac=0.5, coverage=12.0, p_clip_ends=0.3)
    r = sim.generate(cfg, keep_handle=True)
    bam = str(tmp_path / "a.bam")
    sim.write_bam(r, bam, with_seq=with_seq, level=1)
    lin = _bai_linear(bam + ".bai")
    assert len(lin) == 3 and all(len(x) > 0 for x in lin)
    assert all(list(x) == sorted(x) for x in lin)          # monotone in a sorted file
    loci = r.loci.copy()
    loci[::17]["chrom"] = 9                                 # a contig the BAM does not have: no reads
    want = O.refine_batch(r.pileup, loci)
    got, st = O.bgzf_refine_batch(bam, loci, threads=threads, with_stats=True)
    assert np.array_equal(got["start"], want["start"]) and np.array_equal(got["end"], want["end"])
    assert st["records_decoded"] > 0 and st["bytes_inflated"] > 0


def test_bgzf_leg_region_sample(tmp_path):
    """A region BAM (the bench sample) answers the sample's queries like the full pileup."""
    import bgzf_baseline as BB
    cfg = sim.SimConfig(seed=22, n_targets=2, n_loci=200, del_frac=0.5, coverage=10.0)
    r = sim.generate(cfg, keep_handle=True)
    out = BB.run(r, r.loci, n_threads=2, budget_s=0.3, params=Params(), k=40)
    assert out["value_bgzf"] > 0 and out["value_bgzf_1thread"] > 0
    assert "first 40 loci" in out["bgzf_sample"]
