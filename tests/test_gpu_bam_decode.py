"""BAM records decoded on the device (svt_bam_dec_*, svt_bam.inc): the BGZF blocks
go to the GPU compressed, are inflated and their records found (guessed per 64 KiB chunk, proven
on the block_size chain), parsed (CG:B,I restored) and appended to the device pileup.  The loaded
pileup must be the host ingest's (svth_bam_read): same refined results, same index, same
reference work -- for the edge-case fixtures (tests/bamfix.py), simulated BAMs with SEQ/QUAL and
CG tags, batches of any size (records and BGZF blocks split across them), unsorted input; corrupt
and truncated files are errors."""
import numpy as np
import oracle_ffi as O
import pytest

import bamfix
from svtrek_amd import Params, SvtError, host, make_loci, sim

pytestmark = pytest.mark.gpu


def _loci(rng, n_ref, n=400, span=200000):
    return make_loci([(int(rng.choice([1, 2])), int(rng.integers(1, n_ref + 1)), int(p), int(p) + int(d))
                      for p, d in zip(rng.integers(0, span, n), rng.integers(51, 5000, n))])


def _same_as_host(engine_factory, path, loci, batch_bytes=0, pinned=True, params=None):
    pl, info = host.read_bam(path, threads=2)
    dev = engine_factory(params)
    st = host.load_bam_device(dev, path, threads=2, batch_bytes=batch_bytes, pinned=pinned)
    ref = engine_factory(params)
    ref.load_pileup(pl)
    assert st["reads"] == len(pl.pos) and st["records"] == info["records"]
    assert st["cg_restored"] == info["cg_restored"]
    assert dev.load_stats()["span_events"] == ref.load_stats()["span_events"]
    got = dev.refine(loci)
    np.testing.assert_array_equal(got, O.refine_batch(pl, loci, params))
    wd, wr = dev.count_work(loci), ref.count_work(loci)
    assert (wd["reads"], wd["ops_walked"], wd["candidates"]) == (wr["reads"], wr["ops_walked"], wr["candidates"])
    return st


@pytest.mark.parametrize("batch_kb", [0, 256, 64, 9])
def test_fixture_any_batch_size(engine_factory, tmp_path, batch_kb):
    path = str(tmp_path / "f.bam")
    recs, n_ref = bamfix.write(path, seed=21 + batch_kb)
    st = _same_as_host(engine_factory, path, _loci(np.random.default_rng(batch_kb), n_ref), batch_bytes=batch_kb << 10,
                       pinned=batch_kb != 64)
    assert st["batches"] >= (1 if batch_kb == 0 else 3)


def test_sim_bam_with_seq_and_split_reads(engine_factory, tmp_path):
    cfg = sim.SimConfig(seed=31, n_targets=3, n_loci=300, del_frac=0.5, coverage=15, p_clip_ends=0.3, p_exotic=0.05)
    r = sim.generate(cfg, keep_handle=True)
    path = str(tmp_path / "s.bam")
    sim.write_bam(r, path, with_seq=True, level=1)
    st = _same_as_host(engine_factory, path, r.loci, batch_bytes=4 << 20)
    assert st["batches"] >= 2


def test_long_cigars_from_cg_tags(engine_factory, tmp_path):
    """> 65535 CIGAR ops stored as kSmN + CG:B,I (the records span many 64 KiB chunks and batches)."""
    cfg = sim.SimConfig(seed=8, n_targets=1, n_loci=4, coverage=2.0, read_len_mean=200000, read_len_sd=0,
                        read_len_min=150000, rho=1.5, spacing=400000)
    r = sim.generate(cfg, keep_handle=True)
    path = str(tmp_path / "long.bam")
    sim.write_bam(r, path, with_seq=True)
    st = _same_as_host(engine_factory, path, r.loci, batch_bytes=1 << 20)
    assert st["cg_restored"] == int((np.diff(r.pileup.cig_off.astype(np.int64)) > 65535).sum()) > 0


def test_unsorted_bam_is_sorted(engine_factory, tmp_path):
    raw, recs = bamfix.make_bam(seed=7, n_reads=800, unplaced=5)
    # swap two records of contig 1: the file is no longer coordinate-sorted
    hdr_len = len(raw) - sum(len(r["raw"]) for r in recs)
    body = [r["raw"] for r in recs]
    body[10], body[500] = body[500], body[10]
    path = str(tmp_path / "u.bam")
    with open(path, "wb") as f:
        f.write(bamfix.bgzf_blocks(raw[:hdr_len] + b"".join(body)))
    _same_as_host(engine_factory, path, _loci(np.random.default_rng(7), 3))


def test_corrupt_and_truncated(engine_factory, tmp_path):
    raw, recs = bamfix.make_bam(seed=9, n_reads=300, unplaced=0)
    hdr_len = len(raw) - sum(len(r["raw"]) for r in recs)
    bad = bytearray(raw)
    at = hdr_len + sum(len(r["raw"]) for r in recs[:100])
    bad[at:at + 4] = (20).to_bytes(4, "little")        # block_size < 32
    p1 = str(tmp_path / "bad.bam")
    with open(p1, "wb") as f:
        f.write(bamfix.bgzf_blocks(bytes(bad)))
    with pytest.raises((OSError, SvtError), match="corrupt BAM record"):   # (a feed error: the reader's OSError)
        host.load_bam_device(engine_factory(), p1)
    p2 = str(tmp_path / "trunc.bam")
    with open(p2, "wb") as f:
        f.write(bamfix.bgzf_blocks(raw[:len(raw) - 17]))
    with pytest.raises(SvtError, match="truncated"):
        host.load_bam_device(engine_factory(), p2)


def test_params_and_empty_file(engine_factory, tmp_path):
    raw, recs = bamfix.make_bam(seed=13, n_reads=0, unplaced=3)
    path = str(tmp_path / "e.bam")
    with open(path, "wb") as f:
        f.write(bamfix.bgzf_blocks(raw))
    eng = engine_factory()
    st = host.load_bam_device(eng, path)
    assert st["reads"] == 0 and st["records"] == 3
    got = eng.refine(make_loci([(2, 1, 100000, 101000)]))
    assert int(got["start"][0]) == 0xFFFFFFFF
    # a header and no record at all: the decode never allocates a stream, load must still work
    raw0, _ = bamfix.make_bam(seed=14, n_reads=0, unplaced=0)
    path0 = str(tmp_path / "h.bam")
    with open(path0, "wb") as f:
        f.write(bamfix.bgzf_blocks(raw0))
    eng0 = engine_factory()
    st0 = host.load_bam_device(eng0, path0)
    assert st0["reads"] == 0 and st0["records"] == 0
    got0 = eng0.refine(make_loci([(2, 1, 100000, 101000), (1, 2, 500, 0)]))
    assert (got0["start"] == 0xFFFFFFFF).all() and (got0["end"] == 0xFFFFFFFF).all()
    path2 = str(tmp_path / "p.bam")
    recs, n_ref = bamfix.write(path2, seed=17)
    _same_as_host(engine_factory, path2, _loci(np.random.default_rng(17), n_ref),
                  params=Params(wider_interval=3000, narrow_interval=100, consensus_min_count=1))


def test_wrong_guess_rechains_from_the_failing_chunk(engine_factory, tmp_path):
    """A record whose aux array holds copies of another record makes the chunks inside it guess
    a start that is not on the chain: the proof fails there and the batch is re-chained hop by
    hop from that chunk on, with the host parse's result."""
    import random
    import struct
    raw, recs = bamfix.make_bam(seed=41, n_reads=4000, unplaced=0)
    hdr_len = len(raw) - sum(len(r["raw"]) for r in recs)
    rng = random.Random(5)
    k = len(recs) // 2
    fake = recs[3]["raw"]
    payload = fake * (200000 // len(fake) + 1)
    aux = b"XBBC" + struct.pack("<I", len(payload)) + payload
    big = bamfix.record(recs[k]["tid"], recs[k]["pos"], b"giant", [(0, 500)], 0, 500, aux, False, rng)
    body = b"".join(r["raw"] for r in recs[:k]) + big + b"".join(r["raw"] for r in recs[k:])
    path = str(tmp_path / "g.bam")
    with open(path, "wb") as f:
        f.write(bamfix.bgzf_blocks(raw[:hdr_len] + body))
    st = _same_as_host(engine_factory, path, _loci(np.random.default_rng(41), 3))
    n_chunks = (len(body) + 65535) // 65536
    assert st["rechained"] == 1 and 0 < st["rechained_chunks"] < n_chunks


@pytest.mark.parametrize("which", ["middle", "last"])
def test_corrupt_block_reported_by_the_pipelined_feed(engine_factory, tmp_path, which):
    """svt_bam_dec_feed is pipelined one batch deep: a batch's inflate error is found by the call
    that decodes it (the next feed, or svt_bam_dec_load for the last batch).  A block whose ISIZE
    claims one byte more than its DEFLATE data holds must fail the load either way."""
    import struct
    raw, recs = bamfix.make_bam(seed=23, n_reads=3000, unplaced=0)
    data = bytearray(bamfix.bgzf_blocks(raw))
    starts, p = [], 0
    while p + 18 <= len(data):   # BGZF members: BSIZE at offset 16
        starts.append(p)
        p += struct.unpack_from("<H", data, p + 16)[0] + 1
    assert p == len(data) and len(starts) >= 6
    b = starts[len(starts) // 2] if which == "middle" else starts[-2]   # (starts[-1]: the EOF block)
    end = b + struct.unpack_from("<H", data, b + 16)[0] + 1
    isize = struct.unpack_from("<I", data, end - 4)[0]
    struct.pack_into("<I", data, end - 4, isize + 1)
    path = str(tmp_path / f"c_{which}.bam")
    with open(path, "wb") as f:
        f.write(bytes(data))
    with pytest.raises((OSError, SvtError), match="corrupt"):
        host.load_bam_device(engine_factory(), path, batch_bytes=64 << 10)
