"""svt_bgzf_inflate on the device: BGZF blocks inflated one wave per block
(svt_inflate.inc), byte-identical to zlib -- a BAM with SEQ/QUAL written by the simulator's BGZF
writer, and raw DEFLATE streams of every block type (stored / fixed / dynamic), zlib level and
strategy, data kind (tests/deflate_streams.py) and byte alignment of input and output, mixed in
one batch; corrupt streams (truncated, wrong ISIZE, reserved block type, codes zlib rejects) are
reported by block index; the CPU backend (zlib) behind the same ABI agrees."""
import ctypes as C
import os
import random
import zlib

import numpy as np
import pytest

import deflate_streams as D
from svtrek_amd import Engine, Params, sim
from svtrek_amd._lib import BGZF_BLOCK_DTYPE, bind_abi
from svtrek_amd.bgzf import block_table

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _zlib_all(comp: bytes, blocks: np.ndarray) -> bytes:
    return b"".join(zlib.decompress(comp[int(b["coff"]):int(b["coff"]) + int(b["clen"])], -15) for b in blocks)


def test_inflate_sim_bam(engine_factory, tmp_path):
    cfg = sim.SimConfig(seed=9, n_targets=2, n_loci=40, del_frac=0.5, coverage=6.0)
    r = sim.generate(cfg, keep_handle=True)
    path = str(tmp_path / "s.bam")
    sim.write_bam(r, path, with_seq=True, level=1)
    comp = open(path, "rb").read()
    blocks = block_table(comp)
    eng = engine_factory()
    got = eng.bgzf_inflate(comp, blocks)
    assert got.tobytes() == _zlib_all(comp, blocks)
    assert len(blocks) > 50 and eng.last_inflate_ms() > 0


def _batch(streams, rng, out_skew=False):
    """(comp bytes, block table) for [(compressed, plain)], each at a random input alignment
    (and, with out_skew, a random output gap)."""
    comp, rows, u = bytearray(), [], 0
    for z, d in streams:
        comp += bytes(rng.randint(0, 7))
        rows.append((len(comp), u, len(z), len(d)))
        comp += z
        u += len(d) + (rng.randint(0, 5) if out_skew else 0)
    return bytes(comp), np.array(rows, dtype=BGZF_BLOCK_DTYPE)


def test_inflate_every_kind_level_strategy(engine_factory):
    """Every data kind x zlib level x strategy, at random input / output alignments."""
    rng = random.Random(11)
    streams = []
    for kind in D.KINDS:
        d = D.data(kind, rng)
        for level in (0, 1, 6, 9):
            for strat in D.STRATEGIES:
                streams.append((D.deflate(d, level, strat), d))
    rng.shuffle(streams)
    comp, blocks = _batch(streams, rng, out_skew=True)
    got = engine_factory().bgzf_inflate(comp, blocks)
    for (z, d), b in zip(streams, blocks):
        assert got[int(b["uoff"]):int(b["uoff"]) + len(d)].tobytes() == d, (len(z), len(d))


@pytest.mark.parametrize("case", ["truncated", "isize_small", "isize_large", "reserved", "oversubscribed"])
def test_inflate_rejects_corrupt(engine_factory, case):
    """One bad block among good ones is named by index (as zlib rejects it)."""
    rng = random.Random(5)
    good = [(D.deflate(x, 6, zlib.Z_DEFAULT_STRATEGY), x) for x in (rng.randbytes(3000), b"abc" * 900)]
    d = rng.randbytes(5000) + b"xyz" * 500
    z = D.deflate(d, 6, zlib.Z_DEFAULT_STRATEGY)
    bad = {"truncated": (z[:-3], d), "isize_small": (z, d[:-1]), "isize_large": (z, d + b"!"),
           "reserved": (bytes([0x07]) + z[1:], d),
           "oversubscribed": (D.dynamic_block({8: 1, 1: 2, 2: 2}, [8] * 256 + [1], [1], b"SV"), b"SV")}[case]
    if case == "oversubscribed":   # 256 x 2^-8 + 2^-1 > 1
        assert not D.zlib_ok(*bad[:1], len(bad[1]))
    comp, blocks = _batch(good + [bad] + good, rng)
    with pytest.raises(RuntimeError, match="corrupt BGZF block 2"):
        engine_factory().bgzf_inflate(comp, blocks)


def test_inflate_mixed_streams(engine_factory):
    rng = random.Random(3)
    comp, rows, want = bytearray(), [], []
    u = 0
    for i in range(700):
        kind = i % 5
        n = rng.randint(0, 65536)
        d = (rng.randbytes(n) if kind == 0 else bytes(rng.choice(b"ACGT!#+5") for _ in range(n // 8)) * 8 if kind == 1
             else b"xy" * (n // 2) if kind == 2 else bytes(rng.randrange(33, 74) for _ in range(n // 4)) if kind == 3
             else b"")
        d = d[:65536]
        level = rng.choice([0, 1, 6, 9])
        strat = rng.choice([zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE])
        c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strat)
        z = c.compress(d) + c.flush()
        comp += bytes(rng.randint(0, 5))          # any byte alignment
        rows.append((len(comp), u, len(z), len(d)))
        comp += z
        u += len(d)
        want.append(d)
    blocks = np.array(rows, dtype=BGZF_BLOCK_DTYPE)
    eng = engine_factory()
    assert eng.bgzf_inflate(bytes(comp), blocks).tobytes() == b"".join(want)
    # a corrupt block is named; the others are not trusted either
    bad = bytearray(comp)
    k = 123
    bad[int(blocks[k]["coff"]) + int(blocks[k]["clen"]) // 2] ^= 0x5a
    blocks2 = blocks.copy()
    blocks2[k]["ulen"] += 1 if blocks2[k]["ulen"] < 65536 else -1
    with pytest.raises(RuntimeError, match="corrupt BGZF block 123"):
        eng.bgzf_inflate(bytes(comp), blocks2)
    with pytest.raises(RuntimeError, match="outside its buffers"):
        b3 = blocks.copy()
        b3[5]["clen"] = len(comp)
        eng.bgzf_inflate(bytes(comp), b3)


def test_inflate_cpu_backend_agrees(tmp_path):
    cfg = sim.SimConfig(seed=10, n_targets=1, n_loci=20, del_frac=0.5, coverage=5.0)
    r = sim.generate(cfg, keep_handle=True)
    path = str(tmp_path / "c.bam")
    sim.write_bam(r, path, with_seq=True, level=6)
    comp = open(path, "rb").read()
    blocks = block_table(comp)
    with Engine(Params(), device=0) as g:
        a = g.bgzf_inflate(comp, blocks)
    cpu = Engine(Params(), device=0, lib=bind_abi(C.CDLL(os.path.join(ROOT, "oracle", "libsvtrek_cpu.so"))))
    b = cpu.bgzf_inflate(comp, blocks)
    cpu.close()
    assert a.tobytes() == b.tobytes() == _zlib_all(comp, blocks)


def test_inflate_incomplete_codes_as_zlib(engine_factory):
    """Hand-built dynamic blocks on the device: an incomplete code-length code and
    an incomplete literal/length code are rejected as zlib rejects them (the host path and the
    reference's htslib inflate with zlib), a lone 1-bit distance code is accepted."""
    data = b"SVTrek"
    eng = engine_factory()
    for cl, lit, valid in (({9: 1, 1: 2, 2: 2}, [9] * 256 + [1], True), ({9: 1, 1: 2}, [9] * 256 + [1], False),
                           ({9: 1, 2: 2, 1: 2}, [9] * 256 + [2], False)):
        comp = D.dynamic_block(cl, lit, [1], data)
        assert D.zlib_ok(comp, len(data)) == valid
        blocks = np.array([(3, 0, len(comp), len(data))], dtype=BGZF_BLOCK_DTYPE)
        buf = bytes(3) + comp
        if valid:
            assert eng.bgzf_inflate(buf, blocks).tobytes() == data
        else:
            with pytest.raises(RuntimeError, match="corrupt BGZF block 0"):
                eng.bgzf_inflate(buf, blocks)


def test_inflate_crafted_streams(engine_factory):
    """the edge cases of the vector-side decoder -- matches 1921-2048 bytes back with
    lengths 65-258 (the ring's far edge), every distance class, a stored block after a dynamic block
    ending in a far match (and an empty stored block), outputs ending exactly on a 256-byte chunk,
    literal/length and distance codes of 10-15 bits (past the 9-bit root) -- byte-identical to zlib,
    in one batch at random alignments; and ISIZE off by one either way at a chunk boundary is
    reported as zlib would (the stream does not inflate to its ISIZE)."""
    rng = random.Random(23)
    crafted = D.crafted_streams(random.Random(17))
    for z, d, name in crafted:
        assert zlib.decompressobj(-15).decompress(z) == d, name
    streams = [(z, d) for z, d, _ in crafted] * 3
    rng.shuffle(streams)
    comp, blocks = _batch(streams, rng, out_skew=True)
    eng = engine_factory()
    got = eng.bgzf_inflate(comp, blocks)
    for (z, d), b in zip(streams, blocks):
        assert got[int(b["uoff"]):int(b["uoff"]) + len(d)].tobytes() == d, (len(z), len(d))
    good = [(z, d) for z, d, name in crafted if name == "far_edge"]
    for z, d, name in crafted:
        if not name.startswith("chunk_end_"):
            continue
        for delta in (-1, 1):
            if len(d) + delta > 65536:
                continue
            bad = (z, d[:-1] if delta < 0 else d + b"\0")
            c2, b2 = _batch(good + [bad] + good, rng)
            with pytest.raises(RuntimeError, match="corrupt BGZF block 1"):
                eng.bgzf_inflate(c2, b2)
