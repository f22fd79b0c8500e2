"""The BGZF inflate core (svtrek_amd/csrc/svt_inflate.h) on the host: the same source the
device kernel runs (one lane per block), compiled with g++ and checked byte for byte against
zlib -- every DEFLATE block type (stored, fixed, dynamic), zlib's strategies and levels, data
that compresses well and data that does not (BAM SEQ/QUAL-like), every start alignment of the
block data in its words, and corrupt streams (truncated, wrong ISIZE) rejected."""
import ctypes
import os
import random
import subprocess
import zlib

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def shim(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("inf") / "shim.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra", "-Werror", "-Wno-unknown-pragmas",
                    "-I", os.path.join(ROOT, "svtrek_amd", "csrc"), "-o", out,
                    os.path.join(ROOT, "tests", "native", "inflate_shim.cpp")], check=True)
    return ctypes.CDLL(out)


def _inf(lib, comp: bytes, ulen: int, skip: int):
    buf = ctypes.create_string_buffer(bytes(skip) + comp + bytes(8))   # 16-B aligned base
    out = ctypes.create_string_buffer(max(ulen, 1))
    rc = lib.inf_host(ctypes.byref(buf, skip), len(comp), out, ulen, skip)
    return rc, out.raw[:ulen]


def _data(kind: str, rng: random.Random) -> bytes:
    if kind == "random":
        return rng.randbytes(rng.randint(1, 65280))
    if kind == "words":
        return " ".join(rng.choice(["ACGT", "read", "12345", "CIGAR", "\t"]) for _ in range(12000)).encode()[:65280]
    if kind == "repeat":
        return b"ab" * 32000
    if kind == "qual":   # BAM QUAL-like: ~40 symbols, no long matches
        return bytes(rng.choice(range(33, 74)) for _ in range(65280))
    if kind == "seq":    # 4-bit base pairs
        return bytes(rng.choice([0x11, 0x12, 0x14, 0x18, 0x21, 0x22, 0x24, 0x28, 0x41, 0x44, 0x81, 0x88])
                     for _ in range(40000))
    return b"" if kind == "empty" else b"x"


@pytest.mark.parametrize("kind", ["random", "words", "repeat", "qual", "seq", "empty", "one"])
def test_inflate_matches_zlib(shim, kind):
    rng = random.Random(hash(kind) & 0xffff)
    d = _data(kind, rng)
    for level in (0, 1, 6, 9):
        for strat in (zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE):
            c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strat)
            comp = c.compress(d) + c.flush()
            for skip in (0, 3, 5, 15):
                rc, got = _inf(shim, comp, len(d), skip)
                assert rc == 0 and got == d, (level, strat, skip, rc)


def test_inflate_rejects_corrupt(shim):
    d = random.Random(5).randbytes(5000)
    comp = zlib.compress(d, 6)[2:-4]
    assert _inf(shim, comp[:-3], len(d), 1)[0] != 0      # truncated
    assert _inf(shim, comp, len(d) - 1, 2)[0] != 0       # ISIZE too small
    assert _inf(shim, comp, len(d) + 1, 3)[0] != 0       # ISIZE too large
    bad = bytearray(comp)
    bad[0] = 0x07                                          # reserved block type 3
    assert _inf(shim, bytes(bad), len(d), 0)[0] != 0
