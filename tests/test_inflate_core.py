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


def _canonical(lengths: list[int]) -> dict[int, tuple[int, int]]:
    """RFC 1951 3.2.2: symbol -> (code, length) for the non-zero lengths."""
    bl = [0] * 16
    for n in lengths:
        if n:
            bl[n] += 1
    code, nxt = 0, [0] * 16
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    out = {}
    for s, n in enumerate(lengths):
        if n:
            out[s] = (nxt[n], n)
            nxt[n] += 1
    return out


def _dynamic_block(cl_len: dict[int, int], lit_len: list[int], dist_len: list[int], data: bytes) -> bytes:
    """One final dynamic-Huffman DEFLATE block written bit by bit (codes MSB-first, RFC 1951)."""
    bits: list[int] = []

    def put(v: int, n: int):          # an n-bit field, LSB first
        bits.extend((v >> i) & 1 for i in range(n))

    def put_code(code: int, n: int):  # a Huffman code, MSB first
        bits.extend((code >> (n - 1 - i)) & 1 for i in range(n))

    order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
    put(1, 1)
    put(2, 2)
    put(len(lit_len) - 257, 5)
    put(len(dist_len) - 1, 5)
    put(19 - 4, 4)
    for s in order:
        put(cl_len.get(s, 0), 3)
    clc = _canonical([cl_len.get(s, 0) for s in range(19)])
    for n in lit_len + dist_len:
        put_code(*clc[n])
    lc = _canonical(lit_len)
    for b in data:
        put_code(*lc[b])
    put_code(*lc[256])
    bits += [0] * (-len(bits) % 8)
    return bytes(sum(bits[i + k] << k for k in range(8)) for i in range(0, len(bits), 8))


def _zlib_ok(comp: bytes, n: int) -> bool:
    try:
        return len(zlib.decompressobj(-15).decompress(comp)) == n
    except zlib.error:
        return False


def test_inflate_incomplete_codes_as_zlib(shim):
    """zlib's inflate_table rules for incomplete Huffman codes (inftrees.c), which the host path
    (zlib / libdeflate) and the reference's htslib apply: an incomplete code-length code is
    rejected, an incomplete literal/length code is rejected, a single distance code of length 1
    is accepted.  The GPU inflater (the same svt_inflate.h source) must agree on each."""
    data = b"SVTrek"
    lit_ok = [9] * 256 + [1]             # 256 x 2^-9 + 2^-1: complete
    lit_short = [9] * 256 + [2]          # 0.75: incomplete, longest code 9
    cases = [
        ({9: 1, 1: 2, 2: 2}, lit_ok, [1], True),     # complete CL code, one 1-bit distance code: valid
        ({9: 1, 1: 2}, lit_ok, [1], False),          # CL code incomplete (3/4)
        ({9: 1, 2: 2, 1: 2}, lit_short, [1], False),  # literal/length code incomplete
    ]
    for cl, lit, dist, valid in cases:
        comp = _dynamic_block(cl, lit, dist, data)
        assert _zlib_ok(comp, len(data)) == valid, (cl, valid)
        for skip in (0, 7):
            rc, got = _inf(shim, comp, len(data), skip)
            assert (rc == 0 and got == data) == valid, (cl, skip, rc)
