"""Raw DEFLATE test streams for the device inflater (tests/test_gpu_inflate.py): data of every
kind BAM blocks hold (SEQ/QUAL-like, text, runs, incompressible), zlib streams of every level and
strategy, and dynamic blocks written bit by bit with chosen code lengths (incomplete and
over-subscribed codes, which only a hand-built stream contains)."""
import random
import zlib

KINDS = ["random", "words", "repeat", "qual", "seq", "periods", "empty", "one"]
STRATEGIES = (zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE)


def data(kind: str, rng: random.Random) -> bytes:
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
    if kind == "periods":  # runs repeating with every period 1..300: matches of every distance < length
        out = bytearray()
        while len(out) < 60000:
            p = rng.choice([1, 2, 3, 4, 7, 8, 63, 64, 65, 127, 128, 129, 200, 258, 259, 300])
            out += rng.randbytes(p) * rng.randint(2, 12)
        return bytes(out[:65280])
    return b"" if kind == "empty" else b"x"


def canonical(lengths: list[int]) -> dict[int, tuple[int, int]]:
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


def dynamic_block(cl_len: dict[int, int], lit_len: list[int], dist_len: list[int], data: bytes) -> bytes:
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
    clc = canonical([cl_len.get(s, 0) for s in range(19)])
    for n in lit_len + dist_len:
        put_code(*clc[n])
    lc = canonical(lit_len)
    for b in data:
        put_code(*lc[b])
    put_code(*lc[256])
    bits += [0] * (-len(bits) % 8)
    return bytes(sum(bits[i + k] << k for k in range(8)) for i in range(0, len(bits), 8))


def zlib_ok(comp: bytes, n: int) -> bool:
    try:
        return len(zlib.decompressobj(-15).decompress(comp)) == n
    except zlib.error:
        return False


def deflate(d: bytes, level: int, strategy: int) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
    return c.compress(d) + c.flush()
