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


# ---- crafted multi-block streams: matches of chosen length / distance, stored blocks
# after compressed ones, literal/length and distance codes longer than the device's 9-bit root
LEN_BASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115,
            131, 163, 195, 227, 258]
LEN_EXTRA = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DIST_BASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537,
             2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577]
DIST_EXTRA = [0, 0, 0, 0] + [k for k in range(1, 14) for _ in range(2)]


class BitWriter:
    def __init__(self):
        self.bits: list[int] = []

    def put(self, v: int, n: int):        # an n-bit field, LSB first
        self.bits.extend((v >> i) & 1 for i in range(n))

    def put_code(self, code: int, n: int):  # a Huffman code, MSB first
        self.bits.extend((code >> (n - 1 - i)) & 1 for i in range(n))

    def align(self):
        self.bits += [0] * (-len(self.bits) % 8)

    def bytes(self) -> bytes:
        b = self.bits + [0] * (-len(self.bits) % 8)
        return bytes(sum(b[i + k] << k for k in range(8)) for i in range(0, len(b), 8))


def skewed_lengths(n_sym: int, symbols: list[int], k: int) -> list[int]:
    """A complete code over `symbols` (of an alphabet of n_sym): the first k get lengths 1..k, the
    rest share the remaining 2^-k at lengths L and L + 1 (Kraft sum exactly 1), so most codes are
    long.  Needs len(symbols) - k >= 1 and L + 1 <= 15."""
    lens = [0] * n_sym
    head, rest = symbols[:k], symbols[k:]
    for i, s in enumerate(head):
        lens[s] = i + 1
    m = len(rest)
    L = k + m.bit_length() - 1                 # 2^(L-k) <= m < 2^(L-k+1)
    a = 2 ** (L + 1 - k) - m                   # symbols at length L, the others at L + 1
    assert 0 <= a <= m and L + (a < m) <= 15, (m, k, L)
    for i, s in enumerate(rest):
        lens[s] = L if i < a else L + 1
    assert sum(2.0 ** -x for x in lens if x) == 1.0
    return lens


def len_sym(n: int) -> tuple[int, int, int]:
    i = max(j for j in range(29) if LEN_BASE[j] <= n)
    return 257 + i, n - LEN_BASE[i], LEN_EXTRA[i]


def dist_sym(d: int) -> tuple[int, int, int]:
    i = max(j for j in range(30) if DIST_BASE[j] <= d)
    return i, d - DIST_BASE[i], DIST_EXTRA[i]


def write_dynamic(bw: BitWriter, syms: list, final: bool, k_lit: int = 3, k_dist: int = 2) -> None:
    """One dynamic block of `syms` (ints = literals, (length, distance) = matches), with skewed
    codes over exactly the symbols used (plus end-of-block and two spare distance codes)."""
    lit_used = sorted({s for s in syms if isinstance(s, int)} | {len_sym(m[0])[0] for m in syms if not isinstance(m, int)}
                      | {256})
    dist_used = sorted({dist_sym(m[1])[0] for m in syms if not isinstance(m, int)} | {0, 29})
    k_lit = min(k_lit, len(lit_used) - 1)
    k_dist = min(k_dist, len(dist_used) - 1)
    lit_len = skewed_lengths(286, lit_used, k_lit)
    dist_len = skewed_lengths(30, dist_used, k_dist)
    nl = max(s for s in range(286) if lit_len[s]) + 1
    nd = max(s for s in range(30) if dist_len[s]) + 1
    lit_len, dist_len = lit_len[:max(nl, 257)], dist_len[:nd]
    bw.put(1 if final else 0, 1)
    bw.put(2, 2)
    bw.put(len(lit_len) - 257, 5)
    bw.put(len(dist_len) - 1, 5)
    order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
    bw.put(19 - 4, 4)
    cl_len = [4 if s < 16 else 0 for s in range(19)]   # 16 symbols of 4 bits: complete, no run codes
    for s in order:
        bw.put(cl_len[s], 3)
    clc = canonical(cl_len)
    for n in lit_len + dist_len:
        bw.put_code(*clc[n])
    lc, dc = canonical(lit_len), canonical(dist_len)
    for s in syms:
        if isinstance(s, int):
            bw.put_code(*lc[s])
        else:
            ls, lx, ln = len_sym(s[0])
            bw.put_code(*lc[ls])
            bw.put(lx, ln)
            ds, dx, dn = dist_sym(s[1])
            bw.put_code(*dc[ds])
            bw.put(dx, dn)
    bw.put_code(*lc[256])


def write_stored(bw: BitWriter, data: bytes, final: bool) -> None:
    bw.put(1 if final else 0, 1)
    bw.put(0, 2)
    bw.align()
    bw.put(len(data), 16)
    bw.put(len(data) ^ 0xffff, 16)
    for b in data:
        bw.put(b, 8)


def lz_expand(syms: list, out: bytearray) -> None:
    for s in syms:
        if isinstance(s, int):
            out.append(s)
        else:
            n, d = s
            assert 1 <= d <= len(out)
            for _ in range(n):
                out.append(out[-d])


def crafted_streams(rng: random.Random) -> list[tuple[bytes, bytes, str]]:
    """(raw DEFLATE, plain, name) for the cases ADVICE r05 lists."""
    out = []

    def stream(blocks, name):   # blocks: [("dyn", syms) | ("stored", bytes)], the last is final
        bw, plain = BitWriter(), bytearray()
        for i, (kind, x) in enumerate(blocks):
            fin = i == len(blocks) - 1
            if kind == "dyn":
                write_dynamic(bw, x, fin)
                lz_expand(x, plain)
            else:
                write_stored(bw, x, fin)
                plain += x
        out.append((bw.bytes(), bytes(plain), name))

    def lits(n):
        return [rng.randrange(256) for _ in range(n)]

    # matches reaching back 1921..2048 bytes (the far edge of a 2 KiB ring) with lengths 65..258
    syms = lits(2100)
    for _ in range(150):
        syms.append((rng.randint(65, 258), rng.randint(1921, 2048)))
        syms += lits(rng.randint(0, 3))
    stream([("dyn", syms)], "far_edge")
    # every distance class, long lengths, many literals in between
    syms, n = lits(32800), 32800
    while True:
        ln, k = rng.choice([3, 64, 65, 66, 130, 257, 258]), rng.randint(0, 40)
        if n + ln + k > 65536:
            break
        syms.append((ln, rng.randint(1, 32768)))
        syms += lits(k)
        n += ln + k
    stream([("dyn", syms)], "all_distances")
    # a stored block right after a dynamic block that ends in a far match, then more matches
    syms = lits(5000) + [(258, 4097), (200, 3000)]
    syms2 = [(100, 2500), (258, 5555)] + lits(10)
    stream([("dyn", syms), ("stored", bytes(rng.randbytes(777))), ("dyn", syms2)], "stored_after_far")
    stream([("dyn", lits(300) + [(258, 299)]), ("stored", b""), ("stored", rng.randbytes(40))], "stored_empty")
    # outputs ending exactly on 256-byte chunk boundaries (a match overrunning into the next chunk
    # would be caught only at the chunk's store)
    for total in (256, 4096, 65536):
        syms, n = lits(200), 200
        while n < total:
            ln = min(258, total - n)
            if ln < 3:
                syms += lits(ln)
                n += ln
                break
            syms.append((ln, rng.randint(1, min(n, 32768))))
            n += ln
        stream([("dyn", syms)], f"chunk_end_{total}")
    # a literal-heavy block whose codes are all long (literals at 14-15 bits)
    stream([("dyn", lits(20000))], "long_literals")
    return out
