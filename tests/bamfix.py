"""Edge-case BAM fixtures written from scratch (SAM spec 4.2 records in BGZF blocks), independent
of the simulator's writer: records with tid -1 (unplaced), unmapped-but-placed reads (flag 4),
empty CIGARs, CIGARs moved to a CG:B,I tag (the kSmN placeholder htslib's bam_tag2cigar
restores), read names of every length mod 4, aux fields of every type before and after CG.
`expected_pileup` states what an ingest must produce from them (the records a tid >= 0 region
query can yield, htslib bam_endpos, the soft-clip test bits refinement.c:120/:210 read)."""
from __future__ import annotations

import random
import struct
import zlib

import numpy as np

OPS = "MIDNSHP=X"


def bgzf_blocks(data: bytes, block: int = 65280, level: int = 6) -> bytes:
    """BGZF: gzip members of <= 64 KiB each with the BC extra field, then the EOF block."""
    out = bytearray()
    for i in range(0, len(data), block):
        chunk = data[i:i + block]
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        cdata = c.compress(chunk) + c.flush()
        bsize = 12 + 6 + len(cdata) + 8
        out += struct.pack("<BBBBIBBH", 31, 139, 8, 4, 0, 0, 255, 6) + struct.pack("<BBHH", 66, 67, 2, bsize - 1)
        out += cdata + struct.pack("<II", zlib.crc32(chunk) & 0xffffffff, len(chunk))
    out += bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    return bytes(out)


def _aux(rng: random.Random) -> bytes:
    out = b""
    for _ in range(rng.randint(0, 3)):
        t = rng.choice("AcCsSiIfZHB")
        tag = bytes(rng.choice(b"ABXYZ") for _ in range(2))
        if t == "A":
            out += tag + b"A" + b"Q"
        elif t in "cC":
            out += tag + t.encode() + bytes([rng.randrange(256)])
        elif t in "sS":
            out += tag + t.encode() + struct.pack("<H", rng.randrange(65536))
        elif t in "iIf":
            out += tag + t.encode() + struct.pack("<I", rng.randrange(1 << 32))
        elif t in "ZH":
            out += tag + t.encode() + bytes(rng.choice(b"0123456789ABCDEF") for _ in range(rng.randint(0, 9))) + b"\0"
        else:
            sub = rng.choice("cCsSiIf")
            n = rng.randint(0, 5)
            es = {"c": 1, "C": 1, "s": 2, "S": 2, "i": 4, "I": 4, "f": 4}[sub]
            out += tag + b"B" + sub.encode() + struct.pack("<I", n) + bytes(rng.randrange(256) for _ in range(n * es))
    return out


def record(tid: int, pos: int, name: bytes, ops: list[tuple[int, int]], flag: int, l_seq: int, aux: bytes,
           cg: bool, rng: random.Random) -> bytes:
    """One BAM record (with its block_size); cg: the CIGAR moved to a CG:B,I tag and the record
    carrying the placeholder <l_seq>S<reflen>N (htslib's layout for > 65535 ops)."""
    cig = [ln << 4 | op for op, ln in ops]
    if cg:
        rlen = sum(ln for op, ln in ops if op in (0, 2, 3, 7, 8))
        stored = [l_seq << 4 | 4, max(rlen, 1) << 4 | 3]
        aux = aux + b"CGBI" + struct.pack("<I", len(cig)) + struct.pack(f"<{len(cig)}I", *cig) + _aux(rng)
    else:
        stored = cig
    qn = name + b"\0"
    body = struct.pack("<iiBBHHHiiii", tid, pos, len(qn), 60, 4680, len(stored), flag, l_seq, -1, -1, 0)
    body += qn + struct.pack(f"<{len(stored)}I", *stored)
    body += bytes(rng.randrange(256) for _ in range((l_seq + 1) // 2)) + bytes(rng.randrange(33, 74) for _ in range(l_seq))
    body += aux
    return struct.pack("<i", len(body)) + body


def make_bam(seed: int, n_reads: int = 3000, n_ref: int = 3, unplaced: int = 40, seq: bool = True):
    """(BAM bytes, the records as written: list of dicts) -- coordinate-sorted, unplaced last."""
    rng = random.Random(seed)
    recs = []
    for _ in range(n_reads):
        tid = rng.randrange(n_ref)
        pos = rng.randrange(0, 200000)
        kind = rng.random()
        if kind < 0.05:
            ops = []
        else:
            ops = [(rng.choice([0, 0, 0, 1, 2, 4, 5, 7, 8, 3]), rng.randint(1, 120)) for _ in range(rng.randint(1, 40))]
            if rng.random() < 0.3:
                ops = [(4, rng.randint(1, 300))] + ops
            if rng.random() < 0.3:
                ops = ops + [(4, rng.randint(1, 300))]
        l_seq = sum(ln for op, ln in ops if op in (0, 1, 4, 7, 8)) if seq else 0
        flag = rng.choice([0, 16, 256, 2048, 4, 1024])
        cg = bool(ops) and rng.random() < 0.1 and l_seq > 0
        name = bytes(rng.choice(b"ACGTNacgt0123456789:_") for _ in range(rng.randint(1, 40)))
        recs.append(dict(tid=tid, pos=pos, ops=ops, flag=flag, l_seq=l_seq, cg=cg, name=name, aux=_aux(rng)))
    recs.sort(key=lambda r: (r["tid"], r["pos"]))
    for _ in range(unplaced):   # unplaced unmapped reads: tid -1, pos -1, at the end of the file
        recs.append(dict(tid=-1, pos=-1, ops=[], flag=4, l_seq=rng.randint(0, 50) if seq else 0, cg=False,
                         name=b"u%d" % rng.randrange(10 ** 6), aux=_aux(rng)))
    text = b"@HD\tVN:1.6\tSO:coordinate\n" + b"".join(b"@SQ\tSN:%d\tLN:1000000\n" % (t + 1) for t in range(n_ref))
    hdr = b"BAM\1" + struct.pack("<i", len(text)) + text + struct.pack("<i", n_ref)
    for t in range(n_ref):
        nm = b"%d\0" % (t + 1)
        hdr += struct.pack("<i", len(nm)) + nm + struct.pack("<i", 1000000)
    for r in recs:
        r["raw"] = record(r["tid"], r["pos"], r["name"], r["ops"], r["flag"], r["l_seq"], r["aux"], r["cg"], rng)
    return hdr + b"".join(r["raw"] for r in recs), recs


def restored(r: dict) -> bool:
    """htslib's bam_tag2cigar moves the CG array in only when it holds >= n_cigar (here 2) ops."""
    return r["cg"] and len(r["ops"]) >= 2 and r["tid"] >= 0 and r["pos"] >= 0


def expected_pileup(recs: list[dict], n_ref: int):
    """What the ingest must produce: (tid_off, pos, endpos, cig_off, cigar, clip) of the kept reads."""
    keep = [r for r in recs if 0 <= r["tid"] < n_ref and r["pos"] >= 0]
    tid_off = np.zeros(n_ref + 1, dtype=np.int64)
    for r in keep:
        tid_off[r["tid"] + 1] += 1
    tid_off = np.cumsum(tid_off)
    pos, endpos, clip, cig_off, cigar = [], [], [], [0], []
    for r in keep:
        ops = r["ops"]
        if r["cg"] and not restored(r):   # bam_tag2cigar needs >= n_cigar (2) CG ops: the placeholder stays
            ops = [(4, r["l_seq"]), (3, max(sum(ln for op, ln in ops if op in (0, 2, 3, 7, 8)), 1))]
        words = [ln << 4 | op for op, ln in ops]
        rl = 0 if r["flag"] & 4 else sum(ln for op, ln in ops if op in (0, 2, 3, 7, 8))
        pos.append(r["pos"])
        endpos.append(r["pos"] + (rl if rl else 1))
        c = 0
        if words:
            c |= 1 if (words[-1] & 15) == 4 else 0
            c |= 2 if (words[0] & 15) == 4 else 0
        else:   # the bytes refinement.c reads: the NUL-padded name's last word, the byte after the CIGAR
            qn = r["name"] + b"\0"
            padded = (len(qn) + 3) & ~3
            w0 = qn[padded - 4] if padded >= 4 and padded - 4 < len(qn) else 0
            c |= 1 if (w0 & 15) == 4 else 0
            after = 4 + 32 + len(qn)
            c |= 2 if after < len(r["raw"]) and (r["raw"][after] & 15) == 4 else 0
        clip.append(c)
        cigar += words
        cig_off.append(len(cigar))
    return (tid_off, np.array(pos, np.int32), np.array(endpos, np.int32), np.array(cig_off, np.uint64),
            np.array(cigar, np.uint32), np.array(clip, np.uint8))


def write(path: str, seed: int, **kw) -> tuple[list[dict], int]:
    raw, recs = make_bam(seed, **kw)
    with open(path, "wb") as f:
        f.write(bgzf_blocks(raw))
    return recs, kw.get("n_ref", 3)
