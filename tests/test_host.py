"""CPU tests of the host side: BAM ingest round trip, VCF parsing (A1) and printing (A11)
against the oracle restatement, the simvcf golden fixtures, and the C-ABI symbol table."""
import ctypes as C
import os
import re
import sys

import numpy as np
import oracle_ffi as O
import pytest

from svtrek_amd import host, sim
from svtrek_amd._lib import ENGINE_SYMBOLS, LOCUS_DTYPE, RESULT_DTYPE, SVT_NA

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def test_engine_library_exports_every_header_symbol():
    """libsvtrek_hip.so loads (no GPU needed) and exports every svt_* the header declares."""
    hdr = open(os.path.join(ROOT, "include", "svtrek_gpu.h")).read()
    declared = set(re.findall(r"\b(svt_[a-z_]+)\s*\(", hdr))
    assert declared == set(ENGINE_SYMBOLS), declared ^ set(ENGINE_SYMBOLS)
    lib = C.CDLL(os.path.join(ROOT, "svtrek_amd", "libsvtrek_hip.so"))
    for s in declared:
        assert hasattr(lib, s), s
    lib.svt_version.restype = C.c_char_p
    assert b"gfx950" in lib.svt_version()


def test_host_library_exports():
    hdr = open(os.path.join(ROOT, "svtrek_amd", "csrc", "svtrek_host.h")).read()
    L = host.load_host()
    for s in set(re.findall(r"\b(svth_[a-z_0-9]+)\s*\(", hdr)):
        assert hasattr(L, s), s


@pytest.mark.parametrize("with_seq", [False, True])
def test_bam_roundtrip(tmp_path, with_seq):
    cfg = sim.SimConfig(seed=5, n_targets=3, n_loci=30, del_frac=0.5, coverage=8, p_clip_ends=0.3,
                        p_exotic=0.05)
    r = sim.generate(cfg, keep_handle=True)
    path = str(tmp_path / "x.bam")
    sim.write_bam(r, path, with_seq=with_seq)
    pl, info = host.read_bam(path, threads=3)
    assert info["names"] == ["1", "2", "3"]
    assert info["records"] == r.pileup.n_reads
    src = r.pileup
    np.testing.assert_array_equal(pl.tid_off, src.tid_off)
    np.testing.assert_array_equal(pl.pos, src.pos)
    np.testing.assert_array_equal(pl.endpos, src.endpos)
    np.testing.assert_array_equal(pl.cig_off, src.cig_off)
    np.testing.assert_array_equal(pl.cigar, src.cigar)
    # clip bits derived from the CIGAR words (n_cigar >= 1 everywhere here)
    last = (src.cigar[src.cig_off[1:].astype(np.int64) - 1] & 15) == 4
    first = (src.cigar[src.cig_off[:-1].astype(np.int64)] & 15) == 4
    np.testing.assert_array_equal(pl.clip, last.astype(np.uint8) | (first.astype(np.uint8) << 1))


def test_bam_long_cigar_cg_tag(tmp_path):
    """> 65535 CIGAR ops are stored as kSmN + CG:B,I; ingest restores them (htslib bam_tag2cigar)."""
    cfg = sim.SimConfig(seed=8, n_targets=1, n_loci=4, coverage=2.0, read_len_mean=200000, read_len_sd=0,
                        read_len_min=150000, rho=1.5, spacing=400000)
    r = sim.generate(cfg, keep_handle=True)
    nops = np.diff(r.pileup.cig_off.astype(np.int64))
    assert nops.max() > 65535
    path = str(tmp_path / "long.bam")
    sim.write_bam(r, path, with_seq=False)
    pl, info = host.read_bam(path, threads=2)
    assert info["cg_restored"] == int((nops > 65535).sum())
    np.testing.assert_array_equal(pl.cigar, r.pileup.cigar)
    np.testing.assert_array_equal(pl.endpos, r.pileup.endpos)


def _vcf_lines(path):
    with open(path) as f:
        for line in f:
            if len(line) < 2 or line.startswith("#"):
                continue
            yield line.rstrip("\n")


@pytest.mark.parametrize("seed", [1, 7, 2024])
def test_parse_simvcf_golden(seed):
    """Reference simvcf.py output (fixture): product parser == oracle parser; the
    END= match inside CIEND= gives every DEL a huge uint32 end."""
    n_del = 0
    for line in _vcf_lines(os.path.join(GOLD, f"simvcf_seed{seed}.sim.vcf")):
        a1 = host.parse_line(line)
        a2 = O.parse_line(line)
        assert a1[0] == a2[0] and a1[1] == a2[1], (line, a1, a2)
        if a1[0] == 1 and a1[1][0] == 2:
            n_del += 1
            ciend = int(re.search(r"CIEND=(-?\d+)", line).group(1))
            assert a1[1][3] == ciend & 0xFFFFFFFF
    assert n_del > 0


def _fuzz_line(rng):
    chrom = rng.choice(["1", "chr2", "chrX", "X", "0", "-1", "22", "chr07", " 3"])
    pos = rng.choice(["0", "00", "12345", "-5", "abc", " 7", "4294967296", "99999999999", "1e3", "60000"])
    ref = rng.choice(["N", "A", "ACGT" * 13, "ACGT" * 12 + "AC", "ACGT" * 12 + "ACG"])
    alt = rng.choice(["<DEL>", "N", "A", "A,C", "A" * 51, "A" * 50, "AC,A" + "G" * 60, ",,A"])
    keys = []
    if rng.random() < 0.8:
        keys.append("SVTYPE=" + rng.choice(["DEL", "INS", "INV", "DUP", "TRA", "BND", "DEL:ME", "INS:ME",
                                             "del", "CNV", "AVERYLONGTYPENAMEHERE", ""]))
    if rng.random() < 0.5:
        keys.append("CIEND=" + rng.choice(["-40,25", "0,0", "x"]))
    if rng.random() < 0.7:
        keys.append("END=" + rng.choice(["60100", "60050", "60049", "0", "abc", "-3", "999999999999999999999999999999999999"]))
    if rng.random() < 0.2:
        keys.append("SVEND=5")
    rng.shuffle(keys)
    info = ";".join(keys) if keys else "."
    fields = [chrom, pos, "id", ref, alt, "60", "PASS", info]
    if rng.random() < 0.3:
        fields += ["GT", "0/1"]
    sep = "\t\t" if rng.random() < 0.05 else "\t"
    return sep.join(fields)


def test_parse_fuzz_vs_oracle():
    import random
    rng = random.Random(42)
    seen = set()
    for _ in range(4000):
        line = _fuzz_line(rng)
        a1 = host.parse_line(line)
        a2 = O.parse_line(line)
        assert a1[0] == a2[0] and a1[1] == a2[1], (line, a1, a2)
        seen.add(a1[0])
    assert seen == {0, 1, 2}


def test_format_vs_oracle():
    rng = np.random.default_rng(0)
    for _ in range(3000):
        t = int(rng.choice([1, 2, 3, 4, 0]))
        pos = int(rng.integers(0, 2**32))
        end = (pos + int(rng.choice([49, 50, 51, 1000, -5]))) & 0xFFFFFFFF
        loc = np.array([(t, int(rng.integers(-2, 25)), pos, end)], dtype=LOCUS_DTYPE)[0]
        vals = [SVT_NA, int(rng.integers(0, 2**32)), (pos + int(rng.integers(-600, 600))) & 0xFFFFFFFF]
        res = np.array([(int(rng.choice(vals)), int(rng.choice(vals)))], dtype=RESULT_DTYPE)[0]
        a = host.format_result(loc, res)
        lo = np.array([loc], dtype=LOCUS_DTYPE)
        rr = np.array([res], dtype=RESULT_DTYPE)
        buf = C.create_string_buffer(512)
        n = O.lib().orc_format_result(lo.ctypes.data, rr.ctypes.data, buf, 512)
        assert a == buf.raw[:n].decode(), (loc, res)


def test_format_examples():
    loc = np.array([(2, 1, 1000, 5000)], dtype=LOCUS_DTYPE)[0]
    res = np.array([(1003, SVT_NA)], dtype=RESULT_DTYPE)[0]
    assert host.format_result(loc, res) == ("(DEL) chr: 1, org pos: 1000, org end: 5000, ref pos: 1003, "
                                            "ref end: NA, diff pos: 3, diff end: NA\n")
    loc = np.array([(1, 3, 2000, 2001)], dtype=LOCUS_DTYPE)[0]
    assert host.format_result(loc, np.array([(1990, SVT_NA)], dtype=RESULT_DTYPE)[0]) == \
        "(INS) chr: 3, org pos: 2000, ref pos: 1990, diff: -10\n"
    loc = np.array([(3, 1, 100, 900)], dtype=LOCUS_DTYPE)[0]
    assert host.format_result(loc, np.array([(SVT_NA, SVT_NA)], dtype=RESULT_DTYPE)[0]) == \
        "(INV) chr: 1, org pos: 100, org end: 900, ref pos: 4294967295, ref end: 4294967295\n"
    # a DEL of exactly 50 bp reaches the switch but prints nothing (audit.c:190)
    loc = np.array([(2, 1, 100, 150)], dtype=LOCUS_DTYPE)[0]
    assert host.format_result(loc, np.array([(SVT_NA, SVT_NA)], dtype=RESULT_DTYPE)[0]) == ""


@pytest.mark.parametrize("region", [(0, 30000, 0, 90000), (0, 50000, 2, 40000), (1, 0, 1, 1 << 30),
                                    (2, 10 ** 8, 2, 10 ** 8 + 5)])
def test_bam_region_read(tmp_path, region):
    """svth_bam_read_region (BAI linear-index seek): every query inside the region yields
    the same reads as from the whole file, and the read stops at the region end."""
    from svtrek_amd.pileup import Pileup  # noqa: F401
    cfg = sim.SimConfig(seed=31, n_targets=3, n_loci=60, del_frac=0.5, coverage=10.0, p_clip_ends=0.3)
    r = sim.generate(cfg, keep_handle=True)
    path = str(tmp_path / "r.bam")
    sim.write_bam(r, path, with_seq=True, level=1)
    full, _ = host.read_bam(path, threads=2)
    part, info = host.read_bam(path, threads=2, region=region)
    t0, b0, t1, e1 = region
    tids = np.repeat(np.arange(3), np.diff(full.tid_off))
    pt = np.repeat(np.arange(3), np.diff(part.tid_off))
    # nothing at or past the region end; every full-file record overlapping the region is there
    assert not ((pt > t1) | ((pt == t1) & (part.pos >= e1))).any()
    inside = ((tids > t0) | ((tids == t0) & (full.endpos > b0))) & ((tids < t1) | ((tids == t1) & (full.pos < e1)))
    key = lambda t, p, e: set(zip(t.tolist(), p.tolist(), e.tolist()))
    assert key(tids[inside], full.pos[inside], full.endpos[inside]) <= key(pt, part.pos, part.endpos)
    assert info["records"] >= int(inside.sum())


def _zero_empty_bai_windows(bai_path: str, pl) -> int:
    """Rewrite a BAI the way older indexers leave it: linear-index windows no record overlaps
    hold 0 (the sim writer fills them with the next window's offset).  Returns how many."""
    import struct
    data = open(bai_path, "rb").read()
    o = 8
    n_ref = struct.unpack_from("<i", data, 4)[0]
    out = bytearray(data)
    zeroed = 0
    for t in range(n_ref):
        n_bin = struct.unpack_from("<i", data, o)[0]
        o += 4
        for _ in range(n_bin):
            n_chunk = struct.unpack_from("<i", data, o + 4)[0]
            o += 8 + 16 * n_chunk
        n_intv = struct.unpack_from("<i", data, o)[0]
        o += 4
        r0, r1 = int(pl.tid_off[t]), int(pl.tid_off[t + 1])
        cov = np.zeros(n_intv, dtype=bool)
        for p_, e_ in zip(pl.pos[r0:r1], pl.endpos[r0:r1]):
            cov[int(p_) >> 14:((int(e_) - 1) >> 14) + 1] = True
        for k in np.nonzero(~cov)[0]:
            struct.pack_into("<Q", out, o + 8 * int(k), 0)
            zeroed += 1
        o += 8 * n_intv
    open(bai_path, "wb").write(bytes(out))
    return zeroed


def test_bam_region_read_zero_linear_index(tmp_path):
    """a BAI whose empty 16 kb windows hold 0 (older indexers) -- a region
    starting in such a window seeks to the next non-zero entry, never to offset 0 (the
    header), and still yields every record the region overlaps."""
    cfg = sim.SimConfig(seed=33, n_targets=2, n_loci=20, del_frac=0.5, coverage=0.4, spacing=60000)
    r = sim.generate(cfg, keep_handle=True)
    path = str(tmp_path / "z.bam")
    sim.write_bam(r, path, with_seq=False, level=1)
    assert _zero_empty_bai_windows(path + ".bai", r.pileup) > 0
    full, _ = host.read_bam(path, threads=2)
    tids = np.repeat(np.arange(2), np.diff(full.tid_off))
    for t0 in range(2):
        r0, r1 = int(full.tid_off[t0]), int(full.tid_off[t0 + 1])
        gaps = [int(full.endpos[r0:r1][:k + 1].max()) for k in range(r1 - r0 - 1)
                if full.pos[r0 + k + 1] > full.endpos[r0:r0 + k + 1].max() + (1 << 15)]
        for b0 in gaps[:3]:
            b0 += 1 << 14   # a window no record overlaps
            part, _ = host.read_bam(path, threads=2, region=(t0, b0, 1, 1 << 29))
            pt = np.repeat(np.arange(2), np.diff(part.tid_off))
            inside = (tids > t0) | ((tids == t0) & (full.endpos > b0))
            key = lambda t, p, e: set(zip(t.tolist(), p.tolist(), e.tolist()))  # noqa: E731
            assert key(tids[inside], full.pos[inside], full.endpos[inside]) <= key(pt, part.pos, part.endpos)


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_vcf_batch_parse_and_format(threads):
    """svth_vcf_parse / svth_format_batch (multithreaded, '\\n'-aligned pieces) give the
    per-line parse's records and messages and the per-record text, in file order."""
    import random
    rng = random.Random(threads)
    lines = [_fuzz_line(rng) for _ in range(3000)]
    extra = ["", "#comment", "x", "1\t100\t.\tA\t<DEL>\t.\tPASS\tSVTYPE=DUP;END=900", "1\t0x\t.\tA\tT\t.\t.\tEND=5"]
    lines += extra * 50
    rng.shuffle(lines)
    text = ("\n".join(lines) + "\n").encode("latin-1") * 3
    loci, msgs = host.parse_vcf_text(text, threads=threads)
    want, wmsg = [], []
    for raw in text.decode("latin-1").split("\n"):
        line = raw
        if len(line) + 1 < 2 or line.startswith("#"):
            continue
        act, rec, err = host.parse_line(line)
        if act == 2:
            wmsg.append(err)
        if act == 1:
            if rec[0] not in (1, 2, 3):
                wmsg.append("[ERROR] Unkown type.\n")
            want.append(rec)
    assert [tuple(int(x) for x in r) for r in loci] == want
    assert msgs == "".join(wmsg)
    rng2 = np.random.default_rng(threads)
    from svtrek_amd._lib import RESULT_DTYPE
    res = np.zeros(len(loci), dtype=RESULT_DTYPE)
    res["start"] = np.where(rng2.random(len(loci)) < 0.3, 0xFFFFFFFF, rng2.integers(0, 2**32, len(loci)))
    res["end"] = np.where(rng2.random(len(loci)) < 0.3, 0xFFFFFFFF, rng2.integers(0, 2**32, len(loci)))
    assert host.format_batch(loci, res, threads=threads) == "".join(
        host.format_result(loci[k], res[k]) for k in range(len(loci)))


@pytest.mark.parametrize("region", [None, "mid"])
def test_bam_read_with_inflate_callback(tmp_path, region):
    """svth_bam_read_ex with an inflater callback (the CLI's device path; here the CPU backend's
    svt_bgzf_inflate behind the same ABI) reads the same pileup as the host-thread inflate, for
    the whole file and for a BAI region."""
    import ctypes

    from svtrek_amd import Engine, Params
    from svtrek_amd._lib import bind_abi
    cfg = sim.SimConfig(seed=21, n_targets=3, n_loci=60, del_frac=0.5, coverage=8, p_clip_ends=0.3)
    r = sim.generate(cfg, keep_handle=True)
    path = str(tmp_path / "x.bam")
    sim.write_bam(r, path, with_seq=True, level=1)
    reg = None if region is None else (1, 20000, 2, 10 ** 9)
    want, wi = host.read_bam(path, threads=3, region=reg)
    cpu = Engine(Params(), device=0, lib=bind_abi(ctypes.CDLL(os.path.join(ROOT, "oracle", "libsvtrek_cpu.so"))))
    try:
        got, gi = host.read_bam(path, threads=3, region=reg, inflate=cpu, batch_bytes=100_000)   # many batches
    finally:
        cpu.close()
    wi.pop("stage_s"); gi.pop("stage_s")
    assert wi == gi
    for k in ("tid_off", "pos", "endpos", "cig_off", "cigar", "clip"):
        assert np.array_equal(getattr(want, k), getattr(got, k)), k


def _reference_reader(data: bytes) -> list[bytes]:
    """The reader loop of audit.c:294-327, restated over bytes: fgets into a buffer of
    current_size bytes (1 MiB, doubled whenever a line fills it, never shrunk), strlen, the
    skip of a final line that exactly fills the buffer (fgets returns NULL, :317), of lines
    shorter than 2 chars and of '#' lines; the trailing '\\n' stripped."""
    cur, pos, n, out = 1 << 20, 0, len(data), []

    def fgets(cap):
        nonlocal pos
        if pos >= n:
            return None
        room = min(cap - 1, n - pos)
        j = data.find(b"\n", pos, pos + room)
        k = j - pos + 1 if j >= 0 else room
        s = data[pos:pos + k]
        pos += k
        return s

    def strlen(b):
        z = b.find(b"\0")
        return len(b) if z < 0 else z

    while (buf := fgets(cur)) is not None:
        L, skip = strlen(buf), False
        while L == cur - 1 and buf[L - 1:L] != b"\n":
            cur *= 2
            t = fgets(cur - L)
            if t is None:
                skip = True
                break
            buf = buf[:L] + t
            L = strlen(buf)
        if skip or L < 2 or buf[:1] == b"#":
            continue
        line = buf[:L]
        out.append(line[:-1] if line.endswith(b"\n") else line)
    return out


def _padded_record(pos: int, total: int, nl: bool) -> bytes:
    """A DEL record whose line is exactly `total` bytes (the trailing '\\n' included when nl)."""
    head = f"1\t{pos}\t.\tN\t<DEL>\t.\tPASS\tSVTYPE=DEL;END={pos + 900};PAD=".encode()
    return head + b"x" * (total - len(head) - (1 if nl else 0)) + (b"\n" if nl else b"")


@pytest.mark.parametrize("case", ["final_fills_1m", "final_short_by_one", "grown_buffer", "final_fills_2m",
                                  "long_mid", "nul"])
def test_vcf_reader_long_lines_and_nul(case):
    """svth_vcf_parse (threaded; the exact sequential reader once a line reaches 1 MiB) and the
    oracle's orc_audit_text against the reference's reader loop (audit.c:294-327): a final line
    without '\\n' that exactly fills the 1 MiB buffer is dropped; after a longer line has grown the
    buffer to 2 MiB the same line is kept and a 2 MiB - 1 one dropped; a NUL ends a line."""
    body = b"".join(_padded_record(10000 + 5000 * k, 90, True) for k in range(20))
    M = 1 << 20
    tail = {"final_fills_1m": _padded_record(900000, M - 1, False),
            "final_short_by_one": _padded_record(900000, M - 2, False),
            "grown_buffer": _padded_record(800000, M + 300, True) + _padded_record(900000, M - 1, False),
            "final_fills_2m": _padded_record(800000, M + 300, True) + _padded_record(900000, 2 * M - 1, False),
            "long_mid": _padded_record(800000, 3 * M + 7, True) + body,
            "nul": b"1\t700000\t.\tN\t<DEL>\t.\tPASS\tSVTYPE=DEL;END=700900\x00;junk\n" + b"1\t7\0\n"}[case]
    data = body + tail
    want = _reference_reader(data)
    recs = [host.parse_line(w.decode("latin-1")) for w in want]
    want_loci = [r[1] for r in recs if r[0] == 1]
    for threads in (1, 4):
        loci, _ = host.parse_vcf_text(data, threads=threads)
        assert [tuple(int(x) for x in r) for r in loci] == want_loci, (case, threads)
    # the oracle's reader: one printed line per parsed record (an empty pileup: NA results)
    from svtrek_amd.pileup import from_reads
    printed = O.audit_text(data.decode("latin-1"), from_reads(1, [])).splitlines()[1:-1]
    assert len(printed) == len(want_loci), case
    if case == "final_fills_1m":
        assert len(want_loci) == 20   # the final line is dropped
    if case in ("final_short_by_one", "grown_buffer"):
        assert len(want_loci) == 21 + (case == "grown_buffer")


def test_write_bam_regions_is_a_shard_halo(tmp_path):
    """sim.write_bam_regions (tools/e2e_shard.py): the records overlapping a shard's per-contig
    regions refine the shard's loci exactly as the whole pileup does."""
    import oracle_ffi as O
    from svtrek_amd import Params, host, sim
    from svtrek_amd.distributed import shard_rows
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from e2e_shard import shard_regions
    r = sim.generate(sim.SimConfig(seed=29, n_loci=240, n_targets=4, del_frac=0.5, coverage=8), keep_handle=True)
    for rank in range(3):
        loci = r.loci[shard_rows(r.loci, 3, rank)]
        regions = shard_regions(loci, Params())
        assert len({t for t, _, _ in regions}) == len(regions) >= 1
        path = str(tmp_path / f"s{rank}.bam")
        sim.write_bam_regions(r, path, regions, with_seq=True, level=1)
        pl, _ = host.read_bam(path, threads=2)
        assert pl.n_reads < r.pileup.n_reads
        np.testing.assert_array_equal(O.refine_batch(pl, loci).view(np.uint32), O.refine_batch(r.pileup, loci).view(np.uint32))
