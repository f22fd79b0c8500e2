"""The BAM record decode behind svt_bam_dec_*  on the CPU: the record-start guess
(svt_bamrec.h bamrec::plausible, compiled for the host) accepts every true record start, the
host ingest and the CPU backend's decoder read the edge-case fixtures (tests/bamfix.py) exactly
as stated, and the CLI's decode flow (svth_bam_read_device feeding the decoder, batches split
anywhere) gives the host ingest's results.  The device decoder itself: test_gpu_bam_decode.py."""
import ctypes as C
import os
import subprocess
import zlib

import numpy as np
import oracle_ffi as O
import pytest

import bamfix
from svtrek_amd import Engine, Params, host, sim
from svtrek_amd._lib import bind_abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def shim(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("br") / "bamrec_shim.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(ROOT, "svtrek_amd", "csrc"), "-o", out,
                    os.path.join(ROOT, "tests", "native", "bamrec_shim.cpp")], check=True)
    lib = C.CDLL(out)
    lib.bamrec_scan.argtypes = [C.c_void_p, C.c_uint64, C.c_int32, C.c_void_p, C.c_uint64]
    lib.bamrec_scan.restype = C.c_uint64
    return lib


def _inflated(path: str) -> bytes:
    data, out, p = open(path, "rb").read(), [], 0
    while p < len(data):
        bsize = int.from_bytes(data[p + 16:p + 18], "little") + 1
        out.append(zlib.decompress(data[p + 18:p + bsize - 8], -15))
        p += bsize
    return b"".join(out)


def _record_starts(raw: bytes) -> tuple[int, list[int]]:
    """(n_ref, the offsets of every record's block_size word) by walking the header and chain."""
    lt = int.from_bytes(raw[4:8], "little")
    p = 8 + lt
    n_ref = int.from_bytes(raw[p:p + 4], "little")
    p += 4
    for _ in range(n_ref):
        p += 4 + int.from_bytes(raw[p:p + 4], "little") + 4
    starts = []
    while p + 4 <= len(raw):
        starts.append(p)
        p += 4 + int.from_bytes(raw[p:p + 4], "little")
    return n_ref, starts


@pytest.mark.parametrize("src", ["fixture", "sim_seq"])
def test_plausible_accepts_every_record_start(shim, tmp_path, src):
    path = str(tmp_path / "x.bam")
    if src == "fixture":
        bamfix.write(path, seed=3)
    else:
        r = sim.generate(sim.SimConfig(seed=4, n_targets=2, n_loci=30, coverage=6.0), keep_handle=True)
        sim.write_bam(r, path, with_seq=True)
    raw = _inflated(path)
    n_ref, starts = _record_starts(raw)
    buf = C.create_string_buffer(raw, len(raw))
    out = np.zeros(len(raw), dtype=np.uint64)
    k = shim.bamrec_scan(buf, len(raw), n_ref, out.ctypes.data, len(out))
    found = set(out[:k].tolist())
    assert set(starts) <= found                      # every true start is plausible
    assert len(found - set(starts)) <= len(starts) // 100 + 2   # and few false guesses (proven away)


def test_host_ingest_reads_fixture_exactly(tmp_path):
    path = str(tmp_path / "f.bam")
    recs, n_ref = bamfix.write(path, seed=5)
    want = bamfix.expected_pileup(recs, n_ref)
    pl, info = host.read_bam(path, threads=3)
    assert info["records"] == len(recs)
    assert info["cg_restored"] == sum(1 for r in recs if bamfix.restored(r))
    for got, exp in zip((pl.tid_off, pl.pos, pl.endpos, pl.cig_off, pl.cigar, pl.clip), want):
        np.testing.assert_array_equal(got, exp)


def _cpu_engine():
    return Engine(Params(), device=0, lib=bind_abi(C.CDLL(os.path.join(ROOT, "oracle", "libsvtrek_cpu.so"))))


@pytest.mark.parametrize("batch_kb", [0, 64, 7])
def test_cpu_backend_decoder_flow(tmp_path, batch_kb):
    """svth_bam_read_device -> svt_bam_dec_* of the CPU backend, batches of any size (records and
    BGZF blocks split across them): the refined results of the host ingest's pileup."""
    path = str(tmp_path / "d.bam")
    recs, n_ref = bamfix.write(path, seed=11 + batch_kb)
    pl, _ = host.read_bam(path, threads=2)
    rng = np.random.default_rng(batch_kb)
    from svtrek_amd import make_loci
    loci = make_loci([(int(rng.choice([1, 2])), int(rng.integers(1, n_ref + 1)), int(p), int(p) + int(d))
                      for p, d in zip(rng.integers(0, 200000, 300), rng.integers(51, 5000, 300))])
    eng = _cpu_engine()
    st = host.load_bam_device(eng, path, threads=2, batch_bytes=batch_kb << 10, pinned=False)
    assert st["reads"] == len(pl.pos) and st["records"] == len(recs)
    assert st["cg_restored"] == sum(1 for r in recs if bamfix.restored(r))
    np.testing.assert_array_equal(eng.refine(loci), O.refine_batch(pl, loci))
    eng.close()
