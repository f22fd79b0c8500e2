"""SURVEY.md §5 sanitizers, host code only: the product's host C++ (bam_ingest.cpp: BGZF
inflate + record parsing with T threads, CG-tag CIGARs, BAI region reads; vcf_audit.cpp:
multithreaded VCF parse + batch formatting) and the oracle's threaded paths run under
ASan+UBSan and under TSan (drivers in tests/san/, built by svtrek_amd.build.build_sanitizers);
each instrumented run must exit cleanly and agree with the uninstrumented library."""
import glob
import os
import random
import subprocess

import numpy as np
import pytest

from svtrek_amd import build, host, sim

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")


@pytest.fixture(scope="module")
def san():
    return build.build_sanitizers()


def _fnv(vals, h=0xcbf29ce484222325):
    for v in vals:
        h = ((h ^ int(v)) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def _expected_bam(path, threads, region=None):
    pl, info = host.read_bam(path, threads=threads, region=region)
    vals = []
    clip = pl.clip if pl.clip is not None else np.zeros(pl.n_reads, np.uint8)
    for r in range(pl.n_reads):
        vals += [int(pl.pos[r]) & 0xFFFFFFFF, int(pl.endpos[r]) & 0xFFFFFFFF, int(clip[r])]
        vals += pl.cigar[int(pl.cig_off[r]):int(pl.cig_off[r + 1])].tolist()
    return f"reads {pl.n_reads} records {info['records']} cg {info['cg_restored']} bamsum {_fnv(vals):016x}"


def _vcf(tmp_path):
    from test_host import _fuzz_line
    rng = random.Random(5)
    lines = [_fuzz_line(rng) for _ in range(1500)] + ["#x", "", "1\t7\t.\tA\tT\t.\t.\tSVTYPE=BND;END=9"] * 20
    goldens = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "simvcf_seed*.sim.vcf")))
    text = "\n".join(lines) + "\n" + "".join(open(g, encoding="latin-1").read() for g in goldens[:2])
    p = tmp_path / "s.vcf"
    p.write_text(text, encoding="latin-1")
    return str(p)


@pytest.mark.parametrize("kind", ["asan", "tsan"])
@pytest.mark.parametrize("case", ["seq", "cg", "region"])
def test_host_ingest_and_vcf_under_sanitizer(tmp_path, san, kind, case):
    if case == "cg":   # > 65535-op CIGARs stored as CG:B,I (restored at ingest)
        cfg = sim.SimConfig(seed=8, n_targets=1, n_loci=3, coverage=1.5, read_len_mean=200000, read_len_sd=0,
                            read_len_min=150000, rho=1.5, spacing=400000)
    else:
        cfg = sim.SimConfig(seed=9, n_targets=3, n_loci=40, del_frac=0.5, coverage=8.0, p_clip_ends=0.3,
                            p_exotic=0.05)
    r = sim.generate(cfg, keep_handle=True)
    bam = str(tmp_path / "s.bam")
    sim.write_bam(r, bam, with_seq=case != "cg", level=1)
    vcf = _vcf(tmp_path)
    region = (0, 20000, 2, 60000) if case == "region" else None
    args = [san[f"host_{kind}"], bam, vcf, "4"] + ([str(x) for x in region] if region else [])
    p = subprocess.run(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=ENV, timeout=600)
    assert p.returncode == 0, p.stderr.decode()[-4000:]
    assert b"Sanitizer" not in p.stderr and b"runtime error" not in p.stderr, p.stderr.decode()[-4000:]
    got = p.stdout.decode().strip()
    assert got.startswith(_expected_bam(bam, 4, region)), (got, _expected_bam(bam, 4, region))
    loci, msgs = host.parse_vcf_text(open(vcf, "rb").read(), threads=4)
    assert f" loci {len(loci)} " in got and f" msgbytes {len(msgs.encode('latin-1'))} " in got
    if case == "cg":
        assert " cg 0 " not in got


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_oracle_threads_under_sanitizer(tmp_path, san, kind):
    p = subprocess.run([san[f"oracle_{kind}"], str(tmp_path), "4"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       env=ENV, timeout=600)
    assert p.returncode == 0, p.stderr.decode()[-4000:]
    assert b"Sanitizer" not in p.stderr, p.stderr.decode()[-4000:]
    assert b"same 1" in p.stdout
