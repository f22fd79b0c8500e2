"""One ABI, two backends: oracle/libsvtrek_cpu.so implements
include/svtrek_gpu.h on the CPU restatement, so the same calls -- svtrek_amd.Engine over
either library, and the product's CLI (svtrek_main.cpp) linked against either -- run here
without a GPU.  The GPU side of the comparison is tests/test_gpu_parity.py
(test_hip_and_cpu_backends_through_one_abi)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import oracle_ffi as O
import pytest

from svtrek_amd import Engine, Params, make_loci, sim
from svtrek_amd._lib import ENGINE_SYMBOLS, bind_abi

from fuzz import random_loci, random_pileup

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPU_LIB = os.path.join(ROOT, "oracle", "libsvtrek_cpu.so")
CPU_CLI = os.path.join(ROOT, "oracle", "_cpu", "svtrek_cpu")


def cpu_engine(params=None):
    return Engine(params or Params(), device=0, lib=bind_abi(C.CDLL(CPU_LIB)))


def test_cpu_backend_exports_the_header():
    hdr = open(os.path.join(ROOT, "include", "svtrek_gpu.h")).read()
    L = C.CDLL(CPU_LIB)
    for s in set(re.findall(r"\b(svt_[a-z_0-9]+)\s*\(", hdr)) | set(ENGINE_SYMBOLS):
        assert hasattr(L, s), s


@pytest.mark.parametrize("seed", range(4))
def test_cpu_backend_refine_and_work(seed):
    rng = np.random.default_rng(500 + seed)
    pl = random_pileup(rng, n_targets=2, contig_len=60000, n_reads=int(rng.integers(50, 500)), max_ops=60,
                       hot=[int(x) for x in rng.integers(5000, 55000, size=5)])
    loci = random_loci(rng, 300, 2, 60000, [int(x) for x in rng.integers(5000, 55000, size=5)])
    with cpu_engine() as e:
        e.load_pileup(pl)
        got = e.refine(loci)
        work = e.count_work(loci)
    want, w = O.refine_batch(pl, loci, with_work=True)
    assert np.array_equal(got, want)
    assert work["reads"] == w["reads"] and work["ops_walked"] == w["ops_walked"]


def test_cpu_backend_errors():
    with pytest.raises(Exception):
        cpu_engine(Params(consensus_min_count=0))
    with cpu_engine() as e:
        from svtrek_amd import SvtError
        with pytest.raises(SvtError):
            e.refine(make_loci([(2, 1, 1000, 5000)]))   # before load_pileup: SVT_ESTATE


@pytest.mark.parametrize("inflate", ["cpu", "gpu", "gpu-hostparse"])
def test_cli_on_cpu_backend(tmp_path, inflate, monkeypatch):
    """The drop-in CLI's whole flow (BAM ingest, parallel A1 parse beside it, batched refine,
    batch A11 print) linked against the CPU backend: stdout bytes equal the oracle's.
    --inflate gpu runs the ingest's device pipeline in 1 MiB batches: the batches handed to
    svt_bam_dec_* (here the CPU backend's decoder), or -- gpu-hostparse, SVTREK_HOSTPARSE=1 --
    inflated by svt_bgzf_inflate and parsed on the host."""
    monkeypatch.setenv("SVTREK_INFLATE_BATCH_MB", "1")
    if inflate == "gpu-hostparse":
        monkeypatch.setenv("SVTREK_HOSTPARSE", "1")
        inflate = "gpu"
    r = sim.generate(sim.SimConfig(seed=41, n_targets=2, n_loci=150, del_frac=0.5, coverage=10), keep_handle=True)
    bam = str(tmp_path / "c.bam")
    sim.write_bam(r, bam, with_seq=True, level=1)
    vcf = tmp_path / "c.vcf"
    sim.write_vcf(r.loci, str(vcf))
    with open(vcf, "a") as f:
        f.write("1\t5000\t.\tA\t<DUP>\t.\tPASS\tSVTYPE=DUP;END=9000\n1\tx\n")
    p = subprocess.run([CPU_CLI, "audt", "-b", bam, "-v", str(vcf), "-t", "3", "--inflate", inflate], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=300)
    assert p.returncode == 0, p.stderr.decode()
    assert p.stdout.decode("latin-1") == O.audit_text(vcf.read_text(encoding="latin-1"), r.pileup)
    assert "[ERROR] Unkown type." in p.stderr.decode()
