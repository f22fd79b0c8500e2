"""The value-bucketed event index's DESIGN against the oracle, on the CPU (tests/native/bucket_model.c).

The engine's lane path (svt_bucket.inc) answers a window from the events filed in its band's value
buckets, BELOW from per-bucket prefix maxima of one key and ABOVE from bounded walks only when the
vote needs it.  The model restates exactly that on the CPU and votes the band plus the two facts with
the oracle's consensus_pos (refinement.c:41-101): it must equal the oracle's full walk on every
window -- adversarial pileups (every op code, D/I lengths around 50, clip-bit quirks, wrapping
windows, five parameter sets) and simulated workloads -- so that a GPU mismatch could only be a
coding error, never the design.  (The GPU kernels themselves: tests/test_gpu_parity.py.)"""
import os
import subprocess

import numpy as np
import pytest

import fuzz
from svtrek_amd import sim

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PARAMS = [[20000, 10000, 2000, 500, 5, 3], [3000, 1500, 700, 400, 10, 2], [20000, 10000, 2000, 60, 0, 1],
          [5000, 5000, 600, 520, 7, 4], [20000, 10000, 2000, 500, -3, 3]]


@pytest.fixture(scope="module")
def model(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("bkm") / "bucket_model")
    lib = os.path.join(ROOT, "oracle")
    subprocess.run(["gcc", "-O2", "-o", out, os.path.join(ROOT, "tests", "native", "bucket_model.c"), "-L" + lib,
                    "-loracle", "-Wl,-rpath," + lib, "-lpthread"], check=True)
    return out


def _dump(path, pl, loci, prm):
    nt = len(pl.tid_off) - 1
    clip = pl.clip if pl.clip is not None else _clip_bits(pl)
    with open(path, "wb") as f:
        np.array([nt, pl.n_reads, len(pl.cigar), len(loci)], dtype=np.int64).tofile(f)
        np.asarray(pl.tid_off, dtype=np.int64).tofile(f)
        np.asarray(pl.pos, dtype=np.int32).tofile(f)
        np.asarray(pl.endpos, dtype=np.int32).tofile(f)
        np.asarray(pl.cig_off, dtype=np.uint64).tofile(f)
        np.asarray(pl.cigar, dtype=np.uint32).tofile(f)
        np.ascontiguousarray(loci).view(np.uint8).tofile(f)
        np.asarray(clip, dtype=np.uint8).tofile(f)
        np.array(prm, dtype=np.int32).tofile(f)


def _clip_bits(pl):
    off = np.asarray(pl.cig_off, dtype=np.int64)
    cig = np.asarray(pl.cigar, dtype=np.uint32)
    n = off[1:] - off[:-1]
    last = np.where(n > 0, cig[np.maximum(off[1:] - 1, 0)] & 0xF, 0)
    first = np.where(n > 0, cig[np.minimum(off[:-1], max(len(cig) - 1, 0))] & 0xF, 0)
    return ((last == 4).astype(np.uint8) | ((first == 4).astype(np.uint8) << 1)) * (n > 0)


def _run(model, path, bsh=10):
    r = subprocess.run([model, path, str(bsh)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "mismatches 0" in r.stdout, r.stdout
    return r.stdout


@pytest.mark.parametrize("seed", range(1, 16))
def test_bucket_design_fuzz(model, tmp_path, seed):
    rng = np.random.default_rng(seed)
    nt, clen = 2, 60000
    hot = [int(x) for x in rng.integers(2000, clen - 2000, size=int(rng.integers(1, 8)))]
    pl = fuzz.random_pileup(rng, n_targets=nt, contig_len=clen, n_reads=int(rng.integers(50, 600)), hot=hot,
                            p_exotic=float(rng.choice([0.0, 0.1, 0.3])))
    loci = fuzz.random_loci(rng, 300, nt, clen, hot=hot)
    path = str(tmp_path / "f.bin")
    _dump(path, pl, loci, PARAMS[seed % len(PARAMS)])
    for bsh in (4, 10):   # (narrow buckets: more windows read the prefix maxima and walk bucket edges)
        _run(model, path, bsh)


@pytest.mark.parametrize("name,scale", [("cfg4_1m_delins_30x_hifi", 0.01), ("cfg2_10kdel_30x_ont", 0.05),
                                        ("cfg3_50k_delins_30x_ont", 0.01)])
def test_bucket_design_workloads(model, tmp_path, name, scale):
    from dataclasses import replace
    cfg = sim.WORKLOADS[name]
    r = sim.generate(replace(cfg, n_loci=max(1, int(cfg.n_loci * scale))))
    path = str(tmp_path / "w.bin")
    _dump(path, r.pileup, r.loci, PARAMS[0])
    out = _run(model, path)
    assert "redo 0.0000" in out   # every window of the default parameters takes the bucket path
