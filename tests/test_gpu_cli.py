"""End to end: `svtrek audt -b BAM -v VCF` (CLI -> BAM ingest -> C ABI -> HIP) prints
exactly what the CPU oracle's restatement of the reference audit prints."""
import os
import random
import subprocess

import oracle_ffi as O
import pytest

from svtrek_amd import sim
from svtrek_amd.simvcf import resolved_vcf_from_loci, simulate

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "svtrek_amd", "svtrek")


def run_cli(*args, check=True):
    r = subprocess.run([CLI, "audt", *args], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=300)
    if check and r.returncode != 0:
        raise AssertionError(f"svtrek failed rc={r.returncode}\n{r.stderr}")
    return r


@pytest.mark.parametrize("inflate", ["auto", "gpu", "gpu-small-batches"])
def test_cfg1_simvcf_layout(tmp_path, inflate, monkeypatch):
    """BASELINE config 1: 100 DEL via the simvcf transform + 10x long-read BAM, -t 1; the BAM's
    BGZF blocks inflated on the host (auto: a small BAM) or on the GPU (also in 16 MiB batches:
    many batches, partial blocks carried across them)."""
    if inflate == "gpu-small-batches":
        monkeypatch.setenv("SVTREK_INFLATE_BATCH_MB", "16")
    r = sim.generate(sim.WORKLOADS["cfg1_100del_10x"], keep_handle=True)
    bam = str(tmp_path / "cfg1.bam")
    sim.write_bam(r, bam, with_seq=True)
    resolved = resolved_vcf_from_loci(r.loci, r.truth, seed=1)
    vcf_text = "".join(simulate(resolved, random.Random(101)))
    vcf = tmp_path / "cfg1.sim.vcf"
    vcf.write_text(vcf_text)
    out = run_cli("-b", bam, "-v", str(vcf), "-t", "1", "--inflate", inflate.split("-")[0]).stdout
    want = O.audit_text(vcf_text, r.pileup)
    assert out == want
    dels = [l for l in out.splitlines() if l.startswith("(DEL)")]
    assert len(dels) == 100
    # END= matched inside CIEND=: every end window is empty -> "ref end: NA" 
    assert all("ref end: NA" in l for l in dels)
    assert sum("ref pos: NA" not in l for l in dels) > 50


def test_plain_vcf_mixed_types_and_errors(tmp_path):
    r = sim.generate(sim.SimConfig(seed=31, n_targets=2, n_loci=300, del_frac=0.5, coverage=20,
                                   p_clip_ends=0.2), keep_handle=True)
    bam = str(tmp_path / "x.bam")
    sim.write_bam(r, bam, with_seq=False)
    vcf = tmp_path / "x.vcf"
    sim.write_vcf(r.loci, str(vcf), chrom_prefix="chr")
    extra = ("chr1\t30000\tinv1\tN\t<INV>\t.\tPASS\tSVTYPE=INV;END=36000\n"
             "chr1\t40000\tdup1\tN\t<DUP>\t.\tPASS\tSVTYPE=DUP;END=46000\n"
             "chr1\tabc\tbad\tN\t<DEL>\t.\tPASS\tSVTYPE=DEL;END=46000\n"
             "chr2\t50000\tdel50\tN\t<DEL>\t.\tPASS\tSVTYPE=DEL;END=50050\n"
             "chr2\t50000\tdel49\tN\t<DEL>\t.\tPASS\tSVTYPE=DEL;END=50049\n"
             "chr9\t50000\tnocontig\tN\t<DEL>\t.\tPASS\tSVTYPE=DEL;END=60000\n"
             "onlyone\n"
             "x\n")
    text = vcf.read_text() + extra
    vcf.write_text(text)
    res = run_cli("-b", bam, "-v", str(vcf), "-t", "3")
    assert res.stdout == O.audit_text(text, r.pileup)
    assert "[ERROR] Unkown type." in res.stderr
    assert "[ERROR] Conversion error to pos abc" in res.stderr
    assert "VCF: no index at line: onlyone" in res.stderr


def test_nondefault_flags(tmp_path):
    r = sim.generate(sim.SimConfig(seed=41, n_targets=1, n_loci=120, del_frac=0.5, coverage=25), keep_handle=True)
    bam = str(tmp_path / "y.bam")
    sim.write_bam(r, bam)
    vcf = tmp_path / "y.vcf"
    sim.write_vcf(r.loci, str(vcf))
    from svtrek_amd import Params
    p = Params(wider_interval=5000, median_interval=3000, narrow_interval=800, consensus_interval_range=300,
               consensus_interval=8, consensus_min_count=4)
    out = run_cli("-b", bam, "--vcf", str(vcf), "--wider-interval", "5000", "--median-interval", "3000",
                  "--narrow-interval", "800", "--consensus-interval-range", "300", "--consensus-interval", "8",
                  "--consensus-min-count", "4", "--batch", "17").stdout
    assert out == O.audit_text(vcf.read_text(), r.pileup, p)


def test_cli_usage_and_missing_files(tmp_path):
    r = subprocess.run([CLI], stdout=subprocess.PIPE, text=True)
    assert r.returncode == 1 and r.stdout.startswith("Usage: ./svtrek [MODE] [OPTIONS]")
    r = subprocess.run([CLI, "audt", "-h"], stdout=subprocess.PIPE, text=True)
    assert r.returncode == 0 and "--consensus-min-count" in r.stdout
    r = run_cli("-v", str(tmp_path / "none.vcf"), check=False)
    assert r.returncode != 0 and "[ERROR] BAM file is not provided." in r.stderr


def test_audt_dist_single_rank(tmp_path):
    """The torchrun multi-GPU driver (svtrek_amd.audt_dist) at world size 1 prints the same bytes."""
    import sys
    r = sim.generate(sim.SimConfig(seed=51, n_targets=2, n_loci=150, del_frac=0.5, coverage=15), keep_handle=True)
    bam = str(tmp_path / "d.bam")
    sim.write_bam(r, bam)
    vcf = tmp_path / "d.vcf"
    sim.write_vcf(r.loci, str(vcf))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    res = subprocess.run([sys.executable, "-m", "svtrek_amd.audt_dist", "-b", bam, "-v", str(vcf)],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600, cwd=ROOT, env=env)
    assert res.returncode == 0, res.stderr[-2000:]
    assert res.stdout == O.audit_text(vcf.read_text(), r.pileup)


def test_genomic_shards_on_one_device(tmp_path):
    """--devices 0,0,0: three genomic shards, each with its own halo-sliced pileup and its own
    context on GPU 0, print the same bytes as one shard (SURVEY §8(e) partitioning)."""
    r = sim.generate(sim.SimConfig(seed=61, n_targets=3, n_loci=240, del_frac=0.5, coverage=15), keep_handle=True)
    bam = str(tmp_path / "s.bam")
    sim.write_bam(r, bam)
    vcf = tmp_path / "s.vcf"
    sim.write_vcf(r.loci, str(vcf))
    lines = vcf.read_text().splitlines(keepends=True)
    head = [l for l in lines if l.startswith("#")]
    body = [l for l in lines if not l.startswith("#")]
    random.Random(5).shuffle(body)                     # VCF order != genomic order
    text = "".join(head + body)
    vcf.write_text(text)
    want = O.audit_text(text, r.pileup)
    assert run_cli("-b", bam, "-v", str(vcf), "--devices", "0,0,0", "--batch", "50").stdout == want
    assert run_cli("-b", bam, "-v", str(vcf), "--devices", "0,0").stdout == want


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_audt_dist_two_ranks_engine(tmp_path):
    """audt_dist with the real HIP engine in two rank processes (launched by
    torch.distributed.run; on a one-GPU box both ranks share device 0 and the status all-reduce
    and gather go through gloo): per-rank BAI region reads, the engine on each shard, the gather,
    and stdout byte-identical to the oracle's for the whole VCF (audit.c:269-293)."""
    import sys
    r = sim.generate(sim.SimConfig(seed=52, n_targets=3, n_loci=400, del_frac=0.5, coverage=15), keep_handle=True)
    bam = str(tmp_path / "d2.bam")
    sim.write_bam(r, bam)
    vcf = tmp_path / "d2.vcf"
    sim.write_vcf(r.loci, str(vcf))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    res = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                          "-m", "svtrek_amd.audt_dist", "-b", bam, "-v", str(vcf), "-t", "2"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600, cwd=ROOT, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    out = "".join(ln for ln in res.stdout.splitlines(keepends=True) if not ln.startswith("[Gloo]"))
    assert out == O.audit_text(vcf.read_text(), r.pileup)
