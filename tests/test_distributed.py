"""N>1 plumbing on CPU: world_size 2 (and 3) gloo processes shard the loci and gather the
results to rank 0 in VCF order.  The per-rank refinement here is the CPU oracle (test
infrastructure standing in for the GPU, which this container lacks); the genomic
sharding, halo slicing, record packing and gather code is the product's
(svtrek_amd.distributed, svtrek_amd.pileup.halo_slice)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from svtrek_amd.distributed import (PAD_INDEX, genomic_order, pack_records, shard_bounds, shard_rows,
                                    unpack_records)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, seed, outdir):
    import torch.distributed as dist

    import oracle_ffi as O
    from svtrek_amd import sim
    from svtrek_amd.distributed import gather_results
    from svtrek_amd.pileup import halo_slice

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = sim.generate(sim.SimConfig(seed=seed, n_loci=97, n_targets=2, del_frac=0.6, coverage=12))
    rows = shard_rows(r.loci, world, rank)
    mine = r.loci[rows]
    sub = halo_slice(r.pileup, mine, 20000, 10000, 2000)
    assert world == 1 or sub.n_reads < r.pileup.n_reads
    res = gather_results(rows, O.refine_batch(sub, mine), len(r.loci))
    if rank == 0:
        np.save(os.path.join(outdir, "res.npy"), res.view(np.uint32).reshape(-1, 2))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_shard_and_gather(tmp_path, world):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
    mp.spawn(_worker, args=(world, _free_port(), 17, str(tmp_path)), nprocs=world, join=True)
    import oracle_ffi as O
    from svtrek_amd import sim
    r = sim.generate(sim.SimConfig(seed=17, n_loci=97, n_targets=2, del_frac=0.6, coverage=12))
    want = O.refine_batch(r.pileup, r.loci).view(np.uint32).reshape(-1, 2)
    got = np.load(tmp_path / "res.npy")
    np.testing.assert_array_equal(got, want)


def test_shard_bounds_cover_rows_once():
    for n in (0, 1, 7, 97, 1000):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, world, r) for r in range(world)]
            rows = [i for b0, b1 in spans for i in range(b0, b1)]
            assert rows == list(range(n))


def test_genomic_order_is_stable_and_shards_partition():
    from svtrek_amd.pileup import make_loci
    loci = make_loci([(2, 2, 500, 900), (2, 1, 700, 900), (1, 1, 700, 0), (2, 2, 100, 900), (2, 1, 700, 800)])
    assert genomic_order(loci).tolist() == [1, 2, 4, 3, 0]
    for world in (1, 2, 3, 8):
        got = np.concatenate([shard_rows(loci, world, r) for r in range(world)])
        assert got.tolist() == [1, 2, 4, 3, 0]


def test_pack_unpack_records_roundtrip():
    from svtrek_amd._lib import RESULT_DTYPE
    rng = np.random.default_rng(3)
    n, world = 23, 4
    res = np.zeros(n, dtype=RESULT_DTYPE)
    res["start"] = rng.integers(0, 2**32, n, dtype=np.uint64)
    res["end"] = rng.integers(0, 2**32, n, dtype=np.uint64)
    perm = rng.permutation(n)
    per = (n + world - 1) // world
    bufs = [pack_records(perm[b0:b1], res[perm[b0:b1]], per)
            for b0, b1 in (shard_bounds(n, world, r) for r in range(world))]
    assert all(b.shape == (per, 4) for b in bufs)
    assert (bufs[-1][n - per * (world - 1):, 0] == PAD_INDEX).all()
    back = unpack_records(np.concatenate(bufs), n)
    np.testing.assert_array_equal(back.view(np.uint32), res.view(np.uint32))
    with pytest.raises(RuntimeError):
        unpack_records(np.concatenate(bufs[:-1]), n)


@pytest.mark.parametrize("seed", [5, 6])
def test_halo_slice_is_exact(seed):
    """Refining a shard against its halo slice equals refining it against the whole pileup,
    including wrapped windows near the contig start, INS/INV loci, unknown contigs and
    non-default intervals."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
    import oracle_ffi as O
    from svtrek_amd import Params, sim
    from svtrek_amd.pileup import halo_slice, make_loci
    r = sim.generate(sim.SimConfig(seed=seed, n_loci=160, n_targets=3, del_frac=0.5, coverage=10))
    extra = make_loci([(2, 1, 30, 400), (1, 1, 5, 0), (3, 1, 100, 9000), (2, 9, 5000, 9000),
                       (2, 0, 5000, 9000), (2, 2, 0xFFFFFF00, 0xFFFFFFF0)])
    loci = np.concatenate([r.loci, extra])
    for prm in (Params(), Params(wider_interval=3000, median_interval=700, narrow_interval=300)):
        full = O.refine_batch(r.pileup, loci, prm)
        for world in (2, 5):
            for rank in range(world):
                rows = shard_rows(loci, world, rank)
                sub = halo_slice(r.pileup, loci[rows], prm.wider_interval, prm.median_interval,
                                 prm.narrow_interval)
                got = O.refine_batch(sub, loci[rows], prm)
                np.testing.assert_array_equal(got.view(np.uint32), full[rows].view(np.uint32))


def _bench_path_worker(rank, world, port, outdir):
    """bench.py's N > 1 data path on gloo: shard_workload -> per-step 16-B records ->
    PipelinedGather (double-buffered async gathers) -> unpack at rank 0."""
    import torch
    import torch.distributed as dist

    import oracle_ffi as O
    from svtrek_amd import Params, sim
    from svtrek_amd._lib import RECORD_DTYPE
    from svtrek_amd.distributed import PipelinedGather, pack_records, padded_rows, shard_workload

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = sim.generate(sim.SimConfig(seed=23, n_loci=211, n_targets=3, del_frac=0.5, coverage=10))
    rows, sl, sub = shard_workload(r.loci, r.pileup, Params(), world, rank)
    per = padded_rows(len(r.loci), world)
    pg = PipelinedGather(lambda: torch.full((per * RECORD_DTYPE.itemsize // 4,), -1, dtype=torch.int32),
                         world, rank)
    local = O.refine_batch(sub, sl)
    steps = 5
    for i in range(steps):   # each step writes its records into the buffer the pipeline hands out
        buf = pg.buffer(i)
        buf.copy_(torch.from_numpy(pack_records(rows, local, per).view(np.int32).reshape(-1)))
        pg.submit(i)
    pg.drain()
    if rank == 0:
        recs = np.concatenate([p.numpy().view(np.uint32) for p in pg.gathered(steps - 1)])
        np.save(os.path.join(outdir, "recs.npy"), recs)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_bench_shard_and_gather_path(tmp_path, world):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
    mp.spawn(_bench_path_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    import oracle_ffi as O
    from svtrek_amd import sim
    r = sim.generate(sim.SimConfig(seed=23, n_loci=211, n_targets=3, del_frac=0.5, coverage=10))
    recs = np.load(tmp_path / "recs.npy")
    got = unpack_records(recs, len(r.loci))
    np.testing.assert_array_equal(got.view(np.uint32), O.refine_batch(r.pileup, r.loci).view(np.uint32))


def _audt_worker(rank, world, port, bam, outdir, fail_rank, fail_kind="refine"):
    """audt_dist.run_rank on gloo: BAI region read + halo trim per rank, status all-reduce,
    gather; the oracle stands in for the GPU engine (test infrastructure)."""
    import torch.distributed as dist

    import oracle_ffi as O
    from svtrek_amd import Params, audt_dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    loci, _ = audt_dist.parse_vcf(os.path.join(outdir, "c.vcf"), threads=2)
    seen = {}

    def refine(pl, mine):
        if rank == fail_rank and fail_kind == "refine":
            raise ValueError("injected failure")
        seen["reads"] = pl.n_reads
        return O.refine_batch(pl, mine)

    def parse():   # a failure before the shard (VCF parse) must not hang the others
        if rank == fail_rank and fail_kind == "parse":
            raise ValueError("injected failure")
        return loci

    try:
        res = audt_dist.run_rank(bam, parse, Params(), 2, refine, world, rank)
        if rank == 0:
            np.save(os.path.join(outdir, "res.npy"), res.view(np.uint32).reshape(-1, 2))
        np.save(os.path.join(outdir, f"reads{rank}.npy"), np.array([seen.get("reads", 0)]))
    except RuntimeError as e:
        with open(os.path.join(outdir, f"err{rank}.txt"), "w") as f:
            f.write(str(e))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_rank,fail_kind", [(2, -1, ""), (3, -1, ""), (2, 1, "refine"), (3, 0, "parse")])
def test_gloo_audt_dist_region_shards(tmp_path, world, fail_rank, fail_kind):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
    import oracle_ffi as O
    from svtrek_amd import sim
    r = sim.generate(sim.SimConfig(seed=23, n_loci=120, n_targets=3, del_frac=0.5, coverage=10), keep_handle=True)
    bam = str(tmp_path / "c.bam")
    sim.write_bam(r, bam, with_seq=True, level=1)
    sim.write_vcf(r.loci, str(tmp_path / "c.vcf"))
    mp.spawn(_audt_worker, args=(world, _free_port(), bam, str(tmp_path), fail_rank, fail_kind), nprocs=world,
             join=True)
    if fail_rank >= 0:   # every rank stops with an error, none hangs in the gather
        for k in range(world):
            assert (tmp_path / f"err{k}.txt").exists()
        assert "injected failure" in (tmp_path / f"err{fail_rank}.txt").read_text()
        return
    from svtrek_amd import audt_dist
    loci, _ = audt_dist.parse_vcf(str(tmp_path / "c.vcf"))
    want = O.refine_batch(r.pileup, loci).view(np.uint32).reshape(-1, 2)
    np.testing.assert_array_equal(np.load(tmp_path / "res.npy"), want)
    reads = [int(np.load(tmp_path / f"reads{k}.npy")[0]) for k in range(world)]
    assert max(reads) < r.pileup.n_reads   # each rank read only its region of the BAM


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launcher_spawns_ranks_dry_run(world):
    """`bench.py --gpus N` (no WORLD_SIZE in the environment) starts N rank processes itself:
    the gloo dry run shards cfg1, every rank's records reach rank 0 through the gather and
    exactly one JSON line comes out, with n_gpus = N."""
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    bench = os.path.join(os.path.dirname(here), "bench.py")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, bench, "--gpus", str(world), "--dry-run", "--workload", "cfg1_100del_10x",
                        "--steps", "3", "--warmup", "1"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]   # gloo prints "[Gloo] ..." lines
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["gather_ranks"] == world and out["records_verified"] is True
    assert out["config"]["loci_total"] == 100 and out["cpu_baseline"] is None
    assert out["parity_sample"]["loci"] == 100 and out["parity_sample"]["mismatches"] == 0


def test_bench_parity_mismatch_fails_the_run():
    """the bench checks its own records against the oracle after the timed
    loop -- one wrong record on the last rank (a diagnostic flag of the dry run) is reported in
    parity_sample and the run exits non-zero."""
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    bench = os.path.join(os.path.dirname(here), "bench.py")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, bench, "--gpus", "2", "--dry-run", "--workload", "cfg1_100del_10x",
                        "--steps", "2", "--warmup", "1", "--corrupt-record", "7"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode != 0, r.stdout[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["records_verified"] is False and out["parity_sample"]["mismatches"] == 1
    assert "parity self-check failed" in r.stderr


def test_parity_sample_counts_mismatches():
    """bench.parity_sample on gathered record buffers: the sampled rows against the oracle, pads
    skipped, one flipped end counted once, full=True checks every row."""
    import sys
    import numpy as np
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    import bench
    import oracle_ffi as O
    from svtrek_amd import sim
    from svtrek_amd.distributed import padded_rows
    r = sim.generate(sim.SimConfig(seed=31, n_targets=2, n_loci=300, del_frac=0.5, coverage=8.0))
    want = O.refine_batch(r.pileup, r.loci)
    per = padded_rows(len(r.loci), 2)
    parts = []
    for g in range(2):
        rows = shard_rows(r.loci, 2, g)
        parts.append(pack_records(rows, want[rows], per))
    ps = bench.parity_sample(parts, r, np.arange(50), n_random=100, threads=2)
    assert ps["mismatches"] == 0 and 100 <= ps["loci"] <= 150
    assert bench.parity_sample(parts, r, [], full=True, threads=2)["loci"] == 300
    parts[1][5, 2] ^= 1
    ps = bench.parity_sample(parts, r, [], full=True, threads=2)
    assert ps["mismatches"] == 1 and ps["first"]["vcf_row"] == int(parts[1][5, 0])


def test_bench_refuses_world_size_mismatch():
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    bench = os.path.join(os.path.dirname(here), "bench.py")
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, bench, "--gpus", "4", "--dry-run"], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0 and "must agree" in r.stderr


def test_bench_launcher_stops_ranks_on_failure():
    """A rank that fails makes the launcher stop the others and exit non-zero (an unknown
    workload fails every rank before the first collective)."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    bench = os.path.join(os.path.dirname(here), "bench.py")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, bench, "--gpus", "2", "--dry-run", "--workload", "nope"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and not any(ln.startswith("{") for ln in r.stdout.splitlines())


@pytest.mark.parametrize("nbuf", [1, 2, 3, 4])
def test_pipelined_gather_one_buffer_per_step_in_flight(nbuf):
    """bench.py gives the gather one buffer per step in flight (--inflight K, at least two): steps
    i and i + 1 .. i + K - 1 never share a buffer, and gathered(i) is step i's."""
    import torch
    from svtrek_amd.distributed import PipelinedGather
    pg = PipelinedGather(lambda: torch.zeros(4, dtype=torch.int32), 1, 0, enabled=False, nbuf=nbuf)
    k = max(2, nbuf)
    assert pg.n == k
    for i in range(3 * k):
        pg.buffer(i).fill_(i)
        for j in range(max(0, i - k + 1), i):
            assert pg.buffer(j).data_ptr() != pg.buffer(i).data_ptr()
            pg.buffer(j).fill_(j)   # (restore: buffer(j) is handed out again above)
        pg.submit(i)
    pg.drain()
    last = 3 * k - 1
    assert int(pg.gathered(last)[0][0]) == last
