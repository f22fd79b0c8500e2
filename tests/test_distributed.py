"""N>1 plumbing on CPU: world_size 2 (and 3) gloo processes shard the loci and gather the
results to rank 0 in VCF order.  The per-rank refinement here is the CPU oracle (test
infrastructure standing in for the GPU, which this container lacks); the sharding,
padding and gather code is the product's (svtrek_amd.distributed)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from svtrek_amd.distributed import shard_bounds


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, seed, outdir):
    import torch.distributed as dist

    import oracle_ffi as O
    from svtrek_amd import sim
    from svtrek_amd.distributed import run_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = sim.generate(sim.SimConfig(seed=seed, n_loci=97, n_targets=2, del_frac=0.6, coverage=12))
    res = run_sharded(r.loci, lambda l: O.refine_batch(r.pileup, l))
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
