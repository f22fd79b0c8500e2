"""bench.py's N > 1 path with the HIP engine, on the one GPU a test box has.
`bench.py --gpus 2` starts two rank processes; with fewer GPUs than ranks they share device 0
and gather through host memory (gloo) -- the same shard, halo slice, K contexts per rank, launch
streams and multi-buffered gather as the 8-GPU run, checked here against the oracle on every row
of the full cfg4 workload (audit.c:269-293: the reference's T workers, one process per GPU here).
The line is labelled a one-device emulation: it is not a scaling number."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_one_device_full_parity():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--no-cold", "--parity-full"], env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["gather_ranks"] == 2 and out["records_verified"] is True
    ps = out["parity_sample"]
    assert ps["loci"] == out["config"]["loci_total"] == 1_000_000 and ps["mismatches"] == 0
    assert "emulation" in out and "not a scaling number" in out["emulation"]
    assert out["engine_lib"]["path"] == os.path.join("svtrek_amd", "libsvtrek_hip.so")
    assert not out["engine_lib"]["override"]
    print(json.dumps({k: out[k] for k in ("value", "ms_per_step", "n_gpus", "gather_ranks", "emulation")}))
