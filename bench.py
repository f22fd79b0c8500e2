"""bench.py -- refined SV loci/sec on MI355X (BASELINE.json metric), driver contract.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload: BASELINE config 4 by default (cfg4_1m_delins_30x_hifi: 1M DEL+INS calls over 22
contigs, 30x HiFi-like pileup) -- the configuration the >= 100k loci/s target is quoted on.
Every rank generates the same seeded workload; the loci are put in genomic order and rank g
refines the g-th contiguous slice against only the reads its queries can reach
(distributed.shard_workload), so the total work is fixed as N grows
("scaling": "strong").

A step is the whole per-locus path from the resident columnar pileup to refined calls:
  1. the device index build (svt_reindex: every read's CIGAR walked once,
     refinement.c:118-159/:184-221/:295-318): for short reads (cfg4) ix2_census_kernel +
     ix2_emit_kernel, one lane per read, a hipcub scan of the census totals between them;
     for long reads one pass over the stream: index_kernel (the stream walk, events staged
     per range) + a hipcub scan of the range totals + ix_copy_kernel (the staged rows placed)),
  2. one batched refine launch over the rank's slice (svt_refine_device_records:
     refine_lane_kernel + refine_redo_kernel; loci and 16-B result records resident in HBM),
  3. at N > 1, the one collective of the path: an RCCL gather to rank 0 of the slice's 16-B
     {vcf_index, start, end, pad} records, padded to ceil(N_total / N) rows (the gather of step i
     overlaps step i + 1; double-buffered records).
Rank 0 prints ONE JSON line.

roofline (HBM-bound integer work, no MFMA): `achieved` = the step's algorithmic bytes -- what
the engine's own algorithm must move: the index build's (svt_load_stats.index_bytes: the CIGAR
stream -- twice for the lane-per-read build, once for the stream walk --, per-read records and
offsets, the span events written) plus the refine launch's
(svt_work.event_bytes: loci, region queries, span bounds and events, 16-B result records) -- / the
step's mean duration from HIP events on the launch stream; `frac` = achieved / 8 TB/s.
`traffic` = the HBM bytes per step the rocprofv3 PMC passes of this engine version and workload
measured (profiles/traffic.json, tools/make_traffic.py), `frac_hbm` = traffic / step / 8 TB/s,
and `kernels` the same per kernel ({ms from the committed --stats summary, bytes, frac}).
`reference_equivalent` prices the step with SURVEY.md §8(d)'s bytes instead -- what the
reference's per-window CIGAR walk touches (24 B/locus + 12 B/yielded read + 4 B/CIGAR word walked,
svt_count_work): the engine walks each read once where the reference re-walks it per window, so
that rate is an effective one and may pass the peak.  cpu_baseline: the CPU oracle (restatement
of the reference's tpool path) on rank 0's host cores.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
DEFAULT_WORKLOAD = "cfg4_1m_delins_30x_hifi"


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_cores() -> tuple[int, int, float | None]:
    """(cores to use, CPUs in this process's affinity mask, cgroup CPU quota or None)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    n = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return n, aff, quota


def cpu_baseline(res, loci, n_threads: int, budget_s: float = 24.0, sample_loci: int = 1000) -> dict:
    """Time the CPU oracle (reference-shaped restatement, T pthread workers) on a bounded
    sample of the same workload.  Test-infrastructure leg: the only bench use of oracle/."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ffi as O  # noqa: E402

    def timed(n: int, threads: int, min_s: float) -> tuple[float, int]:
        """loci/s over repeated passes on loci[:n] until at least min_s of wall time."""
        done, t0 = 0, time.perf_counter()
        while True:
            O.refine_batch(res.pileup, loci[:n], threads=threads)
            done += n
            dt = time.perf_counter() - t0
            if dt >= min_s:
                return done / dt, done

    n0 = min(len(loci), 500)
    t = time.perf_counter()
    O.refine_batch(res.pileup, loci[:n0], threads=1)
    per_locus_1t = max(time.perf_counter() - t, 1e-6) / n0
    n1 = int(min(len(loci), max(n0, budget_s / 3 / per_locus_1t)))
    v1, d1 = timed(n1, 1, budget_s / 3)
    nt = int(min(len(loci), max(n0, budget_s * 2 / 3 / per_locus_1t * n_threads / 4)))
    vt, dt_ = timed(nt, n_threads, budget_s * 2 / 3)
    out = {
        "value": round(vt, 1), "unit": "loci/s", "cores": n_threads, "kind": "port",
        "sample": f"first {nt} loci of the workload (VCF order), repeated for >= {budget_s * 2 / 3:.0f} s "
                  f"({dt_} loci), {n_threads} pthread workers on {_cpu_model()}; in-memory columnar pileup; "
                  f"1 thread: {v1:.1f} loci/s over {d1} loci (first {n1})",
        "value_inmem": round(vt, 1),
        "value_inmem_1thread": round(v1, 1),
        "cpu_model": _cpu_model(),
    }
    # the BGZF leg: per-thread BAM handle + BAI, per-query linear-index seek,
    # block inflate and record decode, as the reference's htslib calls do -- the baseline value
    import bgzf_baseline as BB  # noqa: E402
    out.update(BB.run(res, loci, n_threads, budget_s=budget_s, k=sample_loci))
    if "value_bgzf" in out:
        out["value"] = out["value_bgzf"]
        out["sample"] = out["bgzf_sample"] + "; in-memory leg (no BGZF): " + out["sample"]
    return out


def _engine_version() -> str:
    from svtrek_amd import version
    return version()


def engine_lib_identity() -> dict:
    """The engine library this process binds (path relative to the repo, sha256, and whether
    SVTREK_ENGINE_LIB named a variant build) -- so an A/B variant cannot pass as the product."""
    import hashlib
    from svtrek_amd._lib import engine_path
    path = engine_path()
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return {"path": os.path.relpath(os.path.realpath(path), ROOT), "sha256": h.hexdigest(),
            "override": bool(os.environ.get("SVTREK_ENGINE_LIB"))}


def parity_sample(parts, res, first_rows, n_random: int = 10000, seed: int = 0, threads: int = 8,
                  full: bool = False) -> dict:
    """Untimed self-check of the timed records (the checker, like cpu_baseline: the only other bench
    use of oracle/): the records of the last step -- `parts`, the gathered {vcf_index, start, end,
    pad} buffers -- against the CPU oracle (refinement.c:327-339 restated) on the rows of the
    cpu_baseline sample (`first_rows`) plus a seeded random sample of n_random of the rows the
    records hold (every row with full=True).  Returns {"loci", "mismatches", ...}."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ffi as O  # noqa: E402
    from svtrek_amd.distributed import PAD_INDEX
    rec = np.concatenate([np.asarray(p).reshape(-1, 4) for p in parts]).astype(np.uint32)
    rec = rec[rec[:, 0] != PAD_INDEX]
    if full:
        pick = np.arange(len(rec))
    else:
        pos = np.full(len(res.loci), -1, dtype=np.int64)
        pos[rec[:, 0].astype(np.int64)] = np.arange(len(rec))
        want = np.asarray(first_rows, dtype=np.int64)
        want = want[pos[want] >= 0]
        rng = np.random.default_rng(seed)
        rnd = rng.choice(len(rec), size=min(n_random, len(rec)), replace=False)
        pick = np.unique(np.concatenate([pos[want], rnd]))
    rows = rec[pick, 0].astype(np.int64)
    want = O.refine_batch(res.pileup, res.loci[rows], threads=threads)
    bad = np.nonzero((rec[pick, 1] != want["start"]) | (rec[pick, 2] != want["end"]))[0]
    out = {"loci": int(len(rows)), "mismatches": int(len(bad)),
           "sample": ("every row the records hold" if full else
                      f"the cpu_baseline sample's rows + {min(n_random, len(rec))} seeded random rows (seed {seed})"),
           "oracle": "oracle/svtrek_oracle.c (CPU restatement of refinement.c / audit.c)"}
    if len(bad):
        k = int(bad[0])
        out["first"] = {"vcf_row": int(rows[k]), "got": [int(rec[pick[k], 1]), int(rec[pick[k], 2])],
                        "want": [int(want["start"][k]), int(want["end"][k])]}
    return out


STEP_KERNELS = ("ix2_census_kernel", "ix2_emit_kernel", "refine_lane_kernel", "refine_redo_kernel")
STREAM_INDEX_KERNELS = ("index_kernel", "ix_copy_kernel")   # the long-read index build (svt_index.inc)
BUCKET_INDEX_KERNELS = ("ixb_lane_kernel",)                  # the value buckets filed from the stream (short reads)
BUCKET_STREAM_KERNELS = ("index_kernel", "ixb_copy_kernel")   # ... from the stream walk's stage (long reads)


def index_kernels(load_stats: dict) -> tuple:
    """The kernels of one svt_reindex for this pileup (the step's index build)."""
    if load_stats.get("bucket_index"):
        return BUCKET_INDEX_KERNELS if load_stats.get("index_kind") == 1 else BUCKET_STREAM_KERNELS
    return STEP_KERNELS[:2] if load_stats.get("index_kind") == 1 else STREAM_INDEX_KERNELS


def _traffic(workload: str, records: bool) -> dict:
    """kernel -> profiles/traffic.json entry (HBM bytes per launch from the committed rocprofv3
    PMC passes, tools/make_traffic.py; "step" = their sum) for this engine version / workload."""
    try:
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return {}
    return {e["kernel"]: e for e in (tj if isinstance(tj, list) else [tj])
            if e.get("engine_version") == _engine_version() and e.get("workload") == workload
            and bool(e.get("records", False)) == records}


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str]) -> int:
    """`bench.py --gpus N` with no WORLD_SIZE in the environment: start N fresh rank processes
    (this script again, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one GPU each) and wait.

    The parent makes no torch / HIP call (it never imports torch), so the ranks are children,
    not an exec of a process that touched the GPU. Rank 0 prints the one JSON line (the
    children share this process's stdout). If any rank exits non-zero the others are
    terminated (by their own PIDs) and the first failing status is returned. This is the
    fan-out of the reference's T tpool workers (audit.c:287-293), one process per GPU."""
    import signal
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                print(f"bench.py: rank {procs.index(p)} exited with status {rc}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.send_signal(signal.SIGTERM)
        if live:
            time.sleep(0.05)
    return status


def dry_run(args, world: int, rank: int) -> int:
    """`--dry-run`: the N-rank plumbing of the bench on the CPU (gloo), no engine. Each rank
    shards the seeded workload exactly as the GPU run does, writes its slice's 16-B records
    (the loci unrefined: start = end = NA) into the multi-buffered gather for K steps, and
    rank 0 checks that every VCF row arrived exactly once and prints the one JSON line. It
    measures nothing (value is the plumbing's own rate) -- it exists so that the launcher, the
    rank environment and the gather are exercised without a GPU (tests/test_distributed.py)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from svtrek_amd import Params, sim
    from svtrek_amd._lib import RECORD_DTYPE, RESULT_DTYPE, SVT_NA
    from svtrek_amd.distributed import PipelinedGather, pack_records, padded_rows, shard_workload, unpack_records

    if world > 1:
        dist.init_process_group("gloo")
    cfg = sim.WORKLOADS[args.workload]
    if args.scale != 1.0:
        from dataclasses import replace
        cfg = replace(cfg, n_loci=max(1, int(cfg.n_loci * args.scale)))
    res = sim.generate(cfg)
    rows, sl, spile = shard_workload(res.loci, res.pileup, Params(), world, rank)
    n_total, per = len(res.loci), padded_rows(len(res.loci), world)
    # the records: the CPU oracle's results for the slice (a stand-in for the engine, so the
    # parity self-check below has real records to check; nothing here is timed as refinement)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ffi as O  # noqa: E402
    local = O.refine_batch(spile, sl, threads=2) if len(sl) else np.zeros(0, dtype=RESULT_DTYPE)
    if args.corrupt_record is not None and rank == world - 1 and len(sl):   # (tests: a mismatch fails the run)
        local = local.copy()
        k = args.corrupt_record % len(sl)
        local["start"][k] = (int(local["start"][k]) + 1) & 0xFFFFFFFF
    recs = torch.from_numpy(pack_records(rows, local, per).view(np.int32).reshape(-1).copy())
    pg = PipelinedGather(lambda: torch.full((per * RECORD_DTYPE.itemsize // 4,), -1, dtype=torch.int32),
                         world, rank, enabled=world > 1, nbuf=max(1, min(4, args.inflight)))   # (as the GPU run's)
    for i in range(args.warmup):
        pg.buffer(i).copy_(recs)
        pg.submit(i)
    pg.drain()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        pg.buffer(i).copy_(recs)
        pg.submit(i)
    pg.drain()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    tt = torch.tensor([wall], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    rc = 0
    if rank == 0:
        parts = [p.numpy().view(np.uint32).reshape(-1, 4) for p in pg.gathered(args.steps - 1)]
        unpack_records(np.concatenate(parts), n_total)
        ranks_seen = sum(int((p[:, 0] != 0xFFFFFFFF).any()) for p in parts)
        ps = parity_sample(parts, res, np.arange(min(n_total, 200)), n_random=500, threads=2)
        rc = 1 if ps["mismatches"] else 0
        print(json.dumps({
            "metric": "refined SV loci/sec (whole node)", "value": round(n_total * args.steps / float(tt.item()), 1),
            "unit": "loci/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(float(tt.item()) / max(args.steps, 1) * 1e3, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "int32",
            "data": "dry run: launcher + shard + gather plumbing on CPU (gloo), no refinement -- not a measurement",
            "dry_run": True,
            "config": {"workload": args.workload, "loci_total": n_total, "loci_per_gpu": len(sl),
                       "parallelism": f"genomic row shard x{world}", "gather": "gloo" if world > 1 else None},
            "gather_ranks": ranks_seen if world > 1 else 1, "records_verified": rc == 0,
            "parity_sample": ps,
            "records_note": "the slice records are the CPU oracle's results (stand-in for the engine)",
            "cpu_baseline": None,
            "cpu_baseline_note": "not timed in a dry run",
        }), flush=True)
        if rc:
            print(f"bench.py: parity self-check failed: {ps['mismatches']} of {ps['loci']} sampled loci differ "
                  f"from the oracle (first: {ps.get('first')})", file=sys.stderr, flush=True)
    if world > 1:
        dist.destroy_process_group()
    return rc


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one GPU each); without WORLD_SIZE in the environment, N > 1 starts the N "
                         "rank processes itself; under torch.distributed.run it must equal WORLD_SIZE")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU plumbing check: launcher, shard, gloo gather and the JSON line, no GPU, no refinement")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default=DEFAULT_WORKLOAD)
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cold", action="store_true")
    ap.add_argument("--inflight", type=int, default=3,
                    help="steps in flight (1-4): K engine contexts and streams, step i + 1's index build beside "
                         "step i's refine")
    ap.add_argument("--no-verify", action="store_true", help="diagnostic builds: skip the records checks")
    ap.add_argument("--parity-full", action="store_true",
                    help="check every timed record against the oracle (default: the cpu_baseline sample + 10k "
                         "seeded random rows)")
    ap.add_argument("--gather-backend", choices=("auto", "nccl", "gloo"), default="auto",
                    help="N > 1: the gather's backend; auto = nccl (RCCL over xGMI) when every rank has its own "
                         "GPU, else gloo through host memory (one-device emulation: ranks share device 0; not a "
                         "scaling number)")
    ap.add_argument("--corrupt-record", type=int, default=None, help=argparse.SUPPRESS)   # tests: dry run only
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-sample-loci", type=int, default=1000,
                    help="loci of the BGZF CPU leg's sample (the first K of contig 1, genomic order; 45000 ~ cfg4's "
                         "whole contig 1 -- the bytes tools/e2e_bench.py --region-sample K writes)")
    ap.add_argument("--emulate-shard", default=None, metavar="N:R",
                    help="diagnostic, one process: run rank R's slice of an N-GPU run (its loci and halo reads) "
                         "alone -- the per-rank work of the multi-GPU bench, measured on one GPU")
    ap.add_argument("--scale", type=float, default=1.0,
                    help="diagnostic: scale the workload's locus count (and so its genome) by this factor")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        if args.emulate_shard:
            ap.error("--emulate-shard runs one rank's slice in one process; it takes no --gpus N > 1")
        return launch_ranks(args.gpus, sys.argv[1:])
    world = int(env_world or "1")
    if world != args.gpus:
        ap.error(f"WORLD_SIZE={world} from the launcher but --gpus {args.gpus}: they must agree")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)

    import numpy as np
    import torch
    import torch.distributed as dist

    from svtrek_amd import Engine, Params, sim
    from svtrek_amd._lib import RECORD_DTYPE
    from svtrek_amd.distributed import PipelinedGather, padded_rows, shard_workload, unpack_records
    # one GPU per rank; fewer GPUs than ranks (a one-GPU box) is the one-device emulation: the ranks
    # share the devices round-robin and gather through host memory (gloo) -- the N-rank code path
    # with the engine, not a scaling number
    ndev = torch.cuda.device_count()
    emulated = world > 1 and ndev < world
    backend = args.gather_backend if args.gather_backend != "auto" else ("gloo" if emulated else "nccl")
    if emulated and backend == "nccl":
        ap.error(f"{world} ranks on {ndev} GPU(s): RCCL needs one GPU per rank (use --gather-backend gloo)")
    dev = torch.device("cuda", (local % ndev) if world > 1 else 0)
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    # ---- the workload (BASELINE config), identical on every rank; this rank's genomic slice
    cfg = sim.WORKLOADS[args.workload]
    if args.scale != 1.0:
        from dataclasses import replace
        cfg = replace(cfg, n_loci=max(1, int(cfg.n_loci * args.scale)))
    t0 = time.perf_counter()
    res = sim.generate(cfg, keep_handle=True)   # the handle writes the CPU baseline's sample BAM
    gen_s = time.perf_counter() - t0
    params = Params()
    t0 = time.perf_counter()
    if args.emulate_shard:
        en, er = (int(x) for x in args.emulate_shard.split(":"))
        rows, sl, spile = shard_workload(res.loci, res.pileup, params, en, er)
    else:
        rows, sl, spile = shard_workload(res.loci, res.pileup, params, world, rank)
    shard_s = time.perf_counter() - t0
    n_total, n = len(res.loci), len(sl)
    per = padded_rows(n_total, world)

    # K steps in flight (--inflight K): K engine contexts, each with the pileup and its own index
    # buffers, and K streams; step i runs on context / stream i % K, so step i + 1's index build
    # overlaps step i's refine.  Every step is the whole work (index build + refine of all loci).
    K = max(1, min(4, args.inflight))
    engs = [Engine(params, device=dev.index) for _ in range(K)]
    t0 = time.perf_counter()
    for e_ in engs:
        e_.load_pileup(spile)
    load_s = (time.perf_counter() - t0) / K
    eng = engs[0]
    load_stats = eng.load_stats()
    work = eng.count_work(sl)   # exact algorithmic work (counting kernel, untimed)

    d_loci = torch.from_numpy(np.ascontiguousarray(sl).view(np.uint8).copy()).to(dev)
    d_index = torch.from_numpy(rows.astype(np.uint32).view(np.int32)).to(dev)
    rec_words = per * RECORD_DTYPE.itemsize // 4
    # launch streams of their own, the first made current (the gather, the events and every
    # torch op of the bench are ordered on the stream of the step they belong to)
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    stream = streams[0]
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    gather = world > 1 and not args.no_gather
    pg = PipelinedGather(lambda: torch.full((rec_words,), -1, dtype=torch.int32, device=dev),   # pads: index ~0
                         world, rank, enabled=gather, nbuf=K,   # (buffer i % max(K, 2) <-> context i % K)
                         host_stage=backend == "gloo")

    def launch(i: int, k: int = 0) -> None:
        engs[k].refine_device_records(d_loci.data_ptr(), n, pg.buffer(i).data_ptr(), d_index.data_ptr(), 0,
                                      streams[k].cuda_stream)

    def step(i: int, k: int = 0) -> None:
        engs[k].reindex(streams[k].cuda_stream)   # the device index: every read's CIGAR walked once
        launch(i, k)                              # the batched refine over the rank's loci

    def run_step(i: int) -> None:
        k = i % K
        with torch.cuda.stream(streams[k]):
            step(i, k)
            pg.submit(i)

    for i in range(args.warmup):
        run_step(i)
    pg.drain()
    for k, e_ in enumerate(engs):
        e_.sync(streams[k].cuda_stream)

    # HIP events: the start on stream 0 after a device-wide sync, an end event per step on its
    # stream; the mean step duration = the last end - the start, / K steps (dispatch gaps and the
    # overlap of steps in flight included)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        run_step(i)
        ev[i].record(streams[i % K])
    pg.drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    for k, e_ in enumerate(engs):
        e_.sync(streams[k].cuda_stream)   # raises on a deferred spill-pool overflow
    step_ms = max(ev0.elapsed_time(e_) for e_ in ev) / args.steps

    t_max = wall
    if world > 1:
        tt = torch.tensor([wall], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())

    # ---- untimed: every VCF row arrives exactly once at rank 0 (last step's records), and the
    # records agree with the CPU oracle on a sample (the whole set with --parity-full)
    last = args.steps - 1
    verified = None
    gather_ranks = None
    parity = None
    rc = 0
    if rank == 0 and (gather or world == 1) and not args.no_verify:
        parts = [p.cpu().numpy().view(np.uint32).reshape(-1, 4) for p in pg.gathered(last)]
        if not args.emulate_shard:
            unpack_records(np.concatenate(parts), n_total)
        gather_ranks = sum(int((p[:, 0] != 0xFFFFFFFF).any()) for p in parts)
        cores_ps = cpu_cores()[0]
        parity = parity_sample(parts, res, rows[:min(len(rows), args.cpu_sample_loci)], threads=cores_ps,
                               full=args.parity_full)
        verified = parity["mismatches"] == 0
        rc = 0 if verified else 1

    # ---- untimed: the two phases on their own (5 runs each), and a step with the Infinity
    # Cache flushed first
    def timed_ms(fn, reps: int = 5) -> list[float]:
        pl = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a_, b_ in pl:
            a_.record(stream)
            fn()
            b_.record(stream)
        torch.cuda.synchronize(dev)
        return sorted(a_.elapsed_time(b_) for a_, b_ in pl)
    index_ms = statistics.median(timed_ms(lambda: eng.reindex(sh)))
    refine_ms = statistics.median(timed_ms(lambda: launch(0)))
    cold_ms = None
    if not args.no_cold:
        flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)   # 4x the 256 MiB MALL
        cold = []
        for k in range(3):
            flush.fill_(k + 1)
            cold += timed_ms(lambda: step(0), 1)
        cold_ms = statistics.median(cold)
        del flush
    eng.sync(sh)

    total_loci = (n if args.emulate_shard else n_total) * args.steps
    value = total_loci / t_max
    ref_bytes = 24 * n + 12 * work["reads"] + 4 * work["ops_walked"]
    ev_bytes = int(work["event_bytes"]) + 12 * n   # records: 16-B result record (not 8) + 4-B row index
    idx_bytes = int(load_stats.get("bucket_bytes" if load_stats.get("bucket_index") else "index_bytes", 0))
    alg_bytes = idx_bytes + ev_bytes               # the engine's algorithmic bytes of one step
    step_s = step_ms * 1e-3
    achieved = alg_bytes / step_s / 1e9
    refine_kernel = "refine_lane_kernel" if (os.environ.get("SVTREK_GATHER", "span") != "span1" and
                                             (os.environ.get("SVTREK_LANE_W") or 2 * n >= 65536)) \
        else "refine_span_kernel"   # the engine's size-based pick (svt_engine.hip, launch)
    tr = {} if (args.scale != 1.0 or world > 1 or args.emulate_shard) else _traffic(args.workload, records=True)
    traffic = int(tr["step"]["hbm_bytes_per_launch"]) if "step" in tr else None
    traffic_src = tr["step"].get("source") if "step" in tr else None
    kernels = {}
    for kname, e in tr.items():
        if kname == "step":
            continue
        ns, b = e.get("avg_ns"), int(e["hbm_bytes_per_launch"])
        kernels[kname] = {"ms": round(ns * 1e-6, 5) if ns else None, "bytes": b,
                          "gbs": round(b / (ns * 1e-9) / 1e9, 1) if ns else None,
                          "frac": round(b / (ns * 1e-9) / 1e9 / HBM_PEAK_GBS, 4) if ns else None}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores, aff, quota = cpu_cores()
        cpu = cpu_baseline(res, sl, args.cpu_threads or cores, sample_loci=args.cpu_sample_loci)
        cpu["affinity_cpus"] = aff
        cpu["cgroup_cpu_quota"] = quota

    if rank == 0:
        out = {
            "metric": "refined SV loci/sec (whole node)",
            "value": round(value, 1),
            "unit": "loci/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded simpileup: HiFi/ONT-like pileup + SV loci; no real BAM)",
            "config": {"workload": args.workload, "loci_total": n_total, "loci_per_gpu": n,
                       "reads_per_gpu": spile.n_reads, "cigar_ops_per_gpu": spile.n_ops,
                       "coverage": cfg.coverage, "read_len_mean": cfg.read_len_mean,
                       "parallelism": f"genomic row shard x{world}",
                       "gather": ("16-B records, RCCL gather to rank 0, overlapped with the next launch"
                                  if backend == "nccl" else "16-B records, gloo gather to rank 0 through host memory")
                       if gather else None,
                       **({"loci_scale": args.scale} if args.scale != 1.0 else {}),
                       **({"emulated_shard": args.emulate_shard} if args.emulate_shard else {})},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "frac_hbm": round(traffic / step_s / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
                         "traffic_gbs": round(traffic / step_s / 1e9, 2) if traffic else None,
                         "traffic_over_alg": round(traffic / alg_bytes, 4) if traffic else None,
                         "traffic_source": traffic_src,
                         "kernels": kernels or None,
                         "alg_bytes_per_launch": alg_bytes,
                         "alg_bytes": "the engine's algorithmic bytes of one step: index build (svt_load_stats."
                                      "index_bytes) + refine launch (svt_work.event_bytes + 12 B/locus records)",
                         "reference_equivalent": {
                             "bytes": ref_bytes, "gbs": round(ref_bytes / step_s / 1e9, 2),
                             "frac": round(ref_bytes / step_s / 1e9 / HBM_PEAK_GBS, 4),
                             "def": "SURVEY 8(d): 24 B/locus + 12 B/yielded read + 4 B/CIGAR word the reference walk "
                                    "consumes (svt_count_work); the engine walks each read once, the reference once "
                                    "per window that yields it, so this is an effective rate, not DRAM traffic"},
                         "kernel": "step = index build (" + ", ".join(index_kernels(load_stats)) + ") + refine (" +
                                   (refine_kernel + (", refine_redo_kernel" if refine_kernel == "refine_lane_kernel"
                                                     else "")) + ")",
                         "step_ms_mean": round(step_ms, 5),
                         "step_ms_timing": "HIP events: start on stream 0, the last step's end, / K",
                         "steps_in_flight": K,
                         "step_ms_cold": round(cold_ms, 5) if cold_ms else None,
                         "phases": {
                             "index_ms": round(index_ms, 5), "refine_ms": round(refine_ms, 5),
                             "index_alg_bytes": idx_bytes,
                             "index_gbs": round(idx_bytes / (index_ms * 1e-3) / 1e9, 2) if idx_bytes else None,
                             "index_bytes_def": ("value buckets (svt_load_stats.bucket_bytes): short reads, the CIGAR "
                                                 "stream once (4 B/op) + 24 B/read (offsets, record) + 28 B/filed event "
                                                 "(16-B event written, its bucket's two 4-B offsets read, 4-B cursor "
                                                 "incremented; a D > 50 op is filed twice); long reads, the stream "
                                                 "walk's stage: the stream once + 32 B/read + 32 B/staged event + 28 B/filed "
                                                 "event"
                                                 if load_stats.get("bucket_index") else
                                                 "lane per read: CIGAR stream twice (4 B/op; census + emit), 65 B/read "
                                                 "(census soff, clip byte, counts; emit counts, soff, rec, offsets), 16 B/span "
                                                 "event; stream walk: the stream once, 56 B/read (soff, rec, staged and "
                                                 "placed offsets), 48 B/span event (staged, read back, placed) "
                                                 "(svt_load_stats.index_bytes)"),
                         },
                         "engine_bytes": {"bytes": ev_bytes, "ms": round(refine_ms, 5),
                                          "gbs": round(ev_bytes / (refine_ms * 1e-3) / 1e9, 2),
                                          "kernel": refine_kernel,
                                          "def": ("the refine launch alone, priced with the value buckets' own bytes: "
                                                  "36 B/locus (locus, 16-B record + 4-B row index) + 12 B/bucket query "
                                                  "(two bucket offsets, one prefix-max key) + 16 B/event of the band's "
                                                  "buckets and of the walks for ABOVE (svt_work)"
                                                  if load_stats.get("bucket_index") else
                                                  "the refine launch alone, priced with the span walk's own bytes: "
                                                  "36 B/locus + 32 B/query + 4 B/search entry + 16 B/span bounds + "
                                                  "16 B/span event (svt_work)")}},
            "index_build": {"index_ms_load": load_stats["index_ms"], "load_ms": load_stats,
                            "value_index_resident": round((n if args.emulate_shard else n_total) / (refine_ms * 1e-3), 1),
                            "note": "value_index_resident: loci/s of the refine launch alone, the index built once "
                                    "(BAI-like amortisation); not the headline"},
            "cpu_baseline": cpu,
            **({} if cpu is not None else {"cpu_baseline_note":
                "timed on rank 0 at N = 1 only (a bounded sample of the same workload); this run has N = "
                f"{world}" if world > 1 else "skipped (--no-cpu-baseline or an emulated shard)"}),
            "work": work,
            "records_verified": verified,
            "parity_sample": parity,
            "gather_ranks": gather_ranks,
            "engine_lib": engine_lib_identity(),
            **({"emulation": f"one-device emulation: {world} ranks on {ndev} GPU(s), gather through host memory "
                             "(gloo) -- the N-rank path with the engine, not a scaling number"} if emulated else {}),
            "setup_s": {"generate": round(gen_s, 2), "shard": round(shard_s, 2), "load_pileup": round(load_s, 2)},
            "pileup_device_bytes": eng.device_bytes,
            "engine_version": _engine_version(),
        }
        print(json.dumps(out), flush=True)
        if rc:
            print(f"bench.py: parity self-check failed: {parity['mismatches']} of {parity['loci']} sampled loci "
                  f"differ from the oracle (first: {parity.get('first')})", file=sys.stderr, flush=True)
    for e_ in engs:
        e_.close()
    if world > 1:
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
