"""bench.py -- refined SV loci/sec on MI355X (BASELINE.json metric), driver contract.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A step = one refinement pass of the HIP engine (svt_refine_device, one batched launch)
over one rank's shard of SV loci, with the pileup and loci already resident in HBM.
N>1: every rank owns its own shard (independent loci, no data-path collective: weak
scaling); each step ends with the one RCCL gather of refined calls to rank 0 that the
multi-GPU path performs.  Rank 0 prints ONE JSON line.

roofline: algorithmic bytes of the timed kernel (refine_event_kernel) per launch =
  16 B/locus in + 8 B/locus out + Σ_windows Σ_yielded reads (12 B + 4 B × CIGAR words walked)
(what the reference's walk touches; counted exactly by svt_count_work) ÷ the
kernel's mean duration, measured with HIP events on the launch stream.  The event walk reads
per-read summaries built once by svt_load_pileup (candidate-op lists, walk ends, chunk index)
instead of every CIGAR word, so `achieved` can exceed the HBM peak; `traffic` (measured HBM
bytes per launch, rocprofv3 PMC, profiles/traffic.json) and `traffic_frac` give the kernel's
physical bandwidth.  cpu_baseline: the CPU oracle (restatement of the reference's tpool path
over the same in-memory pileup) timed on rank 0's host cores on the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(res, n_threads: int, budget_s: float = 20.0) -> dict:
    """Time the CPU oracle (reference-shaped restatement, T pthread workers) on a bounded
    sample of the same workload.  Test-infrastructure leg: the only bench use of oracle/."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ffi as O  # noqa: E402

    loci = res.loci

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
    vt, dt_ = timed(len(loci), n_threads, budget_s * 2 / 3)
    return {
        "value": round(vt, 1), "unit": "loci/s", "cores": n_threads, "kind": "port",
        "sample": f"all {len(loci)} loci of the same workload, repeated for >= {budget_s * 2 / 3:.0f} s "
                  f"({dt_} loci), in-memory columnar pileup (no BGZF inflate), {n_threads} pthread workers on "
                  f"{_cpu_model()}; 1 thread: {v1:.1f} loci/s over {d1} loci (first {n1})",
        "value_1thread": round(v1, 1),
    }


def _engine_version() -> str:
    from svtrek_amd import version
    return version()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="cfg2_10kdel_30x_ont")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--scale", type=float, default=1.0,
                    help="diagnostic: scale the workload's locus count (and so its genome) by this factor")
    ap.add_argument("--replicate", type=int, default=1,
                    help="diagnostic: launch the workload's loci R times per step (tail-effect study)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from svtrek_amd import Engine, Params, sim
    from svtrek_amd._lib import RESULT_DTYPE

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    # ---- synthetic workload (BASELINE config), one shard per rank (weak scaling)
    cfg = sim.WORKLOADS[args.workload]
    if args.scale != 1.0:
        from dataclasses import replace
        cfg = replace(cfg, n_loci=max(1, int(cfg.n_loci * args.scale)))
    if world > 1:
        from dataclasses import replace
        cfg = replace(cfg, seed=cfg.seed + 1000 * rank)
    t0 = time.perf_counter()
    res = sim.generate(cfg)
    gen_s = time.perf_counter() - t0
    n = len(res.loci)

    eng = Engine(Params(), device=dev.index)
    t0 = time.perf_counter()
    eng.load_pileup(res.pileup)
    load_s = time.perf_counter() - t0
    load_stats = eng.load_stats()
    work = eng.count_work(res.loci)   # exact algorithmic work (diagnostic launch, untimed)

    if args.replicate > 1:
        import numpy as np
        res.loci = np.tile(res.loci, args.replicate)
        n = len(res.loci)
        work = {k: v * args.replicate for k, v in work.items()}
    loci_np = res.loci.view("u1").reshape(-1)
    d_loci = torch.from_numpy(loci_np.copy()).to(dev)
    d_out = torch.empty(n * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    gather_list = None
    if world > 1 and not args.no_gather:
        gather_list = [torch.empty_like(d_out) for _ in range(world)] if rank == 0 else None

    def step():
        eng.refine_device(d_loci.data_ptr(), n, d_out.data_ptr(), sh)
        if world > 1 and not args.no_gather:
            dist.gather(d_out, gather_list, dst=0)

    for _ in range(args.warmup):
        step()
    eng.sync(sh)

    # HIP events on the launch stream bracket the timed launches: with N = 1 nothing else runs
    # on that stream, so (end - start) / K is the kernel's average launch duration (plus the
    # few-us dispatch gap between back-to-back launches; no per-launch event packets in the
    # timed loop).  N > 1: per-launch event pairs, since the gathers share the stream order.
    per_launch = world > 1 and not args.no_gather
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps if per_launch else 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if not per_launch:
        ev[0][0].record(stream)
    for i in range(args.steps):
        if per_launch:
            ev[i][0].record(stream)
        eng.refine_device(d_loci.data_ptr(), n, d_out.data_ptr(), sh)
        if per_launch:
            ev[i][1].record(stream)
            dist.gather(d_out, gather_list, dst=0)
    if not per_launch:
        ev[0][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    eng.sync(sh)   # raises on a deferred spill-pool overflow
    if per_launch:
        kern_ms = sorted(a.elapsed_time(b) for a, b in ev)
        kern_mean_ms = sum(kern_ms) / len(kern_ms)
    else:
        kern_mean_ms = ev[0][0].elapsed_time(ev[0][1]) / args.steps
    # per-launch event pairs in a short untimed pass after the timed region (diagnostic: the
    # launch-duration spread; includes each pair's own event-packet overhead)
    pl = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for a_, b_ in pl:
        a_.record(stream)
        eng.refine_device(d_loci.data_ptr(), n, d_out.data_ptr(), sh)
        b_.record(stream)
    torch.cuda.synchronize(dev)
    kern_ms = sorted(a_.elapsed_time(b_) for a_, b_ in pl)

    t_max = wall
    if world > 1:
        tt = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())

    total_loci = n * world * args.steps
    value = total_loci / t_max
    alg_bytes = 24 * n + 12 * work["reads"] + 4 * work["ops_walked"]
    achieved = alg_bytes / (kern_mean_ms * 1e-3) / 1e9

    # HBM traffic of the timed kernel from the committed rocprofv3 PMC passes, when they were
    # taken on this engine version, workload and kernel (tools/gpu_profile.sh -> profiles/traffic.json)
    gather = os.environ.get("SVTREK_GATHER", "event")
    kernel = {"event": "refine_event_kernel", "index": "refine_index_kernel"}.get(gather, "refine_kernel")
    traffic = traffic_src = None
    try:
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
            tj = json.load(f)
        if (tj.get("engine_version") == _engine_version() and tj.get("workload") == args.workload
                and tj.get("kernel") == kernel and args.replicate == 1):
            traffic, traffic_src = int(tj["hbm_bytes_per_launch"]), tj.get("source")
    except (OSError, ValueError, KeyError):
        pass

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            avail = len(os.sched_getaffinity(0))
        except AttributeError:
            avail = os.cpu_count() or 1
        threads = args.cpu_threads or max(1, min(16, avail))
        cpu = cpu_baseline(res, threads)

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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded simpileup: ONT-like pileup + SV loci; no real BAM)",
            "config": {"workload": args.workload, "loci_per_gpu": n, "reads_per_gpu": res.pileup.n_reads,
                       "cigar_ops_per_gpu": res.pileup.n_ops, "coverage": cfg.coverage,
                       "read_len_mean": cfg.read_len_mean, "parallelism": f"loci-shard x{world}",
                       "gather": bool(world > 1 and not args.no_gather),
                       **({"loci_scale": args.scale} if args.scale != 1.0 else {})},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_gbs": round(traffic / (kern_mean_ms * 1e-3) / 1e9, 2) if traffic else None,
                         "traffic_frac": round(traffic / (kern_mean_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                         if traffic else None,
                         "traffic_source": traffic_src,
                         "kernel": kernel, "gather": gather, "kernel_ms_mean": round(kern_mean_ms, 5),
                         "kernel_ms_timing": "per-launch event pairs" if per_launch else
                         "one event pair around the timed launches / K",
                         "kernel_ms_min": round(kern_ms[0], 5),
                         "kernel_ms_mean_event_pairs": round(sum(kern_ms) / len(kern_ms), 5),
                         "alg_bytes_per_launch": alg_bytes,
                         "note": "achieved = the reference walk's bytes (SURVEY 8(d)) / kernel time; the event walk "
                                 "reads load-time per-read summaries instead of every CIGAR word, so achieved can "
                                 "exceed peak; traffic = measured HBM bytes per launch" if gather == "event" else None},
            # the query-independent device index (built once per pileup by svt_load_pileup, like
            # the reference's BAI) is outside the timed step; for transparency, the throughput
            # if every step rebuilt it too: loci / (step time + index-kernel time)
            "index_build": {"index_ms": load_stats["index_ms"], "load_ms": load_stats,
                            "value_if_rebuilt_every_step": round(
                                n * world / (t_max / args.steps + load_stats["index_ms"] * 1e-3), 1)},
            "cpu_baseline": cpu,
            "work": work,
            "setup_s": {"generate": round(gen_s, 2), "load_pileup": round(load_s, 2)},
            "pileup_device_bytes": eng.device_bytes,
            "engine_version": _engine_version(),
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
