"""Allele-consensus (POA) mode throughput on a BASELINE workload's INS calls.

Times svt_poa_consensus (host arrays in and out: the PCIe copies of loci, results and
consensus bases are inside the timed call) over every INS locus of the workload after
refinement, and the CPU oracle (oracle/poa_oracle.c, one thread) on a bounded sample of the
same loci.  Prints one JSON line.  Test/measurement tool: the oracle is the baseline here,
never the thing measured.

    python tools/bench_poa.py [--workload cfg3_50k_delins_30x_ont] [--repeat 3] [--cpu-sample 200]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

from svtrek_amd import SVT_NA, Engine, Params, sim, version  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3_50k_delins_30x_ont")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--cpu-sample", type=int, default=200)
    ap.add_argument("--err-permille", type=int, default=50)
    ap.add_argument("--cap", type=int, default=4096)
    ap.add_argument("--check", type=int, default=50, help="loci checked bit-exactly against the oracle")
    a = ap.parse_args()

    cfg = sim.WORKLOADS[a.workload]
    t0 = time.perf_counter()
    r = sim.generate(cfg, keep_handle=True)
    off, bases = sim.insertion_sequences(r, cfg, err_permille=a.err_permille)
    t_gen = time.perf_counter() - t0
    ins = r.loci[r.loci["type"] == 1]
    eng = Engine(Params())
    eng.load_pileup(r.pileup)
    eng.load_insseq(off, bases)
    refined = eng.refine(ins)
    n_ref = int((refined["start"] != SVT_NA).sum())

    res, out = eng.poa_consensus(ins, refined, cap=a.cap)      # warm-up (scratch allocation)
    times = []
    for _ in range(a.repeat):
        t = time.perf_counter()
        res, out = eng.poa_consensus(ins, refined, cap=a.cap)
        times.append(time.perf_counter() - t)
    gpu_s = min(times)
    done = res["len"] >= 0
    fused = int(res["n_used"][done].sum())
    fused_bases = 0

    import oracle_ffi as O
    pl = r.pileup
    insop = ((pl.cigar & 15) == 1) & ((pl.cigar >> 4) >= 50)
    c = np.concatenate([[0], np.cumsum(insop, dtype=np.int64)])
    ib = c[pl.cig_off[:-1].astype(np.int64)].astype(np.uint64)
    pp = dict(O.POA_DEFAULTS)
    mi = eng.params.median_interval
    idx_done = np.flatnonzero(done)

    def oracle_locus(i):
        s = (int(ins["pos"][i]) - mi) & 0xFFFFFFFF
        e = (int(ins["pos"][i]) + mi) & 0xFFFFFFFF
        sup = O.poa_support(pl, ib, int(ins["chrom"][i]), s, e, int(refined["start"][i]), cap=pp["max_support"])
        seqs = [bases[off[k]:off[k + 1]] for k in sup]
        return O.poa_consensus(seqs), seqs

    mism = 0
    for i in idx_done[:a.check]:
        (want, used), _ = oracle_locus(i)
        if res["n_used"][i] != used or res["len"][i] != len(want) or \
                not np.array_equal(out[i, :min(len(want), a.cap)], want[:a.cap]):
            mism += 1
    sample = idx_done[:a.cpu_sample]
    t = time.perf_counter()
    for i in sample:
        (_, used), seqs = oracle_locus(i)
        fused_bases += sum(len(s) for s in seqs[:used])
    cpu_s = time.perf_counter() - t
    cpu_rate = len(sample) / cpu_s if cpu_s > 0 else None

    print(json.dumps({
        "metric": "INS allele consensus loci/sec (POA mode, 1 GPU)",
        "value": round(len(ins) / gpu_s, 1), "unit": "loci/s",
        "workload": a.workload, "ins_loci": int(len(ins)), "refined_ins": n_ref, "consensus_loci": int(done.sum()),
        "sequences_fused": fused, "deferred_to_full_slots": eng.poa_deferred, "gpu_s": round(gpu_s, 4), "gpu_s_all": [round(x, 4) for x in times],
        "timing": "svt_poa_consensus wall time incl. H2D of loci/results and D2H of consensus bases",
        "parity_checked": int(min(a.check, len(idx_done))), "parity_mismatches": mism,
        "cpu_baseline": {"value": round(cpu_rate, 2) if cpu_rate else None, "unit": "loci/s", "cores": 1,
                         "kind": "port", "sample": f"first {len(sample)} consensus loci, {fused_bases} bases fused"},
        "setup_s": {"generate": round(t_gen, 2)}, "engine_version": version(),
    }))
    eng.close()


if __name__ == "__main__":
    main()
