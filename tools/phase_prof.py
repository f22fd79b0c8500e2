"""Phase attribution of refine_lane_kernel (diagnostic build with -DSVT_PHASE_PROF=1, named by
SVTREK_ENGINE_LIB): every wave adds the wall time of its phases (0: A2/A3 queries, 1: span
walks, 2: sort + vote, 3: redo list) and work counts; printed per launch.

    SVTREK_ENGINE_LIB=variants/x_phase.so python tools/phase_prof.py [--workload W] [--reps 5]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg4_1m_delins_30x_hifi")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from svtrek_amd import Engine, sim
    r = sim.generate(sim.WORKLOADS[a.workload])
    eng = Engine(device=0)
    eng.load_pileup(r.pileup)
    lib = eng.lib
    buf = (C.c_ulonglong * 16)()
    eng.refine(r.loci)
    lib.svt_diag_phase(buf)   # clear (warm-up launch)
    for _ in range(a.reps):
        eng.refine(r.loci)
    if lib.svt_diag_phase(buf):
        print("svt_diag_phase failed", file=sys.stderr)
        return 1
    v = [int(x) / a.reps for x in buf]
    waves = v[4]
    tot = sum(v[:4])
    out = {"workload": a.workload, "waves": waves,
           "phase_us_per_wave": [round(x / waves / 100.0, 3) for x in v[:4]],   # 100 MHz ticks
           "phase_frac": [round(x / tot, 3) for x in v[:4]],
           "walk_windows": v[8], "events": v[9], "walked_alone": v[10], "alone_256ev_steps": v[11],
           "packed_slots": v[12], "nmax<=8": v[13], "nmax<=16": v[14], "nmax<=32": v[15]}
    print(json.dumps(out))
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
