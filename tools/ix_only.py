"""Diagnostic: load a workload's pileup into one engine and rebuild its device index N times
(no refine launch), for PMC passes of the index kernels alone.
    python tools/ix_only.py [--workload NAME] [--builds N]   (SVTREK_ENGINE_LIB picks the engine)"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg4_1m_delins_30x_hifi")
    ap.add_argument("--builds", type=int, default=5)
    args = ap.parse_args()
    from svtrek_amd import Engine, Params, sim
    res = sim.generate(sim.WORKLOADS[args.workload])
    eng = Engine(Params(), device=0)
    eng.load_pileup(res.pileup)
    for _ in range(args.builds):
        eng.reindex(0)
    eng.sync(0)
    print("index builds:", args.builds, eng.load_stats())
    return 0


if __name__ == "__main__":
    sys.exit(main())
