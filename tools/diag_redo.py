"""Diagnostic: how many windows of a workload take refine_lane_kernel's wave-wide phase 3
(needs the -DSVT_DIAG=9 build in SVTREK_ENGINE_LIB; prints the engine's stderr count)."""
import sys
sys.path.insert(0, ".")
from svtrek_amd import Engine, Params, sim  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "cfg4_1m_delins_30x_hifi"
r = sim.generate(sim.WORKLOADS[w])
with Engine(Params(), device=0) as e:
    e.load_pileup(r.pileup)
    e.refine(r.loci)
print("windows", 2 * len(r.loci))
