"""Diagnostic: which windows of a workload leave refine_lane_kernel for the wave-wide
refine_redo_kernel, and why.  Needs the -DSVT_DIAG=11 build in SVTREK_ENGINE_LIB: there each
left-over window's result is 0xF0000000 | reason (1 slow reads / window past 2^31, 2 band
off, 3 band > LV_CAP, 4 stop queue overflow, 5 stop value out of range, 6 band > LV_CAP after
the stop searches)."""
import collections
import sys

import numpy as np

sys.path.insert(0, ".")
from svtrek_amd import Engine, Params, sim  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "cfg4_1m_delins_30x_hifi"
r = sim.generate(sim.WORKLOADS[w])
with Engine(Params(), device=0) as e:
    e.load_pileup(r.pileup)
    got = e.refine(r.loci)
vals = np.concatenate([got["start"], got["end"]])
hits = vals[(vals & 0xF0000000) == 0xF0000000] & 0xFF
print("windows", 2 * len(r.loci), "left over", len(hits), dict(sorted(collections.Counter(hits.tolist()).items())))
