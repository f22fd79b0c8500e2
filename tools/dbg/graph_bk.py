"""Debug: which step of a captured reindex sets the bucket-extent error word."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "oracle"))
import numpy as np, torch
from svtrek_amd import Engine, Params, sim
r = sim.generate(sim.SimConfig(seed=71, n_targets=2, n_loci=3000, del_frac=0.5, coverage=25.0))
eng = Engine(Params(), device=0)
eng.load_pileup(r.pileup)
def chk(tag):
    try:
        eng.sync(); print(tag, "ok", flush=True)
    except Exception as e:
        print(tag, "ERR", e, flush=True)
chk("load")
s = torch.cuda.Stream()
eng.reindex(s.cuda_stream); s.synchronize(); chk("direct on s")
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    eng.reindex(s.cuda_stream)
chk("after capture")
g.replay(); torch.cuda.synchronize(); chk("replay 1")
g.replay(); torch.cuda.synchronize(); chk("replay 2")
eng.reindex(); chk("direct null")
eng.reindex(s.cuda_stream); s.synchronize(); chk("direct s")
