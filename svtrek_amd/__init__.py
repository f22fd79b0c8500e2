"""svtrek_amd -- MI355X-native engine for SVTrek's `audt` SV-refinement hot path.

Product path: include/svtrek_gpu.h (C ABI) implemented by libsvtrek_hip.so (HIP,
gfx950), driven by the `svtrek audt` CLI (csrc/svtrek_main.cpp) or from Python via
Engine.  See DESIGN.md.
"""
from ._lib import LOCUS_DTYPE, RESULT_DTYPE, SVT_DEL, SVT_INS, SVT_INV, SVT_NA  # noqa: F401
from .engine import Engine, Params, SvtError, version  # noqa: F401
from .pileup import Pileup, from_reads, make_loci  # noqa: F401

__all__ = ["Engine", "Params", "SvtError", "Pileup", "from_reads", "make_loci", "version",
           "LOCUS_DTYPE", "RESULT_DTYPE", "SVT_DEL", "SVT_INS", "SVT_INV", "SVT_NA"]
