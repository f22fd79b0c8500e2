import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build every native artefact once per session (no-op when up to date)."""
    from svtrek_amd import build
    build.build_all()
    yield


@pytest.fixture(scope="session")
def engine_factory():
    from svtrek_amd import Engine, Params

    engines = []

    # gather variant -> (SVTREK_GATHER, SVTREK_LANE_W)
    variants = {"span": ("span", "32"), "auto": ("span", None), "span1": ("span1", None)}

    def make(params=None, gather="span", env=None):
        """gather: "span" (span events through refine_lane_kernel<32> at every batch size -- the
        product picks it from 64K windows up), "span1" (one wave per
        window, refine_span_kernel: the product's pick for smaller batches) or "auto" (the product's
        size-based pick).  env: extra engine switches read at svt_open (e.g. SVTREK_IX=stream)."""
        g, lw = variants.get(gather, (gather, None))
        keys = ("SVTREK_GATHER", "SVTREK_LANE_W") + tuple(env or ())
        old = {k: os.environ.get(k) for k in keys}
        os.environ["SVTREK_GATHER"] = g
        os.environ.pop("SVTREK_LANE_W", None)
        if lw:
            os.environ["SVTREK_LANE_W"] = lw
        os.environ.update(env or {})
        try:
            e = Engine(params or Params(), device=0)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        engines.append(e)
        return e

    yield make
    for e in engines:
        e.close()
