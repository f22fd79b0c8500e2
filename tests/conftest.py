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

    def make(params=None, gather="span"):
        """gather: "span" (span events, default), "event" (candidate-op lists), "index" (chunk-index walk),
        "stream" (full CIGAR stream) or "perread" (per-read walk) -- the SVTREK_GATHER variants of the engine."""
        old = os.environ.get("SVTREK_GATHER")
        os.environ["SVTREK_GATHER"] = gather
        try:
            e = Engine(params or Params(), device=0)
        finally:
            if old is None:
                os.environ.pop("SVTREK_GATHER", None)
            else:
                os.environ["SVTREK_GATHER"] = old
        engines.append(e)
        return e

    yield make
    for e in engines:
        e.close()
