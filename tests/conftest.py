import contextlib
import json
import pathlib
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running (large grids)")


@pytest.fixture(scope="session")
def pgmg():
    import _pkgload
    return _pkgload.load()


@pytest.fixture
def plan(pgmg):
    """plan(**cfg): pgmg_config fields applied to every Solver built during this test
    (pgmg.config_overrides; flags are OR-ed), e.g. plan(cross_min_n=9) to run the
    cross-cycle fused finest level on small grids."""
    stack = contextlib.ExitStack()

    def set_(**kw):
        stack.enter_context(pgmg.config_overrides(**kw))

    yield set_
    stack.close()


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def golden_cycles():
    return json.loads((GOLDEN / "cycles.json").read_text())


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def assert_bitwise(a, b, what=""):
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    diff = bits(a) != bits(b)
    if diff.any():
        idx = np.argwhere(diff)
        i = tuple(idx[0])
        raise AssertionError(
            f"{what}: {int(diff.sum())} of {diff.size} words differ; first at {i}: "
            f"{a[i]!r} vs {b[i]!r}; max|d|={np.max(np.abs(a - b)):.3e}")
