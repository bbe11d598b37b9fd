"""GPU: the LDS-DMA build of the cross-cycle finest-level pass (k_postpre_glds: rows
brought into LDS by global_load_lds, three row pairs in flight, counted waits across the
per-pair barrier) is bit-identical to the register-staged k_postpre_lds, on the reference
problem and on a random phi0 with a non-zero boundary, over the band/column edge cases of
several grid sizes.  PGMG_PP_LDS_MODE=3 selects it."""
import os

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


@pytest.fixture
def env():
    saved = {}

    def set_(k, v):
        saved.setdefault(k, os.environ.get(k))
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v

    yield set_
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _run(pgmg, N, cycles, phi0=None, **cfg):
    with pgmg.Solver(N, **cfg) as s:
        s.set_problem(phi0, None)
        s.vcycle(cycles)
        return s.solution(), s.stats_detail()


@pytest.mark.parametrize("N", [65, 129, 257, 513, 1025, 2049, 4097])
@pytest.mark.parametrize("boundary", [False, True])
def test_glds_equals_register_staged(pgmg, env, N, boundary):
    env("PGMG_CROSS_MIN_N", "9")
    phi0 = None
    if boundary:
        rng = np.random.default_rng(N)
        phi0 = rng.uniform(-1, 1, (N, N))
    out = []
    for mode in ("0", "3"):
        env("PGMG_PP_LDS_MODE", mode)
        out.append(_run(pgmg, N, 4, phi0, tail_n=17 if N <= 129 else 65))
    assert_bitwise(out[1][0], out[0][0], f"glds vs lds N={N}")
    assert out[1][1] == out[0][1]


@pytest.mark.parametrize("blocks", ["512", "3072", "6144"])
def test_glds_band_heights(pgmg, env, blocks):
    """Band heights from 2 to ~40 row pairs (the ring wraps at every phase)."""
    env("PGMG_PP_BLOCKS", blocks)
    out = []
    for mode in ("0", "3"):
        env("PGMG_PP_LDS_MODE", mode)
        out.append(_run(pgmg, 4097, 3))
    assert_bitwise(out[1][0], out[0][0], f"blocks={blocks}")
