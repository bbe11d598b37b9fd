"""GPU: the small coarse levels' 2D LDS tile passes (pgmg_coarse.hip, r04) against the
row-marching passes they replace (PGMG_FLAG_NO_CTILE) and against the oracle: bitwise phi and
equal sweep / exit counts for V, W and F cycles, the reference problem and a random RHS with a
non-zero boundary, eps forcing every coarse check to fire (1e3), mixed (1e-2) or never (0),
fp32, speculative and in-stream (PGMG_FLAG_EXACT_DIST) calls, and grids whose coarse interior
is not a multiple of the tile (every N here: Nc - 2 = 2^k - 1)."""
import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _run(pgmg, N, kind, cycles, flags=0, f=None, phi0=None, dtype="f64", **cfg):
    with pgmg.Solver(N, flags=flags, dtype=dtype, **cfg) as s:
        s.set_problem(phi0, f)
        run = {"V": s.vcycle, "W": s.wcycle, "F": s.fcycle}[kind]
        for c in cycles:
            run(c)
        return s.solution(), s.stats()


CASES = [
    ("V", 129, [3], 1e-7), ("V", 513, [2, 1], 1e-7), ("V", 1025, [2], 1e-7),
    ("V", 2049, [3], 1e-7), ("V", 4097, [2], 1e-7), ("V", 513, [30], 1e-7),
    ("V", 257, [4], 1e3), ("V", 257, [4], 1e-2), ("V", 257, [3], 0.0),
    ("W", 129, [2], 1e-7), ("W", 257, [1, 1], 1e-7), ("W", 129, [2], 1e-2),
    ("F", 513, [1], 1e-7), ("F", 1025, [2], 1e-7),
]


@pytest.mark.parametrize("kind,N,cycles,eps", CASES)
def test_tiles_equal_row_marching(pgmg, kind, N, cycles, eps):
    a, sa = _run(pgmg, N, kind, cycles, eps=eps)
    b, sb = _run(pgmg, N, kind, cycles, flags=pgmg.PGMG_FLAG_NO_CTILE, eps=eps)
    assert_bitwise(a, b, f"{kind} N={N} eps={eps}")
    assert sa == sb


@pytest.mark.parametrize("N", [65, 257])
def test_tiles_random_rhs_boundary_vs_oracle(pgmg, oracle_mod, N):
    rng = np.random.default_rng(N + 5)
    f = rng.uniform(-1, 1, (N, N))
    phi0 = np.zeros((N, N))
    phi0[0, :] = rng.uniform(-1, 1, N)
    phi0[:, -1] = rng.uniform(-1, 1, N)
    for kind in ("V", "W"):
        o = oracle_mod.Oracle()
        ref = phi0.copy()
        for _ in range(3):
            (o.v_cycle if kind == "V" else o.w_cycle)(ref, f)
        got, (sw, _) = _run(pgmg, N, kind, [3], f=f, phi0=phi0, tail_n=17)
        assert_bitwise(got, ref, f"{kind} random rhs N={N}")
        assert sw == o.sweeps


def test_tiles_exact_in_stream_and_fp32(pgmg):
    for flags in (pgmg.PGMG_FLAG_EXACT_DIST, pgmg.PGMG_FLAG_NO_GRAPH):
        a, sa = _run(pgmg, 1025, "V", [3], flags=flags)
        b, sb = _run(pgmg, 1025, "V", [3], flags=flags | pgmg.PGMG_FLAG_NO_CTILE)
        assert_bitwise(a, b, f"flags={flags}")
        assert sa == sb
    a, sa = _run(pgmg, 513, "V", [3], dtype="f32")
    b, sb = _run(pgmg, 513, "V", [3], dtype="f32", flags=pgmg.PGMG_FLAG_NO_CTILE)
    assert np.array_equal(a.astype(np.float32).view(np.uint32), b.astype(np.float32).view(np.uint32))
    assert sa == sb
