"""GPU: PGMG_FLAG_L1POST (level 1's post-smooth inside the finest level's cross-cycle pass)
is bitwise the default path -- and so the reference (tests/golden/cycles.json) -- with the
same statistics: analytic and stored RHS, random problems, grids whose level 1 spans one or
many column blocks, fp32, and early-exit checks that fire (the speculative call is rolled
back and rerun in-stream, where the flag does not apply)."""
import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _run(pg, N, cycles, flags=0, problem=(None, None), **kw):
    with pg.Solver(N, flags=flags, **kw) as s:
        s.set_problem(*problem)
        for c in cycles if isinstance(cycles, (list, tuple)) else [cycles]:
            s.vcycle(c)
        return s.solution(), s.stats(), s.residual_norm()


def _same(pg, N, cycles, extra=0, **kw):
    ref = _run(pg, N, cycles, extra, **kw)
    got = _run(pg, N, cycles, extra | pg.PGMG_FLAG_L1POST, **kw)
    assert_bitwise(got[0], ref[0], f"L1POST N={N} flags={extra}")
    assert got[1] == ref[1]
    assert got[2] == ref[2]
    return got


@pytest.mark.parametrize("N,cycles", [(2049, 5), (4097, 3), (4097, [2, 1, 3])])
@pytest.mark.parametrize("stored", [False, True])
def test_l1post_bitwise_default(pgmg, N, cycles, stored):
    _same(pgmg, N, cycles, pgmg.PGMG_FLAG_STORED_RHS if stored else 0)


def test_l1post_matches_reference_golden(pgmg, oracle_mod, golden_cycles):
    case = next(c for c in golden_cycles if c["kind"] == "V" and c["N"] == 4097 and c["eps"] == 1e-7)
    n = min(len(case["cycles"]), 6)
    phi, _, _ = _run(pgmg, 4097, n, pgmg.PGMG_FLAG_L1POST)
    assert oracle_mod.fnv_hash(phi) == case["cycles"][n - 1]["hash"]


@pytest.mark.parametrize("N", [129, 257, 1025])
def test_l1post_small_grids(pgmg, plan, N):
    """Cross-cycle path forced on small grids: level 1 of 65 .. 513 points, one column
    block, bands that reach both frames."""
    plan(cross_min_n=9)
    _same(pgmg, N, 4, tail_n=9)
    _same(pgmg, N, 4, tail_n=33)


def test_l1post_random_problem(pgmg):
    rng = np.random.default_rng(11)
    N = 2049
    phi0 = rng.uniform(-1, 1, (N, N))
    f = rng.uniform(-1, 1, (N, N))
    for a in (phi0, f):
        a[0, :] = a[-1, :] = a[:, 0] = a[:, -1] = 0.0
    _same(pgmg, N, 3, problem=(phi0, f))


@pytest.mark.parametrize("eps", [1.0, 1e3])
def test_l1post_checks_fire(pgmg, eps):
    _same(pgmg, 2049, 4, eps=eps)


def test_l1post_fp32(pgmg):
    ref = _run(pgmg, 2049, 4, dtype="f32")
    got = _run(pgmg, 2049, 4, pgmg.PGMG_FLAG_L1POST, dtype="f32")
    a, b = np.ascontiguousarray(got[0]), np.ascontiguousarray(ref[0])
    assert a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))
    assert got[1] == ref[1]


@pytest.mark.slow
def test_l1post_full_size(pgmg, golden_cycles, oracle_mod):
    case = next((c for c in golden_cycles if c["kind"] == "V" and c["N"] == 16385), None)
    if case is None:
        pytest.skip("no 16385 golden")
    n = min(len(case["cycles"]), 4)
    phi, _, _ = _run(pgmg, 16385, n, pgmg.PGMG_FLAG_L1POST)
    assert oracle_mod.fnv_hash(phi) == case["cycles"][n - 1]["hash"]
