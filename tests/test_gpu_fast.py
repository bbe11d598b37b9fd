"""FAST mode (PGMG_FLAG_FAST): the finest level's cross-cycle pass (N >= 2049) with shared
neighbour sums and FMA residuals, against the EXACT default (itself bitwise the reference).

Tolerance, after 10 V-cycles from phi0 = 0 (scripts/fast_tolerance.py, profiles/r02_c/fast/):
relative L2 and max-abs difference <= 1e-12 for N <= 4097, 2e-12 at 8193 (measured 5.5e-13)
and 3e-11 at 16385 (measured 7.4e-12).  SURVEY §8(c) asks 1e-12 at any N; at 16385 no
reordering can meet it: the residual f - (N-1)^2 (4x - S) carries an absolute rounding error of
(N-1)^2 * ulp(4x) ~ 2e-7 in either order, and the coarse-grid correction passes its smooth part
on, so two valid roundings of the same cycle differ by ~1e-11 relative there.  What FAST must
not change -- the sweep counts (early-exit decisions) and the solution's error against the
analytic solution -- is checked to the digit.  Row strips ignore the flag (bitwise)."""
import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _run(pg, N, cycles, flags, **kw):
    with pg.Solver(N, flags=flags, **kw) as s:
        s.set_problem()
        s.vcycle(cycles)
        return s.solution(), s.stats()[0]


TOL = {2049: 1e-12, 4097: 1e-12, 8193: 2e-12, 16385: 3e-11}


def _check(pgmg, oracle_mod, N, cycles, extra=0):
    ref, sw_ref = _run(pgmg, N, cycles, extra)
    got, sw = _run(pgmg, N, cycles, extra | pgmg.PGMG_FLAG_FAST)
    d = got - ref
    rel = np.linalg.norm(d) / np.linalg.norm(ref)
    assert rel <= TOL[N], rel
    assert np.max(np.abs(d)) <= TOL[N]
    assert sw == sw_ref
    assert not np.array_equal(got.view(np.uint64), ref.view(np.uint64)), "FAST ran the exact pass"
    u = oracle_mod.Oracle().exact(N)
    e_ref = np.linalg.norm(ref - u) / np.linalg.norm(u)
    e_got = np.linalg.norm(got - u) / np.linalg.norm(u)
    assert abs(e_got - e_ref) <= 1e-6 * e_ref, (e_got, e_ref)


@pytest.mark.parametrize("N,cycles", [(2049, 10), (4097, 10), (4097, 3)])
@pytest.mark.parametrize("stored", [False, True])
def test_fast_within_tolerance_of_exact(pgmg, oracle_mod, N, cycles, stored):
    _check(pgmg, oracle_mod, N, cycles, pgmg.PGMG_FLAG_STORED_RHS if stored else 0)


@pytest.mark.slow
@pytest.mark.parametrize("N", [8193, 16385])
def test_fast_large(pgmg, oracle_mod, N):
    _check(pgmg, oracle_mod, N, 10)


def test_fast_ignored_on_strips(pgmg):
    import threading
    N, W = 2049, 2
    ref, _ = _run(pgmg, N, 4, 0)
    hub = pgmg.LoopbackHub(W)
    out, err = [None] * W, [None] * W

    def rank(r):
        try:
            with pgmg.Solver(N, hub=hub, rank=r, flags=pgmg.PGMG_FLAG_FAST) as s:
                s.set_problem()
                s.vcycle(4)
                out[r] = s.solution()
        except Exception as e:  # surfaced below
            err[r] = e

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    hub.close()
    for e in err:
        if e is not None:
            raise e
    assert_bitwise(out[0], ref, "strips with PGMG_FLAG_FAST")
