"""GPU: speculative F-cycles (pgmg_ctx.hip "speculative F-cycles") against the same F-cycles
decided in-stream (PGMG_FLAG_EXACT_DIST) and the oracle.

A call of F-cycles records every bulk early-exit check of its climb -- the V-cycles' passes and
the fused smooth(3)'s three checks -- as "does not fire" and validates them once after the
call; a failed check rolls the call back (the level buffers and statistics restored, the first
climb restarted from the saved tail-top grid) and reruns it in-stream.  Either way the result
is the reference's: phi bitwise, sweep and early-exit counts equal to the in-stream solver
(MultiGrid.hpp:138-183, Smoother.hpp:59-88).  Tolerance: EXACT.
"""
import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _run(pgmg, N, calls, flags=0, phi0=None, f=None, **cfg):
    with pgmg.Solver(N, flags=flags, **cfg) as s:
        s.set_problem(phi0, f) if phi0 is not None else s.set_problem()
        for kind, n in calls:
            {"F": s.fcycle, "V": s.vcycle, "W": s.wcycle}[kind](n)
        return s.solution(), s.stats(), s.dist_info()


@pytest.mark.parametrize("N,calls", [(129, [("F", 1)]), (129, [("F", 3)]), (1025, [("F", 2)]),
                                     (4097, [("F", 1), ("F", 2)]), (2049, [("V", 3), ("F", 2), ("V", 2)]),
                                     (513, [("F", 1), ("W", 1), ("F", 1)]), (257, [("F", 3)]),
                                     (2049, [("F", 4)]), (16385, [("F", 3)])])
def test_fspec_equals_in_stream(pgmg, N, calls):
    """Consecutive F-cycles of one call also exercise k_post_r2 (the finest k_post forming the
    next F-cycle's level-2 restriction, N >= 257), whose 116-column wave tiles form every
    level-2 centre column themselves (lanes 3..60 own the centres)."""
    got, st, info = _run(pgmg, N, calls)
    want, st_x, _ = _run(pgmg, N, calls, flags=pgmg.PGMG_FLAG_EXACT_DIST)
    assert_bitwise(got, want, f"N={N} calls={calls}")
    assert st == st_x
    assert info[1] == 0, info     # the reference problem: no bulk check of an F-cycle fires


def test_fspec_golden_16385(pgmg, oracle_mod, golden_cycles):
    """The reference's two F-cycles at 16385 (kind F in cycles.json), one speculative call."""
    case = next(c for c in golden_cycles if c["kind"] == "F" and c["N"] == 16385)
    with pgmg.Solver(16385) as s:
        s.set_problem()
        s.fcycle(2)
        assert oracle_mod.fnv_hash(s.solution()) == case["cycles"][1]["hash"]
        assert s.stats()[0] == case["cycles"][1]["sweeps"]
        assert s.dist_info()[1] == 0


@pytest.mark.parametrize("eps", [1e5, 1e3, 3.0, 1e-2])
@pytest.mark.parametrize("N", [129, 1025])
def test_fspec_rollback(pgmg, oracle_mod, N, eps):
    """eps at which checks fire (1e5: every one, the bulk levels' included; below it mostly the
    tail's, which decides in its own launch): a speculative call whose bulk check fires is
    rolled back and rerun in-stream (from the saved tail-top grid), bitwise the in-stream
    solver and the oracle; a second call on the problem decides in-stream from the start."""
    calls = [("F", 2), ("F", 1)]
    got, st, info = _run(pgmg, N, calls, eps=eps)
    want, st_x, _ = _run(pgmg, N, calls, eps=eps, flags=pgmg.PGMG_FLAG_EXACT_DIST)
    assert_bitwise(got, want, f"N={N} eps={eps}")
    assert st == st_x
    o = oracle_mod.Oracle(eps=eps)
    ref = np.zeros((N, N))
    for _ in range(3):
        o.f_cycle_outer(ref)
    assert_bitwise(got, ref, f"N={N} eps={eps} oracle")
    assert st[0] == o.sweeps
    if eps >= 1e5:
        assert info[1] == 1, info     # rolled back once, the second call in-stream


def test_fspec_random_boundary_and_rhs(pgmg, oracle_mod):
    """A non-zero Dirichlet boundary and the mt19937_64 RHS (the F-cycle restricts the current
    phi, so the boundary reaches the tail top's grid the rollback restarts from)."""
    N = 513
    rng = np.random.default_rng(11)
    phi0 = np.zeros((N, N))
    phi0[0, :], phi0[-1, :] = rng.uniform(-1, 1, N), rng.uniform(-1, 1, N)
    phi0[:, 0], phi0[:, -1] = rng.uniform(-1, 1, N), rng.uniform(-1, 1, N)
    f = oracle_mod.rhs_mt64(N)
    for eps in (1e-7, 10.0):
        calls = [("V", 2), ("F", 2)]
        got, st, _ = _run(pgmg, N, calls, phi0=phi0, f=f, eps=eps)
        want, st_x, _ = _run(pgmg, N, calls, phi0=phi0, f=f, eps=eps,
                             flags=pgmg.PGMG_FLAG_EXACT_DIST)
        assert_bitwise(got, want, f"eps={eps}")
        assert st == st_x


def test_fspec_fp32(pgmg):
    calls = [("F", 2)]
    got, st, info = _run(pgmg, 1025, calls, dtype="f32")
    want, st_x, _ = _run(pgmg, 1025, calls, dtype="f32", flags=pgmg.PGMG_FLAG_EXACT_DIST)
    assert_bitwise(got, want, "fp32")
    assert st == st_x and info[1] == 0
