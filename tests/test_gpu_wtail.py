"""W-cycles through the LDS tail's speculative paths, against the oracle.

The tail decides some early-exit checks late in W-cycles (pgmg_tail.hip): the gamma coarsest
solves of a 9x9 visit as one Jacobi sequence with one reduction of the summed checks, the 9x9
visit's pre-smooth check after the visit (rollback when it did not fire), the 17x17
pre-smooth check after the restriction.  These eps values drive every branch: 1e3 (every
check fires: the fast paths always hold), 0 (no check fires: every fast path rolls back),
and values between (mixed, visit by visit).  Tolerance: EXACT (bitwise phi, equal sweep
counts), like tests/test_gpu_parity.py.
"""
import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N", [65, 129])
@pytest.mark.parametrize("eps", [1e-7, 1e3, 1e-2, 1e-4, 0.0])
def test_wcycle_eps_against_oracle(pgmg, oracle_mod, N, eps):
    o = oracle_mod.Oracle(eps=eps)
    f = o.rhs(N)
    ref = np.zeros((N, N))
    with pgmg.Solver(N, eps=eps) as s:
        s.set_problem()
        for k in range(4):
            o.w_cycle(ref, f)
            s.wcycle(1)
            assert_bitwise(s.solution(), ref, f"W N={N} eps={eps} cycle={k + 1}")
            assert s.stats()[0] == o.sweeps, (N, eps, k)


@pytest.mark.parametrize("v1,v2", [(2, 1), (1, 2), (0, 1), (1, 0)])
def test_wcycle_other_smoothing_counts(pgmg, oracle_mod, v1, v2):
    """v1/v2 != 1: the fast paths step aside (v1 = 0) or keep the exact post-smooth."""
    N = 129
    for eps in (1e-7, 1e-3):
        o = oracle_mod.Oracle(eps=eps, v1=v1, v2=v2)
        f = o.rhs(N)
        ref = np.zeros((N, N))
        with pgmg.Solver(N, v1=v1, v2=v2, eps=eps) as s:
            s.set_problem()
            for k in range(3):
                o.w_cycle(ref, f)
                s.wcycle(1)
                assert_bitwise(s.solution(), ref, f"W v1={v1} v2={v2} eps={eps} cycle={k + 1}")
                assert s.stats()[0] == o.sweeps, (v1, v2, eps, k)
