"""GPU parity of the F-cycle (full multigrid).

Reference: MultigridTestRunner::run_cycle("F-cycle") (2_part_MG/MultiGridTestRunner.hpp:192-205)
-> MultigridSolver::compute_coarsest_grid + f_cycle (2_part_MG/MultiGrid.hpp:28-55,138-183):
phi is restricted to n_coarse, then each level up is smooth(3) -> prolongation into a zeroed
finer grid -> analytic RHS of the finer grid -> one V-cycle.  Checked bitwise against the
reference goldens (tests/golden/cycles.json, kind "F") and against the C oracle
(oracle/pgmg_oracle.c:orc_f_cycle_outer) for the cases the goldens do not hold.
"""
import numpy as np
import pytest

from conftest import ROOT

GOLD = ROOT / "tests" / "golden"

pytestmark = pytest.mark.gpu


def _golden(golden_cycles, N, eps=1e-7):
    return next(c for c in golden_cycles if c["kind"] == "F" and c["N"] == N and c["eps"] == eps)


def _run_golden(pgmg, oracle_mod, case, **cfg):
    N = case["N"]
    with pgmg.Solver(N, eps=case["eps"], **cfg) as s:
        s.set_problem()
        for row in case["cycles"]:
            s.fcycle(1)
            phi = s.solution()
            tag = f"F N={N} cycle={row['cycle']} cfg={cfg}"
            assert oracle_mod.fnv_hash(phi) == row["hash"], tag
            assert s.stats()[0] == row["sweeps"], tag


@pytest.mark.parametrize("N", [33, 129, 1025])
def test_fcycle_matches_reference_golden(pgmg, oracle_mod, golden_cycles, N):
    _run_golden(pgmg, oracle_mod, _golden(golden_cycles, N))


@pytest.mark.parametrize("tail_n", [5, 9, 17, 33])
def test_fcycle_bulk_levels(pgmg, oracle_mod, golden_cycles, tail_n):
    """A lower tail threshold moves FMG levels from the LDS tail onto the bulk kernels."""
    for N in (33, 129):
        _run_golden(pgmg, oracle_mod, _golden(golden_cycles, N), tail_n=tail_n)


def test_fcycle_full_vectors(pgmg):
    for N, k in ((33, 3), (129, 2)):
        want = np.load(GOLD / f"phi_F{N}_c{k}.npy")
        with pgmg.Solver(N) as s:
            s.set_problem()
            s.fcycle(k)
            got = s.solution()
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), N


def _oracle_f(oracle_mod, N, phi0, cycles, **kw):
    o = oracle_mod.Oracle(**kw)
    phi = phi0.copy()
    for _ in range(cycles):
        o.f_cycle_outer(phi)
    return phi, o


@pytest.mark.parametrize("cfg", [dict(flags=4), dict(v1=2, v2=2), dict(v1=0, v2=3),
                                 dict(eps=1.0), dict(eps=1e3), dict(eps=0.0)],
                         ids=["unfused", "v2", "v0v3", "eps1", "eps1e3", "eps0"])
def test_fcycle_vs_oracle_configs(pgmg, oracle_mod, cfg):
    N = 257
    okw = {k: v for k, v in cfg.items() if k in ("v1", "v2", "eps")}
    want, o = _oracle_f(oracle_mod, N, np.zeros((N, N)), 2, **okw)
    for tail_n in (9, 65):
        with pgmg.Solver(N, tail_n=tail_n, **cfg) as s:
            s.set_problem()
            s.fcycle(2)
            got = s.solution()
            assert s.stats()[0] == o.sweeps, (cfg, tail_n)
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), (cfg, tail_n)


def test_fcycle_from_nonzero_phi_and_after_vcycles(pgmg, oracle_mod):
    """The F-cycle restricts whatever phi holds (user boundary included) and leaves f alone:
    V-cycles after it still solve the user's problem."""
    N = 129
    rng = np.random.default_rng(11)
    phi0 = rng.standard_normal((N, N))
    f = rng.standard_normal((N, N))
    o = oracle_mod.Oracle()
    want = phi0.copy()
    o.f_cycle_outer(want)
    o.v_cycle(want, f)
    o.f_cycle_outer(want)
    with pgmg.Solver(N) as s:
        s.set_problem(phi0, f)
        s.fcycle(1)
        s.vcycle(1)
        s.fcycle(1)
        got = s.solution()
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_fcycle_nonunit_domain(pgmg, oracle_mod):
    """a != 1: the F-cycle's h chain starts at 1/(n_coarse-1) (MultiGridTestRunner.hpp:195),
    not a/(N-1) as the V-cycle's does."""
    N = 129
    o = oracle_mod.Oracle(a=2.0, p=1.0, q=3.0)
    want = np.zeros((N, N))
    o.f_cycle_outer(want)
    with pgmg.Solver(N, a=2.0, p=1.0, q=3.0, tail_n=17) as s:
        s.set_problem()
        s.fcycle(1)
        got = s.solution()
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_fcycle_tiny_grids(pgmg, oracle_mod):
    for N in (5, 9, 17):
        want, _ = _oracle_f(oracle_mod, N, np.zeros((N, N)), 2)
        with pgmg.Solver(N) as s:
            s.set_problem()
            s.fcycle(2)
            got = s.solution()
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), N


def test_fcycle_cross_context(pgmg, oracle_mod, golden_cycles, plan):
    """A context that runs cross-cycle fused V-cycles (swapped ping-pong buffers) still
    runs F-cycles on its current solution."""
    plan(cross_min_n=9)
    N = 257
    o = oracle_mod.Oracle()
    f = o.rhs(N)
    want = np.zeros((N, N))
    o.v_cycle(want, f)
    o.f_cycle_outer(want)
    o.v_cycle(want, f)
    o.v_cycle(want, f)
    with pgmg.Solver(N) as s:
        s.set_problem()
        s.vcycle(1)
        s.fcycle(1)
        s.vcycle(2)
        got = s.solution()
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


@pytest.mark.slow
def test_fcycle_4097_vs_oracle(pgmg, oracle_mod):
    N = 4097
    want, o = _oracle_f(oracle_mod, N, np.zeros((N, N)), 1)
    with pgmg.Solver(N) as s:
        s.set_problem()
        s.fcycle(1)
        got = s.solution()
        assert s.stats()[0] == o.sweeps
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


@pytest.mark.parametrize("N", [129, 2049])
def test_fcycle_regenerated_rhs_equals_stored(pgmg, N):
    """The F-cycle's level-0 passes regenerate the FMG chain's analytic RHS in-kernel;
    PGMG_FLAG_STORED_RHS streams it: identical words over repeated F-cycles (the cached
    level-0 RHS, the assigned prolongation and the zeroed frames included)."""
    out = []
    for flags in (0, pgmg.PGMG_FLAG_STORED_RHS):
        with pgmg.Solver(N, flags=flags) as s:
            s.set_problem()
            s.fcycle(2)
            s.vcycle(1)       # the V-cycle after an F-cycle uses the problem's own f again
            out.append((s.solution(), s.stats()))
    assert np.array_equal(out[0][0].view(np.uint64), out[1][0].view(np.uint64))
    assert out[0][1] == out[1][1]


def test_vcycle_graph_after_fused_smooth3_swaps(pgmg, oracle_mod):
    """The F-cycle's fused smooth(3) makes levels 1.. trade their A/B buffers; a V-cycle
    hipGraph captured before must be dropped and recaptured (N < 2049: graph replay)."""
    N = 513
    rng = np.random.default_rng(5)
    f = rng.standard_normal((N, N))
    f[0, :] = f[-1, :] = f[:, 0] = f[:, -1] = 0.0
    o = oracle_mod.Oracle()
    want = np.zeros((N, N))
    for _ in range(3):
        o.v_cycle(want, f)
    o.f_cycle_outer(want)
    for _ in range(3):
        o.v_cycle(want, f)
    with pgmg.Solver(N) as s:
        s.set_problem(None, f)
        s.vcycle(3)          # eager first cycle, then a captured graph
        s.fcycle(1)
        s.vcycle(3)
        got = s.solution()
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
