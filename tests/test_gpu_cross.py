"""GPU: cross-cycle fusion of the finest level (k_postpre: post-smooth of cycle k and
pre-smooth + residual + restriction of cycle k+1 in one pass) is bit-identical to the
reference over multi-cycle calls, including both speculative early-exit rare paths.

pgmg_config.cross_min_n lowers the grid size from which the finest level is cross-fused so
small grids exercise it (default 2049)."""

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


@pytest.fixture
def cross_everywhere(pgmg):
    with pgmg.config_overrides(cross_min_n=9):
        yield


def _golden(golden_cycles, kind, N, eps=1e-7):
    return next(c for c in golden_cycles if c["kind"] == kind and c["N"] == N and c["eps"] == eps)


@pytest.mark.parametrize("N,eps,tail_n", [(129, 1e-7, 65), (129, 1e-7, 9), (513, 1e-7, 65),
                                          (33, 1e-7, 17), (129, 1e3, 65), (257, 1.0, 9),
                                          (65, 0.0, 33), (257, 1e-7, 17)])
def test_cross_multicycle_call_matches_golden(pgmg, oracle_mod, golden_cycles, cross_everywhere,
                                              N, eps, tail_n):
    case = _golden(golden_cycles, "V", N, eps)
    with pgmg.Solver(N, eps=eps, tail_n=tail_n) as s:
        assert s.stats_detail()[2] >= 0, "cross-cycle fusion not active"
        s.set_problem()
        k = len(case["cycles"])
        s.vcycle(k)                     # ONE call: k_pre, (children, k_postpre) x k-1, k_post
        phi = s.solution()
        assert oracle_mod.fnv_hash(phi) == case["cycles"][-1]["hash"]
        assert s.stats()[0] == case["cycles"][-1]["sweeps"]
        # and the context continues correctly after the buffer rotation
        if k >= 2:
            s.set_problem()
            s.vcycle(k - 1)
            s.vcycle(1)
            assert oracle_mod.fnv_hash(s.solution()) == case["cycles"][-1]["hash"]


def test_cross_rare_paths_fire_and_match_oracle(pgmg, oracle_mod, cross_everywhere):
    """Sweep eps on a random problem until both rare paths of k_postpre have fired."""
    rng = np.random.default_rng(3)
    N = 129
    phi0 = rng.uniform(-1, 1, (N, N))
    f = rng.uniform(-1, 1, (N, N)) * 1e-3
    for a in (phi0, f):
        a[0, :] = a[-1, :] = a[:, 0] = a[:, -1] = 0.0
    seen = [0, 0]
    for eps in [10 ** (k / 12.0) for k in range(96, -24, -1)]:
        if seen[0] > 0 and seen[1] > 0:
            break
        o = oracle_mod.Oracle(eps=eps)
        ref = phi0.copy()
        for _ in range(6):
            o.v_cycle(ref, f)
        with pgmg.Solver(N, eps=eps, tail_n=17) as s:
            s.set_problem(phi0, f)
            s.vcycle(6)
            assert_bitwise(s.solution(), ref, f"eps={eps}")
            d = s.stats_detail()
            assert d[0] == o.sweeps, (eps, d, o.sweeps)
            seen[0] += d[2]
            seen[1] += d[3]
    assert seen[0] > 0 and seen[1] > 0, seen


def test_cross_wcycle(pgmg, oracle_mod, golden_cycles, cross_everywhere):
    case = _golden(golden_cycles, "W", 129)
    with pgmg.Solver(129, tail_n=17) as s:
        s.set_problem()
        s.wcycle(3)
        assert oracle_mod.fnv_hash(s.solution()) == case["cycles"][-1]["hash"]


def test_cross_default_threshold_large_grid(pgmg, oracle_mod, golden_cycles):
    case = _golden(golden_cycles, "V", 4097)
    with pgmg.Solver(4097) as s:
        assert s.stats_detail()[2] >= 0
        s.set_problem()
        s.vcycle(3)
        assert oracle_mod.fnv_hash(s.solution()) == case["cycles"][2]["hash"]
        assert s.stats()[0] == case["cycles"][2]["sweeps"]


def test_cross_rare_paths_nonzero_boundary(pgmg, oracle_mod, cross_everywhere):
    """The rare paths rebuild the iterate in the scratch grid S; S must carry phi's
    Dirichlet boundary (set_problem mirrors it), or a non-zero boundary goes wrong."""
    rng = np.random.default_rng(5)
    N = 129
    phi0 = rng.uniform(-1, 1, (N, N))          # boundary included
    f = rng.uniform(-1, 1, (N, N)) * 1e-3
    seen = [0, 0]
    for eps in [10 ** (k / 12.0) for k in range(96, -24, -1)]:
        if seen[0] > 0 and seen[1] > 0:
            break
        o = oracle_mod.Oracle(eps=eps)
        ref = phi0.copy()
        for _ in range(6):
            o.v_cycle(ref, f)
        with pgmg.Solver(N, eps=eps, tail_n=17) as s:
            s.set_problem(phi0, f)
            s.vcycle(6)
            assert_bitwise(s.solution(), ref, f"eps={eps}")
            d = s.stats_detail()
            seen[0] += d[2]
            seen[1] += d[3]
    assert seen[0] > 0 and seen[1] > 0, seen


@pytest.mark.parametrize("N,dtype", [(513, "f64"), (2049, "f64"), (513, "f32")])
def test_regenerated_rhs_equals_stored_rhs(pgmg, cross_everywhere, N, dtype):
    """With the analytic RHS, k_postpre regenerates f in-kernel (fx[i] * sy[j]); the same
    multi-cycle call with PGMG_FLAG_STORED_RHS streams the stored f: identical words."""
    out = []
    for flags in (0, pgmg.PGMG_FLAG_STORED_RHS):
        with pgmg.Solver(N, dtype=dtype, flags=flags) as s:
            s.set_problem()
            gen = s.fine_pass_bytes(3) < s.fine_pass_bytes(0)
            assert gen == (flags == 0)
            s.vcycle(4)
            out.append((s.solution(), s.stats_detail()))
    assert_bitwise(out[0][0], out[1][0], f"regenerated vs stored f, N={N} {dtype}")
    assert out[0][1] == out[1][1]


def test_regenerated_rhs_rare_paths(pgmg, oracle_mod, cross_everywhere):
    """Analytic f (regenerated in k_postpre) with a random phi0 and eps swept until both
    k_postpre rare paths fire: bitwise to the oracle."""
    rng = np.random.default_rng(9)
    N = 129
    phi0 = rng.uniform(-1, 1, (N, N)) * 1e-3
    phi0[0, :] = phi0[-1, :] = phi0[:, 0] = phi0[:, -1] = 0.0
    seen = [0, 0]
    for eps in [10 ** (k / 12.0) for k in range(72, -36, -1)]:
        if seen[0] > 0 and seen[1] > 0:
            break
        o = oracle_mod.Oracle(eps=eps)
        f = o.rhs(N)
        ref = phi0.copy()
        for _ in range(6):
            o.v_cycle(ref, f)
        with pgmg.Solver(N, eps=eps, tail_n=17) as s:
            s.set_problem(phi0, None)
            s.vcycle(6)
            assert_bitwise(s.solution(), ref, f"eps={eps}")
            d = s.stats_detail()
            assert d[0] == o.sweeps, (eps, d, o.sweeps)
            seen[0] += d[2]
            seen[1] += d[3]
    assert seen[0] > 0 and seen[1] > 0, seen
