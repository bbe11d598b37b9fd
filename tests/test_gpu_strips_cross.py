"""GPU: cross-cycle fusion of the finest level on row strips (k_postpre per rank, one
grouped halo exchange of phi and the coarse correction, one allreduce of three sums
per cycle) is bit-identical to one GPU and to the oracle, including both speculative
early-exit rare paths and non-zero Dirichlet boundaries.

Ranks are threads sharing the one GPU (loopback transport, see test_gpu_strips.py).
PGMG_CROSS_MIN_N=9 cross-fuses every grid size so small strips exercise it; each
Solver.vcycle(k) call is ONE multi-cycle call (k_pre, (children, k_postpre) x k-1,
children, k_post).
"""
import threading

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def cross_everywhere(pgmg):
    with pgmg.config_overrides(cross_min_n=9):
        yield


def _ranks(pgmg, world, N, cycles, problem=(None, None), **cfg):
    hub = pgmg.LoopbackHub(world)
    out, err = [None] * world, [None] * world

    def work(r):
        try:
            with pgmg.Solver(N, hub=hub, rank=r, **cfg) as s:
                s.set_problem(*problem)
                s.vcycle(cycles)
                out[r] = (s.solution(), s.stats_detail())
        except Exception as e:  # surfaced below
            err[r] = e

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    hub.close()
    for e in err:
        if e is not None:
            raise e
    return out


def _single(pgmg, N, cycles, problem=(None, None), **cfg):
    with pgmg.Solver(N, **cfg) as s:
        s.set_problem(*problem)
        s.vcycle(cycles)
        return s.solution(), s.stats_detail()


@pytest.mark.parametrize("world,N,gather_n", [(2, 1025, 65), (3, 1025, 129), (4, 1025, 65),
                                              (2, 2049, 1025), (8, 2049, 129), (4, 4097, 257)])
def test_strips_cross_bitwise_equal_single_gpu(pgmg, world, N, gather_n):
    ref = _single(pgmg, N, 4)
    assert ref[1][2] >= 0, "cross-cycle fusion not active"
    outs = _ranks(pgmg, world, N, 4, gather_n=gather_n)
    for r, (phi, det) in enumerate(outs):
        assert det[2] >= 0, "cross-cycle fusion not active on the strips"
        assert_bitwise(phi, ref[0], f"rank {r} of {world}")
    assert outs[0][1][:2] == ref[1][:2]


def test_strips_cross_matches_reference_golden(pgmg, oracle_mod, golden_cycles):
    case = next(c for c in golden_cycles if c["kind"] == "V" and c["N"] == 4097)
    k = case["cycles"][-1]["cycle"]
    outs = _ranks(pgmg, 4, 4097, k, gather_n=257)
    assert oracle_mod.fnv_hash(outs[0][0]) == case["cycles"][-1]["hash"]
    assert outs[0][1][0] == case["cycles"][-1]["sweeps"]


@pytest.mark.parametrize("world", [2, 4])
def test_strips_cross_rare_paths_and_boundary(pgmg, oracle_mod, world):
    """Random problem with a non-zero boundary; eps swept until both k_postpre rare paths
    have fired on the strips.  Every rank must equal the oracle word for word."""
    rng = np.random.default_rng(11)
    N = 257
    phi0 = rng.uniform(-1, 1, (N, N))
    f = rng.uniform(-1, 1, (N, N)) * 1e-3
    f[0, :] = f[-1, :] = f[:, 0] = f[:, -1] = 0.0
    seen = [0, 0]
    for eps in [10 ** (k / 10.0) for k in range(80, -20, -1)]:
        if seen[0] > 0 and seen[1] > 0:
            break
        o = oracle_mod.Oracle(eps=eps)
        ref = phi0.copy()
        for _ in range(5):
            o.v_cycle(ref, f)
        single = _single(pgmg, N, 5, problem=(phi0, f), eps=eps, tail_n=9)
        assert_bitwise(single[0], ref, f"1 GPU eps={eps}")
        outs = _ranks(pgmg, world, N, 5, problem=(phi0, f), eps=eps, tail_n=9, gather_n=33)
        for r, (phi, det) in enumerate(outs):
            assert_bitwise(phi, ref, f"rank {r} eps={eps}")
        det = outs[0][1]   # rank 0 also runs the gathered levels: it sees every sweep
        # exits <= oracle: a check after a smoother's final sweep is not evaluated (no effect)
        assert det[0] == o.sweeps and det[1] <= o.early_exits, (eps, det, o.sweeps)
        seen[0] += outs[0][1][2]
        seen[1] += outs[0][1][3]
    assert seen[0] > 0 and seen[1] > 0, seen


def test_strips_cross_fp32(pgmg):
    ref = _single(pgmg, 1025, 3, dtype="f32")
    outs = _ranks(pgmg, 4, 1025, 3, gather_n=65, dtype="f32")
    for r, (phi, _) in enumerate(outs):
        assert_bitwise(phi, ref[0], f"fp32 rank {r}")


def _ranks_info(pgmg, world, N, cycles, problem=(None, None), **cfg):
    hub = pgmg.LoopbackHub(world)
    out, err = [None] * world, [None] * world

    def work(r):
        try:
            with pgmg.Solver(N, hub=hub, rank=r, **cfg) as s:
                s.set_problem(*problem)
                s.vcycle(cycles)
                out[r] = (s.solution(), s.stats_detail(), s.dist_info())
        except Exception as e:  # surfaced below
            err[r] = e

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    hub.close()
    for e in err:
        if e is not None:
            raise e
    return out


def test_speculative_decisions_no_rollback_and_exact_mode(pgmg):
    """The reference problem: every distributed check is ruled out locally (huge norms),
    so the speculative call is never rolled back; PGMG_FLAG_EXACT_DIST (one allreduce per
    check) gives the same words and statistics."""
    ref = _single(pgmg, 2049, 4)
    spec = _ranks_info(pgmg, 4, 2049, 4, gather_n=129)
    exact = _ranks_info(pgmg, 4, 2049, 4, gather_n=129, flags=pgmg.PGMG_FLAG_EXACT_DIST)
    for r in range(4):
        assert spec[r][2] == (True, 0), spec[r][2]
        assert exact[r][2] == (False, 0), exact[r][2]
        assert_bitwise(spec[r][0], ref[0], f"speculative rank {r}")
        assert_bitwise(exact[r][0], ref[0], f"exact rank {r}")
    assert spec[0][1][:2] == exact[0][1][:2] == ref[1][:2]


def test_speculative_rollback_when_a_check_can_fire(pgmg, oracle_mod):
    """eps above every norm: every check fires, no rank can rule any out, the call is
    rolled back and rerun exactly; the result is the oracle's."""
    N, eps = 513, 1e9
    o = oracle_mod.Oracle(eps=eps)
    f = o.rhs(N)
    ref = np.zeros((N, N))
    for _ in range(3):
        o.v_cycle(ref, f)
    outs = _ranks_info(pgmg, 2, N, 3, eps=eps, tail_n=17, gather_n=33)
    for r, (phi, det, info) in enumerate(outs):
        assert_bitwise(phi, ref, f"rank {r}")
        assert info[0] and info[1] >= 1, info
    assert outs[0][1][0] == o.sweeps
