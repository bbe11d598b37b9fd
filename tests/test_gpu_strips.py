"""GPU: the row-strip decomposition (multi-rank path) is bit-identical to one GPU.

Ranks run as threads of this process sharing the one GPU of the test box, connected
by the library's loopback transport (PGMG_FLAG_LOOPBACK): same halo / allreduce /
gather-scatter messages as the RCCL transport, which RCCL itself cannot exercise
here (it refuses two ranks on one device).  The decomposition, halo depths, global
early-exit decision and the rank-0 coarse collapse are all the production code.
"""
import threading

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _run_ranks(pgmg, world, N, cycles, kind="V", **cfg):
    hub = pgmg.LoopbackHub(world)
    out = [None] * world
    err = [None] * world

    def work(r):
        try:
            with pgmg.Solver(N, hub=hub, rank=r, **cfg) as s:
                s.set_problem(*_problem.get(r, (None, None)))
                for _ in range(cycles):
                    (s.vcycle if kind == "V" else s.wcycle)(1)
                out[r] = (s.solution(), s.stats(), s.residual_norm())
        except Exception as e:  # surfaced below
            err[r] = e

    _problem = cfg.pop("problem", {})
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


def _single(pgmg, N, cycles, kind="V", problem=(None, None), **cfg):
    with pgmg.Solver(N, **cfg) as s:
        s.set_problem(*problem)
        for _ in range(cycles):
            (s.vcycle if kind == "V" else s.wcycle)(1)
        return s.solution(), s.stats(), s.residual_norm()


@pytest.mark.parametrize("world,N,gather_n", [(2, 1025, 65), (4, 1025, 65), (2, 2049, 257),
                                              (3, 1025, 129), (8, 4097, 129)])
def test_strips_vcycle_bitwise_equal_single_gpu(pgmg, world, N, gather_n):
    ref = _single(pgmg, N, 3)
    outs = _run_ranks(pgmg, world, N, 3, gather_n=gather_n)
    for r, (phi, stats, res) in enumerate(outs):
        assert_bitwise(phi, ref[0], f"rank {r} of {world}")
        assert abs(res - ref[2]) <= 1e-12 * ref[2]
    assert outs[0][1][0] == ref[1][0]     # rank 0 counts every level's sweeps once


def test_strips_match_reference_golden(pgmg, oracle_mod, golden_cycles):
    case = next(c for c in golden_cycles if c["kind"] == "V" and c["N"] == 4097)
    outs = _run_ranks(pgmg, 4, 4097, 3, gather_n=257)
    assert oracle_mod.fnv_hash(outs[0][0]) == case["cycles"][2]["hash"]


@pytest.mark.parametrize("eps", [1e3, 1.0])
def test_strips_early_exit_global_decision(pgmg, eps):
    """Forced / mixed early exits: all ranks must take the same (global) decision."""
    N = 1025
    ref = _single(pgmg, N, 4, eps=eps, tail_n=9)
    outs = _run_ranks(pgmg, 4, N, 4, eps=eps, tail_n=9, gather_n=33)
    for phi, stats, _ in outs:
        assert_bitwise(phi, ref[0], f"eps={eps}")
    assert outs[0][1] == ref[1]


def test_strips_unfused_and_wcycle(pgmg):
    N = 1025
    ref = _single(pgmg, N, 2, flags=pgmg.PGMG_FLAG_UNFUSED)
    outs = _run_ranks(pgmg, 2, N, 2, gather_n=65, flags=pgmg.PGMG_FLAG_UNFUSED)
    assert_bitwise(outs[1][0], ref[0], "unfused strips")
    ref = _single(pgmg, 513, 1, kind="W")
    outs = _run_ranks(pgmg, 2, 513, 1, kind="W", gather_n=65)
    assert_bitwise(outs[0][0], ref[0], "W strips")


def test_strips_other_smoothing_counts(pgmg):
    N = 1025
    ref = _single(pgmg, N, 2, v1=2, v2=0, eps=5.0, tail_n=17)
    outs = _run_ranks(pgmg, 2, N, 2, v1=2, v2=0, eps=5.0, tail_n=17, gather_n=65)
    assert_bitwise(outs[0][0], ref[0], "v1=2 v2=0 strips")


def test_strips_random_problem(pgmg):
    rng = np.random.default_rng(7)
    N = 1025
    phi0 = rng.uniform(-1, 1, (N, N))
    f = rng.uniform(-1, 1, (N, N))
    for a in (phi0, f):
        a[0, :] = a[-1, :] = a[:, 0] = a[:, -1] = 0.0
    ref = _single(pgmg, N, 2, problem=(phi0, f))
    outs = _run_ranks(pgmg, 4, N, 2, gather_n=65, problem={r: (phi0, f) for r in range(4)})
    for phi, _, _ in outs:
        assert_bitwise(phi, ref[0], "random strips")


@pytest.mark.parametrize("recompute", ["1", "0"])
@pytest.mark.parametrize("kind,eps", [("V", 1e-7), ("V", 1.0), ("W", 1e-7)])
def test_strips_extended_post_rows(pgmg, plan, recompute, kind, eps):
    """k_post of the levels below the finest computes kPostExt rows past its strip instead
    of exchanging the coarse correction: thin strips (16 rows at the deepest distributed
    level), with and without the recomputed pre-smoothed iterate, V and W cycles, forced
    coarse early exits — bitwise equal to one GPU."""
    if recompute == "0":
        plan(flags=pgmg.PGMG_FLAG_NO_RECOMPUTE)
    N = 1025
    ref = _single(pgmg, N, 2, kind=kind, eps=eps, tail_n=17)
    outs = _run_ranks(pgmg, 8, N, 2, kind=kind, eps=eps, tail_n=17, gather_n=65)
    for r, (phi, stats, _) in enumerate(outs):
        assert_bitwise(phi, ref[0], f"rank {r} recompute={recompute} {kind} eps={eps}")
    assert outs[0][1] == ref[1]
