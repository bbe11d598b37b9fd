"""GPU: speculative calls (the early-exit checks of a V/W-cycle call are recorded and
validated once after the call instead of being decided by a fix-up launch after every
fused pass) give exactly the in-stream path's words and statistics: without a firing
check, across validated segments, after a rollback, for W-cycles, and after an F-cycle
rewrote the boundary frame of the level-0 buffers (the speculative cycles rotate through
the scratch grid S, which must mirror it).

PGMG_FLAG_EXACT_DIST selects the in-stream decisions; pgmg_config.spec_segment caps the
cycles per validated segment.
"""

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _run(pgmg, N, calls, problem=(None, None), cycle="v", **cfg):
    with pgmg.Solver(N, **cfg) as s:
        s.set_problem(*problem)
        for k in calls:
            getattr(s, f"{cycle}cycle")(k)
        return s.solution(), s.stats_detail(), s.dist_info()


@pytest.mark.parametrize("N,calls", [(2049, [5]), (4097, [3, 1]), (513, [4, 2])])
def test_speculative_equals_in_stream(pgmg, plan, N, calls):
    plan(cross_min_n=9)
    spec = _run(pgmg, N, calls)
    exact = _run(pgmg, N, calls, flags=pgmg.PGMG_FLAG_EXACT_DIST)
    assert spec[2] == (True, 0), spec[2]
    assert exact[2] == (False, 0), exact[2]
    assert_bitwise(spec[0], exact[0], f"N={N}")
    assert spec[1] == exact[1]


def test_speculative_segments_match_golden(pgmg, oracle_mod, golden_cycles, plan):
    """Seven cycles in one call validated in segments of two (each segment restarts the
    cross-fused chain: k_pre, k_postpre..., k_post) equal the reference's seven."""
    plan(cross_min_n=9)
    plan(spec_segment=int("2"))
    case = next(c for c in golden_cycles if c["kind"] == "V" and c["N"] == 513 and c["eps"] == 1e-7)
    k = min(7, len(case["cycles"]))
    phi, det, info = _run(pgmg, 513, [k])
    assert info == (True, 0)
    assert oracle_mod.fnv_hash(phi) == case["cycles"][k - 1]["hash"]
    assert det[0] == case["cycles"][k - 1]["sweeps"]


@pytest.mark.parametrize("seg", ["0", "1", "3"])
def test_speculative_rollback_then_in_stream(pgmg, oracle_mod, plan, seg):
    """eps above every norm, so every check fires: the first call is rolled back and rerun
    with in-stream decisions, later calls decide in-stream; every word is the oracle's."""
    plan(cross_min_n=9)
    if seg != "0":
        plan(spec_segment=int(seg))
    rng = np.random.default_rng(21)
    N, eps = 129, 1e9
    phi0 = rng.uniform(-1, 1, (N, N))
    f = rng.uniform(-1, 1, (N, N)) * 1e-3
    f[0, :] = f[-1, :] = f[:, 0] = f[:, -1] = 0.0
    o = oracle_mod.Oracle(eps=eps)
    ref = phi0.copy()
    for _ in range(6):
        o.v_cycle(ref, f)
    with pgmg.Solver(N, eps=eps, tail_n=17) as s:
        s.set_problem(phi0, f)
        s.vcycle(4)
        s.vcycle(2)
        assert_bitwise(s.solution(), ref, "after rollback")
        sp, rb = s.dist_info()
        assert sp and rb == 1, (sp, rb)
        assert s.stats_detail()[0] == o.sweeps
        assert o.early_exits > 0
        # a new problem speculates again (and, eps above every norm, rolls back again)
        s.set_problem()
        s.vcycle(2)
        assert s.dist_info()[1] == 2


def test_speculative_wcycle(pgmg, oracle_mod, golden_cycles, plan):
    plan(cross_min_n=9)
    case = next(c for c in golden_cycles if c["kind"] == "W" and c["N"] == 129)
    # W-cycles revisit the coarse levels until their checks fire (the reference's 129 W-cycle
    # exits 147 times in its first cycle): they decide in-stream, never roll back
    phi, _, info = _run(pgmg, 129, [len(case["cycles"])], cycle="w", tail_n=17)
    assert info[1] == 0
    assert oracle_mod.fnv_hash(phi) == case["cycles"][-1]["hash"]
    spec = _run(pgmg, 1025, [2], cycle="w")
    exact = _run(pgmg, 1025, [2], cycle="w", flags=pgmg.PGMG_FLAG_EXACT_DIST)
    assert_bitwise(spec[0], exact[0], "W 1025")
    assert spec[1] == exact[1]


def test_speculative_after_fcycle_nonzero_boundary(pgmg, plan):
    """F-cycle zeroes the frame of the level-0 buffers (reference semantics); the scratch
    grid the speculative V-cycles rotate through must follow, or the boundary of later
    V-cycles goes wrong."""
    plan(cross_min_n=9)
    rng = np.random.default_rng(8)
    N = 257
    phi0 = rng.uniform(-1, 1, (N, N))
    f = rng.uniform(-1, 1, (N, N))
    out = []
    for flags in (0, pgmg.PGMG_FLAG_EXACT_DIST):
        with pgmg.Solver(N, flags=flags) as s:
            s.set_problem(phi0, f)
            s.vcycle(2)
            s.fcycle(1)
            s.vcycle(3)
            out.append((s.solution(), s.stats_detail()))
    assert_bitwise(out[0][0], out[1][0], "F then V")
    assert out[0][1] == out[1][1]


def test_speculative_30_cycles_golden(pgmg, oracle_mod, golden_cycles, plan):
    """The reference's 30-cycle run at N = 513 (early exits from cycle 12 on, 112 in all)
    in segments of 5: the segments before the first firing check are kept, the one that
    contains it is rolled back and the rest of the call runs in-stream."""
    plan(cross_min_n=9)
    plan(spec_segment=int("5"))
    case = next(c for c in golden_cycles if c["kind"] == "V" and c["N"] == 513 and c["eps"] == 1e-7)
    last = case["cycles"][-1]
    phi, det, info = _run(pgmg, 513, [30])
    assert oracle_mod.fnv_hash(phi) == last["hash"]
    # exits <= the oracle's: a check after a smoother's final sweep is not evaluated here
    # (it cannot change anything)
    assert det[0] == last["sweeps"] and det[1] <= last["exits"]
    assert info[0] and info[1] <= 1


def test_speculation_predicts_firing_levels(pgmg):
    """The reference problem at N = 2049: the levels above the tail reach eps after ~27
    V-cycles.  After a short call the per-level decay predicts it, so a long call marks
    those levels in-stream up front instead of rolling back; words equal the in-stream
    run's."""
    out = []
    for flags in (0, pgmg.PGMG_FLAG_EXACT_DIST):
        with pgmg.Solver(2049, flags=flags) as s:
            s.set_problem()
            s.vcycle(3)
            s.vcycle(40)
            out.append((s.solution(), s.stats_detail(), s.dist_info(), s.spec_levels()))
    (phi, det, info, mask), (ref, rdet, _, rmask) = out
    assert info == (True, 0), info
    assert mask & ~1 and not mask & 1, bin(mask)   # coarse levels in-stream, level 0 speculating
    assert rmask & 1
    assert_bitwise(phi, ref, "2049 x 43")
    assert det == rdet
