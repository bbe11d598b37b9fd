"""GPU: the carry (r06, include/pgmg.h above pgmg_vcycle; pgmg_ctx.hip "carry").

A speculative V call on the context's own grids ends with the carry pass, which also runs the
next cycle's pre-smooth, residual and restriction; the next pgmg_vcycle on the same problem
starts from them.  Entries that only read the problem keep the carry, every entry that changes
phi, f, eps, the flags or the cycle kind drops it.  Whatever the interleaving, phi and the
statistics must be the uncarried path's, bit for bit: the oracle (the CPU restatement of the
reference's MultigridSolver, pinned to the compiled reference by tests/test_oracle_golden.py)
runs the same sequence, and wherever the state is "k V-cycles from phi0 = 0 at eps = 1e-7" the
reference's own FNV-64 fixture (tests/golden/cycles.json) is checked too.

Reference semantics: MultigridSolver::v_cycle (2_part_MG/MultiGrid.hpp:57-94),
JacobiSmoother::smooth's per-sweep early exit (Smoother.hpp:59-88),
ParallelTestRunner::run_v_cycle's one-call-per-cycle loop (3_part_parallel/
ParallelTestRunner.cu:172-173).
"""

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu

EPS = 1e-7

# (op, arg): "v" k cycles, "res" pgmg_residual_norm, "sol" pgmg_get_solution (compared),
# "hash" pgmg_solution_hash, "set" pgmg_set_problem (phi0 = 0, analytic f), "eps" pgmg_set_eps,
# "f" pgmg_fcycle, "w" pgmg_wcycle.  30 cycle calls.
SEQ = [("v", 1), ("res", None), ("v", 1), ("sol", None), ("v", 1), ("res", None), ("v", 2),
       ("hash", None), ("v", 1), ("v", 1), ("sol", None), ("v", 3), ("res", None), ("v", 1),
       ("set", None), ("v", 1), ("v", 1), ("res", None), ("v", 1), ("eps", 1e-6), ("v", 1),
       ("sol", None), ("v", 1), ("f", 1), ("v", 1), ("res", None), ("v", 1), ("eps", EPS),
       ("v", 2), ("w", 1), ("v", 1), ("v", 1), ("sol", None), ("set", None), ("v", 1),
       ("res", None), ("v", 1), ("v", 1), ("f", 1), ("v", 1), ("v", 1), ("hash", None), ("v", 1),
       ("res", None), ("v", 1), ("sol", None), ("v", 2), ("v", 1)]


def _golden(golden_cycles, N):
    for c in golden_cycles:
        if c["kind"] == "V" and c["N"] == N and c["eps"] == EPS:
            return c["cycles"]
    return None


def _run_sequence(pgmg, oracle_mod, golden_cycles, N, seq, **cfg):
    gold = _golden(golden_cycles, N)
    o = oracle_mod.Oracle(eps=EPS)
    f = o.rhs(N)
    phi = np.zeros((N, N))
    base = 0
    pure = 0          # V-cycles from phi0 = 0 at eps = 1e-7 with nothing else in between (-1: no)
    checked_gold = 0
    calls = 0
    with pgmg.Solver(N, **cfg) as s:
        s.set_problem()

        def compare(what):
            nonlocal checked_gold
            assert_bitwise(s.solution(), phi, what)
            assert s.stats()[0] == o.sweeps - base, (what, s.stats()[0], o.sweeps - base)
            if pure > 0 and gold is not None and pure <= len(gold):
                assert oracle_mod.fnv_hash(phi) == gold[pure - 1]["hash"], (what, pure)
                assert o.sweeps - base == gold[pure - 1]["sweeps"], (what, pure)
                checked_gold += 1

        for i, (op, arg) in enumerate(seq):
            what = f"N={N} step {i} {op}({arg})"
            if op == "v":
                s.vcycle(arg)
                for _ in range(arg):
                    o.v_cycle(phi, f)
                pure = pure + arg if pure >= 0 else -1
                calls += 1
            elif op == "w":
                s.wcycle(arg)
                for _ in range(arg):
                    o.w_cycle(phi, f)
                pure = -1
                calls += 1
            elif op == "f":
                s.fcycle(arg)
                for _ in range(arg):
                    o.f_cycle_outer(phi)
                pure = -1
                calls += 1
            elif op == "set":
                s.set_problem()
                phi[:] = 0.0
                base = o.sweeps
                pure = 0 if o.c.eps == EPS else -1
            elif op == "eps":
                s.set_eps(arg)
                o.c.eps = arg
                pure = -1
            elif op == "res":
                got = s.residual_norm()
                r = oracle_mod.residual(phi, f, 1.0 / (N - 1))
                r[0, :] = r[-1, :] = r[:, 0] = r[:, -1] = 0.0
                want = float(np.sqrt(np.sum(r * r)))
                assert abs(got - want) <= 1e-12 * max(want, 1e-300), (what, got, want)
            elif op == "sol":
                compare(what)
            elif op == "hash":
                assert s.solution_hash(0) == oracle_mod.fnv_hash(phi), what
        compare(f"N={N} end")
        info = s.carry_info()
        rb = s.dist_info()[1]
    return info, checked_gold, calls, rb


@pytest.mark.parametrize("N", [513, 4097])
def test_carry_interleaved_api_sequence(pgmg, oracle_mod, golden_cycles, plan, N):
    """30+ cycle calls interleaved with residual_norm, get_solution, solution_hash,
    set_problem, set_eps, fcycle and wcycle: bitwise the oracle after every reading entry,
    sweep counts equal, the reference's fixture wherever the state is pure V-cycles."""
    if N < 2049:
        plan(cross_min_n=9)
    info, gold, calls, rb = _run_sequence(pgmg, oracle_mod, golden_cycles, N, SEQ)
    assert calls >= 30
    took, made, dropped = info
    assert took >= 10 and made >= took, info
    assert gold >= 2, gold


def test_carry_off_gives_the_same_words(pgmg, plan):
    """PGMG_FLAG_NO_CARRY: the same phi and statistics over one-cycle calls; with the carry
    on every call after the first takes it."""
    plan(cross_min_n=9)
    out = []
    for fl in (0, pgmg.PGMG_FLAG_NO_CARRY):
        with pgmg.Solver(1025, flags=fl) as s:
            s.set_problem()
            for _ in range(12):
                s.vcycle(1)
            s.vcycle(3)
            s.vcycle(1)
            out.append((s.solution(), s.stats_detail(), s.carry_info()))
    assert_bitwise(out[0][0], out[1][0], "carry vs no carry")
    assert out[0][1] == out[1][1]
    took, made, dropped = out[0][2]
    assert took >= 10 and made >= took, out[0][2]
    assert out[1][2] == (0, 0, 0), out[1][2]


def test_carry_dropped_when_its_check_could_fire(pgmg, oracle_mod, plan):
    """eps above every norm: every check fires, the first call rolls back (no carry made),
    later calls decide in-stream; a problem whose finest checks fire late drops carries
    whose pre-smooth check could fire.  Every word is the oracle's."""
    plan(cross_min_n=9)
    rng = np.random.default_rng(5)
    N = 257
    phi0 = rng.uniform(-1, 1, (N, N))
    f = rng.uniform(-1, 1, (N, N)) * 1e-3
    f[0, :] = f[-1, :] = f[:, 0] = f[:, -1] = 0.0
    for eps in (1e9, 2e-2, 5e-3):
        o = oracle_mod.Oracle(eps=eps)
        ref = phi0.copy()
        with pgmg.Solver(N, eps=eps, tail_n=17) as s:
            s.set_problem(phi0, f)
            for k in range(10):
                s.vcycle(1)
                o.v_cycle(ref, f)
                assert_bitwise(s.solution(), ref, f"eps={eps} call {k}")
                assert s.stats()[0] == o.sweeps, (eps, k)


def test_carry_then_rollback(pgmg, oracle_mod, plan):
    """A call that took a carry and is then rolled back (a coarse check predicted "does not
    fire" fires: spec_segment = 1 forces a validation per cycle, eps near the coarse norms)
    reruns from phi with its own k_pre: bitwise the oracle, rollbacks counted."""
    plan(cross_min_n=9, spec_segment=1)
    N = 513
    for eps in (1e-3, 3e-5, 1e-6):
        o = oracle_mod.Oracle(eps=eps)
        f = o.rhs(N)
        ref = np.zeros((N, N))
        with pgmg.Solver(N, eps=eps) as s:
            s.set_problem()
            for k in range(14):
                s.vcycle(1 if k % 3 else 2)
                for _ in range(1 if k % 3 else 2):
                    o.v_cycle(ref, f)
            assert_bitwise(s.solution(), ref, f"eps={eps}")
            assert s.stats()[0] == o.sweeps


def test_carry_full_size_single_calls(pgmg, golden_cycles):
    """N = 16385, 25 one-cycle calls (the reference harness's shape, the bench's
    context_single_calls leg): the reference's hash and sweep count after 25 cycles, every
    call after the first starting from the carry."""
    gold = _golden(golden_cycles, 16385)
    with pgmg.Solver(16385) as s:
        s.set_problem()
        for _ in range(25):
            s.vcycle(1)
        assert s.solution_hash(0) == gold[24]["hash"]
        assert s.stats()[0] == gold[24]["sweeps"]
        took, made, dropped = s.carry_info()
        assert took >= 20 and made >= took, (took, made, dropped)


def test_spin_wait_gives_the_same_words(pgmg, golden_cycles):
    """The validation's wait polls the reply word in pinned memory (pgmg_ctx.hip reply_wait);
    PGMG_FLAG_NO_SPIN waits on the stream instead: the same phi, statistics and carries over
    one-cycle calls at 4097, and the reference's hash after 12 cycles."""
    gold = _golden(golden_cycles, 4097)
    out = []
    for fl in (0, pgmg.PGMG_FLAG_NO_SPIN):
        with pgmg.Solver(4097, flags=fl) as s:
            s.set_problem()
            for _ in range(12):
                s.vcycle(1)
                s.residual_norm()
            assert s.solution_hash(0) == gold[11]["hash"]
            out.append((s.solution(), s.stats_detail(), s.carry_info()))
    assert_bitwise(out[0][0], out[1][0], "spin vs stream wait")
    assert out[0][1] == out[1][1]
    assert out[0][2] == out[1][2]


@pytest.mark.parametrize("variant", ["stored", "fast", "fast_stored", "f32", "f32_stored"])
@pytest.mark.parametrize("N", [1025, 4097])
def test_carry_forms_equal_uncarried(pgmg, plan, variant, N):
    """Every compiled form of the carry pass and of the recompute form (f streamed or
    regenerated, FAST, fp32) against the same calls with PGMG_FLAG_NO_CARRY: the same phi and
    statistics, bit for bit -- the recompute form's two stages reproduce the carry pass's
    pre-smooth exactly.  FAST (a tolerance mode: its cross-cycle passes use shared-sum
    expressions, its k_pre / k_post the reference's, so where a call starts and ends moves the
    last bits) is held to tests/test_gpu_fast.py's tolerance, 1e-12 relative, and equal sweeps."""
    plan(cross_min_n=9)
    flags = {"stored": pgmg.PGMG_FLAG_STORED_RHS, "fast": pgmg.PGMG_FLAG_FAST,
             "fast_stored": pgmg.PGMG_FLAG_FAST | pgmg.PGMG_FLAG_STORED_RHS,
             "f32": 0, "f32_stored": pgmg.PGMG_FLAG_STORED_RHS}[variant]
    dtype = "f32" if variant.startswith("f32") else "f64"
    out = []
    for fl in (flags, flags | pgmg.PGMG_FLAG_NO_CARRY):
        with pgmg.Solver(N, flags=fl, dtype=dtype) as s:
            s.set_problem()
            for k in range(10):
                s.vcycle(1)
                if k % 4 == 3:
                    s.residual_norm()
            s.vcycle(3)
            s.vcycle(1)
            out.append((s.solution(), s.stats_detail(), s.carry_info()))
    if variant.startswith("fast"):
        d = out[0][0] - out[1][0]
        rel = np.linalg.norm(d) / np.linalg.norm(out[1][0])
        assert rel <= 1e-12 and np.abs(d).max() <= 1e-12, (variant, rel)
    else:
        assert_bitwise(out[0][0], out[1][0], f"{variant} carry vs no carry")
    assert out[0][1] == out[1][1]
    took, made, dropped = out[0][2]
    assert took >= 9 and made >= took, out[0][2]
    assert out[1][2] == (0, 0, 0)
