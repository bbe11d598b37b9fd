"""GPU: randomised differential test of the speculative calls.

The speculative machinery -- per-call check logs validated after the call, rollbacks, segment
planning, per-cycle speculation windows, levels predicted to fire, W-cycle plans -- may only
change WHEN a check is decided, never what the reference's smoother does (Smoother.hpp:59-88:
after every sweep, stop when ||r|| < eps).  Hand-picked cases cover its branches
(test_gpu_spec.py, test_gpu_spec_fire.py); here a fixed-seed generator draws 40 problems over
the dimensions where a rollback or a prediction bug would hide:
  * N in {33 .. 2049} (and 4097 once), the cross-cycle fused finest level forced on
    (cross_min_n = 33) so every context speculates, tail_n in {9, 17, 33, 65};
  * eps log-uniform in [1e-10, 1e3] (from "never fires" to "every check fires");
  * the reference RHS or the mt19937_64 robustness RHS, with or without a random Dirichlet
    boundary;
  * 1 .. 6 calls of V, W or F cycles summing to 1 .. 40 cycles, spec_segment in {0, 2, 3, 5};
and every case is compared with the oracle (oracle/pgmg_oracle.c, pinned to the compiled
reference) -- phi bitwise, sweep counts equal -- and with the same calls decided in-stream
(PGMG_FLAG_EXACT_DIST: no speculation) -- phi, sweep and early-exit counts equal.  (The
oracle's exit count also books a check after a smoother's LAST sweep, which decides nothing;
the library books the exits that stop a smoother early.)  A failure names its case index;
re-run that index alone (-k) to reproduce it."""
import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu

SEED = 20261017
NCASES = 40


def _draw_cases():
    rng = np.random.default_rng(SEED)
    cases = []
    sizes = [33, 65, 129, 257, 513, 1025, 2049]
    for i in range(NCASES):
        N = 4097 if i == NCASES - 1 else int(rng.choice(sizes, p=[.12, .16, .2, .2, .16, .1, .06]))
        eps = float(10.0 ** rng.uniform(-10, 3))
        rhs = "mt" if rng.random() < 0.35 else "ref"
        boundary = rng.random() < 0.25
        ncalls = int(rng.integers(1, 7))
        budget = int(rng.integers(ncalls, 41))
        # W and F cycles are expensive in the oracle on big grids: cap their cycle counts
        calls = []
        left = budget
        for k in range(ncalls):
            kind = str(rng.choice(["V", "W", "F"], p=[0.6, 0.25, 0.15]))
            if kind == "W" and N > 513:
                kind = "V"
            n = left if k == ncalls - 1 else int(rng.integers(1, max(2, left - (ncalls - k - 1)) + 1))
            n = max(1, min(n, left - (ncalls - k - 1)))
            if kind != "V":
                n = min(n, 3)
            calls.append((kind, n))
            left -= n
            if left <= 0:
                break
        tail_n = int(rng.choice([9, 17, 33, 65]))
        seg = int(rng.choice([0, 2, 3, 5]))
        cases.append(dict(idx=i, N=N, eps=eps, rhs=rhs, boundary=boundary, calls=calls,
                          tail_n=min(tail_n, N), spec_segment=seg, bseed=int(rng.integers(1 << 30))))
    return cases


CASES = _draw_cases()


def _problem(oracle_mod, c):
    N = c["N"]
    f = oracle_mod.rhs_mt64(N) if c["rhs"] == "mt" else oracle_mod.Oracle().rhs(N)
    phi0 = np.zeros((N, N))
    if c["boundary"]:
        r = np.random.default_rng(c["bseed"])
        phi0[0, :] = r.uniform(-1, 1, N)
        phi0[-1, :] = r.uniform(-1, 1, N)
        phi0[:, 0] = r.uniform(-1, 1, N)
        phi0[:, -1] = r.uniform(-1, 1, N)
    return f, phi0


@pytest.mark.parametrize("c", CASES, ids=[f"case{c['idx']}-N{c['N']}" for c in CASES])
def test_speculative_calls_random(pgmg, oracle_mod, c):
    f, phi0 = _problem(oracle_mod, c)
    o = oracle_mod.Oracle(eps=c["eps"])
    want = phi0.copy()
    for kind, n in c["calls"]:
        for _ in range(n):
            if kind == "V":
                o.v_cycle(want, f)
            elif kind == "W":
                o.w_cycle(want, f)
            else:
                o.f_cycle_outer(want)
    runs = []
    for flags in (0, pgmg.PGMG_FLAG_EXACT_DIST):
        with pgmg.Solver(c["N"], eps=c["eps"], cross_min_n=33, tail_n=c["tail_n"],
                         spec_segment=c["spec_segment"], flags=flags) as s:
            s.set_problem(phi0, f)
            for kind, n in c["calls"]:
                {"V": s.vcycle, "W": s.wcycle, "F": s.fcycle}[kind](n)
            runs.append((s.solution(), s.stats(), s.dist_info()))
    (got, (sweeps, exits), (spec, _)), (exact, st_exact, (spec_x, _)) = runs
    # the first context speculated (when it has a bulk level above the tail), the second not
    assert spec == (c["N"] > c["tail_n"]) and not spec_x
    assert_bitwise(got, want, f"case {c['idx']}: {c}")
    assert_bitwise(exact, want, f"case {c['idx']} in-stream")
    assert sweeps == o.sweeps, (c, sweeps, o.sweeps)
    assert (sweeps, exits) == st_exact, (c, (sweeps, exits), st_exact)


def test_random_cases_cover_the_space():
    """The draw spans what it claims (a guard against a generator edit that narrows it)."""
    eps = [c["eps"] for c in CASES]
    assert min(eps) < 1e-8 and max(eps) > 10
    kinds = {k for c in CASES for k, _ in c["calls"]}
    assert kinds == {"V", "W", "F"}
    assert any(sum(n for _, n in c["calls"]) >= 25 for c in CASES)
    assert any(len(c["calls"]) >= 4 for c in CASES)
    assert any(c["N"] == 4097 for c in CASES) and any(c["N"] == 33 for c in CASES)
