"""GPU: error paths leave a usable context behind.

An F-cycle on row strips that fails half-way (a transport error injected on every rank at
the same exchange through the loopback hub's test hook) must undo everything it changed on
the context — the level h chain, the level-0 RHS swap, the climb's regenerated-RHS level and
the per-level RHS swap — so that set_problem + V-cycles afterwards are the reference's
(advisor r01: state left set on an error path silently changes later V-cycles)."""
import threading

import pytest

pytestmark = pytest.mark.gpu


def _two_ranks(pgmg, N, fail_at, golden_hash, **cfg):
    hub = pgmg.LoopbackHub(2)
    res, err = [None, None], [None, None]

    def run(r):
        try:
            with pgmg.Solver(N, hub=hub, rank=r, **cfg) as s:
                s.set_problem()
                hub.fail(r, fail_at)
                failed = False
                try:
                    s.fcycle(1)
                    s.sync()
                except pgmg.PgmgError:
                    failed = True
                hub.fail(r, 0)
                s.set_problem()
                s.vcycle(3)
                phi = s.gather_solution(0, r == 0)
                res[r] = (failed, phi)
        except Exception as e:  # surfaced below
            err[r] = e

    ts = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    hub.close()
    for e in err:
        if e is not None:
            raise e
    return res


def test_vcycles_after_failed_fcycle_on_strips(pgmg, oracle_mod, golden_cycles):
    N = 1025
    case = next(c for c in golden_cycles if c["kind"] == "V" and c["N"] == N and c["eps"] == 1e-7)
    want = case["cycles"][2]["hash"]
    failures = 0
    for fail_at in (1, 2, 4, 7, 11):
        res = _two_ranks(pgmg, N, fail_at, want, gather_n=65, tail_n=17)
        assert res[0][0] == res[1][0], "ranks disagree on the failure"
        failures += res[0][0]
        assert oracle_mod.fnv_hash(res[0][1]) == want, f"V-cycles after a failed F-cycle (at {fail_at})"
    assert failures >= 3, "the injected failures did not hit the F-cycle"
