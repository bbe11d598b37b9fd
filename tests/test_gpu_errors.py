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


def test_span_check_bounds(pgmg):
    """The allocation registry behind the fused passes' read/write span checks
    (pgmg_check_span; DESIGN.md §2 "Read extents"): a level grid covers kHalo = 10 rows above
    and below its N rows, 15 elements before element (0, 0) and 512 elements of slack past
    its last halo row; one element outside is refused.  (Every other GPU test runs the same
    check before each fused launch: a false refusal would fail it.)"""
    import ctypes as C
    N = 1025
    with pgmg.Solver(N) as s:
        s.set_problem()
        ptr, pitch, row0, rows = C.c_void_p(), C.c_int(), C.c_int(), C.c_int()
        pgmg.check(s.lib.pgmg_phi_device(s.h, C.byref(ptr), C.byref(pitch), C.byref(row0),
                                         C.byref(rows)), "pgmg_phi_device")
        P = pitch.value
        assert P >= N and rows.value == N

        def span(r0, r1, c0, c1):
            return s.lib.pgmg_check_span(ptr, P, 8, r0, r1, c0, c1)

        assert span(-10, N + 9, -15, P - 1) == pgmg.PGMG_OK          # halos + offset
        assert span(N + 10, N + 10, 0, 511 - 15) == pgmg.PGMG_OK     # the slack
        assert span(-11, 0, 0, 0) == pgmg.PGMG_ERR_STATE             # above the top halo
        assert span(-10, -10, -16, 0) == pgmg.PGMG_ERR_STATE         # before the allocation
        assert span(N + 10, N + 10, 0, P - 1) == pgmg.PGMG_ERR_STATE  # past the slack
        assert span(0, 0, 0, 0) == pgmg.PGMG_OK
        # the check works on the grid's own allocation, not on neighbouring ones
        assert span(-10, 10 * N, 0, 0) == pgmg.PGMG_ERR_STATE
