"""GPU: the fp32 variant (PGMG_PRECISION_FP32; BASELINE config 5).

The reference is fp64-only, so the fp32 variant has two checks:

1. Bitwise against the fp32 restatement of mg_cpu_exec (oracle/liboracle_f32.so: the
   same C source compiled with -DORC_REAL=float — every grid value and operation in
   fp32, h*h and 1/(h*h) rounded once from fp64, norms accumulated in fp64).  The
   kernels keep the reference's expression order with -ffp-contract=off, so the fp32
   pass equals the fp32 oracle word for word, exactly as the fp64 pass equals the
   reference.  The only order-dependent value is again the early-exit norm.
2. A stated tolerance against fp64 (the library's fp64 path, itself bitwise equal to
   the reference goldens):  ||phi32 - phi64||_2 / ||phi64||_2 after 3 V-cycles from
   phi0 = 0 is at most FP32_TOL[N].  Calibrated on the fp32 oracle (2.9e-7 at N=33,
   7.5e-7 at 129, 5.8e-6 at 513, 1.7e-5 at 1025, 2.6e-4 at 2049): the fp32 round-off
   of the residual f - (1/h^2) A x grows like N^2, so the tolerance is per grid size.
"""
import threading

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu

# ||phi32 - phi64|| / ||phi64|| after 3 V-cycles (about 4x the oracle's measured value)
FP32_TOL = {33: 2e-6, 129: 4e-6, 513: 3e-5, 1025: 1e-4, 2049: 1.2e-3}


def _f32_oracle(oracle_mod, kind, N, cycles, phi0=None, f=None, **kw):
    o = oracle_mod.Oracle(dtype="f32", **kw)
    f = o.rhs(N) if f is None else np.ascontiguousarray(f, dtype=np.float32)
    phi = np.zeros((N, N), np.float32) if phi0 is None else np.array(phi0, np.float32)
    for _ in range(cycles):
        {"V": o.v_cycle, "W": o.w_cycle}[kind](phi, f) if kind != "F" else o.f_cycle_outer(phi)
    return phi.astype(np.float64), o


@pytest.mark.parametrize("N,tail_n,mode", [(9, 65, "fused"), (33, 17, "fused"), (129, 65, "fused"),
                                           (129, 9, "fused"), (513, 65, "fused"),
                                           (129, 33, "unfused"), (257, 17, "cross"),
                                           (513, 65, "cross"), (129, 17, "norecompute"),
                                           (2049, 65, "fused"), (1025, 65, "cross"),
                                           (2049, 33, "cross_stored"), (4097, 65, "cross")])
def test_fp32_vcycle_bitwise_vs_fp32_oracle(pgmg, oracle_mod, plan, N, tail_n, mode):
    cfg = dict(dtype="f32", tail_n=tail_n)
    if mode == "unfused":
        cfg["flags"] = pgmg.PGMG_FLAG_UNFUSED
    if mode in ("cross", "cross_stored"):
        # the cross-cycle finest pass (fp32: k_postpre_lds<float>, two columns per lane; several
        # column blocks from N = 1025 on, the analytic f regenerated or, stored, streamed)
        plan(cross_min_n=9)
    if mode == "cross_stored":
        cfg["flags"] = pgmg.PGMG_FLAG_STORED_RHS
    if mode == "norecompute":
        cfg["flags"] = pgmg.PGMG_FLAG_NO_RECOMPUTE
    cycles = 3
    ref, o = _f32_oracle(oracle_mod, "V", N, cycles)
    with pgmg.Solver(N, **cfg) as s:
        assert s.elem_bytes == 4
        s.set_problem()
        if mode in ("cross", "cross_stored"):
            assert s.stats_detail()[2] >= 0, "cross-cycle fusion not active"
            s.vcycle(cycles)
        else:
            for _ in range(cycles):
                s.vcycle(1)
        got = s.solution()
        assert s.stats()[0] == o.sweeps
    assert_bitwise(got, ref, f"fp32 V N={N} {mode}")


@pytest.mark.parametrize("kind,N,cycles", [("W", 33, 2), ("W", 129, 2), ("F", 33, 2),
                                           ("F", 129, 1), ("F", 1025, 1)])
def test_fp32_w_and_f_cycles_bitwise_vs_fp32_oracle(pgmg, oracle_mod, kind, N, cycles):
    ref, o = _f32_oracle(oracle_mod, kind, N, cycles)
    with pgmg.Solver(N, dtype="f32") as s:
        s.set_problem()
        for _ in range(cycles):
            (s.wcycle if kind == "W" else s.fcycle)(1)
        assert_bitwise(s.solution(), ref, f"fp32 {kind} N={N}")
        assert s.stats()[0] == o.sweeps


def test_fp32_early_exit_rare_paths_bitwise(pgmg, oracle_mod, plan):
    """Random problem, eps swept until early exits fire on bulk and tail levels and both
    k_postpre rare paths have run: still bitwise equal to the fp32 oracle."""
    plan(cross_min_n=9)
    rng = np.random.default_rng(7)
    N = 129
    phi0 = rng.uniform(-1, 1, (N, N))
    f = rng.uniform(-1, 1, (N, N)) * 1e-3
    for a in (phi0, f):
        a[0, :] = a[-1, :] = a[:, 0] = a[:, -1] = 0.0
    phi0 = phi0.astype(np.float32).astype(np.float64)   # representable in fp32
    f = f.astype(np.float32).astype(np.float64)
    exits = 0
    seen = [0, 0]
    for eps in [10 ** (k / 8.0) for k in range(64, -16, -1)]:
        if exits > 0 and seen[0] > 0 and seen[1] > 0:
            break
        ref, o = _f32_oracle(oracle_mod, "V", N, 5, phi0=phi0, f=f, eps=eps)
        with pgmg.Solver(N, dtype="f32", eps=eps, tail_n=17) as s:
            s.set_problem(phi0, f)
            s.vcycle(5)
            assert_bitwise(s.solution(), ref, f"fp32 eps={eps}")
            d = s.stats_detail()
            assert d[0] == o.sweeps and d[1] <= o.early_exits, (eps, d, o.sweeps, o.early_exits)
            exits += d[1]
            seen[0] += d[2]
            seen[1] += d[3]
    assert exits > 0 and seen[0] > 0 and seen[1] > 0, (exits, seen)


@pytest.mark.parametrize("N", sorted(FP32_TOL))
def test_fp32_within_stated_tolerance_of_fp64(pgmg, N):
    sols = {}
    for dt in ("f64", "f32"):
        with pgmg.Solver(N, dtype=dt) as s:
            s.set_problem()
            s.vcycle(3)
            sols[dt] = s.solution()
    d = np.linalg.norm(sols["f32"] - sols["f64"]) / np.linalg.norm(sols["f64"])
    assert d <= FP32_TOL[N], (N, d)


@pytest.mark.parametrize("exact", [False, True])
def test_fp32_strips_bitwise_equal_single_gpu(pgmg, plan, exact):
    """Row strips (loopback transport, 4 ranks) in fp32: same words as one GPU in fp32
    (halo rows and gathered levels move 4-byte elements).  exact: every check decided
    in-stream (PGMG_FLAG_EXACT_DIST) with the cross-cycle finest pass on, so the strips run
    k_postpre_lds<float>'s third sum (R2)."""
    N, world = 1025, 4
    if exact:
        plan(cross_min_n=9, flags=pgmg.PGMG_FLAG_EXACT_DIST)
    with pgmg.Solver(N, dtype="f32") as s:
        s.set_problem()
        s.vcycle(3)
        ref = s.solution()
    hub = pgmg.LoopbackHub(world)
    out, err = [None] * world, [None] * world

    def work(r):
        try:
            with pgmg.Solver(N, hub=hub, rank=r, gather_n=65, dtype="f32") as s:
                s.set_problem()
                s.vcycle(3)
                out[r] = s.solution()
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
    for r in range(world):
        assert_bitwise(out[r], ref, f"fp32 rank {r}")


@pytest.mark.slow
def test_fp32_full_size_first_cycle(pgmg):
    """N = 16385 (the bench grid): the first fp32 V-cycle from phi0 = 0 agrees with fp64
    to 1e-6 (measured 8.7e-8).  Later cycles do not: at h = 1/16384 the fp32 residual
    f - (1/h^2)(4x - ...) carries a round-off of ~(1/h^2) ulp(1) ~ 16 per point against
    f ~ 20, so fp32 stalls at ~0.11 relative error (profiles/r01_fp32/fp32_sweep.json);
    this is the tolerance sweep's finding, not a defect of the kernels (which are bitwise
    equal to the fp32 oracle)."""
    N = 16385
    sols = {}
    for dt in ("f64", "f32"):
        with pgmg.Solver(N, dtype=dt) as s:
            s.set_problem()
            s.vcycle(1)
            sols[dt] = s.solution()
    d = np.linalg.norm(sols["f32"] - sols["f64"]) / np.linalg.norm(sols["f64"])
    assert d <= 1e-6, d
