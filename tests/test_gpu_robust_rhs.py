"""GPU: SURVEY §8(d)'s robustness input -- f uniform in [-1, 1) from std::mt19937_64 seed
12345, boundary 0 (oracle.rhs_mt64, pinned to libstdc++ by tests/golden/mt_rhs.json),
phi0 = 0 -- through the default paths, bitwise against the C oracle with equal sweep
counts: the cross-fused speculative finest level with a stored (user) f at 2049, a long
run at 513 whose coarse checks fire (rollbacks), W-cycles, fp32 and loopback strips."""
import threading

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _oracle(oracle_mod, N, calls, kind="V", dtype="f64"):
    f = oracle_mod.rhs_mt64(N, dtype=dtype)
    o = oracle_mod.Oracle(dtype=dtype)
    phi = np.zeros((N, N), dtype=f.dtype)
    for _ in range(sum(calls)):
        (o.v_cycle if kind == "V" else o.w_cycle)(phi, f)
    return f, phi, o.sweeps


def _gpu(pgmg, N, f, calls, kind="V", **kw):
    with pgmg.Solver(N, **kw) as s:
        s.set_problem(None if f is None else np.zeros_like(f), f)
        for c in calls:
            (s.vcycle if kind == "V" else s.wcycle)(c)
        return s.solution(), s.stats()[0]


@pytest.mark.parametrize("N,calls", [(2049, [3]), (2049, [1, 2]), (513, [5, 25]), (4097, [3])])
def test_robust_rhs_vcycle(pgmg, oracle_mod, N, calls):
    f, ref, sw = _oracle(oracle_mod, N, calls)
    got, gsw = _gpu(pgmg, N, f, calls)
    assert_bitwise(got, ref, f"mt64 RHS N={N} calls={calls}")
    assert gsw == sw


def test_robust_rhs_wcycle(pgmg, oracle_mod):
    f, ref, sw = _oracle(oracle_mod, 513, [2], kind="W")
    got, gsw = _gpu(pgmg, 513, f, [2], kind="W")
    assert_bitwise(got, ref, "mt64 RHS W 513")
    assert gsw == sw


def test_robust_rhs_fp32(pgmg, oracle_mod):
    f, ref, sw = _oracle(oracle_mod, 513, [3], dtype="f32")
    got, gsw = _gpu(pgmg, 513, f, [3], dtype="f32")
    got = np.ascontiguousarray(got, dtype=np.float32)
    assert np.array_equal(got.view(np.uint32), np.ascontiguousarray(ref).view(np.uint32))
    assert gsw == sw


def test_robust_rhs_strips(pgmg, oracle_mod):
    N, W = 2049, 4
    f, ref, _ = _oracle(oracle_mod, N, [3])
    hub = pgmg.LoopbackHub(W)
    out, err = [None] * W, [None] * W

    def work(r):
        try:
            with pgmg.Solver(N, hub=hub, rank=r, gather_n=257) as s:
                s.set_problem(np.zeros_like(f), f)
                s.vcycle(3)
                out[r] = s.solution()
        except Exception as e:  # surfaced below
            err[r] = e

    ts = [threading.Thread(target=work, args=(r,)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    hub.close()
    for e in err:
        if e is not None:
            raise e
    for r in range(W):
        assert_bitwise(out[r], ref, f"mt64 RHS strips rank {r}")


@pytest.mark.parametrize("N", [2049, 4097])
def test_robust_rhs_fast_tolerance(pgmg, oracle_mod, N):
    """FAST mode on a rough RHS: the same tolerance against the exact default as on the
    analytic one (test_gpu_fast.TOL), equal sweep counts."""
    f = oracle_mod.rhs_mt64(N)
    ref, sw = _gpu(pgmg, N, f, [10])
    got, gsw = _gpu(pgmg, N, f, [10], flags=pgmg.PGMG_FLAG_FAST)
    d = got - ref
    rel = np.linalg.norm(d) / np.linalg.norm(ref)
    print(f"N={N} FAST vs exact on the mt64 RHS: rel {rel:.3e} max-abs {np.max(np.abs(d)):.3e}")
    assert rel <= 1e-12 and np.max(np.abs(d)) <= 1e-12 * max(1.0, np.max(np.abs(ref)))
    assert gsw == sw
