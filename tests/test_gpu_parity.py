"""GPU parity: the HIP path (through the C ABI) against the reference's goldens and the oracle.

Tolerance: EXACT.  All fp64 arithmetic keeps the reference's expression order and the
library is built with -ffp-contract=off, so phi must be bit-identical to mg_cpu_exec
(compared through the FNV-64 hash of every IEEE word, or word by word).  The only
order-dependent quantity is the smoother's early-exit norm (a parallel sum instead of
the reference's sequential one); it can only matter when ||r|| lands within ~1e-15
relative of eps, which none of these cases does.
"""
import numpy as np
import pytest

from conftest import GOLDEN, assert_bitwise

pytestmark = pytest.mark.gpu


def _golden(golden_cycles, kind, N, eps=1e-7):
    for c in golden_cycles:
        if c["kind"] == kind and c["N"] == N and c["eps"] == eps:
            return c
    raise KeyError((kind, N, eps))


def _run_against_golden(pgmg, oracle_mod, case, **cfg):
    kind, N, eps = case["kind"], case["N"], case["eps"]
    with pgmg.Solver(N, eps=eps, **cfg) as s:
        s.set_problem()
        for row in case["cycles"]:
            (s.vcycle if kind == "V" else s.wcycle)(1)
            phi = s.solution()
            tag = f"{kind} N={N} eps={eps} cycle={row['cycle']} cfg={cfg}"
            assert oracle_mod.fnv_hash(phi) == row["hash"], tag
            sweeps, exits = s.stats()
            assert sweeps == row["sweeps"], tag
            assert exits <= row["exits"], tag


@pytest.mark.parametrize("N", [33, 65, 129, 257, 513, 1025, 2049, 4097])
def test_vcycle_matches_reference_golden(pgmg, oracle_mod, golden_cycles, N):
    _run_against_golden(pgmg, oracle_mod, _golden(golden_cycles, "V", N))


@pytest.mark.parametrize("tail_n", [5, 9, 17, 33])
def test_vcycle_bulk_kernels_on_small_levels(pgmg, oracle_mod, golden_cycles, tail_n):
    """Moving the tail threshold down runs the multi-kernel path on N = 9..65 levels."""
    for N in (33, 129, 257):
        _run_against_golden(pgmg, oracle_mod, _golden(golden_cycles, "V", N), tail_n=tail_n)


@pytest.mark.parametrize("eps,N,tail_n", [(1e3, 129, 65), (1e3, 129, 5), (1.0, 257, 65),
                                          (1.0, 257, 9), (0.0, 65, 65), (0.0, 65, 5)])
def test_vcycle_early_exit_paths(pgmg, oracle_mod, golden_cycles, eps, N, tail_n):
    """Forced and mixed smoother early exits (Smoother.hpp:84-88) in bulk and tail."""
    _run_against_golden(pgmg, oracle_mod, _golden(golden_cycles, "V", N, eps), tail_n=tail_n)


def test_vcycle_30_cycles_early_exit_regime(pgmg, oracle_mod, golden_cycles):
    """N=513 over 30 cycles: coarse levels start exiting early from ~cycle 13."""
    _run_against_golden(pgmg, oracle_mod, _golden(golden_cycles, "V", 513))
    _run_against_golden(pgmg, oracle_mod, _golden(golden_cycles, "V", 513), tail_n=9)


@pytest.mark.parametrize("N", [33, 129, 513])
def test_wcycle_matches_reference_golden(pgmg, oracle_mod, golden_cycles, N):
    _run_against_golden(pgmg, oracle_mod, _golden(golden_cycles, "W", N))
    if N <= 129:
        _run_against_golden(pgmg, oracle_mod, _golden(golden_cycles, "W", N), tail_n=9)


@pytest.mark.parametrize("name", ["phi_V33_c3.npy", "phi_V129_c30.npy", "phi_V65_c4_eps0.npy",
                                  "phi_V129_c8_eps1000.npy", "phi_W129_c3.npy"])
def test_full_vectors(pgmg, name):
    stem = name[4:-4]
    kind, parts = stem[0], stem[1:].split("_")
    N, k = int(parts[0]), int(parts[1][1:])
    eps = float(parts[2][3:]) if len(parts) > 2 else 1e-7
    ref = np.load(GOLDEN / name, allow_pickle=False)
    with pgmg.Solver(N, eps=eps) as s:
        s.set_problem()
        (s.vcycle if kind == "V" else s.wcycle)(k)
        assert_bitwise(s.solution(), ref, name)


@pytest.mark.parametrize("N,cycles", [(129, 30), (513, 30), (1025, 3)])
def test_unfused_path_matches_golden(pgmg, oracle_mod, golden_cycles, N, cycles):
    """One kernel per sweep (the general path) gives the same bits as the fused passes."""
    case = _golden(golden_cycles, "V", N)
    case = dict(case, cycles=case["cycles"][:cycles])
    _run_against_golden(pgmg, oracle_mod, case, flags=pgmg.PGMG_FLAG_UNFUSED)
    _run_against_golden(pgmg, oracle_mod, case, flags=pgmg.PGMG_FLAG_UNFUSED, tail_n=9)


@pytest.mark.parametrize("v1,v2,N", [(2, 0, 257), (0, 3, 129), (3, 2, 129), (2, 2, 65)])
def test_other_smoothing_counts_against_oracle(pgmg, oracle_mod, v1, v2, N):
    """v1/v2 != 1 (general path, odd sweep counts, several early-exit checks per call)."""
    for eps, tail_n in ((1e-7, 65), (1e-7, 9), (5.0, 9)):
        o = oracle_mod.Oracle(eps=eps, v1=v1, v2=v2)
        f = o.rhs(N)
        ref = np.zeros((N, N))
        with pgmg.Solver(N, v1=v1, v2=v2, eps=eps, tail_n=tail_n) as s:
            s.set_problem()
            for k in range(4):
                o.v_cycle(ref, f)
                s.vcycle(1)
                assert_bitwise(s.solution(), ref, f"v1={v1} v2={v2} eps={eps} tail={tail_n} k={k}")
                assert s.stats()[0] == o.sweeps


def test_graph_replay_equals_eager(pgmg):
    out = []
    for flags in (0, pgmg.PGMG_FLAG_NO_GRAPH, pgmg.PGMG_FLAG_TIME_FINE):
        with pgmg.Solver(1025, flags=flags) as s:
            s.set_problem()
            s.vcycle(3)
            out.append(s.solution())
    assert_bitwise(out[0], out[1], "graph vs eager")
    assert_bitwise(out[0], out[2], "graph vs timed eager")


def test_random_problem_against_oracle(pgmg, oracle_mod):
    """Seeded random phi0 / f (boundary 0) — not the analytic RHS."""
    rng = np.random.default_rng(12345)
    for N, tail_n in ((257, 65), (257, 9), (129, 5)):
        phi0 = rng.uniform(-1, 1, (N, N))
        f = rng.uniform(-1, 1, (N, N))
        for a in (phi0, f):
            a[0, :] = a[-1, :] = a[:, 0] = a[:, -1] = 0.0
        o = oracle_mod.Oracle()
        ref = phi0.copy()
        for _ in range(3):
            o.v_cycle(ref, f)
        with pgmg.Solver(N, tail_n=tail_n) as s:
            s.set_problem(phi0, f)
            s.vcycle(3)
            assert_bitwise(s.solution(), ref, f"random N={N} tail_n={tail_n}")
            assert s.stats()[0] == o.sweeps


def test_residual_norm_matches_oracle(pgmg, oracle_mod):
    N = 513
    phi, _ = oracle_mod.run_cycles("V", N, 2)
    with pgmg.Solver(N) as s:
        s.set_problem()
        s.vcycle(2)
        got = s.residual_norm()
    f = oracle_mod.Oracle().rhs(N)
    want = oracle_mod.norm(oracle_mod.residual(phi, f, 1.0 / (N - 1)))
    assert abs(got - want) <= 1e-12 * want   # parallel vs sequential summation order


@pytest.mark.slow
def test_vcycle_16385_golden(pgmg, oracle_mod, golden_cycles):
    """Full-size roofline configuration: one V-cycle, hash of all 268M words."""
    _run_against_golden(pgmg, oracle_mod, _golden(golden_cycles, "V", 16385))


# ---- op level (Parallel::Compute* mirror) ----------------------------------

@pytest.mark.parametrize("N", [17, 33, 65])
def test_ops_match_reference_kats(pgmg, N):
    import torch
    z = np.load(GOLDEN / f"ops_N{N}.npz", allow_pickle=False)
    dev = torch.device("cuda:0")
    t = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa
    x, f, e = t(z["x"]), t(z["f"]), t(z["e"])
    h, eps = float(z["h"]), float(z["eps"])
    r = torch.zeros_like(x)
    pgmg.ops.residual(r, x, f, h)
    torch.cuda.synchronize()
    assert_bitwise(r.cpu().numpy(), z["residual"], "residual")
    Nc = e.shape[0]
    c = torch.zeros((Nc, Nc), dtype=torch.float64, device=dev)
    pgmg.ops.restrict(x, c)
    torch.cuda.synchronize()
    assert_bitwise(c.cpu().numpy(), z["restrict"], "restrict")
    p = x.clone()
    pgmg.ops.prolong(e, p)
    torch.cuda.synchronize()
    assert_bitwise(p.cpu().numpy(), z["prolong"], "prolong")
    for it, key in ((1, "smooth1"), (10, "smooth10")):
        s = x.clone()
        pgmg.ops.jacobi(s, f, h, it, eps=eps)
        torch.cuda.synchronize()
        assert_bitwise(s.cpu().numpy(), z[key], key)


def test_op_jacobi_early_exit_and_norm(pgmg, oracle_mod):
    import torch
    N = 65
    h = 1.0 / (N - 1)
    o = oracle_mod.Oracle(eps=1e-7)
    f = o.rhs(N)
    dev = torch.device("cuda:0")
    for eps in (1e-7, 1e2, 1e6, -1.0):
        x = np.zeros((N, N))
        oo = oracle_mod.Oracle(eps=eps if eps >= 0 else -1.0)
        n_ref = oo.smooth(x, f, h, 20)
        xt = torch.zeros((N, N), dtype=torch.float64, device=dev)
        ft = torch.tensor(f, device=dev)
        n = pgmg.ops.jacobi(xt, ft, h, 20, eps=eps)
        assert n == n_ref, eps
        assert_bitwise(xt.cpu().numpy(), x, f"jacobi eps={eps}")
    v = torch.tensor(f, device=dev)
    assert abs(pgmg.ops.norm(v) - oracle_mod.norm(f)) <= 1e-13 * oracle_mod.norm(f)


def test_op_rhs_bitwise(pgmg, oracle_mod):
    import torch
    N = 257
    f = torch.zeros((N, N), dtype=torch.float64, device="cuda:0")
    pgmg.ops.rhs(f, 1.0 / (N - 1))
    torch.cuda.synchronize()
    assert_bitwise(f.cpu().numpy(), oracle_mod.Oracle().rhs(N), "rhs")


def test_op_jacobi_concurrent_streams(pgmg, oracle_mod):
    """The op-level API keeps one scratch set (partials, flags, ping-pong buffer) per stream:
    smoothers of different problems enqueued on two streams at once, without syncs between
    them, each equal to the oracle bit for bit (with one shared set, the second stream's
    partial sums and early-exit flags overwrote the first's)."""
    import torch
    dev = torch.device("cuda:0")
    probs = []
    for seed, N, eps in ((1, 257, 1e-3), (2, 513, 1e-2)):
        rng = np.random.default_rng(seed)
        f = rng.uniform(-1, 1, (N, N))
        f[0, :] = f[-1, :] = f[:, 0] = f[:, -1] = 0.0
        h = 1.0 / (N - 1)
        x = np.zeros((N, N))
        n_ref = oracle_mod.Oracle(eps=eps).smooth(x, f, h, 40)
        probs.append((N, h, eps, f, x, n_ref))
    streams = [torch.cuda.Stream(device=dev) for _ in probs]
    outs = []
    for (N, h, eps, f, _, _), st in zip(probs, streams):
        xt = torch.zeros((N, N), dtype=torch.float64, device=dev)
        ft = torch.tensor(f, device=dev)
        torch.cuda.synchronize()
        outs.append((xt, ft, st))
    # interleave: both ops enqueued before either is waited for
    for rep in range(3):
        for i, (xt, ft, st) in enumerate(outs):
            N, h, eps, f, _, _ = probs[i]
            xt.zero_()
            torch.cuda.synchronize()
            # sweeps_done = NULL: the op returns without waiting for its stream
            pgmg.check(pgmg.load().pgmg_jacobi(C_ptr(xt), None, C_ptr(ft), N, N, h, 40, eps,
                                               None, C_stream(st)), "pgmg_jacobi")
        torch.cuda.synchronize()
        for i, (xt, _, _) in enumerate(outs):
            assert_bitwise(xt.cpu().numpy(), probs[i][4], f"stream {i} rep {rep}")
    # and with the sweep count (synchronous form), per stream
    for i, (xt, ft, st) in enumerate(outs):
        N, h, eps, f, _, n_ref = probs[i]
        xt.zero_()
        torch.cuda.synchronize()
        assert pgmg.ops.jacobi(xt, ft, h, 40, eps=eps, stream=C_stream(st)) == n_ref
    # releasing a stream's scratch set: the next op on it allocates a fresh one
    for i, (xt, ft, st) in enumerate(outs):
        pgmg.check(pgmg.load().pgmg_ops_release(C_stream(st)), "pgmg_ops_release")
        pgmg.check(pgmg.load().pgmg_ops_release(C_stream(st)), "pgmg_ops_release")  # no-op
        N, h, eps, f, x_ref, n_ref = probs[i]
        xt.zero_()
        torch.cuda.synchronize()
        assert pgmg.ops.jacobi(xt, ft, h, 40, eps=eps, stream=C_stream(st)) == n_ref
        assert_bitwise(xt.cpu().numpy(), x_ref, f"stream {i} after release")
        pgmg.check(pgmg.load().pgmg_ops_release(C_stream(st)), "pgmg_ops_release")


def C_stream(st):
    import ctypes
    return ctypes.c_void_p(st.cuda_stream)


def C_ptr(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())


@pytest.mark.parametrize("N", [9, 33, 129, 1025])
def test_symmetric_prolongation_kat(pgmg, oracle_mod, N):
    """gpu_exec's prolungator_kernel (Parallel_Method.cu:79-138; symmetric, boundary := 0):
    pgmg_prolong(mode=PGMG_PROLONG_SYMMETRIC) on random coarse and fine grids (boundary
    included) is bitwise the oracle's restatement (orc_prolong_sym, the whole grid covered)."""
    import torch
    rng = np.random.default_rng(1000 + N)
    Nc = (N - 1) // 2 + 1
    c = rng.standard_normal((Nc, Nc))
    f = rng.standard_normal((N, N))
    ct = torch.tensor(c, device="cuda:0")
    ft = torch.tensor(f, device="cuda:0")
    pgmg.ops.prolong(ct, ft, mode=pgmg.PGMG_PROLONG_SYMMETRIC)
    torch.cuda.synchronize()
    assert_bitwise(ft.cpu().numpy(), oracle_mod.prolong_sym(f, c), f"prolong_sym N={N}")


@pytest.mark.slow
def test_vcycle_32769_oracle_hash(pgmg, oracle_mod):
    """N = 32769 (BASELINE config 4's grid, one GPU, ~45 GB of HBM): one V-cycle from
    phi0 = 0 is bitwise the oracle's.  The hash comes from oracle/mg_cpu_exec_port (our C
    restatement; 75 s on one core): `mg_cpu_exec_port V 32769 1 1e-7` -> relerr
    0.17198606950442494, hash 034c7979d0b231c7, 63 sweeps -- the reference's own
    MultigridSolver gives the same (profiles/r06/ref32769/V.out).  Also exercises 32-bit index headroom (N * pitch ~ 1.07e9)."""
    N = 32769
    with pgmg.Solver(N) as s:
        s.set_problem()
        s.vcycle(1)
        phi = s.solution()
        assert s.stats()[0] == 63
    assert oracle_mod.fnv_hash(phi) == "034c7979d0b231c7"


@pytest.mark.parametrize("N,nt", [(33, 32), (33, 16), (129, 32), (1025, 32), (1025, 16), (9, 32)])
def test_symmetric_prolongation_launch_grid(pgmg, oracle_mod, N, nt):
    """Parallel::ComputeProlungator's thread grid (Parallel_Method.cu:191-197: max(1, N /
    num_thread) blocks of num_thread per side): for N = 2^k + 1 > num_thread the last fine
    row and column are never written.  pgmg_prolong_grid(..., num_thread) is bitwise the
    oracle's orc_prolong_sym with that extent on random grids whose last row/column are
    non-zero (N = 9 < 32: one block covers everything)."""
    import torch
    rng = np.random.default_rng(2000 + N + nt)
    Nc = (N - 1) // 2 + 1
    c = rng.standard_normal((Nc, Nc))
    f = rng.standard_normal((N, N))
    ct = torch.tensor(c, device="cuda:0")
    ft = torch.tensor(f, device="cuda:0")
    pgmg.ops.prolong(ct, ft, mode=pgmg.PGMG_PROLONG_SYMMETRIC, num_thread=nt)
    torch.cuda.synchronize()
    got = ft.cpu().numpy()
    assert_bitwise(got, oracle_mod.prolong_sym(f, c, num_thread=nt), f"prolong_sym N={N} nt={nt}")
    if N > nt:
        assert np.array_equal(got[-1, :], f[-1, :]) and np.array_equal(got[:, -1], f[:, -1])
