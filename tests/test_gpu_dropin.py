"""GPU: device-resident problems (pgmg_set_problem_device) — the reference's memory contract.

ParallelMultiGridSolver::v_cycle(phi, f, N, h) (3_part_parallel/Parallel_Mg.cu:21-60) updates
in place arrays the caller keeps in device-accessible memory (ParallelTestRunner.cu:162-163).
Here phi and f are device arrays in the reference layout; with phi from pgmg_alloc_grid on a
cross-fused context the finest passes read and write it in place, any other device pointer is
staged on the device.  Every case is bitwise the oracle (the C restatement pinned to the
reference) or the reference's own golden hashes, with equal sweep counts."""
import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _oracle_phi(oracle_mod, N, cycles, f=None, phi0=None, kind="V"):
    o = oracle_mod.Oracle()
    f = o.rhs(N) if f is None else f
    phi = np.zeros((N, N)) if phi0 is None else phi0.copy()
    for _ in range(cycles):
        (o.v_cycle if kind == "V" else o.w_cycle)(phi, f)
    return phi, o.sweeps


def _device_run(pgmg, N, calls, f_host=None, phi0=None, kind="V", foreign=False, **cfg):
    """calls: cycles per call; returns (phi, sweeps, inplace)."""
    import torch
    keep = []
    if foreign:   # a device pointer the library did not allocate: staged path
        phi = torch.zeros((N, N), dtype=torch.float64, device="cuda")
        if phi0 is not None:
            phi.copy_(torch.from_numpy(phi0))
        keep.append(phi)
    else:
        phi = pgmg.DeviceGrid(N, phi0)
        keep.append(phi)
    fdev = None
    if f_host is not None:
        fdev = pgmg.DeviceGrid(N, f_host)
        keep.append(fdev)
    torch.cuda.synchronize()
    with pgmg.Solver(N, **cfg) as s:
        s.set_problem_device(phi, fdev)
        bound, inplace = s.device_info()
        assert bound
        for c in calls:
            (s.vcycle if kind == "V" else s.wcycle)(c)
        sweeps = s.stats()[0]
        via_ctx = s.solution()           # pgmg_get_solution reads the bound phi
    got = phi.cpu().numpy() if foreign else phi.download()
    assert_bitwise(via_ctx, got, "pgmg_get_solution of the bound phi")
    for k in keep:
        if not foreign and hasattr(k, "close"):
            k.close()
    return got, sweeps, inplace


@pytest.mark.parametrize("N,calls", [(2049, [1, 1]), (2049, [2]), (4097, [1, 1, 1])])
def test_inplace_default_sizes(pgmg, golden_cycles, N, calls):
    """The cross-fused sizes with the analytic f (regenerated): in place, bitwise the
    reference's hash after every call pattern."""
    got, _, inplace = _device_run(pgmg, N, calls)
    assert inplace
    want = next(c for c in golden_cycles if c["kind"] == "V" and c["N"] == N and c["eps"] == 1e-7)
    from oracle import fnv_hash
    assert fnv_hash(got) == want["cycles"][sum(calls) - 1]["hash"]


@pytest.mark.parametrize("calls", [[1] * 6, [3, 1, 2], [30]])
def test_inplace_small_grid_long_runs(pgmg, oracle_mod, calls):
    """N = 513 with the cross-fused finest level forced on (cross_min_n): 1-cycle calls, split
    calls and a 30-cycle call whose coarse checks fire (in-stream levels, rollbacks)."""
    N = 513
    want, sw = _oracle_phi(oracle_mod, N, sum(calls))
    got, gsw, inplace = _device_run(pgmg, N, calls, cross_min_n=33)
    assert inplace
    assert_bitwise(got, want, f"device in place N={N} calls={calls}")
    assert gsw == sw


def test_inplace_thirty_single_calls_with_spec_segments(pgmg, oracle_mod):
    """30 one-cycle calls at 129 (every check of the levels above the tail eventually fires:
    the deferred last pass must follow in-stream rollbacks too), segments of 2."""
    N = 129
    want, sw = _oracle_phi(oracle_mod, N, 30)
    got, gsw, inplace = _device_run(pgmg, N, [1] * 30, cross_min_n=33, tail_n=17, spec_segment=2)
    assert inplace
    assert_bitwise(got, want, "30 single calls")
    assert gsw == sw


def test_inplace_user_rhs_and_boundary(pgmg, oracle_mod):
    """A caller's f (the mt19937_64 robustness RHS) and a non-zero Dirichlet boundary on phi:
    the frame the passes pass through comes from the caller's phi at every call."""
    N = 513
    f = oracle_mod.rhs_mt64(N)
    rng = np.random.default_rng(7)
    phi0 = np.zeros((N, N))
    phi0[0, :] = rng.uniform(-1, 1, N)
    phi0[-1, :] = rng.uniform(-1, 1, N)
    phi0[:, 0] = rng.uniform(-1, 1, N)
    phi0[:, -1] = rng.uniform(-1, 1, N)
    want, sw = _oracle_phi(oracle_mod, N, 4, f=f, phi0=phi0)
    got, gsw, inplace = _device_run(pgmg, N, [1, 2, 1], f_host=f, phi0=phi0, cross_min_n=33)
    assert inplace
    assert_bitwise(got, want, "user f + boundary, in place")
    assert gsw == sw


def test_staged_foreign_pointer(pgmg, oracle_mod):
    """A device pointer the library did not allocate (a torch tensor): staged, same bits."""
    N = 513
    want, sw = _oracle_phi(oracle_mod, N, 3)
    got, gsw, inplace = _device_run(pgmg, N, [1, 2], foreign=True, cross_min_n=33)
    assert not inplace
    assert_bitwise(got, want, "torch tensor phi, staged")
    assert gsw == sw


def test_staged_small_and_wcycle(pgmg, oracle_mod):
    """Contexts without cross-cycle fusion (N < 2049 by default) stage; W-cycles too."""
    for kind, N, calls in (("V", 129, [1, 1, 1]), ("W", 129, [1, 2])):
        want, sw = _oracle_phi(oracle_mod, N, sum(calls), kind=kind)
        got, gsw, inplace = _device_run(pgmg, N, calls, kind=kind)
        assert not inplace
        assert_bitwise(got, want, f"staged {kind} {N}")
        assert gsw == sw


def test_inplace_wcycle(pgmg, oracle_mod):
    N = 257
    want, sw = _oracle_phi(oracle_mod, N, 2, kind="W")
    got, gsw, inplace = _device_run(pgmg, N, [1, 1], kind="W", cross_min_n=33)
    assert inplace
    assert_bitwise(got, want, "W in place")
    assert gsw == sw


def test_fp32_staged(pgmg, oracle_mod):
    N = 257
    o = oracle_mod.Oracle(dtype="f32")
    f = o.rhs(N)
    phi = np.zeros((N, N), dtype=np.float32)
    for _ in range(3):
        o.v_cycle(phi, f)
    got, gsw, inplace = _device_run(pgmg, N, [1, 2], dtype="f32", cross_min_n=33)
    assert not inplace
    assert np.array_equal(got.astype(np.float32).view(np.uint32), phi.view(np.uint32))
    assert got.dtype == np.float64 and gsw == o.sweeps


def test_rebinding_and_unbinding(pgmg, oracle_mod):
    """set_problem (host arrays) unbinds; binding again restarts from the caller's phi."""
    N = 513
    want1, _ = _oracle_phi(oracle_mod, N, 2)
    with pgmg.DeviceGrid(N) as phi, pgmg.Solver(N, cross_min_n=33) as s:
        s.set_problem_device(phi)
        s.vcycle(2)
        assert_bitwise(phi.download(), want1, "bound")
        s.set_problem()
        assert s.device_info() == (False, False)
        s.vcycle(2)
        assert_bitwise(s.solution(), want1, "host problem after unbinding")
        assert_bitwise(phi.download(), want1, "the caller's phi untouched by unbound calls")


def test_device_binding_errors(pgmg):
    import ctypes as C
    with pgmg.Solver(129) as s:
        host = np.zeros((129, 129))
        with pytest.raises(pgmg.PgmgError):
            s.set_problem_device(host.ctypes.data)   # host memory
    assert pgmg.load().pgmg_free_grid(C.c_void_p(12345)) == -1   # PGMG_ERR_ARG


@pytest.mark.slow
def test_inplace_full_size_single_calls(pgmg, golden_cycles):
    """BASELINE's N = 16385 as the reference's entry drives it: 20 one-cycle calls on the
    caller's device phi, in place, analytic f regenerated — the reference's hash after 20."""
    got, _, inplace = _device_run(pgmg, 16385, [1] * 20)
    assert inplace
    want = next(c for c in golden_cycles if c["kind"] == "V" and c["N"] == 16385)
    from oracle import fnv_hash
    assert fnv_hash(got) == want["cycles"][19]["hash"]


@pytest.mark.parametrize("foreign", [False, True])
def test_fcycle_on_bound_problem(pgmg, foreign):
    """pgmg_fcycle on a device-bound problem: the F-cycle restricts and climbs
    on the level-0 grids, so the caller's phi -- updated in place by the V-cycles before it -- is
    staged in and the result written back.  V, F, V, F on the bound phi is bitwise the same
    sequence on a host problem, and pgmg_get_solution / the hash read the bound result."""
    import torch
    N = 513
    seq = [("V", 1), ("F", 1), ("V", 2), ("F", 1), ("F", 3)]   # F x 3: k_post_r2 between them
    with pgmg.Solver(N, cross_min_n=33) as s:
        s.set_problem()
        for k, n in seq:
            (s.vcycle if k == "V" else s.fcycle)(n)
        want, want_sw = s.solution(), s.stats()[0]
    if foreign:
        phi = torch.zeros((N, N), dtype=torch.float64, device="cuda")
    else:
        phi = pgmg.DeviceGrid(N)
    torch.cuda.synchronize()
    with pgmg.Solver(N, cross_min_n=33) as s:
        s.set_problem_device(phi)
        assert s.device_info() == (True, not foreign)
        for k, n in seq:
            (s.vcycle if k == "V" else s.fcycle)(n)
            got = phi.cpu().numpy() if foreign else phi.download()
            assert_bitwise(s.solution(), got, f"bound phi after {k}")
        assert s.stats()[0] == want_sw
    assert_bitwise(got, want, f"V/F sequence on a bound phi (foreign={foreign})")
    if not foreign:
        phi.close()


def test_bound_call_waits_for_default_stream_work(pgmg, oracle_mod):
    """A bound call orders the context's (non-blocking) stream after the caller's outstanding
    null-stream work: phi is written by a copy queued on torch's default
    stream behind a long kernel chain, and the cycle is called without any synchronisation."""
    import torch
    N = 513
    rng = np.random.default_rng(11)
    phi0 = np.zeros((N, N))
    phi0[1:-1, 1:-1] = rng.uniform(-1, 1, (N - 2, N - 2))
    want, sw = _oracle_phi(oracle_mod, N, 1, phi0=phi0)
    src = torch.tensor(phi0, device="cuda")
    phi = torch.zeros((N, N), dtype=torch.float64, device="cuda")
    big = torch.randn((4096, 4096), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    with pgmg.Solver(N, cross_min_n=33) as s:
        s.set_problem_device(phi)
        assert torch.cuda.current_stream().cuda_stream == 0   # the null stream
        for _ in range(4):              # ~tens of ms of fp64 GEMMs on the null stream
            big = big @ big
            big = big / big.abs().max()
        phi.copy_(src)                  # queued behind them, not yet done
        s.vcycle(1)                     # no torch.cuda.synchronize() before the call
        assert s.stats()[0] == sw
    assert_bitwise(phi.cpu().numpy(), want, "phi written on the null stream before the call")
