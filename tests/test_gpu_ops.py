"""GPU: the op-level entries (pgmg_jacobi / residual / restrict / prolong_grid) -- the
reference's Parallel::ComputeJacobi / ComputeResidual / ComputeRestriction /
ComputeProlungator (3_part_parallel/Parallel_Method.cu:144-199) -- on ragged and edge-case
shapes, bitwise against the oracle (oracle/pgmg_oracle.c, pinned to the compiled reference).

The kernels march row bands with column pairs per lane on the caller's layout (pitch W, any
alignment).  Since r05 the sweeps without checks run IN PLACE on x (k_op_sweep_ip /
k_op_sweep2_ip: the tile-edge outputs other workgroups read are deferred to a side buffer and
scattered after the pass); a checked call with an odd sweep count runs its first sweep in place
and the rest ping-pong, seeding only the ping-pong buffer's boundary.  These cases cover what
that can get wrong: even and odd W (the last lane pair is whole or half boundary), W not a
multiple of the 512-column block, many column blocks and row bands (deferred rows and columns
meeting at tile corners), H != W, the smallest grids, every sweep-count parity, checks that fire
at the first or a later sweep, a caller ping-pong buffer full of NaN (nothing may read what the
op did not write), and the caller's non-zero boundary."""
import ctypes as C

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _t(a):
    import torch
    return torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda:0")


def _orc_smooth(oracle_mod, x, f, h, num_iter, eps):
    H, W = x.shape
    o = oracle_mod.Oracle(eps=eps)
    work = np.zeros(H * W)
    n = oracle_mod.lib().orc_jacobi_smooth(C.byref(o.c), oracle_mod._p(x), oracle_mod._p(f), W, H,
                                           h, num_iter, oracle_mod._p(work))
    return n


SHAPES = [(3, 3), (3, 4), (4, 3), (5, 5), (5, 6), (9, 130), (130, 9), (129, 128), (200, 257),
          (257, 513), (64, 1030), (33, 1025)]


@pytest.mark.parametrize("H,W", SHAPES)
def test_jacobi_ragged_shapes(pgmg, oracle_mod, H, W):
    import torch
    rng = np.random.default_rng(H * 7919 + W)
    x0 = rng.uniform(-1, 1, (H, W))          # non-zero boundary too
    f = rng.uniform(-1, 1, (H, W))
    h = 1.0 / (max(H, W) - 1)
    for v in (0, 1, 2, 5):
        for eps in (-1.0, 1e6):
            x = x0.copy()
            n_ref = _orc_smooth(oracle_mod, x, f, h, v, eps)
            xt = _t(x0)
            tmp = torch.full_like(xt, float("nan"))
            n = pgmg.ops.jacobi(xt, _t(f), h, v, eps=eps, tmp=tmp)
            assert n == n_ref, (H, W, v, eps)
            assert_bitwise(xt.cpu().numpy(), x, f"jacobi {H}x{W} v={v} eps={eps}")


@pytest.mark.parametrize("H,W", [(1031, 1537), (700, 2053), (2049, 2049), (4097, 1030),
                                 (517, 4100)])
def test_jacobi_in_place_tiles(pgmg, oracle_mod, H, W):
    """Grids of several column blocks (512 columns for the single sweep, 480 for the paired
    pass) and many row bands: every deferred tile edge, bitwise the oracle, for 1 .. 4 sweeps
    without checks (single, paired, single + paired, two paired passes) and 3 sweeps with
    checks (the first in place, then ping-pong)."""
    import torch
    rng = np.random.default_rng(H * 13 + W)
    x0 = rng.uniform(-1, 1, (H, W))
    f = rng.uniform(-1, 1, (H, W))
    h = 1.0 / (max(H, W) - 1)
    ft = _t(f)
    for v, eps in ((0, -1.0), (1, -1.0), (2, -1.0), (3, -1.0), (2, 1e-30), (2, 1e9)):
        x = x0.copy()
        n_ref = _orc_smooth(oracle_mod, x, f, h, v, eps)
        xt = _t(x0)
        tmp = torch.full_like(xt, float("nan"))
        n = pgmg.ops.jacobi(xt, ft, h, v, eps=eps, tmp=tmp)
        assert n == n_ref, (H, W, v, eps)
        assert_bitwise(xt.cpu().numpy(), x, f"in-place jacobi {H}x{W} v={v} eps={eps}")


def test_jacobi_in_place_repeated_calls(pgmg, oracle_mod):
    """Back-to-back in-place calls on one stream share the side buffer: 7 calls of 1 .. 3
    sweeps equal the oracle's 7 smoother calls."""
    import torch
    H, W = 1500, 1800
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, (H, W))
    f = rng.uniform(-1, 1, (H, W))
    h = 1.0 / (W - 1)
    xt, ft = _t(x), _t(f)
    for k in range(7):
        v = k % 3
        _orc_smooth(oracle_mod, x, f, h, v, -1.0)
        pgmg.ops.jacobi(xt, ft, h, v, eps=-1.0)
    torch.cuda.synchronize()
    assert_bitwise(xt.cpu().numpy(), x, "7 in-place calls")


@pytest.mark.parametrize("N", [65, 257, 1025])
def test_jacobi_checks_fire_mid_call(pgmg, oracle_mod, N):
    """eps between the norms of the first sweeps: the check fires after some sweep k > 1 and
    the speculative sweep k+1 is undone; every later sweep skips."""
    import torch
    rng = np.random.default_rng(N)
    f = np.zeros((N, N))
    f[1:-1, 1:-1] = rng.uniform(-1, 1, (N - 2, N - 2))
    h = 1.0 / (N - 1)
    # norms of the first sweeps from x = 0, then eps between the 3rd and 4th
    norms = []
    x = np.zeros((N, N))
    for _ in range(6):
        _orc_smooth(oracle_mod, x, f, h, 0, -1.0)
        norms.append(oracle_mod.norm(oracle_mod.residual(x, f, h)))
    for eps in (0.5 * (norms[2] + norms[3]), 0.5 * (norms[0] + norms[1])):
        for v in (5, 6):
            x = np.zeros((N, N))
            n_ref = _orc_smooth(oracle_mod, x, f, h, v, eps)
            assert 1 < n_ref < v + 1
            xt = torch.zeros((N, N), dtype=torch.float64, device="cuda:0")
            n = pgmg.ops.jacobi(xt, _t(f), h, v, eps=eps)
            assert n == n_ref, (eps, v)
            assert_bitwise(xt.cpu().numpy(), x, f"jacobi N={N} v={v} fired after {n_ref}")


@pytest.mark.parametrize("H,W", SHAPES)
def test_residual_ragged_shapes(pgmg, oracle_mod, H, W):
    import torch
    rng = np.random.default_rng(H * 31 + W)
    x = rng.uniform(-1, 1, (H, W))
    f = rng.uniform(-1, 1, (H, W))
    h = 1.0 / (max(H, W) - 1)
    want = np.full((H, W), 3.25)             # the boundary of r is untouched
    ref = np.zeros((H, W))
    oracle_mod.lib().orc_residual(oracle_mod._p(ref), oracle_mod._p(x), oracle_mod._p(f), W, H, h)
    want[1:-1, 1:-1] = ref[1:-1, 1:-1]
    r = torch.full((H, W), 3.25, dtype=torch.float64, device="cuda:0")
    pgmg.ops.residual(r, _t(x), _t(f), h)
    torch.cuda.synchronize()
    assert_bitwise(r.cpu().numpy(), want, f"residual {H}x{W}")


@pytest.mark.parametrize("Nf", [5, 9, 17, 129, 1025, 2049])
def test_restrict_sizes(pgmg, oracle_mod, Nf):
    import torch
    rng = np.random.default_rng(Nf)
    fine = rng.uniform(-1, 1, (Nf, Nf))
    Nc = (Nf - 1) // 2 + 1
    want = np.full((Nc, Nc), -2.5)           # the coarse boundary is untouched
    ref = oracle_mod.restrict(fine)
    want[1:-1, 1:-1] = ref[1:-1, 1:-1]
    c = torch.full((Nc, Nc), -2.5, dtype=torch.float64, device="cuda:0")
    pgmg.ops.restrict(_t(fine), c)
    torch.cuda.synchronize()
    assert_bitwise(c.cpu().numpy(), want, f"restrict {Nf}")


@pytest.mark.parametrize("Nf", [5, 9, 17, 129, 1025, 2049])
def test_prolong_cpu_form_sizes(pgmg, oracle_mod, Nf):
    rng = np.random.default_rng(100 + Nf)
    Nc = (Nf - 1) // 2 + 1
    fine = rng.uniform(-1, 1, (Nf, Nf))
    coarse = rng.uniform(-1, 1, (Nc, Nc))
    ft = _t(fine)
    pgmg.ops.prolong(_t(coarse), ft, mode=pgmg.PGMG_PROLONG_REFERENCE)
    assert_bitwise(ft.cpu().numpy(), oracle_mod.prolong(fine, coarse), f"prolong {Nf}")


@pytest.mark.parametrize("Nf,nt", [(5, 0), (17, 0), (17, 4), (1025, 0), (1025, 32), (2049, 16),
                                   (2049, 32), (513, 1000)])
def test_prolong_symmetric_sizes(pgmg, oracle_mod, Nf, nt):
    rng = np.random.default_rng(200 + Nf + nt)
    Nc = (Nf - 1) // 2 + 1
    fine = rng.uniform(-1, 1, (Nf, Nf))
    coarse = rng.uniform(-1, 1, (Nc, Nc))
    ft = _t(fine)
    pgmg.ops.prolong(_t(coarse), ft, mode=pgmg.PGMG_PROLONG_SYMMETRIC, num_thread=nt)
    want = oracle_mod.prolong_sym(fine, coarse, num_thread=nt if nt else None)
    assert_bitwise(ft.cpu().numpy(), want, f"prolong_sym {Nf} nt={nt}")


def test_jacobi_full_size_against_oracle_window(pgmg, oracle_mod):
    """N = 16385 (BASELINE's grid; the pitch is odd, so every other row's lane pairs are 8-byte
    aligned): two sweeps with the reference's analytic f from x = 0, compared bitwise with the
    oracle on a window of rows (a sweep's row j depends only on rows j-2 .. j+2 of x0 = 0)."""
    import torch
    N = 16385
    h = 1.0 / (N - 1)
    x = torch.zeros((N, N), dtype=torch.float64, device="cuda:0")
    f = torch.empty_like(x)
    pgmg.ops.rhs(f, h)
    assert pgmg.ops.jacobi(x, f, h, 1, eps=-1.0) == 2
    rows = [0, 1, 2, 3, 4097, 8192, 16381, 16382, 16383, 16384]
    got = x[rows].cpu().numpy()
    fwin = {r: f[max(0, r - 3):min(N, r + 4)].cpu().numpy() for r in rows}
    del x, f
    torch.cuda.empty_cache()
    for r in rows:
        lo, hi = max(0, r - 3), min(N, r + 4)
        # the oracle on rows lo..hi-1 of the full-width grid, x0 = 0, Dirichlet rows at the cut:
        # rows further than 2 from the cut are exact
        xs = np.zeros((hi - lo, N))
        fs = np.ascontiguousarray(fwin[r])
        _orc_smooth(oracle_mod, xs, fs, h, 1, -1.0)
        if r in (0, N - 1):
            assert np.all(got[rows.index(r)] == 0.0)
        elif r - lo >= 2 or lo == 0:
            if hi - r > 2 or hi == N:
                assert_bitwise(got[rows.index(r)], xs[r - lo], f"row {r}")
