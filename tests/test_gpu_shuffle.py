"""GPU: grids of 256 MB and more built from shuffled physical chunks (HIP virtual memory;
pgmg_ctx.hip "Shuffled physical placement", the one-GPU default since r06) hold and move the
same words as plain hipMalloc grids (PGMG_FLAG_NO_SHUFFLE): host uploads of phi and f, the
runtime's 2D copies avoided on them (set_problem, get_solution, the staged device-array path),
V-cycles, the residual norm and the carry -- at N = 8193 (537 MB level-0 grids)."""

import numpy as np
import pytest
import torch

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu

N = 8193


def _problem():
    rng = np.random.default_rng(7)
    phi0 = rng.uniform(-1, 1, (N, N))
    phi0[0, :] = phi0[-1, :] = phi0[:, 0] = phi0[:, -1] = 0.25
    f = rng.uniform(-1, 1, (N, N))
    return phi0, f


@pytest.mark.parametrize("staged", [False, True])
def test_shuffled_grids_equal_plain(pgmg, staged):
    phi0, f = _problem()
    out = []
    for fl in (0, pgmg.PGMG_FLAG_NO_SHUFFLE):
        with pgmg.Solver(N, flags=fl) as s:
            if staged:   # a torch tensor: the staged device path (kernel copies in and out)
                tphi = torch.from_numpy(phi0).cuda()
                tf = torch.from_numpy(f).cuda()
                s.set_problem_device(tphi, tf)
                s.vcycle(1)
                s.vcycle(2)
                got = tphi.cpu().numpy()
            else:
                s.set_problem(phi0, f)
                s.vcycle(1)
                s.vcycle(2)
                got = s.solution()
            out.append((got, s.stats(), s.residual_norm()))
    assert_bitwise(out[0][0], out[1][0], f"staged={staged}")
    assert out[0][1] == out[1][1]
    assert out[0][2] == out[1][2]


def test_shuffled_against_oracle(pgmg, oracle_mod):
    """Two V-cycles at 8193 from the analytic problem: bitwise the oracle and its sweeps."""
    with pgmg.Solver(N) as s:
        s.set_problem()
        s.vcycle(2)
        got = s.solution()
        sw = s.stats()[0]
    ref, o = oracle_mod.run_cycles("V", N, 2)
    assert_bitwise(got, ref, "8193 V x2")
    assert sw == o.sweeps
