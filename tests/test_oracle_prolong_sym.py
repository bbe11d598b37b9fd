"""CPU: the oracle's restatement of the reference GPU path's symmetric prolongation
(`prolungator_kernel`, 3_part_parallel/Parallel_Method.cu:79-138; launched by
Parallel::ComputeProlungator, :188-199).

No golden vector exists for it (the kernel is CUDA and cannot be built here), so it is
pinned by two properties the reference source fixes:
* on fine rows/columns 2 .. N-2 its four cases are the same expressions, in the same order,
  as the CPU `MultigridSolver::prolongation` (2_part_MG/MultiGrid.hpp:208-226), whose
  restatement (orc_prolong) is pinned bit for bit to the compiled reference;
* row/column 1 get the interpolation the CPU path skips, every boundary point the thread grid
  covers is set to 0, and the points outside the reference's floor-sized grid are untouched.
"""
import numpy as np
import pytest

from conftest import assert_bitwise


@pytest.mark.parametrize("N", [5, 9, 17, 33, 129])
def test_prolong_sym_equals_cpu_prolongation_inside(oracle_mod, N):
    rng = np.random.default_rng(N)
    Nc = (N - 1) // 2 + 1
    coarse = rng.standard_normal((Nc, Nc))
    fine = rng.standard_normal((N, N))
    sym = oracle_mod.prolong_sym(fine, coarse)
    ref = oracle_mod.prolong(fine, coarse)
    assert_bitwise(sym[2:N - 1, 2:N - 1], ref[2:N - 1, 2:N - 1], f"interior N={N}")
    # the boundary the thread grid covers is zeroed
    assert np.all(sym[0] == 0) and np.all(sym[-1] == 0)
    assert np.all(sym[:, 0] == 0) and np.all(sym[:, -1] == 0)
    # row 1 (odd): vertical / 4-corner interpolation between coarse rows 0 and 1
    for x in range(1, N - 1):
        cx = x // 2
        if x % 2 == 0:
            want = fine[1, x] + 0.5 * (coarse[0, cx] + coarse[1, cx])
        else:
            want = fine[1, x] + 0.25 * (coarse[0, cx] + coarse[0, cx + 1] + coarse[1, cx] +
                                        coarse[1, cx + 1])
        assert sym[1, x] == want, x


def test_prolong_sym_hand_values(oracle_mod):
    """A 3x3 block of ones on a 5x5 coarse grid, prolongated into a zero 9x9 grid."""
    c = np.zeros((5, 5))
    c[1:4, 1:4] = 1.0
    f = oracle_mod.prolong_sym(np.zeros((9, 9)), c)
    assert np.all(f[2:7, 2:7] == 1.0)
    assert f[1, 1] == 0.25 and f[1, 2] == 0.5 and f[7, 7] == 0.25 and f[1, 7] == 0.25


def test_prolong_sym_reference_launch_extent(oracle_mod):
    """ComputeProlungator launches max(1, N / num_thread) blocks per axis: for N = 2^k + 1 >
    num_thread the grid is N - 1 wide and the last boundary row/column keep their values;
    for N <= num_thread one block covers everything."""
    rng = np.random.default_rng(7)
    N, Nc = 33, 17
    coarse = rng.standard_normal((Nc, Nc))
    fine = rng.standard_normal((N, N))
    got = oracle_mod.prolong_sym(fine, coarse, num_thread=16)
    full = oracle_mod.prolong_sym(fine, coarse)
    assert_bitwise(got[:N - 1, :N - 1], full[:N - 1, :N - 1], "covered part")
    assert_bitwise(got[N - 1], fine[N - 1], "last row untouched")
    assert_bitwise(got[:, N - 1], fine[:, N - 1], "last column untouched")
    small = oracle_mod.prolong_sym(fine[:9, :9], coarse[:5, :5], num_thread=16)
    assert_bitwise(small, oracle_mod.prolong_sym(fine[:9, :9], coarse[:5, :5]), "one block")
