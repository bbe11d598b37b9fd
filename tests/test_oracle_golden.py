"""CPU: pin the oracle (oracle/pgmg_oracle.c) to the reference's own outputs.

The golden fixtures in tests/golden/ were produced by the reference's CPU multigrid
(2_part_MG/MultiGrid.hpp, Smoother.hpp, DynamicGridUtils.hpp) compiled unmodified by
oracle/Makefile and driven by oracle/ref_harness.cpp (tests/golden/make_golden.py).
"""
import numpy as np
import pytest

from conftest import GOLDEN, assert_bitwise

MAX_N_CPU = 1025  # keep the CPU suite to a few minutes


def _cases(golden_cycles):
    return [c for c in golden_cycles if c["N"] <= MAX_N_CPU]


def test_golden_cycles_hashes(oracle_mod, golden_cycles):
    """Every cycle's FNV hash, centre value, residual norm and sweep count match."""
    checked = 0
    for case in _cases(golden_cycles):
        kind, N, eps = case["kind"], case["N"], case["eps"]
        o = oracle_mod.Oracle(eps=eps)
        f = o.rhs(N)
        phi = np.zeros((N, N))
        h = 1.0 / (N - 1)
        for row in case["cycles"]:
            if kind == "V":
                o.v_cycle(phi, f)
            elif kind == "W":
                o.w_cycle(phi, f)
            else:
                o.f_cycle_outer(phi)
            tag = f"{kind} N={N} eps={eps} cycle={row['cycle']}"
            assert oracle_mod.fnv_hash(phi) == row["hash"], tag
            assert phi[N // 2, N // 2] == row["center"], tag
            assert o.sweeps == row["sweeps"], tag
            assert o.early_exits == row["exits"], tag
            r = oracle_mod.residual(phi, f, h)
            assert oracle_mod.norm(r) == row["res"], tag
            assert o.rel_error(phi) == row["relerr"], tag
            checked += 1
    assert checked > 100


@pytest.mark.parametrize("name", sorted(p.name for p in GOLDEN.glob("phi_*.npy")))
def test_golden_phi_vectors(oracle_mod, name):
    stem = name[len("phi_"):-len(".npy")]
    kind, rest = stem[0], stem[1:]
    parts = rest.split("_")
    N = int(parts[0])
    k = int(parts[1][1:])
    eps = float(parts[2][3:]) if len(parts) > 2 else 1e-7
    ref = np.load(GOLDEN / name, allow_pickle=False)
    phi, _ = oracle_mod.run_cycles(kind, N, k, eps=eps)
    assert_bitwise(phi, ref, name)


@pytest.mark.parametrize("N", [17, 33, 65])
def test_golden_ops(oracle_mod, N):
    z = np.load(GOLDEN / f"ops_N{N}.npz", allow_pickle=False)
    x, f, e, h, eps = z["x"], z["f"], z["e"], float(z["h"]), float(z["eps"])
    assert_bitwise(oracle_mod.residual(x, f, h), z["residual"], "residual")
    assert_bitwise(oracle_mod.restrict(x), z["restrict"], "restrict")
    assert_bitwise(oracle_mod.prolong(x, e), z["prolong"], "prolong")
    for it, key in ((1, "smooth1"), (10, "smooth10")):
        o = oracle_mod.Oracle(eps=eps)
        s = x.copy()
        o.smooth(s, f, h, it)
        assert_bitwise(s, z[key], key)


def test_prolongation_quirk(oracle_mod):
    """interior-ones 5x5 coarse -> fine row/col 1 stay 0, Nf-2 gets 0.5."""
    c = np.zeros((5, 5))
    c[1:4, 1:4] = 1.0
    fine = oracle_mod.prolong(np.zeros((9, 9)), c)
    assert np.all(fine[1, :] == 0) and np.all(fine[:, 1] == 0)
    assert np.all(fine[2:7, 2:7] == 1.0)
    assert np.all(fine[7, 2:7] == 0.5) and np.all(fine[2:7, 7] == 0.5)


def test_restriction_of_ones(oracle_mod):
    c = oracle_mod.restrict(np.ones((9, 9)))
    assert np.all(c[1:4, 1:4] == 1.0)
    assert c[0].sum() == 0 and c[-1].sum() == 0 and c[:, 0].sum() == 0 and c[:, -1].sum() == 0
