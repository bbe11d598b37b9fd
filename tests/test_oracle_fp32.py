"""CPU: the fp32 restatement of mg_cpu_exec (oracle/liboracle_f32.so, -DORC_REAL=float),
the checker of the library's PGMG_PRECISION_FP32 variant.

The reference has no fp32 path, so this oracle is pinned as a tolerance against the
reference's own fp64 goldens (tests/golden/, made by the compiled reference): the phi
vectors the goldens hold for N <= 129 and the relative errors for larger N.  It also
must share the fp64 oracle's control flow (same sweep count on the reference problem).
"""
import numpy as np
import pytest

from conftest import GOLDEN


def _golden(golden_cycles, kind, N, eps=1e-7):
    return next(c for c in golden_cycles if c["kind"] == kind and c["N"] == N and c["eps"] == eps)


def test_fp32_oracle_is_float(oracle_mod):
    assert oracle_mod.lib("f32").orc_real_size() == 4
    assert oracle_mod.lib("f64").orc_real_size() == 8


@pytest.mark.parametrize("kind,N,cycles,tol", [("V", 33, 3, 2e-6), ("V", 65, 3, 2e-6),
                                               ("V", 129, 1, 2e-6), ("W", 33, 3, 2e-6),
                                               ("W", 129, 3, 4e-6), ("F", 33, 3, 4e-6),
                                               ("F", 129, 2, 4e-6)])
def test_fp32_oracle_within_tolerance_of_reference_vectors(oracle_mod, kind, N, cycles, tol):
    ref = np.load(GOLDEN / f"phi_{kind}{N}_c{cycles}.npy", allow_pickle=False)
    phi, _ = oracle_mod.run_cycles(kind, N, cycles, dtype="f32")
    assert phi.dtype == np.float32
    d = np.linalg.norm(phi.astype(np.float64) - ref) / np.linalg.norm(ref)
    assert 0 < d <= tol, d      # > 0: really computed in fp32


@pytest.mark.parametrize("N", [33, 129, 513, 1025])
def test_fp32_oracle_tracks_reference_relerr_and_sweeps(oracle_mod, golden_cycles, N):
    """First <= 3 cycles from phi0 = 0 (no early exit fires in either precision there;
    over long runs fp64 exits early on coarse levels once ||r|| < 1e-7, while the fp32
    round-off floor of the residual keeps fp32 above it — a real difference)."""
    case = _golden(golden_cycles, "V", N)
    row = [r for r in case["cycles"] if r["cycle"] <= 3][-1]
    phi, o = oracle_mod.run_cycles("V", N, row["cycle"], dtype="f32")
    assert abs(o.rel_error(phi) - row["relerr"]) <= 1e-3 * row["relerr"]
    assert o.sweeps == row["sweeps"] and o.early_exits == row["exits"] == 0
