"""GPU, ranks as separate processes: the row-strip decomposition end to end across process
boundaries — every rank its own process and context on GPU 0, halos, gathered coarse rows
and reductions moved by the host-staged transport over a gloo group (PGMG_FLAG_HOST_TRANSPORT;
RCCL refuses two ranks on one device, and the pool's boxes have one GPU).  phi after the
cycles is bitwise the reference's (FNV-64 of tests/golden/cycles.json), sweep counts equal
the single-GPU ones, and the transport really carried the exchanges."""
import pytest

from mp_workers import run_world, solve_worker

pytestmark = pytest.mark.gpu


def _golden(golden_cycles, kind, N, k):
    c = next(c for c in golden_cycles if c["kind"] == kind and c["N"] == N and c["eps"] == 1e-7)
    return c["cycles"][k - 1]


CASES = [
    # (kind, N, world, cycles, cfg)
    ("V", 4097, 2, 3, {}),                                  # level 0..2049 on strips (cross-fused)
    ("V", 1025, 3, 3, {"gather_n": 65, "tail_n": 17}),      # deep strips, 3 ranks
    ("V", 1025, 2, 3, {"gather_n": 65, "exact": True}),     # one allreduce per check
    ("W", 513, 2, 1, {"gather_n": 65, "tail_n": 17}),
    ("F", 1025, 2, 1, {"gather_n": 129}),
]


@pytest.mark.parametrize("kind,N,world,cycles,cfg", CASES)
def test_multiprocess_strips_bitwise(pgmg, golden_cycles, kind, N, world, cycles, cfg):
    res = run_world(solve_worker, world, N, kind, cycles, cfg, timeout=240)
    want = _golden(golden_cycles, kind, N, cycles)
    assert res[0]["hash"] == want["hash"], (kind, N, world)
    assert all(r["sweeps"] == want["sweeps"] for r in res), [r["sweeps"] for r in res]
    assert all(r["calls"] > 0 for r in res)      # the exchanges went through the callbacks
    assert all(r["dist"] == res[0]["dist"] for r in res)
