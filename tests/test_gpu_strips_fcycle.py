"""GPU: the F-cycle (full multigrid, MultiGridTestRunner.hpp:192-205 -> f_cycle) on row
strips is bit-identical to one GPU: the restriction of phi runs on every rank's own rows
(one halo row exchanged) and the first replicated level is assembled by one all-to-all;
the climb computes the analytic RHS of its strip (and halo rows) locally, zeroes the frame
rows it holds, prolongates its rows (one coarse halo row) and runs the V-cycle and the three
smoothing sweeps of each level distributed.  BASELINE config 5 is FMG + W-cycles on 8 GPUs:
both are checked, at worlds 2, 4 and 8, with the reference's F goldens.

Ranks are threads sharing the one GPU (loopback transport, see test_gpu_strips.py)."""
import threading

import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _ranks(pgmg, world, N, calls, problem=(None, None), **cfg):
    hub = pgmg.LoopbackHub(world)
    out, err = [None] * world, [None] * world

    def work(r):
        try:
            with pgmg.Solver(N, hub=hub, rank=r, **cfg) as s:
                s.set_problem(*problem)
                for kind, k in calls:
                    getattr(s, f"{kind}cycle")(k)
                out[r] = (s.solution(), s.stats_detail())
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
    return out


def _single(pgmg, N, calls, problem=(None, None), **cfg):
    with pgmg.Solver(N, **cfg) as s:
        s.set_problem(*problem)
        for kind, k in calls:
            getattr(s, f"{kind}cycle")(k)
        return s.solution(), s.stats_detail()


@pytest.mark.parametrize("world,N,gather_n", [(2, 1025, 65), (4, 1025, 129), (8, 2049, 129),
                                              (4, 4097, 1025), (3, 513, 33)])
def test_strips_fcycle_bitwise_equal_single_gpu(pgmg, world, N, gather_n):
    calls = [("f", 2)]
    ref = _single(pgmg, N, calls)
    outs = _ranks(pgmg, world, N, calls, gather_n=gather_n)
    for r, (phi, det) in enumerate(outs):
        assert_bitwise(phi, ref[0], f"rank {r} of {world}")
    assert outs[0][1][:2] == ref[1][:2]


def test_strips_fcycle_reference_golden(pgmg, oracle_mod, golden_cycles):
    case = next(c for c in golden_cycles if c["kind"] == "F" and c["N"] == 1025)
    k = case["cycles"][-1]["cycle"]
    outs = _ranks(pgmg, 4, 1025, [("f", k)], gather_n=65)
    assert oracle_mod.fnv_hash(outs[0][0]) == case["cycles"][-1]["hash"]


@pytest.mark.parametrize("world", [2, 8])
def test_strips_fmg_then_wcycles(pgmg, world):
    """BASELINE config 5's shape: an FMG start, then W-cycles (and V-cycles), on strips."""
    calls = [("f", 1), ("w", 2), ("v", 2)]
    ref = _single(pgmg, 2049, calls)
    outs = _ranks(pgmg, world, 2049, calls, gather_n=129)
    for r, (phi, _) in enumerate(outs):
        assert_bitwise(phi, ref[0], f"rank {r}")


def test_strips_fcycle_nonzero_boundary_fp32(pgmg):
    """A random phi0 with a non-zero boundary (the F-cycle zeroes the frame it holds), and
    the fp32 variant."""
    rng = np.random.default_rng(4)
    N = 1025
    phi0 = rng.uniform(-1, 1, (N, N))
    for dtype in ("f64", "f32"):
        calls = [("v", 1), ("f", 1), ("v", 2)]
        ref = _single(pgmg, N, calls, (phi0, None), dtype=dtype)
        outs = _ranks(pgmg, 4, N, calls, (phi0, None), gather_n=65, dtype=dtype)
        for r, (phi, _) in enumerate(outs):
            assert_bitwise(phi, ref[0], f"{dtype} rank {r}")
