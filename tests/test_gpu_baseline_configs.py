"""GPU: every BASELINE.json config in the exact call shapes bench.py times, bit for bit against
the reference's fixtures (tests/golden/cycles.json, tests/golden/fp32_big.json).

One test per config id (BASELINE.json "configs"):
  config0_513            mg_cpu_exec's V-cycle at N = 513 (a CPU config: the HIP path run on it
                         against the reference's 30-cycle hashes)
  config1_4097           1 GPU, N = 4097: bench.py's other_configs leg, 3 + 40 cycles per
                         repetition on one context (set_problem restarts), 43-cycle hash
  config2_16385          1 GPU, N = 16385 (the roofline run): the headline leg's warmup 5 +
                         steps 20 with the per-pass timing events, and the general-RHS leg
  config3_32769          N = 32769: one GPU in bench.py's 1 + 5 shape, and 8 row strips
                         (loopback ranks on the one GPU of the test box: the production strip
                         code; RCCL cannot host two ranks on one device)
  config4_fmg_w_32769    FMG start + one W-cycle at N = 32769, fp64 on one GPU against the
                         hash; fp32 on 8 strips bitwise fp32 on one GPU, within the tolerance
                         sweep's distance of fp64
Beside them, the bench's other timed shapes: multi-F-cycle calls at 16385 (bench.py --cycle F:
2 + 20, k_post_r2 between consecutive F-cycles) and fp32 V-cycles at 16385 (bench.py --dtype
f32) against the fp32 restatement's hashes.

Hashes: FNV-64 over phi's IEEE words; the V/F/G 16385 rows come from the compiled
reference (oracle/_ref/ref_harness), the 32769 rows from oracle/mg_cpu_exec_port (the C
restatement), confirmed bitwise in r06 by the reference's own MultigridSolver run at 32769 on a
GPU box's host (profiles/r06/ref32769/), fp32 rows from oracle/liboracle_f32.so.
Tolerance: EXACT (bitwise phi, equal sweep counts) except the stated fp32-vs-fp64 bound.
Reference: /root/reference/2_part_MG/MultiGrid.hpp:57-183.
"""
import json
import pathlib
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"


def _rows(golden_cycles, kind, N, need):
    for c in golden_cycles:
        if c["kind"] == kind and c["N"] == N and c["eps"] == 1e-7 and len(c["cycles"]) >= need:
            return c["cycles"]
    pytest.skip(f"no golden for {kind} N={N} with {need} cycles (make_golden.py --big)")


def _check_hash(got_hash, sweeps, rows, k, what):
    want = rows[k - 1]
    assert got_hash == want["hash"], f"{what}: phi differs from the reference after cycle {k}"
    assert sweeps == want["sweeps"], (what, sweeps, want["sweeps"])


def _ranks(pgmg, world, N, work, **cfg):
    """`world` loopback ranks in threads; work(solver) runs the cycles; phi is gathered to
    rank 0 only (a full host copy per rank would be 8.6 GB each at 32769)."""
    hub = pgmg.LoopbackHub(world)
    out, err = [None] * world, [None] * world

    def run(r):
        try:
            with pgmg.Solver(N, hub=hub, rank=r, **cfg) as s:
                s.set_problem()
                work(s)
                phi = s.gather_solution(0, r == 0)
                out[r] = (phi, s.stats())
        except Exception as e:  # surfaced below
            err[r] = e

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=900)
    hub.close()
    for e in err:
        if e is not None:
            raise e
    return out


# ---------------------------------------------------------------------------- configs[0]
@pytest.mark.parametrize("calls", [[30], [2, 28], [1] * 30])
def test_config0_513(pgmg, golden_cycles, calls):
    """configs[0] (N = 512^2, 2 pre/post sweeps): the HIP path over the reference's 30 cycles
    (coarse checks fire from cycle ~12), one call, bench-like warmup + steps, one-cycle calls."""
    rows = _rows(golden_cycles, "V", 513, 30)
    with pgmg.Solver(513) as s:
        s.set_problem()
        for k in calls:
            s.vcycle(k)
        _check_hash(s.solution_hash(0), s.stats()[0], rows, 30, f"config0 calls={calls}")


# ---------------------------------------------------------------------------- configs[1]
def test_config1_4097(pgmg, golden_cycles):
    """bench.py other_configs: `with Solver(4097)`, per repetition set_problem, vcycle(3),
    vcycle(40); the timed call's result is the reference's 43-cycle phi."""
    rows = _rows(golden_cycles, "V", 4097, 43)
    with pgmg.Solver(4097) as s:
        for rep in range(2):
            s.set_problem()
            s.vcycle(3)
            s.vcycle(40)
            _check_hash(s.solution_hash(0), s.stats()[0], rows, 43, f"config1 rep {rep}")
            assert s.dist_info()[1] == 0, s.dist_info()   # no rollback on the reference problem


# ---------------------------------------------------------------------------- configs[2]
def test_config2_16385(pgmg, golden_cycles):
    """The headline leg (bench.py --warmup 5 --steps 20, with PGMG_FLAG_TIME_FINE's per-pass
    events) on the cross-fused finest level with the analytic f regenerated in-kernel."""
    rows = _rows(golden_cycles, "V", 16385, 25)
    with pgmg.Solver(16385, flags=pgmg.PGMG_FLAG_TIME_FINE) as s:
        assert s.fused, "not the cross-fused path"
        for rep in range(2):
            s.set_problem()
            assert s.fine_pass_bytes(3) < s.fine_pass_bytes(0), "f not regenerated in-kernel"
            s.vcycle(5)
            s.vcycle(20)
            assert s.dist_info()[0], "speculative decisions off"
            _check_hash(s.solution_hash(0), s.stats()[0], rows, 25, f"config2 rep {rep}")


def test_config2_16385_stored_rhs(pgmg, golden_cycles):
    """bench.py's general-RHS leg (f streamed from HBM, 24 B/pt), same 5 + 20 shape."""
    rows = _rows(golden_cycles, "V", 16385, 25)
    with pgmg.Solver(16385, flags=pgmg.PGMG_FLAG_STORED_RHS) as s:
        s.set_problem()
        assert s.fine_pass_bytes(3) > s.fine_pass_bytes(0), "f regenerated despite the flag"
        s.vcycle(5)
        s.vcycle(20)
        _check_hash(s.solution_hash(0), s.stats()[0], rows, 25, "config2 stored f")


# ---------------------------------------------------------------------------- configs[3]
def test_config3_32769_one_gpu(pgmg, golden_cycles):
    """configs[3]'s grid on one GPU in bench.py's shape (1 + 5 cycles, two calls)."""
    rows = _rows(golden_cycles, "V", 32769, 6)
    with pgmg.Solver(32769) as s:
        s.set_problem()
        s.vcycle(1)
        s.vcycle(5)
        _check_hash(s.solution_hash(0), s.stats()[0], rows, 6, "config3 one GPU 1 + 5")


def test_config3_32769_8_strips(pgmg, oracle_mod, golden_cycles):
    """configs[3]: N = 32769 on 8 row strips, one vcycle(2) call per rank (cross-fused finest
    level per strip, speculative decisions, halo rows through the transport)."""
    rows = _rows(golden_cycles, "V", 32769, 2)
    out = _ranks(pgmg, 8, 32769, lambda s: s.vcycle(2))
    _check_hash(oracle_mod.fnv_hash(out[0][0]), out[0][1][0], rows, 2, "config3 8 strips")


# ---------------------------------------------------------------------------- configs[4]
def test_config4_fmg_w_32769_fp64(pgmg, golden_cycles):
    """bench.py other_configs: set_problem, fcycle(1), wcycle(1) at N = 32769, fp64."""
    rows = _rows(golden_cycles, "G", 32769, 2)
    with pgmg.Solver(32769) as s:
        s.set_problem()
        s.fcycle(1)
        s.wcycle(1)
        _check_hash(s.solution_hash(0), s.stats()[0], rows, 2, "config4 FMG + W fp64")


def test_config4_fmg_w_32769_fp32_vs_fp64(pgmg, oracle_mod, golden_cycles):
    """configs[4]'s fp32 half: FMG start + one W-cycle at N = 32769 in fp32 on 8 row strips is
    bitwise the fp32 run on one GPU (pointwise arithmetic), and its distance from the fp64
    result (itself the reference's hash) is the one the sweep measured
    (profiles/r02_fp32/fp32_sweep.json, kind G cycle 2: 0.02353 relative; fp32's residual
    round-off, (N-1)^2 ulp(x), dominates at this size).
    Tolerance: relative L2 difference <= 0.03 (the measured 0.0235 plus margin)."""
    N = 32769

    def work(s):
        s.fcycle(1)
        s.wcycle(1)

    out = _ranks(pgmg, 8, N, work, dtype="f32")
    phi8 = out[0][0]
    with pgmg.Solver(N, dtype="f32") as s:
        s.set_problem()
        work(s)
        phi1 = s.solution()
        st1 = s.stats()
    assert np.array_equal(phi8.view(np.uint64), phi1.view(np.uint64)), "fp32: 8 strips != 1 GPU"
    assert out[0][1][0] == st1[0]
    del phi8
    rows = _rows(golden_cycles, "G", N, 2)
    with pgmg.Solver(N) as s:
        s.set_problem()
        work(s)
        phi64 = s.solution()
        _check_hash(oracle_mod.fnv_hash(phi64), s.stats()[0], rows, 2, "config4 fp64 half")
    rel = float(np.linalg.norm(phi1 - phi64) / np.linalg.norm(phi64))
    print(f"fp32 vs fp64 after FMG + W at 32769: {rel:.6e} relative (sweep: 2.3532e-02)")
    assert rel <= 0.03, rel


# ------------------------------------------------------- the bench's other timed shapes
def test_multi_fcycle_16385(pgmg, oracle_mod, golden_cycles):
    """bench.py --cycle F (2 + 20 F-cycles in two calls: speculative F-cycles, k_post_r2
    forming the next F-cycle's level-2 restriction) against the reference's 22 F-cycles."""
    rows = _rows(golden_cycles, "F", 16385, 22)
    with pgmg.Solver(16385) as s:
        s.set_problem()
        s.fcycle(2)
        s.fcycle(20)
        _check_hash(s.solution_hash(0), s.stats()[0], rows, 22, "F 2 + 20 at 16385")
        assert s.dist_info()[1] == 0


def test_fp32_vcycle_16385(pgmg):
    """bench.py --dtype f32's shape at the headline grid (a fresh problem, a 5-cycle warmup
    call, then a 20-cycle call that starts from the warmup call's carry) against the fp32
    restatement of the reference (tests/golden/fp32_big.json, make_fp32_golden.py: 25 cycles):
    bitwise phi and equal sweep counts after cycles 1, 5 and 25, so the packed-fp32
    k_postpre_lds<float> is pinned over a long call with speculative decisions."""
    import sys
    sys.path.insert(0, str(GOLDEN))
    from make_fp32_golden import hash_f32
    path = GOLDEN / "fp32_big.json"
    case = next(c for c in json.loads(path.read_text()) if c["kind"] == "V" and c["N"] == 16385)
    assert len(case["cycles"]) >= 25
    with pgmg.Solver(16385, dtype="f32") as s:
        s.set_problem()
        s.vcycle(1)
        _check_hash(hash_f32(s.solution()), s.stats()[0], case["cycles"], 1, "fp32 c1")
        s.set_problem()
        s.vcycle(5)
        _check_hash(hash_f32(s.solution()), s.stats()[0], case["cycles"], 5, "fp32 c5")
        s.vcycle(20)
        _check_hash(hash_f32(s.solution()), s.stats()[0], case["cycles"], 25, "fp32 c25")
