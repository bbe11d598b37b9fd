"""GPU: the C++ mirror of the reference entry (host/gpu_exec: ParallelTestRunner ->
ParallelMultiGridSolver -> C ABI) prints the reference's lines and files, and its
solutions are bitwise the reference goldens (FNV-64 of phi after 3 V- and 3 W-cycles,
alpha = 3; the relative error line to the 6 digits std::cout prints)."""
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, assert_bitwise

pytestmark = pytest.mark.gpu

EXE = ROOT / "parallel-geometric-multigrid-for-poisson-problem_amd" / "host" / "gpu_exec"


def _golden_relerr(golden_cycles, kind, N, k):
    c = next(c for c in golden_cycles if c["kind"] == kind and c["N"] == N and c["eps"] == 1e-7)
    return c["cycles"][k - 1]["relerr"]


def _golden_hash(golden_cycles, kind, N, k):
    c = next(c for c in golden_cycles if c["kind"] == kind and c["N"] == N and c["eps"] == 1e-7)
    return c["cycles"][k - 1]["hash"]


def test_gpu_exec_matches_reference(tmp_path, golden_cycles):
    out = subprocess.run([str(EXE), "--n", "33,129", "--cycles", "3", "--hash"], cwd=tmp_path,
                         capture_output=True, text=True, timeout=300, check=True).stdout
    errs = [float(x) for x in re.findall(r"Final Relative L2 Error: (\S+)", out)]
    hashes = re.findall(r"phi FNV-64: ([0-9a-f]{16})", out)
    assert len(errs) == 4 and len(hashes) == 4, out
    cases = [("V", 33), ("W", 33), ("V", 129), ("W", 129)]
    for got, (kind, N) in zip(errs, cases):
        w = _golden_relerr(golden_cycles, kind, N, 3)
        assert float(f"{w:.6g}") == got, (got, w)   # std::cout default precision
    for got, (kind, N) in zip(hashes, cases):
        # the whole mirror path (device arrays bound to the cached context -- staged below
        # N = 2049 --, W through ParallelMultiGridSolver::w_cycle) bitwise the reference
        assert got == _golden_hash(golden_cycles, kind, N, 3), (kind, N)
    for name in ("timings_parallel_v_cycle.txt", "timings_parallel_w_cycle.txt"):
        rows = (tmp_path / "OUTPUT_RESULT" / name).read_text().split("\n")
        assert [r.split()[0] for r in rows if r] == ["33", "129"]


def test_gpu_exec_op_timings(tmp_path):
    """plotTimeSequentialVsParallel (ParallelTestRunner.cu:98-125, save_to_file.hpp:62-89):
    GPU and CPU timing files for every op, one row per (num_thread, N); the CPU side only
    below N = 4096, as in the reference."""
    out = subprocess.run([str(EXE), "--n", "65", "--cycles", "1", "--ops"], cwd=tmp_path,
                         capture_output=True, text=True, timeout=300, check=True).stdout
    assert "N: 65" in out
    for op in ("residual", "jacobi", "restriction", "prolungator"):
        for side in ("gpu", "cpu"):
            rows = (tmp_path / "OUTPUT_RESULT" / f"timings_{op}_{side}.txt").read_text().split("\n")
            rows = [r.split() for r in rows if r]
            assert [r[:2] for r in rows] == [["16", "65"], ["32", "65"]], (op, side)
            assert all(float(r[2]) >= 0 for r in rows)


def test_gpu_exec_err_vector(tmp_path, oracle_mod):
    """run_w_cycles_err_vector_iteration (ParallelTestRunner.cu:143-150) writes the last
    W-cycle run's phi - u in save_errors_vector_to_file_last_iteration_gpu's format
    (save_vector_err_file.hpp:63-83: the length, then one value per line at std::cout's
    default precision): equal to the reference's 3 W-cycles at N = 33 (golden phi)."""
    out = subprocess.run([str(EXE), "--err-vector", "33", "--cycles", "3"], cwd=tmp_path,
                         capture_output=True, text=True, timeout=300, check=True).stdout
    assert "Final Relative L2 Error" in out
    lines = (tmp_path / "OUTPUT_RESULT" / "ERR_VECTOR" / "iteration_last_gpu.txt").read_text().split()
    assert int(lines[0]) == 33 * 33 and len(lines) == 1 + 33 * 33
    phi = np.load(GOLDEN / "phi_W33_c3.npy")
    err = (phi - oracle_mod.Oracle().exact(33)).ravel()
    want = [float(f"{e:.6g}") for e in err]
    assert [float(x) for x in lines[1:]] == want


def test_mirror_honours_h(pgmg, oracle_mod):
    """ParallelMultiGridSolver::v_cycle(phi, f, N, h) takes h from the caller
    (Parallel_Mg.cu:21; MultiGrid.hpp:57): pgmg_config.h0 carries it, and a V-cycle with a
    mesh width other than 1/(N-1) is bitwise the oracle's with that h."""
    N = 129
    h = 0.7 / (N - 1)
    o = oracle_mod.Oracle()
    f = o.rhs(N)
    ref = np.zeros((N, N))
    o.v_cycle(ref, f, h)
    o.v_cycle(ref, f, h)
    with pgmg.Solver(N, h0=h) as s:
        s.set_problem(None, f)
        s.vcycle(2)
        got = s.solution()
        sweeps, _ = s.stats()
    assert_bitwise(got, ref, "V-cycles with h0")
    assert sweeps == o.sweeps


REF_EXE = ROOT / "oracle" / "_ref" / "gpu_exec_ref"


@pytest.mark.skipif(not REF_EXE.exists(), reason="oracle/_ref/gpu_exec_ref not built "
                    "(make -C oracle ref, in a container with the reference tree)")
def test_reference_main_on_mirror(tmp_path, golden_cycles):
    """The reference's OWN gpu_exec main (3_part_parallel/main.cu with INTEGRATION.md's two
    edits, built by oracle/ref_gpu_exec.sh against host/ and libpgmg.so): its default run
    (N = 33 ... 2049, 3 V- then 3 W-cycles per N, alpha = 3) on the MI355X prints the
    reference's errors (every golden there is) and writes its timing files."""
    out = subprocess.run([str(REF_EXE)], cwd=tmp_path, capture_output=True, text=True,
                         timeout=600, check=True).stdout
    errs = [float(x) for x in re.findall(r"Final Relative L2 Error: (\S+)", out)]
    Ns = [33, 65, 129, 257, 513, 1025, 2049]
    assert len(errs) == 2 * len(Ns), out
    checked = 0
    for i, N in enumerate(Ns):
        for j, kind in enumerate(("V", "W")):
            c = next((c for c in golden_cycles if c["kind"] == kind and c["N"] == N
                      and c["eps"] == 1e-7 and len(c["cycles"]) >= 3), None)
            if c is None:
                continue
            assert float(f"{c['cycles'][2]['relerr']:.6g}") == errs[2 * i + j], (kind, N)
            checked += 1
    assert checked >= 7
    for name in ("timings_parallel_v_cycle.txt", "timings_parallel_w_cycle.txt"):
        rows = (tmp_path / "OUTPUT_RESULT" / name).read_text().split("\n")
        assert [int(r.split()[0]) for r in rows if r] == Ns


@pytest.mark.parametrize("args", [["--n", "2049", "--cycles", "2", "--v-only"],
                                  ["--n", "129", "--cycles", "3", "--v-only", "--host-arrays"],
                                  ["--n", "2049", "--cycles", "2", "--v-only", "--mixed-dphi-hf"],
                                  ["--n", "129", "--cycles", "3", "--v-only", "--mixed-hphi-df"]])
def test_gpu_exec_array_modes(tmp_path, golden_cycles, args):
    """The mirror's v_cycle on device arrays in place (N = 2049: cross-fused), on host arrays
    (--host-arrays), and mixed: a device phi with a host f binds phi and a device
    copy of f; a host phi with a device f reads f back and takes the host path.  Every mode
    gives the reference's hash."""
    out = subprocess.run([str(EXE), "--hash"] + args, cwd=tmp_path, capture_output=True,
                         text=True, timeout=300, check=True).stdout
    N, k = int(args[1]), int(args[3])
    mode = re.findall(r"phi arrays: (.+)", out)[0].strip()
    host = "--host-arrays" in args or "--mixed-hphi-df" in args
    assert mode == ("host" if host else "device, in place"), mode
    assert re.findall(r"phi FNV-64: ([0-9a-f]{16})", out)[0] == _golden_hash(golden_cycles, "V", N, k)
