"""CPU: the reference-side switch-over of INTEGRATION.md §2 compiles and links.

oracle/ref_gpu_exec.sh applies exactly the two documented edits to the reference's own
3_part_parallel/main.cu (the ParallelTestRunner include and the CUDA warm-up block) and builds
it with g++ against the C++ mirror (host/) and libpgmg.so — no CUDA, no shims.  Needs the
reference tree (this container); the GPU run of the result is tests/test_gpu_exec.py."""
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
REF_MAIN = pathlib.Path("/root/reference/3_part_parallel/main.cu")
LIB = ROOT / "parallel-geometric-multigrid-for-poisson-problem_amd" / "libpgmg.so"


@pytest.mark.skipif(not REF_MAIN.exists(), reason="reference tree absent")
@pytest.mark.skipif(not LIB.exists(), reason="libpgmg.so not built")
def test_reference_main_builds_against_mirror(tmp_path):
    out = tmp_path / "gpu_exec_ref"
    subprocess.run([str(ROOT / "oracle" / "ref_gpu_exec.sh"), str(out)], check=True,
                   capture_output=True, text=True, timeout=300)
    assert out.exists()
    deps = subprocess.run(["ldd", str(out)], capture_output=True, text=True).stdout
    assert "libpgmg.so" in deps and "cuda" not in deps.lower()
    syms = subprocess.run(["nm", "-u", str(out)], capture_output=True, text=True).stdout
    # the mirror's calls into the C ABI, nothing of the CUDA runtime
    for s in ("pgmg_create", "pgmg_set_problem_device", "pgmg_vcycle", "pgmg_wcycle",
              "pgmg_alloc_grid", "pgmg_device_sync"):
        assert s in syms, s
    assert "cuda" not in syms.lower()


@pytest.mark.skipif(not REF_MAIN.exists(), reason="reference tree absent")
def test_documented_edits_are_the_applied_ones():
    """INTEGRATION.md §2 shows the same two edits the recipe applies."""
    doc = (ROOT / "INTEGRATION.md").read_text()
    recipe = (ROOT / "oracle" / "ref_gpu_exec.sh").read_text()
    for needle in ('#include "ParallelTestRunner.hpp"', "pgmg_device_sync();"):
        assert needle in doc and needle in recipe
    src = REF_MAIN.read_text()
    assert src.count('#include "ParallelTestRunner.cu"') == 1
    assert "cudaMallocManaged(&tmp" in src and "cudaFree(tmp);" in src
