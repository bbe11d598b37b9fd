"""CPU: the oracle's CLI and the reference's own CPU multigrid harness under
AddressSanitizer + UBSan ("CPU tests under -fsanitize=address,undefined").

oracle/Makefile `sanitize` builds both with -fsanitize=address,undefined
-fno-sanitize-recover=all; every run must exit 0 with no sanitizer report and print the same
lines (relative error, residual, centre value, FNV-64 of phi, sweep and exit counts) as the
unsanitized builds.  LeakSanitizer stays on for our oracle; the reference harness runs with
detect_leaks=0 because the reference leaks three arrays per level and cycle by design
(SURVEY Q5).  The library's host code under the same sanitizers needs a GPU:
tests/test_gpu_sanitize.py.
"""
import os
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
ORC = ROOT / "oracle"
CASES = [("V", 65, 3, "1e-7"), ("W", 65, 2, "1e-7"), ("F", 129, 2, "1e-7"), ("G", 65, 2, "1e-7"),
         ("V", 129, 4, "1000"), ("V", 33, 3, "0")]


@pytest.fixture(scope="module")
def san_build():
    subprocess.run(["make", "-C", str(ORC), "-s", "all", "sanitize"], check=True,
                   capture_output=True, timeout=600)
    return ORC / "_san"


def _lines(exe, args, env=None):
    p = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=300,
                       env={**os.environ, **(env or {})})
    assert p.returncode == 0, (exe, args, p.stderr[-3000:])
    assert "runtime error" not in p.stderr and "Sanitizer" not in p.stderr, p.stderr[-3000:]
    # drop the wall-clock field
    return [l.rsplit(" seconds", 1)[0] for l in p.stdout.splitlines() if l.startswith("cycle")]


@pytest.mark.parametrize("kind,N,cycles,eps", CASES)
def test_oracle_under_asan_ubsan(san_build, kind, N, cycles, eps):
    args = [kind, str(N), str(cycles), eps]
    got = _lines(san_build / "mg_cpu_exec_port", args, {"ASAN_OPTIONS": "detect_leaks=1"})
    want = _lines(ORC / "mg_cpu_exec_port", args)
    assert got == want and len(got) == cycles


@pytest.mark.skipif(not pathlib.Path("/root/reference/2_part_MG").exists(),
                    reason="reference tree absent")
@pytest.mark.parametrize("kind,N,cycles,eps", CASES[:4])
def test_reference_harness_under_asan_ubsan(san_build, kind, N, cycles, eps):
    args = [kind, str(N), str(cycles), eps]
    got = _lines(san_build / "ref_harness", args, {"ASAN_OPTIONS": "detect_leaks=0"})
    want = _lines(ORC / "_ref" / "ref_harness", args)
    assert got == want and len(got) == cycles
