"""CPU: bench.py's launcher (`--gpus N` without a launcher starts N ranks itself; a mismatch
between --gpus and the world size, or too few devices, exits non-zero).  VERDICT r03 #1: the
driver's 8-GPU scaling run must measure what it claims."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = str(ROOT / "bench.py")
OFF = ["--cpu-baseline", "off", "--pmc", "off", "--trace", "off"]


def _env(**kw):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PGMG_BENCH_SOLO", "PGMG_BENCH_TRANSPORT",
              "PGMG_BENCH_LAUNCH_STUB"):
        e.pop(k, None)
    e.update(kw)
    return e


def test_gpus_n_launches_n_ranks():
    # --n: an abbreviation of the launcher's own options (--nnodes, ...), forwarded as --N
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--n", "4097"] + OFF,
                       capture_output=True, text=True, timeout=300,
                       env=_env(PGMG_BENCH_LAUNCH_STUB="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(x["stub_rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 for x in lines)
    assert sorted(x["local_rank"] for x in lines) == [0, 1]
    assert all(x["n"] == 4097 for x in lines)


def test_gpus_mismatch_with_world_size_fails():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"] + OFF, capture_output=True,
                       text=True, timeout=120,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_gpus_more_than_devices_fails():
    """No GPU in this container: --gpus 2 without a harness transport exits 2 with a message
    instead of timing one GPU and printing n_gpus: 1."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"] + OFF, capture_output=True,
                       text=True, timeout=300, env=_env())
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs 2 GPUs" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_options_listed():
    """The options the driver's runs and DESIGN.md name exist (a rename would silently fall
    back to argparse's prefix matching or fail only on the GPU box)."""
    r = subprocess.run([sys.executable, BENCH, "--help"], capture_output=True, text=True,
                       timeout=120, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    for opt in ("--gpus", "--steps", "--warmup", "--big-grid", "--other-configs", "--cycle",
                "--save-profiles", "--trace", "--pmc", "--cpu-baseline", "--ops"):
        assert opt in r.stdout, opt


def test_op_cases_build_and_match_kernel_names():
    """bench.py's per-op study table builds (every case callable) and each case's trace-key
    matcher picks the kernels that call launches (bench.kernel_key form: no spaces) -- a stub library on the CPU,
    no GPU."""
    import importlib
    sys.path.insert(0, str(ROOT))
    bench = importlib.import_module("bench")

    class Ops:
        def __getattr__(self, name):
            return lambda *a, **k: None

    class PG:
        ops = Ops()
        PGMG_PROLONG_SYMMETRIC, PGMG_PROLONG_REFERENCE = 1, 0

    cases, keep = bench.op_cases(PG(), 33, device="cpu")
    assert len(cases) == 8 and len(keep) == 6
    for _, call, nbytes, keys, sweeps in cases:
        call()
        assert nbytes > 0 and callable(keys)
    names = {
        0: "k_op_sweep_ip<16,true,true>", 1: "k_op_sweep2_ip<8,true,true>",
        2: "k_op_sweep2_ip<8,true,true>", 3: "k_op_sweep<16,true,false,true>",
        4: "k_op_residual<16>", 5: "k_op_restrict<8>", 6: "k_op_prolong<1>", 7: "k_op_prolong<0>",
    }
    for i, k in names.items():
        assert cases[i][3](k), (i, k)
    assert not cases[0][3]("k_op_sweep2_ip<8,true,true>")
    assert not cases[1][3]("k_op_sweep_ip<16,true,true>")
    assert cases[2][3]("k_op_sweep_ip<16,true,true>")
