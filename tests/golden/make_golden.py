#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own CPU multigrid.

Run in the build container only (needs /root/reference and `make -C oracle ref`):

    python tests/golden/make_golden.py [--big]

The reference (2_part_MG/MultiGrid.hpp + Smoother.hpp + DynamicGridUtils.hpp) is compiled
unmodified by oracle/Makefile into oracle/_ref/ref_harness; this script only runs it and
stores inputs/outputs as data:

  cycles.json        per-cycle relerr / residual norm / centre value / FNV-64 hash of phi /
                     cumulative sweep and early-exit counts, for V, W and F cycles
  phi_<K><N>_c<k>.npy  full phi vectors for small N (N <= 129)
  ops_N<N>.npz       seeded random inputs and the reference's residual, restriction,
                     prolongation and smoother outputs (op-level known-answer tests)
"""
import argparse
import json
import os
import pathlib
import subprocess
import tempfile

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
REPO = HERE.parent.parent
HARNESS = REPO / "oracle" / "_ref" / "ref_harness"

# (kind, N, cycles, eps, dump_phi_at)
CASES = [
    ("V", 33, 30, 1e-7, [1, 3, 30]),
    ("V", 65, 3, 1e-7, [3]),
    ("V", 129, 30, 1e-7, [1, 30]),
    ("V", 257, 3, 1e-7, []),
    ("V", 513, 30, 1e-7, []),
    ("V", 1025, 3, 1e-7, []),
    ("V", 2049, 2, 1e-7, []),
    ("V", 4097, 43, 1e-7, []),    # BASELINE configs[1]: the bench times 3 + 40 cycles
    ("V", 129, 8, 1e3, [8]),     # every smoother exits after its first sweep
    ("V", 257, 5, 1.0, []),      # mixed early exits
    ("V", 65, 4, 0.0, [4]),      # never exits
    ("W", 33, 3, 1e-7, [3]),
    ("W", 129, 3, 1e-7, [3]),
    ("W", 513, 1, 1e-7, []),
    ("F", 33, 3, 1e-7, [3]),
    ("F", 129, 2, 1e-7, [2]),
    ("F", 1025, 1, 1e-7, []),
]
# Full-size cases (python make_golden.py --big: ~45 min on one core, <= 60 GB RSS).
# (kind, N, cycles, tool): tool "ref" = the compiled reference (oracle/_ref/ref_harness,
# whose leak reclaimer keeps its RSS at ~9 grids); "port" = oracle/mg_cpu_exec_port, our C
# restatement, pinned bit for bit to the reference up to N = 16385 by the cases above and
# used at N = 32769, where the reference needs more host memory than the build container
# has.  Kind G = FMG start + W-cycles (BASELINE config 5): cycle 1 an F-cycle, then W.
BIG = [("V", 16385, 30, "ref"),     # every cycle count the bench can time (warmup + steps)
       ("F", 16385, 22, "ref"),     # bench.py --cycle F: warmup 2 + steps 20
       ("G", 16385, 2, "ref"),
       ("V", 32769, 6, "port"),     # BASELINE config 4's grid (the bench times 1 + 5 cycles)
       ("G", 32769, 2, "port")]     # BASELINE config 5's grid
PORT = REPO / "oracle" / "mg_cpu_exec_port"


def parse(line):
    t = line.split()
    d = {t[i]: t[i + 1] for i in range(0, len(t) - 1, 2)}
    return {
        "cycle": int(d["cycle"]),
        "relerr": float(d["relerr"]),
        "res": float(d["res"]),
        "center": float(d["center"]),
        "hash": d["hash"],
        "sweeps": int(d["sweeps"]),
        "exits": int(d["exits"]),
    }


def big_case(kind, N, cycles, tool, ingest=None):
    """One BIG case: run the tool (or read its saved stdout, ingest/<kind><N>.txt, produced by
    exactly `<tool> <kind> <N> <cycles> 1e-7`)."""
    exe = HARNESS if tool == "ref" else PORT
    if ingest:
        path = pathlib.Path(ingest) / f"{kind}{N}.txt"
        out = path.read_text() if path.exists() else ""
        if sum(l.startswith("cycle") for l in out.splitlines()) < cycles:
            print(f"skipping {kind} {N}: {path} incomplete")
            return None
    else:
        out = subprocess.run([str(exe), kind, str(N), str(cycles), "1e-7"],
                             check=True, capture_output=True, text=True).stdout
    rows = [parse(l) for l in out.splitlines() if l.startswith("cycle")]
    assert len(rows) == cycles, (kind, N, len(rows))
    src = ("oracle/_ref/ref_harness (the reference's MultigridSolver)" if tool == "ref"
           else "oracle/mg_cpu_exec_port (C restatement)")
    return {"kind": kind, "N": N, "eps": 1e-7, "cycles": rows, "source": src}


def run_case(kind, N, cycles, eps, dumps, tmp):
    rows = []
    # one run for the stats; phi dumps need a run per dump point (harness dumps the last cycle)
    out = subprocess.run([str(HARNESS), kind, str(N), str(cycles), repr(eps)],
                         check=True, capture_output=True, text=True).stdout
    rows = [parse(l) for l in out.splitlines() if l.startswith("cycle")]
    for k in dumps:
        path = os.path.join(tmp, "phi.bin")
        subprocess.run([str(HARNESS), kind, str(N), str(k), repr(eps), path],
                       check=True, capture_output=True)
        phi = np.fromfile(path, dtype="<f8").reshape(N, N)
        tag = "" if eps == 1e-7 else f"_eps{eps:g}"
        np.save(HERE / f"phi_{kind}{N}_c{k}{tag}.npy", phi)
    return {"kind": kind, "N": N, "eps": eps, "cycles": rows}


def make_ops(N, seed, tmp):
    rng = np.random.default_rng(seed)
    Nc = (N - 1) // 2 + 1
    h = 1.0 / (N - 1)
    x = rng.uniform(-1.0, 1.0, (N, N))
    f = rng.uniform(-1.0, 1.0, (N, N))
    e = rng.uniform(-1.0, 1.0, (Nc, Nc))
    for a in (x, f, e):   # Dirichlet boundary 0
        a[0, :] = a[-1, :] = a[:, 0] = a[:, -1] = 0.0
    eps = 1e-7
    pin = os.path.join(tmp, "in.bin")
    pout = os.path.join(tmp, "out.bin")
    np.concatenate([x.ravel(), f.ravel(), e.ravel()]).astype("<f8").tofile(pin)
    subprocess.run([str(HARNESS), "O", str(N), repr(h), repr(eps), pin, pout], check=True)
    o = np.fromfile(pout, dtype="<f8")
    L, Lc = N * N, Nc * Nc
    parts = np.split(o, np.cumsum([L, Lc, L, L]))
    np.savez(HERE / f"ops_N{N}.npz", N=N, h=h, eps=eps, x=x, f=f, e=e,
             residual=parts[0].reshape(N, N), restrict=parts[1].reshape(Nc, Nc),
             prolong=parts[2].reshape(N, N), smooth1=parts[3].reshape(N, N),
             smooth10=parts[4].reshape(N, N))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true", help="also run the full-size BIG cases")
    ap.add_argument("--ingest", metavar="DIR",
                    help="with --big: read the BIG cases' stdout from DIR/<kind><N>.txt")
    ap.add_argument("--big-only", action="store_true", help="skip the small cases")
    args = ap.parse_args()
    if not HARNESS.exists():
        raise SystemExit("build the reference harness first: make -C oracle ref")
    prev = []
    jpath = HERE / "cycles.json"
    if jpath.exists():
        prev = json.loads(jpath.read_text())
    res = []
    with tempfile.TemporaryDirectory() as tmp:
        if not args.big_only:
            res = [run_case(*c, tmp) for c in CASES]
            for N, seed in ((17, 1), (33, 12345), (65, 7)):
                make_ops(N, seed, tmp)
    if args.big or args.big_only:
        res += [r for r in (big_case(*c, ingest=args.ingest) for c in BIG) if r is not None]
    keys = {(r["kind"], r["N"], r["eps"]) for r in res}
    res += [r for r in prev if (r["kind"], r["N"], r["eps"]) not in keys]
    res.sort(key=lambda r: (r["kind"], r["N"], r["eps"]))
    jpath.write_text(json.dumps(res, indent=1) + "\n")
    print(f"wrote {len(res)} cases to {jpath}")


if __name__ == "__main__":
    main()
