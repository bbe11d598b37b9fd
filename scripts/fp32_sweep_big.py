#!/usr/bin/env python3
"""fp32-vs-fp64 tolerance sweep at N = 32769 (BASELINE config 5's grid) on one GPU.

The same measurements as scripts/fp32_sweep.py for the grid where a full host copy is
8.6 GB: V-cycles, F-cycles and the FMG start + W-cycle sequence ("G"), after every cycle
the relative L2 error against the exact solution for both precisions and
||phi32 - phi64|| / ||phi64||, computed in row chunks (the exact solution is separable).
Appends its rows to the JSON document given by --merge (or prints them).

    python scripts/fp32_sweep_big.py [--n 32769] [--cycles 2] [--merge profiles/.../fp32_sweep.json]
"""
import argparse
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
CH = 2048   # rows per chunk


def stats(phi, ref, N):
    """(||phi - u||/||u||, ||phi - ref||/||ref||, max|phi - ref|) by row chunks"""
    x = np.sin(np.pi * np.arange(N) / (N - 1))
    e2 = u2 = d2 = r2 = 0.0
    mx = 0.0
    for a in range(0, N, CH):
        b = min(N, a + CH)
        u = np.outer(x[a:b], x)
        p = phi[a:b]
        e2 += float(np.sum((p - u) ** 2))
        u2 += float(np.sum(u * u))
        if ref is not None:
            d = p - ref[a:b]
            d2 += float(np.sum(d * d))
            r2 += float(np.sum(ref[a:b] ** 2))
            mx = max(mx, float(np.max(np.abs(d))))
    return (e2 / u2) ** 0.5, ((d2 / r2) ** 0.5 if ref is not None else None), mx


def run(pg, N, kind, cycles, dtype):
    with pg.Solver(N, dtype=dtype) as s:
        s.set_problem()
        for c in range(cycles):
            if kind == "V":
                s.vcycle(1)
            elif kind == "F" or (kind == "G" and c == 0):
                s.fcycle(1)
            else:
                s.wcycle(1)
            yield c + 1, s.solution()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32769)
    ap.add_argument("--cycles", type=int, default=2)
    ap.add_argument("--kinds", default="V,F,G")
    ap.add_argument("--merge", default="")
    args = ap.parse_args()
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    N = args.n
    rows = []
    for kind in args.kinds.split(","):
        p64 = {}
        for c, phi in run(pg, N, kind, args.cycles, "f64"):
            p64[c] = (stats(phi, None, N)[0], phi)
        for c, phi in run(pg, N, kind, args.cycles, "f32"):
            e32, d, mx = stats(phi, p64[c][1], N)
            row = {"N": N, "kind": kind, "cycle": c, "relerr_f64": p64[c][0], "relerr_f32": e32,
                   "diff_f32_f64": d, "maxabs_f32_f64": mx}
            rows.append(row)
            print(json.dumps(row), flush=True)
        del p64
    if args.merge:
        p = pathlib.Path(args.merge)
        doc = json.loads(p.read_text())
        doc["rows"] = [r for r in doc["rows"] if r["N"] != N] + rows
        doc.setdefault("notes", []).append(
            f"N={N} rows: scripts/fp32_sweep_big.py (kind G = FMG start then W-cycles)")
        p.write_text(json.dumps(doc, indent=1) + "\n")


if __name__ == "__main__":
    main()
