#!/usr/bin/env python3
"""fp32-vs-fp64 tolerance sweep (BASELINE config 5) on one GPU.

For each grid N and cycle kind (V, W, F) from the reference's problem (phi0 = 0,
f = analytic RHS): after every cycle, the relative L2 error against the exact solution
for both precisions, ||phi32 - phi64|| / ||phi64||, and the V-cycle rate of each
precision.  Writes one JSON document (stdout, or --out).

    python scripts/fp32_sweep.py [--sizes 129,513,...] [--cycles 8] [--out file.json]
"""
import argparse
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def exact(N):
    x = np.sin(np.pi * np.arange(N) / (N - 1))
    return np.outer(x, x)


def relerr(phi, u):
    return float(np.linalg.norm(phi - u) / np.linalg.norm(u))


def run(pg, N, kind, cycles, dtype):
    out = []
    with pg.Solver(N, dtype=dtype) as s:
        s.set_problem()
        step = {"V": s.vcycle, "W": s.wcycle, "F": s.fcycle}[kind]
        for _ in range(cycles):
            step(1)
            out.append(s.solution())
    return out


def rate(pg, N, dtype, steps):
    with pg.Solver(N, dtype=dtype) as s:
        s.set_problem()
        s.vcycle(2)
        s.sync()
        t = time.perf_counter()
        s.vcycle(steps)
        s.sync()
        return steps / (time.perf_counter() - t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="129,513,1025,2049,4097,8193,16385")
    ap.add_argument("--cycles", type=int, default=8)
    ap.add_argument("--kinds", default="V,W,F")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch  # noqa: F401  (ROCm runtime first, see _capi.load)
    import _pkgload
    pg = _pkgload.load()
    doc = {"problem": "phi0=0, f=2 pi^2 sin(pi x) sin(pi y), eps=1e-7, v1=v2=1", "rows": []}
    for N in [int(n) for n in args.sizes.split(",")]:
        u = exact(N)
        for kind in args.kinds.split(","):
            # W-cycles cost ~3^depth coarse visits; keep them to the smaller grids
            if kind == "W" and N > 4097:
                continue
            k = args.cycles if N <= 4097 else max(2, args.cycles // 2)
            p64 = run(pg, N, kind, k, "f64")
            p32 = run(pg, N, kind, k, "f32")
            for c in range(k):
                row = {"N": N, "kind": kind, "cycle": c + 1,
                       "relerr_f64": relerr(p64[c], u), "relerr_f32": relerr(p32[c], u),
                       "diff_f32_f64": float(np.linalg.norm(p32[c] - p64[c]) /
                                             np.linalg.norm(p64[c])),
                       "maxabs_f32_f64": float(np.max(np.abs(p32[c] - p64[c])))}
                doc["rows"].append(row)
                print(json.dumps(row), file=sys.stderr, flush=True)
            del p64, p32
        steps = 20 if N >= 4097 else 100
        r = {"N": N, "vcycles_per_s_f64": rate(pg, N, "f64", steps),
             "vcycles_per_s_f32": rate(pg, N, "f32", steps)}
        doc.setdefault("rates", []).append(r)
        print(json.dumps(r), file=sys.stderr, flush=True)
    text = json.dumps(doc, indent=1)
    if args.out:
        pathlib.Path(args.out).write_text(text)
    else:
        print(text)


if __name__ == "__main__":
    main()
