#!/usr/bin/env python3
"""Per-sweep cost of the LDS tail: the coarsest solve alone (N = n_coarse) with
coarse_iter = k and no early exit; the slope over k is the cost of one sweep + norm."""
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    out = []
    for N in (5, 9, 17, 33, 65):
        pts = []
        for k in (10, 210):
            with pg.Solver(N, n_coarse=N, coarse_iter=k, eps=-1.0, tail_n=65) as s:
                s.set_problem()
                s.vcycle(3)
                s.sync()
                reps = 200
                t = time.perf_counter()
                s.vcycle(reps)
                s.sync()
                pts.append((time.perf_counter() - t) / reps * 1e6)
        out.append({"N": N, "us_k10": round(pts[0], 2), "us_k210": round(pts[1], 2),
                    "us_per_sweep": round((pts[1] - pts[0]) / 200, 3)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
