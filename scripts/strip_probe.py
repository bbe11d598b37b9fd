#!/usr/bin/env python3
"""Per-rank compute time of the row-strip decomposition, measured on ONE GPU.

    python scripts/strip_probe.py [--n 16385] [--worlds 1,2,4,8] [--steps 20]

For each world size W, one rank (the first and a middle one) runs alone with
PGMG_FLAG_SOLO (null transport: no messages, local allreduces), so the time per
V-cycle is that rank's compute share of a W-GPU run without the communication
(RCCL latency over xGMI is not measured here).  The values computed are meaningless.
Prints one JSON line per (W, rank).
"""
import argparse
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16385)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gather-n", type=int, default=0)
    args = ap.parse_args()
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    for W in [int(w) for w in args.worlds.split(",")]:
        for r in sorted({0, W // 2}) if W > 1 else [0]:
            kw = dict(device=0)
            if W > 1:
                kw.update(rank=r, world=W, flags=pg.PGMG_FLAG_SOLO)
                if args.gather_n:
                    kw["gather_n"] = args.gather_n
            s = pg.Solver(args.n, **kw)
            s.set_problem()
            s.vcycle(args.warmup)
            s.sync()
            t0 = time.perf_counter()
            s.vcycle(args.steps)
            s.sync()
            dt = (time.perf_counter() - t0) / args.steps
            lo, hi, ld = pg.plan_strips(args.n, W, r, 65, args.gather_n or 1025)
            print(json.dumps({"N": args.n, "world": W, "rank": r, "rows": [lo, hi],
                              "dist_levels": ld, "ms_per_cycle": round(dt * 1e3, 4),
                              "dist_info": list(s.dist_info())}), flush=True)
            s.close()


if __name__ == "__main__":
    main()
