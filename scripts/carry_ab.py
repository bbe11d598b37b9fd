#!/usr/bin/env python3
"""Same-box A/B of the carry (pgmg_ctx.hip "carry"): the headline call shape (a fresh problem,
a W-cycle warmup call, then a K-cycle call, timed) and one-cycle calls, with and without
PGMG_FLAG_NO_CARRY, interleaved over R rounds.  One JSON line per (round, variant, shape).

    python scripts/carry_ab.py [--n 16385] [--rounds 3] [--warmup 5] [--steps 20]
"""
import argparse
import json
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16385)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--variants", default="carry,no_carry",
                    help="comma list of: carry (default flags), no_carry, no_spin")
    a = ap.parse_args()
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    flags = {"carry": 0, "no_carry": pg.PGMG_FLAG_NO_CARRY, "no_spin": pg.PGMG_FLAG_NO_SPIN}
    variants = {k: flags[k] for k in a.variants.split(",")}
    solvers = {k: pg.Solver(a.n, flags=v) for k, v in variants.items()}
    for r in range(a.rounds):
        for name, s in solvers.items():
            # the headline shape: 5 repetitions, median
            ts = []
            for _ in range(5):
                s.set_problem()
                s.vcycle(a.warmup)
                s.sync()
                t0 = time.perf_counter()
                s.vcycle(a.steps)
                s.sync()
                ts.append(time.perf_counter() - t0)
            h = s.solution_hash(0)
            print(json.dumps({"round": r, "variant": name, "shape": f"{a.warmup}+{a.steps}",
                              "v_per_s": round(a.steps / statistics.median(ts), 3),
                              "ms_per_cycle": [round(t * 1e3 / a.steps, 4) for t in ts],
                              "hash": h, "carry": s.carry_info()}), flush=True)
            # one-cycle calls
            s.set_problem()
            for _ in range(a.warmup):
                s.vcycle(1)
            s.sync()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                s.vcycle(1)
            s.sync()
            dt = time.perf_counter() - t0
            print(json.dumps({"round": r, "variant": name, "shape": "single calls",
                              "v_per_s": round(a.steps / dt, 3), "hash": s.solution_hash(0),
                              "carry": s.carry_info()}), flush=True)
    for s in solvers.values():
        s.close()


if __name__ == "__main__":
    main()
