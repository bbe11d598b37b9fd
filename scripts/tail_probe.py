#!/usr/bin/env python3
"""Time the LDS tail alone: gamma-cycles on a grid that is entirely tail (N <= tail_n),
one k_tail launch per cycle; env PGMG_TAIL_WAVE_N selects the wave-mode threshold."""
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
    for N in (17, 33, 65):
        for kind in ("V", "W"):
            with pg.Solver(N, tail_n=65) as s:
                s.set_problem()
                run = s.vcycle if kind == "V" else s.wcycle
                run(5)
                s.sync()
                reps = 400
                t = time.perf_counter()
                run(reps)
                s.sync()
                dt = (time.perf_counter() - t) / reps
                out.append({"N": N, "kind": kind, "us_per_cycle": round(dt * 1e6, 2),
                            "device_us": round(s.last_elapsed_ms() * 1e3 / reps, 2),
                            "sweeps": s.stats()[0]})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
