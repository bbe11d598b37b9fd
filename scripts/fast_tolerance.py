#!/usr/bin/env python3
"""FAST mode (PGMG_FLAG_FAST) against the EXACT default: relative L2 and max-abs difference of
phi after `cycles` V-cycles from phi0 = 0, per N (the data behind tests/test_gpu_fast.py's
tolerance).  python scripts/fast_tolerance.py [cycles]"""
import json
import pathlib
import sys

import numpy as np

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent.parent))


def main():
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    cycles = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    for N in (2049, 4097, 8193, 16385):
        sols = []
        for flags in (0, pg.PGMG_FLAG_FAST):
            with pg.Solver(N, flags=flags) as s:
                s.set_problem()
                s.vcycle(cycles)
                sols.append((s.solution(), s.stats()[0]))
        (ref, sr), (got, sg) = sols
        d = got - ref
        print(json.dumps({"N": N, "cycles": cycles,
                          "rel_l2": float(np.linalg.norm(d) / np.linalg.norm(ref)),
                          "max_abs": float(np.max(np.abs(d))), "sweeps_equal": sr == sg,
                          "eps_n2": float(np.finfo(np.float64).eps * (N - 1) ** 2)}), flush=True)


if __name__ == "__main__":
    main()
