#!/usr/bin/env python3
"""Where the LDS tail's time goes: PGMG_TAIL_PROF=1 cycle counters per stage kind for one
W-cycle (and one V-cycle) at N (default 4097).  python scripts/tail_prof.py [N]"""
import ctypes as C
import json
import os
import pathlib
import sys

os.environ["PGMG_TAIL_PROF"] = "1"
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

NAMES = ["wave hand-offs", "block smooth", "block res+restrict", "block prolong", "kernel",
         "launches", "wave smooth", "wave res+restrict+prolong"]


def main():
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    lib = pg.load()
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4097
    buf = (C.c_ulonglong * 16)()
    for kind in ("W", "V"):
        with pg.Solver(N) as s:
            s.set_problem()
            (s.wcycle if kind == "W" else s.vcycle)(1)
            s.sync()
            lib.pgmg_tail_prof(buf, 1)
            (s.wcycle if kind == "W" else s.vcycle)(1)
            s.sync()
            assert lib.pgmg_tail_prof(buf, 1) == 0
            w9 = list(buf)[8:16]
            v = list(buf)[:8]
            k = v[4] or 1
            if w9[7]:
                print(json.dumps({"w9_visits": w9[7], "w9_cycles_per_visit": {
                    n: round(w9[i] / w9[7], 1) for i, n in enumerate(
                        ["smooth (both)", "res+restrict", "coarsest solves", "prolong"])},
                    "w17_cycles_per_visit": {n: round(w9[4 + i] / (w9[7] / 3), 1) for i, n in enumerate(
                        ["smooth (both)", "res+restrict", "prolong"])}}))
            print(json.dumps({"N": N, "cycle": kind, "launches": v[5],
                              "cycles_per_launch": v[4] / max(v[5], 1),
                              "share": {NAMES[i]: round(v[i] / k, 4) for i in (0, 1, 2, 3, 6, 7)}}))


if __name__ == "__main__":
    main()
