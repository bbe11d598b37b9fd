#!/usr/bin/env python3
"""Where a W-cycle's time goes: run under `rocprofv3 --kernel-trace --stats`, then
`--analyse DIR`: per kernel, launches, total and mean time of the timed call (N = 4097, a fresh
problem, 2 W-cycles, then 5 timed)."""
import argparse
import collections
import csv
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def child(n):
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    with pg.Solver(n) as s:
        s.set_problem()
        s.wcycle(2)
        s.sync()
        t0 = time.perf_counter()
        s.wcycle(5)
        s.sync()
        print("ms per W-cycle", (time.perf_counter() - t0) * 200.0, flush=True)


def analyse(d):
    rows = []
    for f in pathlib.Path(d).rglob("*kernel_trace.csv"):
        rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))]
    rows.sort()
    tot = collections.defaultdict(lambda: [0, 0])
    for s0, s1, n in rows:
        k = n.split("(")[0].replace("void ", "")[:70]
        tot[k][0] += 1
        tot[k][1] += s1 - s0
    span = (rows[-1][1] - rows[0][0]) / 1e6
    busy = sum(v[1] for v in tot.values()) / 1e6
    print(f"{len(rows)} launches, span {span:.1f} ms, busy {busy:.1f} ms")
    for k, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:15]:
        print(f"{t / 1e6:9.2f} ms {c:7d} x {t / c / 1e3:8.2f} us  {k}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyse", default="")
    ap.add_argument("--n", type=int, default=4097)
    a = ap.parse_args()
    if a.analyse:
        analyse(a.analyse)
    else:
        child(a.n)
