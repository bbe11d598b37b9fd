#!/usr/bin/env python3
"""Kernel-trace child for the carry probe: per context (carry on, PGMG_FLAG_NO_CARRY), three
repetitions of the headline shape (fresh problem, 5-cycle call, 20-cycle call), with a marker
kernel-free sync between.  Run under `rocprofv3 --kernel-trace --output-format csv`; the
analysis (scripts/carry_trace.py --analyse DIR) lists every k_postpre launch's duration in
order per context."""
import argparse
import csv
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def child():
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    for fl in (0, pg.PGMG_FLAG_NO_CARRY, 0):
        with pg.Solver(16385, flags=fl) as s:
            for _ in range(3):
                s.set_problem()
                s.vcycle(5)
                s.sync()
                s.vcycle(20)
                s.sync()


def analyse(d):
    f = list(pathlib.Path(d).rglob("*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    runs, cur = [], []
    last_end = None
    for r in rows:
        name = r["Kernel_Name"]
        if "k_postpre_lds" not in name:
            continue
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        cur.append(("C" if "130>" in name else "P", (t1 - t0) / 1e3, (t0 - last_end) / 1e3 if last_end else 0))
        last_end = t1
    print(len(cur), "k_postpre launches")
    for i in range(0, len(cur), 24):
        seg = cur[i:i + 24]
        print(" ".join(f"{k}{d:.0f}" for k, d, _ in seg))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyse", default="")
    a = ap.parse_args()
    if a.analyse:
        analyse(a.analyse)
    else:
        child()
