#!/usr/bin/env python3
"""Is the finest pass's speed a property of the context's memory (which grids it got) rather
than of the carry?  In one process, contexts are created one after another in the order given
(c: carry on, n: PGMG_FLAG_NO_CARRY), each running R repetitions of the headline shape with
events around every finest pass; optionally a dummy device buffer of G GiB is allocated and
freed first.  One JSON line per repetition: the mean k_postpre launch (ms).

    python scripts/order_probe.py --order ncnc [--dummy-gib 0]
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
    ap.add_argument("--order", default="ncnc")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dummy-gib", type=float, default=0.0)
    ap.add_argument("--keep", action="store_true", help="keep every context alive until the end")
    a = ap.parse_args()
    import ctypes as C
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    lib = pg.load()
    if a.dummy_gib > 0:
        p = C.c_void_p()
        pg.check(lib.pgmg_device_alloc(C.byref(p), int(a.dummy_gib * (1 << 30))), "alloc")
        pg.check(lib.pgmg_device_free(p), "free")
    keep = []
    for i, ch in enumerate(a.order):
        fl = pg.PGMG_FLAG_TIME_FINE | (pg.PGMG_FLAG_NO_CARRY if ch == "n" else 0)
        s = pg.Solver(16385, flags=fl)
        for r in range(a.reps):
            s.set_problem()
            s.vcycle(5)
            s.sync()
            for w in range(5):
                s.fine_pass_time(w)
            t0 = time.perf_counter()
            s.vcycle(20)
            s.sync()
            dt = time.perf_counter() - t0
            print(json.dumps({"ctx": i, "kind": ch, "rep": r, "ms_per_cycle": round(dt * 50, 4),
                              "k_postpre_ms": round(s.fine_pass_time(3)[1], 4),
                              "dummy_gib": a.dummy_gib}), flush=True)
        if a.keep:
            keep.append(s)
        else:
            s.close()
    for s in keep:
        s.close()


if __name__ == "__main__":
    main()
