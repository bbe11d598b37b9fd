#!/usr/bin/env python3
"""Where a one-cycle call's time goes (the reference harness's loop shape, with the carry):
run under `rocprofv3 --kernel-trace --memory-copy-trace --output-format csv`, then
`--analyse DIR`: per call, the GPU busy time (kernels + copies), the idle gaps inside the call
and between calls, and the carry pass."""
import argparse
import csv
import pathlib
import re
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def child():
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    with pg.Solver(16385) as s:
        s.set_problem()
        for _ in range(5):
            s.vcycle(1)
        s.sync()
        t0 = time.perf_counter()
        for _ in range(10):
            s.vcycle(1)
        s.sync()
        print("wall ms per call", (time.perf_counter() - t0) * 100.0, flush=True)


def analyse(d):
    ev = []
    for pat in ("*kernel_trace.csv", "*memory_copy_trace.csv"):
        for f in pathlib.Path(d).rglob(pat):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name") or r.get("Direction") or "copy"
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    ev.sort()
    # the calls: split at the carry passes (one per call, its last finest pass: a k_postpre_lds
    # whose OPT has bit 128)
    def is_carry(name):
        m = re.search(r"k_postpre_lds<[^>]*, (\d+)>", name)
        return m is not None and int(m.group(1)) & 128
    carry = [i for i, e in enumerate(ev) if is_carry(e[2])]
    print(len(ev), "events,", len(carry), "carry passes")
    for a, b in zip(carry[-11:-1], carry[-10:]):
        seg = ev[a + 1:b + 1]
        t0, t1 = ev[a][1], ev[b][1]
        busy = 0
        last = t0
        gaps = []
        for s0, s1, n in seg:
            if s0 > last:
                gaps.append((s0 - last, n))
            busy += max(0, s1 - max(s0, last))
            last = max(last, s1)
        gaps.sort(reverse=True)
        print(f"call {(t1 - t0) / 1e3:8.1f} us  busy {busy / 1e3:8.1f}  idle {(t1 - t0 - busy) / 1e3:7.1f}  "
              f"carry pass {(ev[b][1] - ev[b][0]) / 1e3:7.1f}  biggest gaps (us, before): " +
              ", ".join(f"{g / 1e3:.1f} {n[:28]}" for g, n in gaps[:4]))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyse", default="")
    a = ap.parse_args()
    if a.analyse:
        analyse(a.analyse)
    else:
        child()
