#!/usr/bin/env python3
"""Where a V-cycle's time goes, kernel by kernel, INCLUDING the gaps between dependent
launches (measurement tool, not product code).

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 scripts/cycle_timeline.py --child [--n 16385]
    python3 scripts/cycle_timeline.py --parse OUT [--cycles 10]

The child runs set_problem + 3 warmup cycles + ONE call of `--cycles` V-cycles (the bench's
timed call).  The parser takes the kernels of that last call (after the last k_pre of the
finest level), groups them by kernel symbol and level (grid size), and prints per cycle:
kernel time, the idle gap before each kernel (previous kernel's end -> this start) and the
share of the cycle each takes.
"""
import argparse
import csv
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def child(args):
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    kw = {"flags": args.flags} if args.flags else {}
    if args.world > 1:   # one rank of a row-strip job alone (PGMG_FLAG_SOLO: null transport)
        kw.update(rank=args.rank, world=args.world, flags=kw.get("flags", 0) | pg.PGMG_FLAG_SOLO)
    with pg.Solver(args.n, **kw) as s:
        s.set_problem()
        run = {"W": s.wcycle, "F": s.fcycle, "G": s.wcycle}.get(args.kind, s.vcycle)
        # G: BASELINE configs[4]'s shape -- one F-cycle (the FMG start), then the timed W call
        (s.fcycle if args.kind == "G" else run)(3 if args.kind == "V" else 1)
        s.sync()
        if args.kind in ("F", "G") or args.whole:   # a marker kernel before the timed call
            torch.full((64,), 1.0, device=f"cuda:{torch.cuda.current_device()}")
            torch.cuda.synchronize()
        run(args.cycles)
        s.sync()


def parse(args):
    files = list(pathlib.Path(args.parse).rglob("*kernel_trace.csv"))
    rows = list(csv.DictReader(open(files[0])))
    ks = []
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pgmg::", "")
        gx, gy = int(r.get("Grid_Size_X", 0) or 0), int(r.get("Grid_Size_Y", 0) or 0)
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, gx, gy))
    ks.sort()
    marks = [i for i, k in enumerate(ks) if "FillFunctor" in k[2]]
    if (args.kind in ("F", "G") or args.whole) and marks:
        # F, G, --whole: the timed call is everything after the child's marker kernel (a
        # speculative V call may be split into segments, each starting with a level-0 k_pre)
        seg = ks[marks[-1] + 1:]
    else:
        # the timed call starts at the first finest-level k_pre after the warmup call
        starts = [i for i, k in enumerate(ks) if k[2].startswith("k_pre<double, false, true")]
        i0 = starts[-1]
        seg = ks[i0:]
        # cut at the last finest-level k_post
        ends = [i for i, k in enumerate(seg) if k[2].startswith("k_post<double, true")]
        seg = seg[:ends[-1] + 1] if ends else seg
    total = seg[-1][1] - seg[0][0]
    agg = {}
    prev_end = seg[0][0]
    for (t0, t1, name, gx, gy) in seg:
        key = f"{name} grid {gx}x{gy}"
        a = agg.setdefault(key, {"calls": 0, "busy_ns": 0, "gap_ns": 0})
        a["calls"] += 1
        a["busy_ns"] += t1 - t0
        a["gap_ns"] += max(0, t0 - prev_end)
        prev_end = max(prev_end, t1)
    busy = sum(a["busy_ns"] for a in agg.values())
    gap = sum(a["gap_ns"] for a in agg.values())
    c = args.cycles
    out = {"cycles": c, "us_per_cycle": total / c / 1e3, "busy_us_per_cycle": busy / c / 1e3,
           "gap_us_per_cycle": gap / c / 1e3, "kernels": []}
    for k, a in sorted(agg.items(), key=lambda kv: -(kv[1]["busy_ns"] + kv[1]["gap_ns"])):
        out["kernels"].append({"kernel": k, "calls_per_cycle": a["calls"] / c,
                               "busy_us_per_cycle": round(a["busy_ns"] / c / 1e3, 2),
                               "gap_us_per_cycle": round(a["gap_ns"] / c / 1e3, 2)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--parse")
    ap.add_argument("--n", type=int, default=16385)
    ap.add_argument("--cycles", type=int, default=10)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--kind", default="V", choices=["V", "W", "F", "G"])
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--whole", action="store_true",
                    help="V: the whole timed call (marker kernel before it), not the last segment")
    ap.add_argument("--rank", type=int, default=0)
    a = ap.parse_args()
    if a.child:
        child(a)
    else:
        parse(a)
