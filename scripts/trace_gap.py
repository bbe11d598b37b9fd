#!/usr/bin/env python3
"""Does rocprofv3 --kernel-trace itself slow the headline call down? (r04)  Runs bench.py's
timed-call shape (pre-warm calls, a fresh problem, warmup cycles, `steps` cycles in one call)
and prints the call's ms per V-cycle from stream events.  Run it plain and under
`rocprofv3 --kernel-trace -- python3 scripts/trace_gap.py` on the same box: if the traced run's
own event time is slower by the same ~4 % as the trace's kernel durations, the gap between
bench.py's event-timed and rocprof-timed `k_postpre_lds` is the profiler's.

    python scripts/trace_gap.py [--n 16385] [--steps 20] [--warmup 2] [--prewarm 4] [--reps 3]

--ab: instead, contexts with and without PGMG_FLAG_TIME_FINE (events between the finest
passes) interleaved over rounds, a fresh context each time, as bench.py's legs do.
--ctx K: K fresh plain contexts one after another, `reps` calls each: the spread between
contexts against the spread within one (does the allocation a context gets set its speed?).
"""
import argparse
import json
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=16385)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=2)
ap.add_argument("--prewarm", type=int, default=4)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--tag", default="plain")
ap.add_argument("--ab", type=int, default=0, help="rounds of the TIME_FINE A/B")
ap.add_argument("--ctx", type=int, default=0, help="fresh contexts for the per-context spread")
args = ap.parse_args()

import torch  # noqa: E402
import _pkgload  # noqa: E402

pg = _pkgload.load()


def call_ms(s):
    s.set_problem()
    s.vcycle(max(args.warmup, 0))
    s.sync()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    s.vcycle(args.steps)
    s.sync()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / args.steps


if args.ctx:
    per = []
    with pg.Solver(args.n, dtype="f64") as s:
        for _ in range(args.prewarm):
            call_ms(s)
    for k in range(args.ctx):
        with pg.Solver(args.n, dtype="f64") as s:
            per.append([round(call_ms(s), 4) for _ in range(args.reps)])
        print(json.dumps({"ctx": k, "ms_per_cycle": per[-1]}), flush=True)
    med = [statistics.median(v) for v in per]
    print(json.dumps({"n": args.n, "ctx_medians": med, "between_pct": round(
        100 * (max(med) - min(med)) / statistics.median(med), 2), "within_pct_max": round(
        max(100 * (max(v) - min(v)) / statistics.median(v) for v in per), 2)}), flush=True)
    sys.exit(0)
if args.ab:
    res = {"plain": [], "time_fine": []}
    for rnd in range(args.ab):
        for name, fl in (("plain", 0), ("time_fine", pg.PGMG_FLAG_TIME_FINE)):
            with pg.Solver(args.n, dtype="f64", flags=fl) as s:
                if rnd == 0:
                    for _ in range(args.prewarm):
                        call_ms(s)
                res[name] += [round(call_ms(s), 4) for _ in range(args.reps)]
    print(json.dumps({"n": args.n, **res, **{k + "_median": round(statistics.median(v), 4)
                                             for k, v in res.items()}}), flush=True)
    sys.exit(0)
ms = []
with pg.Solver(args.n, dtype="f64") as s:
    for _ in range(args.prewarm):
        s.set_problem()
        s.vcycle(args.steps)
        s.sync()
    for _ in range(args.reps):
        s.set_problem()
        s.vcycle(max(args.warmup, 0))
        s.sync()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        s.vcycle(args.steps)
        s.sync()
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b) / args.steps)
print(json.dumps({"tag": args.tag, "n": args.n, "ms_per_cycle": [round(x, 4) for x in ms],
                  "median": round(statistics.median(ms), 4)}), flush=True)
