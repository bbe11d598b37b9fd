#!/usr/bin/env python3
"""Interleaved A/B of the out-of-place op kernels' launch forms (measurement build,
PGMG_LIB=...libpgmg_ab.so): ms per pgmg_residual / pgmg_restrict / pgmg_prolong call at
N = 16385 on reference-layout arrays, events around each call (median of 5); one JSON line per
(variant, round).  frac: SURVEY §8(d)'s algorithmic bytes / call time / 8 TB/s.

    PGMG_LIB=... python scripts/op_misc_ab.py [--rounds 3] NAME[:VAR=v,...] ...
"""
import argparse
import json
import os
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=16385)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("variants", nargs="+")
args = ap.parse_args()
import torch  # noqa: E402
import _pkgload  # noqa: E402

pg = _pkgload.load()
n = args.n
h = 1.0 / (n - 1)
nc = (n - 1) // 2 + 1
x = torch.zeros((n, n), dtype=torch.float64, device="cuda:0")
f = torch.empty_like(x)
pg.ops.rhs(f, h)
r = torch.zeros_like(x)
c = torch.zeros((nc, nc), dtype=torch.float64, device="cuda:0")
e = torch.ones((nc, nc), dtype=torch.float64, device="cuda:0")
fine, coarse = float((n - 2) ** 2), float((nc - 2) ** 2)
OPS = {"residual": (lambda: pg.ops.residual(r, x, f, h), 24 * fine),
       "restrict": (lambda: pg.ops.restrict(r, c), 8 * fine + 8 * coarse),
       "prolong": (lambda: pg.ops.prolong(e, r, mode=pg.PGMG_PROLONG_REFERENCE), 16 * fine + 8 * coarse)}
vs = []
for v in args.variants:
    name, _, envs = v.partition(":")
    vs.append((name, dict(q.split("=", 1) for q in envs.split(",") if q)))
knobs = {k for _, env in vs for k in env}
for rnd in range(args.rounds):
    for name, env in vs:
        for k in knobs:
            os.environ.pop(k, None)
        os.environ.update(env)
        row = {"variant": name, "round": rnd}
        for op, (call, nbytes) in OPS.items():
            call()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                call()
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b))
            ms = statistics.median(ts)
            row[op + "_ms"] = round(ms, 5)
            row[op + "_frac"] = round(nbytes / (ms * 1e-3) / 8e12, 4)
        print(json.dumps(row), flush=True)
