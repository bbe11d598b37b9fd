#!/usr/bin/env python3
"""A/B of rows in flight for the op-level residual and interior copy (r04; measurement build
PGMG_LIB=.../libpgmg_ab.so): ms of pgmg_residual and of pgmg_jacobi(v = 0) (one sweep + the
interior copy back) at N = 16385 on reference-layout arrays, variants interleaved over rounds.

    PGMG_LIB=... python scripts/op_ru_ab.py [--rounds 3]
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
ap.add_argument("--restrict-prolong", action="store_true",
                help="time restriction and prolongation instead (PGMG_OPRS_U)")
args = ap.parse_args()

import torch  # noqa: E402
import _pkgload  # noqa: E402

pg = _pkgload.load()
n = args.n
h = 1.0 / (n - 1)
x = torch.zeros((n, n), dtype=torch.float64, device="cuda:0")
f = torch.empty_like(x)
pg.ops.rhs(f, h)
r = torch.empty_like(x)
tmp = torch.empty_like(x)
fine = float(n - 2) ** 2
nc = (n - 1) // 2 + 1
coarse = float(nc - 2) ** 2
c = torch.zeros((nc, nc), dtype=torch.float64, device="cuda:0")
e = torch.zeros((nc, nc), dtype=torch.float64, device="cuda:0")
variants = [{}, {"PGMG_OPR_U": 8}, {"PGMG_OPR_U": 16, "PGMG_OPR_BLOCKS": 2048},
            {"PGMG_OPC_U": 16}, {"PGMG_OPC_U": 16, "PGMG_OPC_BLOCKS": 1024}]
if args.restrict_prolong:
    # (r04: PGMG_OPP_U = 4, a batched prolongation, measured slower and removed)
    variants = [{}, {"PGMG_OPRS_U": 4}, {"PGMG_OPRS_BLOCKS": 2048}]
keys = sorted({k for v in variants for k in v})


def timed(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


for rnd in range(args.rounds):
    for var in variants:
        for k in keys:
            os.environ.pop(k, None)
        for k, v in var.items():
            os.environ[k] = str(v)
        if args.restrict_prolong:
            ms_rs = timed(lambda: pg.ops.restrict(r, c))
            ms_p = timed(lambda: pg.ops.prolong(e, r, mode=pg.PGMG_PROLONG_SYMMETRIC, num_thread=32))
            print(json.dumps({"variant": var or "base", "round": rnd, "restrict_ms": round(ms_rs, 4),
                              "restrict_frac": round((8 * fine + 8 * coarse) / ms_rs / 1e9 / 8.0, 4),
                              "prolong_ms": round(ms_p, 4),
                              "prolong_frac": round((16 * fine + 8 * coarse) / ms_p / 1e9 / 8.0, 4)}),
                  flush=True)
            continue
        ms_r = timed(lambda: pg.ops.residual(r, x, f, h))
        ms_j = timed(lambda: pg.ops.jacobi(x, f, h, 0, eps=-1.0, tmp=tmp))
        print(json.dumps({"variant": var or "base", "round": rnd, "residual_ms": round(ms_r, 4),
                          "residual_frac": round(24 * fine / ms_r / 1e9 / 8.0, 4),
                          "jacobi_v0_ms": round(ms_j, 4)}), flush=True)
