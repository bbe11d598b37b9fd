#!/usr/bin/env python3
"""A/B of the in-place op-level Jacobi (r05: k_op_sweep_ip / k_op_sweep2_ip + the deferred
tile-edge scatter) against the r04 ping-pong form with its interior copy-back, on the
measurement build (PGMG_LIB=.../libpgmg_ab.so, `make ab`): ms per pgmg_jacobi CALL at
N = 16385 on reference-layout arrays for v = 0 (one sweep), v = 1 (two sweeps, the
reference's ComputeJacobi in the V-cycle) and v = 20, variants interleaved over rounds, one
JSON line per measurement; frac = 24 B per interior point per sweep / call time / 8 TB/s.

    PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so \\
        python scripts/op_ip_ab.py [--n 16385] [--rounds 2]
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
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--quick", action="store_true", help="defaults and the ping-pong form only")
ap.add_argument("--only-inplace", action="store_true", help="the in-place default only")
ap.add_argument("--nth", action="store_true", help="the single in-place sweep's workgroup size")
args = ap.parse_args()

import torch  # noqa: E402
import _pkgload  # noqa: E402

pg = _pkgload.load()
n = args.n
h = 1.0 / (n - 1)
x = torch.zeros((n, n), dtype=torch.float64, device="cuda:0")
f = torch.empty_like(x)
pg.ops.rhs(f, h)
tmp = torch.empty_like(x)
byt = 24.0 * (n - 2) ** 2

KNOBS = ("PGMG_OP_INPLACE", "PGMG_OPIP_U", "PGMG_OPIP_BLOCKS", "PGMG_OP2IP_U", "PGMG_OP2IP_BLOCKS",
         "PGMG_OPIP_BAR", "PGMG_OP2IP_BAR", "PGMG_OPIP_NTH", "PGMG_OP2IP_NTH")
variants = [{"PGMG_OP_INPLACE": 0}, {"PGMG_OP_INPLACE": 1},
            {"PGMG_OP_INPLACE": 1, "PGMG_OPIP_BAR": 0, "PGMG_OP2IP_BAR": 0}]
if args.only_inplace:
    variants = [{"PGMG_OP_INPLACE": 1}]
elif args.nth:
    variants = [{"PGMG_OP_INPLACE": 1}, {"PGMG_OPIP_NTH": 256},
                {"PGMG_OP2IP_NTH": 512}, {"PGMG_OP2IP_NTH": 512, "PGMG_OP2IP_BLOCKS": 512},
                {"PGMG_OP2IP_NTH": 512, "PGMG_OP2IP_BLOCKS": 2048}]
elif not args.quick:
    for u, b in ((16, 2048), (8, 1024), (8, 2048)):
        variants.append({"PGMG_OP_INPLACE": 1, "PGMG_OPIP_BAR": 0, "PGMG_OPIP_U": u,
                         "PGMG_OPIP_BLOCKS": b})
    for u, b in ((4, 2048), (8, 2048)):
        variants.append({"PGMG_OP_INPLACE": 1, "PGMG_OP2IP_BAR": 0, "PGMG_OP2IP_U": u,
                         "PGMG_OP2IP_BLOCKS": b})

def timed(v):
    pg.ops.jacobi(x, f, h, v, eps=-1.0, tmp=tmp, count=os.environ.get("AB_COUNT") == "1")
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        pg.ops.jacobi(x, f, h, v, eps=-1.0, tmp=tmp, count=os.environ.get("AB_COUNT") == "1")
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


for rnd in range(args.rounds):
    for var in variants:
        for k in KNOBS:
            os.environ.pop(k, None)
        for k, v in var.items():
            os.environ[k] = str(v)
        row = dict(var, round=rnd)
        for v in (0, 1, 20):
            ms = timed(v)
            row[f"v{v}_ms"] = round(ms, 5)
            row[f"v{v}_frac"] = round(byt * (v + 1) / (ms * 1e-3) / 1e9 / 8000.0, 4)
        print(json.dumps(row), flush=True)
