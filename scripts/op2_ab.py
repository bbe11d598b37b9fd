#!/usr/bin/env python3
"""A/B of the paired-sweep pass (k_op_sweep2: two Jacobi sweeps per pass for pgmg_jacobi
without early-exit checks) against single sweeps, at N = 16385 on reference-layout arrays:
ms per sweep of pgmg_jacobi(v = 19: 20 sweeps, eps < 0), launch geometry variants on the
measurement build (PGMG_LIB=.../libpgmg_ab.so), interleaved rounds, one JSON line each."""
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
v = 19
variants = [{"PGMG_OP_FUSE2": 0}]
for u, blocks in ((8, 1024), (8, 2048), (4, 1536), (4, 3072), (4, 6144)):
    for nt in (0, 1):
        variants.append({"PGMG_OP_FUSE2": 1, "PGMG_OP2_U": u, "PGMG_OP2_BLOCKS": blocks, "PGMG_OP_NT": nt})
keys = sorted({k for var in variants for k in var})
for rnd in range(args.rounds):
    for var in variants:
        for k in keys:
            os.environ.pop(k, None)
        for k, val in var.items():
            os.environ[k] = str(val)
        pg.ops.jacobi(x, f, h, 1, eps=-1.0, tmp=tmp)
        ts = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            pg.ops.jacobi(x, f, h, v, eps=-1.0, tmp=tmp)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) / (v + 1))
        ms = statistics.median(ts)
        print(json.dumps(dict(var, round=rnd, ms_per_sweep=round(ms, 5),
                              frac_per_sweep=round(byt / ms / 1e9 / 8.0, 4))), flush=True)
