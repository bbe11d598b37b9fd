#!/usr/bin/env python3
"""A/B of the op-level Jacobi sweep's launch geometry (PGMG_OP_OV, PGMG_OP_BLOCKS, PGMG_OP_U, PGMG_OP_NT)
on the measurement build (PGMG_LIB=.../libpgmg_ab.so, `make ab`): ms per sweep of
pgmg_jacobi(v = 100, no early exit) at N = 16385 on reference-layout arrays, variants
interleaved over rounds, one JSON line per measurement.

    PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so \\
        python scripts/op_ab.py [--n 16385] [--rounds 2]
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
ap.add_argument("--v", type=int, default=20)
ap.add_argument("--rows", action="store_true",
                help="single sweeps only (PGMG_OP_FUSE2=0): rows of loads in flight U = 4 / 8 / 16 "
                     "at one round of resident workgroups each")
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
variants = []
# one round of resident workgroups: k_op_sweep U=8 4 waves/SIMD (1024 WGs), U=4 7 (1792);
# k_op_sweep_ov U=8 5 (1280), U=4 8 (2048)
for ov, u, blocks in ((0, 8, 1024), (0, 8, 2048), (0, 4, 1792), (1, 8, 1280), (1, 8, 2560),
                      (1, 4, 2048), (1, 4, 4096), (1, 8, 8192)):
    for nt in (0, 1):
        variants.append({"PGMG_OP_OV": ov, "PGMG_OP_BLOCKS": blocks, "PGMG_OP_U": u,
                         "PGMG_OP_NT": nt})
if args.rows:
    # U = 8: 120 VGPRs, 4 waves per SIMD (1024 resident); U = 16: 214, 2 (512); U = 4: 70, 7 (1792)
    variants = [{"PGMG_OP_FUSE2": 0, "PGMG_OP_OV": 0, "PGMG_OP_BLOCKS": b, "PGMG_OP_U": u,
                 "PGMG_OP_NT": 1} for u, b in ((8, 1024), (16, 512), (16, 1024), (4, 1792))]
for rnd in range(args.rounds):
    for var in variants:
        for k, v in var.items():
            os.environ[k] = str(v)
        pg.ops.jacobi(x, f, h, 1, eps=-1.0, tmp=tmp)
        ts = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            pg.ops.jacobi(x, f, h, args.v, eps=-1.0, tmp=tmp)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) / (args.v + 1))
        ms = statistics.median(ts)
        print(json.dumps(dict(var, round=rnd, ms_per_sweep=round(ms, 5),
                              tbps=round(byt / ms / 1e9, 3), frac=round(byt / ms / 1e9 / 8.0, 4))),
              flush=True)
