#!/usr/bin/env python3
"""Per-level measurement of the coarse bulk passes (k_pre / k_post of levels 8193 ... 129
under a 16385 V-cycle): duration, HBM bytes and instruction mix per launch, from rocprofv3.

    python scripts/level_pmc.py run  [--n 16385] [--out DIR]   # profiles, then summarises
    python scripts/level_pmc.py child [--n 16385]               # the profiled program

`run` makes one rocprofv3 pass per group (kernel trace; FETCH_SIZE; WRITE_SIZE; eight SQ
counters), each as its own `timeout -s KILL` child, and prints one JSON line per (kernel,
level): launches, average duration, HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB; the
gfx950 corrections bench.py uses), GB/s, the algorithmic bytes (levels below the finest are
entered with x0 = 0: k_pre reads f and writes rc, 8 + 2 B per point; k_post reads f and the
coarse correction and writes x2, 8 + 2 + 8 B per point; the finest k_postpre_lds 20 B per
point), VALU instructions per wave and the share of wave cycles parked (SQ_WAIT_ANY) or
issuing (SQ_ACTIVE_INST_ANY).
Levels are told apart by their launch grid (fused_geometry in pgmg_fused.hip, restated)."""
import argparse
import collections
import csv
import json
import math
import os
import pathlib
import shutil
import subprocess
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parent.parent
# SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (issue stalls) +
# SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES (MI355X_MICROARCH.md's PMC table)
SQ = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_WAVE_CYCLES",
      "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"]


def fused_grid(N):
    """Work-items of a k_pre / k_post launch on a level of N points (one GPU)."""
    rows = (N - 1) // 2
    pts = 2 * rows * N
    target = min(3072, max(512, pts // 21845)) if pts > (1 << 23) else max(256, pts // 8192)
    waves = (N - 2 + 119) // 120
    wpb = min(waves, 4)
    gx = (waves + wpb - 1) // wpb
    gymax = max(1, target // gx)
    r = max(2, (rows + gymax - 1) // gymax)
    r = max(1, min(r, rows))
    gy = (rows + r - 1) // r
    return gx * 64 * wpb * gy


def short(name):
    return name.split("(")[0].replace("void ", "").replace("pgmg::", "")


def child(a):
    sys.path.insert(0, str(ROOT))
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    with pg.Solver(a.n) as s:
        s.set_problem()
        s.vcycle(2)
        s.sync()
        s.vcycle(4)
        s.sync()


def rows_of(d, pattern):
    f = list(pathlib.Path(d).rglob(pattern))
    return list(csv.DictReader(open(f[0]))) if f else []


def grid_total(row):
    if "Grid_Size" in row:
        return int(row["Grid_Size"])
    return int(row.get("Grid_Size_X", 1)) * int(row.get("Grid_Size_Y", 1)) * int(row.get("Grid_Size_Z", 1))


def run(a):
    prof = shutil.which("rocprofv3")
    out = pathlib.Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    base = ["timeout", "-s", "KILL", "120", prof, "--output-format", "csv"]
    prog = ["--", sys.executable, str(pathlib.Path(__file__).resolve()), "child", "--n", str(a.n)]
    passes = {"trace": ["--kernel-trace"], "fetch": ["--pmc", "FETCH_SIZE"],
              "write": ["--pmc", "WRITE_SIZE"], "sq": ["--pmc"] + SQ}
    dirs = {}
    for k, opt in passes.items():
        d = tempfile.mkdtemp(prefix=f"lvl_{k}_")
        r = subprocess.run(base + opt + ["-d", d, "-o", "run"] + prog, capture_output=True, text=True,
                           timeout=150)
        (out / f"{k}.log").write_text(r.stdout[-4000:] + r.stderr[-4000:])
        if r.returncode != 0:
            print(json.dumps({"pass": k, "rc": r.returncode}), flush=True)
            sys.exit(1)
        dirs[k] = d
    levels = {}
    N = a.n // 2 + 1
    while N >= 129:
        levels[fused_grid(N)] = N
        N = N // 2 + 1
    dur = collections.defaultdict(list)
    for row in rows_of(dirs["trace"], "*kernel_trace.csv"):
        key = (short(row["Kernel_Name"]), grid_total(row))
        dur[key].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3)
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for k in ("fetch", "write", "sq"):
        for row in rows_of(dirs[k], "*counter_collection.csv"):
            key = (short(row["Kernel_Name"]), grid_total(row))
            ctr[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = []
    for key, ds in sorted(dur.items()):
        name, g = key
        fine = name.startswith("k_postpre_lds<")
        if not fine and (not (name.startswith("k_pre<") or name.startswith("k_post<")) or g not in levels):
            continue
        Nl = a.n if fine else levels[g]
        c = {n: sum(v) / len(v) for n, v in ctr[key].items()}
        us = sum(ds) / len(ds)
        hbm = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024.0
        alg = (20.0 if fine else 10.0 if name.startswith("k_pre<") else 18.0) * Nl * Nl
        waves = c.get("SQ_WAVES", 0)
        d = {"kernel": name, "N": Nl, "launches": len(ds), "avg_us": round(us, 2),
             "hbm_bytes": hbm, "hbm_GBps": round(hbm / us * 1e-3, 1), "alg_bytes": alg,
             "alg_GBps": round(alg / us * 1e-3, 1), "traffic_ratio": round(hbm / alg, 3) if alg else None,
             "valu_per_wave": round(c.get("SQ_INSTS_VALU", 0) / waves, 1) if waves else None,
             "valu_per_point": round(c.get("SQ_INSTS_VALU", 0) * 64 / (Nl * Nl), 2),
             "lds_per_wave": round(c.get("SQ_INSTS_LDS", 0) / waves, 1) if waves else None,
             "wait_frac": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3) if c.get("SQ_WAVE_CYCLES") else None,
             "active_frac": round(c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3) if c.get("SQ_WAVE_CYCLES") else None,
             "waves": waves, "counters": c}
        res.append(d)
        print(json.dumps(d), flush=True)
    (out / "levels.json").write_text(json.dumps(res, indent=1))
    for d in dirs.values():
        shutil.rmtree(d, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "child"])
    ap.add_argument("--n", type=int, default=16385)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "level_pmc"))
    a = ap.parse_args()
    (child if a.mode == "child" else run)(a)


if __name__ == "__main__":
    main()
