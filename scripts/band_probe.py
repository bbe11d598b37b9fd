#!/usr/bin/env python3
"""Level-1 band height A/B (measurement build, -DPGMG_TUNING): the headline shape -- a fresh
problem, a 5-cycle call, a timed 20-cycle call, 5 repetitions -- in a child process per value of
PGMG_FUSED_BLOCKS_BIG (fused_geometry's workgroup target for the k_pre / k_post levels of
N >= 8193: taller bands re-read fewer halo rows, fewer workgroups fill the chip less), values
interleaved over R rounds; per child the median ms per cycle and the per-pass event times of
the instrumented repetitions are not needed: one JSON line per (round, value).

    PGMG_LIB=.../libpgmg_ab.so python3 scripts/band_probe.py --values 0,1536,2048
"""
import argparse
import json
import os
import pathlib
import statistics
import subprocess
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def child(a):
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    ts = []
    run = {"V": lambda s, k: s.vcycle(k), "F": lambda s, k: s.fcycle(k)}[a.cycle]
    warm = 5 if a.cycle == "V" else 2
    with pg.Solver(a.n) as s:
        for _ in range(5):
            s.set_problem()
            run(s, warm)
            s.sync()
            t0 = time.perf_counter()
            run(s, 20)
            s.sync()
            ts.append((time.perf_counter() - t0) / 20 * 1e3)
        h = s.solution_hash(0)
    print(json.dumps({"ms_per_cycle": [round(t, 4) for t in ts], "median": round(statistics.median(ts), 4),
                      "hash": h}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16385)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--values", default="0,1536,2048")
    ap.add_argument("--knob", default="PGMG_FUSED_BLOCKS_BIG",
                    help="the measurement build's knob to set (PGMG_PP_BLOCKS: k_postpre's "
                         "workgroup target)")
    ap.add_argument("--cycle", default="V", choices=["V", "F"])
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a)
    for r in range(a.rounds):
        for v in a.values.split(","):
            env = dict(os.environ)
            if v == "off":     # the knob set to 0 (a switch whose default is on)
                env[a.knob] = "0"
            elif v != "0":     # 0: the knob unset (the library's default)
                env[a.knob] = v
            p = subprocess.run([sys.executable, __file__, "--child", "--n", str(a.n), "--cycle", a.cycle], env=env,
                               capture_output=True, text=True, timeout=300)
            line = p.stdout.strip().splitlines()[-1] if p.stdout.strip() else "{}"
            d = json.loads(line)
            d.update({"round": r, "knob": a.knob, "value": v, "rc": p.returncode})
            if p.returncode:
                d["stderr"] = p.stderr[-800:]
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
