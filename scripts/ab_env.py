#!/usr/bin/env python3
"""Interleaved A/B of measurement-build knobs (libpgmg_ab.so, -DPGMG_TUNING): each variant's
environment in its own child process, rounds interleaved, V-cycles/s (and optionally W) per
grid, each run hash-checked against the reference's fixture.  Measurement tool.

    PGMG_LIB=.../libpgmg_ab.so python3 scripts/ab_env.py --rounds 3 \
        "base:" "nolds:PGMG_LDS_MIN_N=1000000"
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
    out = {}
    for spec in a.grids.split(","):
        kind, n = spec[0], int(spec[1:])
        steps = a.steps if kind in ("V", "F") else max(1, a.steps // 10)
        ts = []
        flags = int(os.environ.get("AB_FLAGS", "0"))   # pgmg_config.flags of the variant
        kw = {"flags": flags} if flags else {}
        if os.environ.get("AB_TAIL_N"):                # pgmg_config.tail_n of the variant
            kw["tail_n"] = int(os.environ["AB_TAIL_N"])
        with pg.Solver(n, **kw) as s:
            run = {"V": s.vcycle, "W": s.wcycle, "F": s.fcycle}[kind]
            for _ in range(3):
                s.set_problem()
                run({"V": 3, "W": 1, "F": 2}[kind])
                s.sync()
                t0 = time.perf_counter()
                run(steps)
                s.sync()
                ts.append(time.perf_counter() - t0)
            h = s.solution_hash(0)
        out[spec] = {"per_s": round(steps / statistics.median(ts), 3), "hash": h}
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--grids", default="V16385,V4097")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    if a.child:
        return child(a)
    variants = []
    for v in a.variants or ["base:"]:
        name, envs = v.split(":", 1)
        env = dict(kv.split("=", 1) for kv in envs.split(";") if kv)
        variants.append((name, env))
    for r in range(a.rounds):
        for name, env in variants:
            e = dict(os.environ)
            e.update(env)
            p = subprocess.run([sys.executable, __file__, "--child", "--grids", a.grids,
                                "--steps", str(a.steps)], env=e, capture_output=True, text=True,
                               timeout=600)
            line = next((l for l in p.stdout.splitlines() if l.startswith("{")), None)
            if line is None:
                print(json.dumps({"round": r, "variant": name, "failed": p.stderr[-1500:]}), flush=True)
                sys.exit(1)
            print(json.dumps({"round": r, "variant": name, **json.loads(line)}), flush=True)


if __name__ == "__main__":
    main()
