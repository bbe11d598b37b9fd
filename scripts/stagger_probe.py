#!/usr/bin/env python3
"""Does the placement of the level-0 grids change the finest pass's speed?  Measurement tool
(libpgmg_probe.so: scripts/build_variant.sh probe, -DPGMG_TUNING).

For each PGMG_GRID_STAGGER value (bytes; level-0 grid k's origin shifted by k times it) a
child process runs the headline shape -- a fresh problem, a 5-cycle call, a timed 20-cycle call
-- R times with and without the carry, with events around every finest pass
(PGMG_FLAG_TIME_FINE), and prints per repetition the ms per cycle, the mean k_postpre launch
and the level-0 grid roles of each segment (PGMG_ROLE_TRACE).

    PGMG_LIB=.../libpgmg_probe.so python3 scripts/stagger_probe.py --staggers 0,4096,65536
"""
import argparse
import json
import os
import pathlib
import subprocess
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def child(a):
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    for carry in (True, False):
        fl = pg.PGMG_FLAG_TIME_FINE | (0 if carry else pg.PGMG_FLAG_NO_CARRY)
        with pg.Solver(a.n, flags=fl) as s:
            for r in range(a.reps):
                s.set_problem()
                s.vcycle(5)
                s.sync()
                for w in range(5):
                    s.fine_pass_time(w)
                print(f"REP {r} carry {int(carry)}", file=sys.stderr, flush=True)
                t0 = time.perf_counter()
                s.vcycle(20)
                s.sync()
                dt = time.perf_counter() - t0
                pp = s.fine_pass_time(3)
                cp = s.fine_pass_time(4)
                print(json.dumps({"variant": os.environ.get("PROBE_VARIANT", ""),
                                  "stagger": int(os.environ.get("PGMG_GRID_STAGGER", "0")),
                                  "carry": carry, "rep": r, "ms_per_cycle": round(dt * 50, 4),
                                  "k_postpre_ms": round(pp[1], 4), "n": pp[0],
                                  "carry_pass_ms": round(cp[1], 4),
                                  "hash": s.solution_hash(0)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16385)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--staggers", default="0,4096,65536")
    ap.add_argument("--variants", default="",
                    help="NAME:ENV=VAL+ENV=VAL,... (instead of --staggers): the measurement "
                         "build's environment knobs per variant")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a)
    specs = ([(f"stagger{st}", {"PGMG_GRID_STAGGER": st}) for st in a.staggers.split(",")]
             if not a.variants else
             [(v.split(":")[0], dict(kv.split("=") for kv in v.split(":")[1].split("+") if kv))
              for v in a.variants.split(",")])
    for name, extra in specs:
        st = extra.get("PGMG_GRID_STAGGER", "0")
        env = dict(os.environ, PGMG_ROLE_TRACE="1", PROBE_VARIANT=name, **extra)
        r = subprocess.run([sys.executable, __file__, "--child", "--n", str(a.n), "--reps", str(a.reps)],
                           env=env, capture_output=True, text=True, timeout=600)
        print(r.stdout, end="", flush=True)
        roles = [l for l in r.stderr.splitlines() if l.startswith("roles") or l.startswith("REP")]
        print(json.dumps({"variant": name, "stagger": int(st), "rc": r.returncode,
                          "roles": roles[-60:], "stderr": r.stderr[-1500:] if r.returncode else ""}),
              flush=True)


if __name__ == "__main__":
    main()
