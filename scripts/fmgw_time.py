#!/usr/bin/env python3
"""BASELINE configs[4]'s cycle timed per variant (measurement tool): set_problem, one F-cycle
(the FMG start), then ONE W-cycle, each timed by the host clock around a synchronised call,
phi's FNV-64 after both checked against the reference's hash (tests/golden/cycles.json, kind
G).  Variants are environment settings of the measurement build (PGMG_LIB=...libpgmg_ab.so),
each run in its own process, interleaved over rounds; one JSON line per run.

    PGMG_LIB=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so \\
        python scripts/fmgw_time.py [--n 32769] [--rounds 2] NAME[:VAR=v,...] ...
"""
import argparse
import json
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent

CHILD = r"""
import json, sys, time
sys.path.insert(0, %(root)r)
import torch  # noqa
import _pkgload
pg = _pkgload.load()
with pg.Solver(%(n)d) as s:
    s.set_problem()
    s.sync()
    t0 = time.perf_counter(); s.fcycle(1); s.sync(); t1 = time.perf_counter()
    s.wcycle(1); s.sync(); t2 = time.perf_counter()
    print(json.dumps({"f_s": t1 - t0, "w_s": t2 - t1, "hash": s.solution_hash(0),
                      "sweeps": s.stats()[0], "modes": s.spec_visit_modes(),
                      "rollbacks": s.dist_info()[1]}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32769)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    want = None
    for c in json.loads((ROOT / "tests" / "golden" / "cycles.json").read_text()):
        if c["kind"] == "G" and c["N"] == a.n and len(c["cycles"]) >= 2:
            want = c["cycles"][1]["hash"]
    vs = []
    for v in a.variants:
        name, _, envs = v.partition(":")
        vs.append((name, dict(e.split("=", 1) for e in envs.split(",") if e)))
    for rnd in range(a.rounds):
        for name, env in vs:
            e = dict(os.environ)
            e.update(env)
            out = subprocess.run([sys.executable, "-c", CHILD % {"root": str(ROOT), "n": a.n}],
                                 env=e, capture_output=True, text=True, timeout=600)
            line = next((l for l in out.stdout.splitlines() if l.startswith("{")), None)
            if line is None:
                print(json.dumps({"variant": name, "round": rnd, "error": out.stderr[-1500:]}),
                      flush=True)
                sys.exit(1)
            d = json.loads(line)
            d.update(variant=name, round=rnd, parity=(d["hash"] == want) if want else None)
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
