#!/usr/bin/env python3
"""Interleaved A/B of library builds and tuning knobs on the finest-level passes.

    python scripts/pp_ab.py [--n 16385] [--rounds 3] NAME=LIB[:VAR=v[,VAR=v...]] ...

LIB is a libpgmg build (e.g. parallel-.../libpgmg_ab.so, built with `make ab`); VAR=v are
environment knobs the measurement build reads (pgmg_internal.h: tuning_int), AB_FLAGS=n:
PGMG_FLAG_* bits OR-ed into the solver's flags, or AB_TAIL_N=n: the solver's tail_n.  Every
variant runs in its own process (set_problem, 2 warmup V-cycles, 20 timed in one call
with per-pass hipEvents); the rounds interleave the variants so box drift hits all alike.
Prints one JSON line per run: k_postpre / k_pre / k_post ms per launch, ms per V-cycle,
and whether phi matches the reference's hash after 22 cycles (tests/golden/cycles.json).
"""
import argparse
import json
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent

CHILD = r"""
import json, os, sys, time
sys.path.insert(0, %(root)r)
import torch  # noqa
import _pkgload
pg = _pkgload.load()
N = %(n)d
K = %(steps)d
kw = {"tail_n": int(os.environ["AB_TAIL_N"])} if os.environ.get("AB_TAIL_N") else {}
with pg.Solver(N, flags=pg.PGMG_FLAG_TIME_FINE | int(os.environ.get("AB_FLAGS", "0")), dtype=%(dtype)r, **kw) as s:
    s.set_problem()
    run = {"V": s.vcycle, "W": s.wcycle, "F": s.fcycle}[%(kind)r]
    run(2); s.sync()
    for w in range(4): s.fine_pass_time(w)
    t0 = time.perf_counter(); run(K); s.sync(); t1 = time.perf_counter()
    r = {w: s.fine_pass_time(w) for w in range(4)}
    h = s.solution_hash(0)
    st = s.stats()
print(json.dumps({"ms_cycle": (t1 - t0) * 1e3 / K, "pp": r[3][1], "pre": r[1][1],
                  "post": r[2][1], "hash": h, "sweeps": st[0]}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16385)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--kind", default="V")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--dtype", default="f64", help="f32: no hash check (the fixtures are fp64)")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    want = None
    for c in [] if a.dtype != "f64" else json.loads((ROOT / "tests" / "golden" / "cycles.json").read_text()):
        if c["kind"] == a.kind and c["N"] == a.n and c["eps"] == 1e-7 and len(c["cycles"]) >= 2 + a.steps:
            want = c["cycles"][1 + a.steps]["hash"]
    vs = []
    for v in a.variants:
        name, rest = v.split("=", 1)
        lib, _, envs = rest.partition(":")
        env = dict(e.split("=", 1) for e in envs.split(",") if e)
        vs.append((name, lib, env))
    for rnd in range(a.rounds):
        for name, lib, env in vs:
            e = dict(os.environ)
            e.update(env)
            if lib:
                e["PGMG_LIB"] = str((ROOT / lib).resolve())
            out = subprocess.run([sys.executable, "-c", CHILD % {"root": str(ROOT), "n": a.n, "kind": a.kind, "steps": a.steps, "dtype": a.dtype}],
                                 env=e, capture_output=True, text=True, timeout=300)
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
