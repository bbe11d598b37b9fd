#!/usr/bin/env python3
"""Sweep launch variants of the fused smoother passes in ONE process (interleaved rounds).

For every variant (environment knobs read by pgmg_fused.hip at launch time) it checks
bit-parity at N=4097 against the reference golden hash, then times the finest-level
k_pre / k_post kernels and the whole V-cycle at N=16385 with hipEvents.

    python scripts/tune_fused.py [--n 16385] [--rounds 3]
"""
import argparse
import itertools
import json
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16385)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--cycles", type=int, default=10)
    ap.add_argument("--variants", default="")
    args = ap.parse_args()
    import torch  # noqa: F401
    import _pkgload
    import oracle
    pg = _pkgload.load()
    golden = {(c["kind"], c["N"], c["eps"]): c for c in
              json.loads((ROOT / "tests/golden/cycles.json").read_text())}
    if args.variants:
        variants = [dict(kv.split("=") for kv in v.split(",")) for v in args.variants.split(";")]
    else:
        variants = [dict(PGMG_FUSED_PAIRS=str(p), PGMG_FUSED_BLOCKS=str(b),
                         PGMG_FUSED_MAX_ROWS=str(m))
                    for p, b, m in itertools.product((1, 2), (1024, 2048, 4096), (64, 512))]

    def apply(v):
        for k in ("PGMG_FUSED_PAIRS", "PGMG_FUSED_BLOCKS", "PGMG_FUSED_MAX_ROWS",
                  "PGMG_FUSED_MIN_ROWS"):
            os.environ.pop(k, None)
        os.environ.update(v)

    # parity per variant
    g = golden[("V", 4097, 1e-7)]
    for v in variants:
        apply(v)
        with pg.Solver(4097, flags=pg.PGMG_FLAG_NO_GRAPH) as s:
            s.set_problem()
            s.vcycle(len(g["cycles"]))
            h = oracle.fnv_hash(s.solution())
        ok = h == g["cycles"][-1]["hash"]
        print(json.dumps({"variant": v, "parity_4097": ok}), flush=True)
        if not ok:
            raise SystemExit("parity failure")

    s = pg.Solver(args.n, flags=pg.PGMG_FLAG_TIME_FINE)
    s.set_problem()
    res = {json.dumps(v): [] for v in variants}
    for r in range(args.rounds):
        for v in variants:
            apply(v)
            s.vcycle(2)
            s.sync()
            for w in (0, 1, 2):
                s.fine_pass_time(w)
            s.vcycle(args.cycles)
            s.sync()
            ms = s.last_elapsed_ms() / args.cycles
            _, pre = s.fine_pass_time(1)
            _, post = s.fine_pass_time(2)
            res[json.dumps(v)].append((ms, pre, post))
    nf = (args.n - 2) ** 2
    out = []
    for k, vals in res.items():
        vals.sort()
        ms, pre, post = vals[len(vals) // 2]
        b = 24.0 * nf + 2.0 * nf
        out.append({"variant": json.loads(k), "vcycle_ms": round(ms, 4),
                    "vcycles_per_s": round(1e3 / ms, 2), "k_pre_ms": round(pre, 4),
                    "k_post_ms": round(post, 4), "k_pre_GBps": round(b / pre / 1e6, 1),
                    "k_post_GBps": round(b / post / 1e6, 1),
                    "min_vcycle_ms": round(min(x[0] for x in vals), 4)})
    out.sort(key=lambda d: d["vcycle_ms"])
    for o in out:
        print(json.dumps(o), flush=True)
    s.close()


if __name__ == "__main__":
    main()
