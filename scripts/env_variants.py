#!/usr/bin/env python3
"""Run bench.py once per environment variant (separate processes, interleaved twice) and
print the finest-level kernel times: scripts/env_variants.py VAR=v1,v2,... [VAR2=...]"""
import itertools
import json
import os
import subprocess
import sys


def main():
    axes = []
    for a in sys.argv[1:]:
        k, vs = a.split("=", 1)
        axes.append([(k, v) for v in vs.split(",")])
    combos = list(itertools.product(*axes)) if axes else [()]
    for rep in range(2):
        for combo in combos:
            env = dict(os.environ)
            env.update(dict(combo))
            out = subprocess.run([sys.executable, "bench.py", "--steps", "20", "--warmup", "3",
                                  "--cpu-baseline", "off"], env=env, capture_output=True,
                                 text=True, timeout=300)
            line = next((l for l in out.stdout.splitlines() if l.startswith("{")), None)
            if line is None:
                print(combo, "FAILED", out.stderr[-2000:], flush=True)
                sys.exit(1)
            d = json.loads(line)
            ks = [d["roofline"]] + d.get("roofline_other", [])
            print(rep, dict(combo), "V/s=%.1f" % d["value"],
                  " ".join("%s=%.4fms" % (k["kernel"].split(" ")[0], k["ms_per_launch"]) for k in ks),
                  flush=True)


if __name__ == "__main__":
    main()
