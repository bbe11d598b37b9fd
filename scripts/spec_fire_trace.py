"""Segment planning and predicted-to-fire trace of one long call (PGMG_SPEC_TRACE=1, needs the
measurement build libpgmg_ab.so via PGMG_LIB): python scripts/spec_fire_trace.py N CYCLES"""
import os
import pathlib
import sys
import time

os.environ["PGMG_SPEC_TRACE"] = "1"
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: F401,E402
import _pkgload  # noqa: E402

pg = _pkgload.load()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 2049
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
if len(sys.argv) > 3 and sys.argv[3] == "W":   # W-cycles: calls of K cycles, the plan per call
    # PGMG_TRACE_FLAGS: pgmg_config.flags (e.g. 32768 = PGMG_FLAG_NO_SPEC_FIRE: no W plans)
    flags = int(os.environ.get("PGMG_TRACE_FLAGS", "0"))
    with pg.Solver(N, flags=flags) as s:
        s.set_problem()
        total = 0.0
        for i in range(int(sys.argv[4]) if len(sys.argv) > 4 else 6):
            t0 = time.perf_counter()
            s.wcycle(K)
            s.sync()
            dt = time.perf_counter() - t0
            total += dt if i > 0 else 0.0
            print(f"N={N} W call {i} x{K}: {K / dt:.2f} W/s modes={s.spec_visit_modes()} "
                  f"dist={s.dist_info()} sweeps={s.stats()} hash={s.solution_hash(0)}",
                  file=sys.stderr, flush=True)
        print(f"N={N} flags={flags}: calls 1.. {K * i / total:.3f} W/s", file=sys.stderr, flush=True)
    sys.exit(0)
with pg.Solver(N) as s:
    s.set_problem()
    s.vcycle(3)
    s.sync()
    print("--- long call", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    s.vcycle(K)
    s.sync()
    dt = time.perf_counter() - t0
    print(f"N={N} K={K} {K / dt:.1f} V/s fire={bin(s.spec_fire_levels())} "
          f"spec={bin(s.spec_levels())} dist={s.dist_info()}", file=sys.stderr, flush=True)
