"""Speculative calls on the reference problem: at which V-cycle does the first bulk-level
early-exit check fire (vcycle(1) calls), and does a warmup + one long call (the bench's
shape) run without a rollback (levels predicted to fire go in-stream first)?"""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: F401,E402
import _pkgload  # noqa: E402

pg = _pkgload.load()
for N, cap in ((2049, 60), (4097, 60), (16385, 60)):
    with pg.Solver(N) as s:
        s.set_problem()
        first = None
        for k in range(1, cap + 1):
            s.vcycle(1)
            if s.dist_info()[1] > 0:
                first = k
                break
        print(f"N={N}: vcycle(1) calls: first rollback at cycle {first}, in-stream mask "
              f"{bin(s.spec_levels())}", flush=True)
    for warm, K in ((2, 20), (3, 40), (2, 60)):
        with pg.Solver(N) as s:
            s.set_problem()
            s.vcycle(warm)
            s.sync()
            t = time.perf_counter()
            s.vcycle(K)
            s.sync()
            dt = time.perf_counter() - t
            print(f"N={N}: warmup {warm} + {K}: {K / dt:.1f} V/s, rollbacks {s.dist_info()[1]}, "
                  f"mask {bin(s.spec_levels())}", flush=True)
