#!/usr/bin/env python3
"""Run a few V-cycles at N (measurement child for rocprofv3 passes; PGMG_LIB picks the build)."""
import sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import _pkgload

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16385
K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
pg = _pkgload.load()
with pg.Solver(N) as s:
    s.set_problem()
    s.vcycle(2)
    s.vcycle(K)
    s.sync()
print("done", N, K, s is not None)
