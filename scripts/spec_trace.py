"""Per-level check norms seen by the speculation policy (PGMG_SPEC_TRACE=1), N = 2049:
vcycle(1) x 40 (each call is one validated segment)."""
import os
import pathlib
import sys

os.environ["PGMG_SPEC_TRACE"] = "1"
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: F401,E402
import _pkgload  # noqa: E402

pg = _pkgload.load()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 2049
with pg.Solver(N) as s:
    s.set_problem()
    for k in range(1, 61):
        print(f"--- call {k}", file=sys.stderr, flush=True)
        s.vcycle(1)
        if s.dist_info()[1]:
            print(f"rollback at call {k}", file=sys.stderr, flush=True)
            break
