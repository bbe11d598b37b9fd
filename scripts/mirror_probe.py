"""Which part of the gpu_exec mirror path (per-call set_problem(phi, f) + vcycle(1) +
get_solution, explicit host f, h0) changes phi's bits against the golden V-cycles?"""
import sys
import pathlib
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "oracle"))
import torch  # noqa
import _pkgload
import oracle
pg = _pkgload.load()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 33
o = oracle.Oracle()
f = o.rhs(N)
ref = np.zeros((N, N))
for _ in range(3):
    o.v_cycle(ref, f)
want = oracle.fnv_hash(ref)


def run(tag, per_call, fhost, h0):
    kw = {"h0": 1.0 / (N - 1)} if h0 else {}
    with pg.Solver(N, **kw) as s:
        phi = np.zeros((N, N))
        if per_call:
            for _ in range(3):
                s.set_problem(phi, f if fhost else None)
                s.vcycle(1)
                phi = s.solution()
        else:
            s.set_problem(None, f if fhost else None)
            s.vcycle(1); s.vcycle(1); s.vcycle(1)
            phi = s.solution()
    h = oracle.fnv_hash(phi)
    print(f"{tag:40s} {h} {'OK' if h == want else 'DIFF'} max|d|={np.max(np.abs(phi - ref)):.3e}",
          flush=True)


for per_call in (False, True):
    for fhost in (False, True):
        for h0 in (False, True):
            run(f"per_call={per_call} fhost={fhost} h0={h0}", per_call, fhost, h0)
