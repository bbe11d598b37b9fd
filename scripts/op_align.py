#!/usr/bin/env python3
"""What the caller's odd pitch costs the op-level Jacobi sweep: ms per sweep of
pgmg_jacobi(v = 20, no early exit) on H = 16385 rows of
  * W = 16385 (the reference layout: every other row's lane pairs 8-byte aligned),
  * W = 16386 at offset 0 (every row's pairs 8-byte aligned only),
  * W = 16386 at offset +1 element (every row's pairs 16-byte aligned),
interleaved over rounds; one JSON line each."""
import json
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
import _pkgload  # noqa: E402

pg = _pkgload.load()
H = 16385
v = 20


def arrays(W, off):
    n = H * W + 2
    st = [torch.zeros(n, dtype=torch.float64, device="cuda:0") for _ in range(3)]
    x, f, t = (s[off:off + H * W].view(H, W) for s in st)
    f.fill_(1.0)
    return st, x, f, t


for rnd in range(3):
    for W, off in ((16385, 0), (16386, 0), (16386, 1), (16385, 1)):
        st, x, f, t = arrays(W, off)
        h = 1.0 / (W - 1)
        pg.ops.jacobi(x, f, h, 1, eps=-1.0, tmp=t)
        ts = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            pg.ops.jacobi(x, f, h, v, eps=-1.0, tmp=t)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) / (v + 1))
        ms = statistics.median(ts)
        byt = 24.0 * (H - 2) * (W - 2)
        print(json.dumps({"W": W, "offset": off, "round": rnd, "ms_per_sweep": round(ms, 5),
                          "frac": round(byt / ms / 1e9 / 8.0, 4)}), flush=True)
        del st, x, f, t
        torch.cuda.empty_cache()
