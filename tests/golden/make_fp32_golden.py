#!/usr/bin/env python3
"""fp32 fixtures at the bench's grid size (BASELINE configs[4]'s "fp32 vs fp64" half).

The reference is fp64-only, so the fp32 variant is pinned to the fp32 restatement of the
oracle (oracle/liboracle_f32.so: pgmg_oracle.c built with -DORC_REAL=float), which the GPU
suite already checks bitwise at N <= 1025 (tests/test_gpu_fp32.py).  This script runs that
restatement at N = 16385 and stores, per cycle, the FNV-64 hash of phi's own fp32 words
(hash_f32: consecutive pairs of 4-byte words as one 64-bit word, a zero word appended to an
odd count) and the cumulative sweep / early-exit counts:

    python tests/golden/make_fp32_golden.py            # -> tests/golden/fp32_big.json

~20 s per V-cycle on one core; 4.3 GB of host memory.
"""
import json
import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent / "oracle"))
import oracle  # noqa: E402

CASES = [("V", 16385, 25)]


def hash_f32(a):
    """FNV-64 (oracle.fnv_hash) over the fp32 words of `a` taken two at a time: every bit of
    every word enters the hash (widening to fp64 first would leave 29 zero bits per word)."""
    w = np.ascontiguousarray(a, dtype=np.float32).ravel()
    if w.size & 1:
        w = np.concatenate([w, np.zeros(1, np.float32)])
    return oracle.fnv_hash(w.view(np.float64))


def main():
    out = []
    for kind, N, cycles in CASES:
        o = oracle.Oracle(eps=1e-7, dtype="f32")
        f = o.rhs(N)
        phi = np.zeros((N, N), dtype=np.float32)
        rows = []
        for k in range(cycles):
            {"V": o.v_cycle, "W": o.w_cycle}[kind](phi, f)
            rows.append({"cycle": k + 1, "hash": hash_f32(phi), "sweeps": o.sweeps,
                         "exits": o.early_exits,
                         "centre": float(phi[N // 2, N // 2])})
            print(kind, N, rows[-1], flush=True)
        out.append({"kind": kind, "N": N, "eps": 1e-7, "dtype": "f32",
                    "source": "oracle/liboracle_f32.so (fp32 restatement of the reference)",
                    "cycles": rows})
    (HERE / "fp32_big.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
