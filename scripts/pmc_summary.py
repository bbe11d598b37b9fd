#!/usr/bin/env python3
"""Summarise rocprofv3 runs into profiles/<tag>/ and profiles/pmc_fine.json.

Inputs (from scripts/gpu_session.sh steps prof/pmc): gpurun_out/prof/run_kernel_stats.csv,
gpurun_out/pmc_fetch/run_counter_collection.csv, gpurun_out/pmc_write/...

HBM bytes per launch of the finest-level kernels = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024):
on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced streaming reads
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16 B/lane stores.
"""
import csv
import collections
import json
import pathlib
import re
import shutil
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
OUT = ROOT / "gpurun_out"


def norm_name(n):
    m = re.search(r"pgmg::(k_\w+)(<[^>]*>)?", n)
    if not m:
        return n
    t = (m.group(2) or "").replace(" ", "")
    # the full template argument list, as bench.py's symbol keys spell it
    return m.group(1) + t


def is_finest(k):
    """Finest-level kernel symbols (normalised): k_postpre*, k_pre<T,false,true>,
    k_post<T,true,PAIRS,false>, k_sweep<T,X0,NORM,true>."""
    return bool(k.startswith("k_postpre") or re.match(r"k_pre<\w+,false,true[,>]", k) or
                re.match(r"k_post<\w+,true,\d+,false[,>]", k) or
                re.match(r"k_sweep<\w+,\w+,\w+,true>$", k))


def main(tag, N=16385):
    dst = ROOT / "profiles" / tag
    dst.mkdir(parents=True, exist_ok=True)
    for src, name in (("prof/run_kernel_stats.csv", "kernel_stats.csv"),
                      ("pmc_fetch/run_counter_collection.csv", "pmc_fetch.csv"),
                      ("pmc_write/run_counter_collection.csv", "pmc_write.csv"),
                      ("bench.log", "bench.log"), ("prof.log", "prof.log")):
        if (OUT / src).exists():
            shutil.copy(OUT / src, dst / name)
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f, ctr in (("pmc_fetch.csv", "FETCH_SIZE"), ("pmc_write.csv", "WRITE_SIZE")):
        p = dst / f
        if not p.exists():
            continue
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == ctr:
                vals[norm_name(r["Kernel_Name"])][ctr].append(float(r["Counter_Value"]))
    stats = {}
    if (dst / "kernel_stats.csv").exists():
        for r in csv.DictReader(open(dst / "kernel_stats.csv")):
            stats[norm_name(r["Name"])] = float(r["AverageNs"]) / 1e6
    kernels = []
    for k, v in sorted(vals.items()):
        if not is_finest(k):
            continue  # finest-level symbols only (FINE template argument; k_postpre always)
        if not v.get("FETCH_SIZE") or not v.get("WRITE_SIZE"):
            continue
        fetch = sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"])
        write = sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"])
        b = 2 * fetch * 1024 + write * 1024
        kernels.append({"kernel": k, "N": N, "fetch_size_kib": fetch, "write_size_kib": write,
                        "hbm_bytes_per_launch": b,
                        "avg_ms_rocprof": stats.get(k)})
    import hashlib
    lib = ROOT / "parallel-geometric-multigrid-for-poisson-problem_amd" / "libpgmg.so"
    build = ("libpgmg.so sha256:" + hashlib.sha256(lib.read_bytes()).hexdigest()[:16]
             if lib.exists() else None)
    summary = {"tag": tag, "N": N, "build": build,
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                         "bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB), gfx950 read correction",
               "kernels": kernels}
    (dst / "pmc_summary.json").write_text(json.dumps(summary, indent=1) + "\n")
    (ROOT / "profiles" / "pmc_fine.json").write_text(json.dumps(summary, indent=1) + "\n")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "latest")
