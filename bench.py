#!/usr/bin/env python3
"""Benchmark: V-cycles/s of the fp64 2D-Poisson geometric-multigrid V-cycle at N=16385
(16384^2 cells) on MI355X, plus the fine-grid Jacobi sweep's HBM roofline fraction.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 16385]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A "step" is one V-cycle of the reference's mg_cpu_exec semantics (2+2 Jacobi sweeps
with the per-sweep residual-norm early exit, full-weighting restriction, the reference
prolongation, recursion to N=5) on the synthetic problem the reference itself solves:
phi0 = 0, f = analytic RHS.  All inputs are resident in HBM before the timed region.
With N GPUs the same grid is split into row strips (strong scaling, RCCL halo exchange);
value = V-cycles of the whole job per second.

Prints ONE JSON line on rank 0.  See DESIGN.md "Measurement" for every field.
"""
import argparse
import json
import os
import pathlib
import platform
import shutil
import subprocess
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
METRIC = "V-cycles/sec + fine-grid stencil HBM GB/s, 2D Poisson N=16384², fp64"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=16385, help="points per side (2^k+1)")
    ap.add_argument("--timing", choices=["graph", "events"], default="events",
                    help="events: eager launches with hipEvents around every fine sweep")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-n", type=int, default=0, help="grid for the CPU sample (default = --n)")
    ap.add_argument("--cycle", choices=["V", "W", "F"], default="V",
                    help="V (the headline), W (alpha=3 recursions) or F (full multigrid) cycles")
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64",
                    help="f64: the reference's precision (the headline); f32: the fp32 variant")
    return ap.parse_args()


def cpu_baseline(n, cycles=1, kind="V"):
    """The reference's own CPU multigrid (MultigridSolver::v_cycle of mg_cpu_exec, compiled
    from its sources by oracle/Makefile into oracle/_ref/ref_harness, 1 thread) on the host:
    a bounded sample of the same workload (one cycle of the same kind at the same N).
    Without that binary: the oracle (our C restatement, oracle/mg_cpu_exec_port)."""
    ref = ROOT / "oracle" / "_ref" / "ref_harness"
    port = ROOT / "oracle" / "mg_cpu_exec_port"
    if ref.exists():
        exe, what = ref, "reference"
    else:
        exe, what = port, "port"
        if not exe.exists():
            subprocess.run(["make", "-C", str(ROOT / "oracle"), "-s",
                            str(exe)], check=True, capture_output=True)
    cmd = [str(exe), kind, str(n), str(cycles), "1e-7"]
    if shutil.which("taskset"):
        cmd = ["taskset", "-c", "0"] + cmd
    out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
    secs = [float(l.split("seconds")[1].split()[0]) for l in out.splitlines() if "seconds" in l]
    t = sum(secs) / len(secs)
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    src = ("the reference's MultigridSolver (2_part_MG/MultiGrid.hpp) via oracle/_ref/ref_harness"
           if what == "reference" else "oracle/mg_cpu_exec_port (our C restatement)")
    return {"value": round(1.0 / t, 6), "unit": f"{kind}-cycles/s", "cores": 1, "kind": what,
            "sample": f"{cycles} {kind}-cycle(s) at N={n}, phi0=0, analytic f; {src}, g++/gcc -O2 "
                      f"single thread (taskset -c 0); {t:.2f} s per {kind}-cycle; host {model}"}


def pmc_traffic(n, key):
    """HBM bytes per launch of the kernel symbol `key` (normalised as scripts/pmc_summary.py
    does, e.g. k_postpre_lds<double,false,true>) at grid n, from the committed rocprofv3 PMC
    summary (profiles/pmc_fine.json: FETCH_SIZE/WRITE_SIZE passes with the gfx950
    corrections of MI355X_MICROARCH.md)."""
    p = ROOT / "profiles" / "pmc_fine.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        for k in d.get("kernels", []):
            if int(k.get("N", 0)) == n and k.get("kernel", "") == key:
                return k.get("hbm_bytes_per_launch")
    except (ValueError, OSError):
        pass
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # CPU baseline first, before this process touches the GPU (it runs a child process)
    cpu = None
    if world == 1 and rank == 0 and args.cpu_baseline == "auto" and args.dtype == "f64":
        try:
            cpu = cpu_baseline(args.cpu_n or args.n, kind=args.cycle)
        except Exception as e:  # reported, not fatal
            cpu = {"value": None, "unit": "V-cycles/s", "cores": 1, "kind": "port",
                   "sample": f"failed: {e}"}
    import torch  # noqa: F401  (loads the ROCm runtime first; see _capi.load)
    import _pkgload
    pg = _pkgload.load()

    dist = None
    uid = None
    # PGMG_BENCH_SOLO=1 (harness test on a one-GPU box only): every rank on device 0 with the
    # null transport (PGMG_FLAG_SOLO: no messages, results meaningless); the line says so
    solo = world > 1 and os.environ.get("PGMG_BENCH_SOLO") == "1"
    device = 0 if (world == 1 or solo) else local_rank
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(device)
        dist.init_process_group("gloo")
        t = torch.tensor(list(pg.unique_id()) if rank == 0 else [0] * 128, dtype=torch.uint8)
        dist.broadcast(t, 0)
        uid = bytes(t.tolist())

    flags = pg.PGMG_FLAG_TIME_FINE if args.timing == "events" else 0
    if solo:
        flags |= pg.PGMG_FLAG_SOLO
    kw = dict(flags=flags, device=device, dtype=args.dtype)
    if world > 1:
        kw.update(rank=rank, world=world, uid=uid)
    s = pg.Solver(args.n, **kw)
    s.set_problem()
    bulk, tail_top = s.levels()

    def barrier():
        if dist is not None:
            dist.barrier()

    # warmup (also builds the hipGraph in graph mode)
    run = {"V": s.vcycle, "W": s.wcycle, "F": s.fcycle}[args.cycle]
    run(max(args.warmup, 0))
    s.sync()
    for w in (0, 1, 2, 3):  # drop warmup events
        s.fine_pass_time(w)
    barrier()
    s.sync()
    t0 = time.perf_counter()
    run(args.steps)
    t_enq = time.perf_counter()   # host time to enqueue the steps (asynchronous launches)
    s.sync()
    barrier()
    t1 = time.perf_counter()
    dt = t1 - t0
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    dev_ms = s.last_elapsed_ms()
    spec_info, spec_mask = s.dist_info(), s.spec_levels()
    vbytes = s.vcycle_bytes()
    n = N = args.n
    gen = s.fused and s.fine_pass_bytes(3) < s.fine_pass_bytes(0)   # f regenerated in-kernel
    T = "double" if args.dtype == "f64" else "float"
    r2 = world > 1 and not s.dist_info()[0]   # k_postpre sums r(x2)^2: exact strip decisions
    passes = []
    if s.fused:
        # algorithmic bytes per launch from the library (pgmg_fine_pass_bytes): each input
        # read once, each output written once
        for which, name, key in (
                (3, "k_postpre (finest level, between cycles: prolongation + 2+2 Jacobi sweeps "
                    "+ residual + restriction, fused" + ("; f regenerated in-kernel" if gen else "")
                    + ")", f"k_postpre_lds<{T},{'true' if r2 else 'false'},"
                           f"{'true' if gen else 'false'}>"),
                (1, "k_pre<false,true> (finest level: 2 Jacobi sweeps + residual + restriction, "
                    "fused)", f"k_pre<{T},false,true,2,{'true' if gen else 'false'},false>"),
                (2, "k_post<true> (finest level: prolongation + 2 Jacobi sweeps, fused)",
                 f"k_post<{T},true,2,false,true>" if gen else f"k_post<{T},true,2,false>")):
            cnt, ms = s.fine_pass_time(which)
            passes.append((name, s.fine_pass_bytes(which), cnt, ms, key))
    else:
        cnt, ms = s.fine_pass_time(0)
        passes.append(("k_sweep<false,false,true> (finest-level Jacobi sweep)",
                       s.fine_pass_bytes(0), cnt, ms, f"k_sweep<{T},false,false,true>"))
    if not passes or passes[0][2] == 0:   # graph mode: time the kernel separately
        ms = s.bench_sweep(20)
        passes = [("k_sweep<false,false,true> (finest-level Jacobi sweep, timed apart)",
                   s.fine_pass_bytes(0), 20, ms, f"k_sweep<{T},false,false,true>")]
    roof = []
    for name, nbytes, cnt, ms, key in passes:
        ach = nbytes / (ms * 1e-3) / 1e9 if ms > 0 else None
        roof.append({"bound": "hbm", "kernel": name, "symbol": key,
                     "achieved": round(ach, 2) if ach else None, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4) if ach else None,
                     "traffic": (pmc_traffic(N, key) if world == 1 else None),
                     "bytes_per_launch": nbytes, "launches_timed": cnt,
                     "ms_per_launch": round(ms, 5)})
    # the dominant kernel: largest total time over the timed region
    roof = [r for r in roof if r["launches_timed"]]
    roof.sort(key=lambda r: -(r["ms_per_launch"] or 0) * r["launches_timed"])
    sweep_eq = None
    if s.fused and roof and roof[0]["achieved"]:
        # the same pass counted as the separate 24 B/pt sweeps it replaces
        nsw = 4 if roof[0]["kernel"].startswith("k_postpre") else 2
        sweep_eq = round(nsw * s.fine_pass_bytes(0) / (roof[0]["ms_per_launch"] * 1e-3) / 1e9, 2)

    if rank == 0:
        value = args.steps / dt
        metric = METRIC if args.dtype == "f64" else METRIC.replace(", fp64", ", fp32 variant")
        if args.cycle != "V":
            metric = metric.replace("V-cycles/sec", f"{args.cycle}-cycles/sec")
        if args.n != 16385:
            metric = metric.replace("16384²", f"{args.n - 1}²")
        line = {
            "metric": metric,
            "value": round(value, 4),
            "unit": f"{args.cycle}-cycles/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic: the reference's own problem, phi0=0, f=2*pi^2*sin(pi x)sin(pi y)",
            "config": {
                "workload": f"{args.cycle}-cycle N={n} ({n - 1}^2 cells), 2+2 Jacobi (v1=v2=1), 11 coarsest "
                            f"sweeps, eps=1e-7 early exit, {bulk} bulk levels + one-workgroup LDS "
                            f"tail from N={tail_top} to N=5",
                "N": n, "bulk_levels": bulk, "tail_top": tail_top,
                "parallelism": "single-gpu" if world == 1 else (
                    f"row-strips x{world} (SOLO null transport on one GPU: harness test, "
                    f"not a measurement)" if solo else f"row-strips x{world} (RCCL halos)"),
                "timing": args.timing,
            },
            "roofline": roof[0],
            "roofline_other": roof[1:],
            "fine_sweep_equivalent_gbps": sweep_eq,
            "vcycle_algorithmic_gbps": round(vbytes / (dt / args.steps) / 1e9, 2),
            "vcycle_device_ms": round(dev_ms / args.steps, 4),
            "host_enqueue_ms_per_step": round((t_enq - t0) * 1e3 / args.steps, 4),
            # early-exit checks recorded and validated after each call (DESIGN.md §3 point 8)
            "speculative_checks": {"enabled": spec_info[0], "rollbacks": spec_info[1],
                                   "in_stream_level_mask": spec_mask},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    s.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
