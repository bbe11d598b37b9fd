#!/usr/bin/env python3
"""Benchmark: V-cycles/s of the fp64 2D-Poisson geometric-multigrid V-cycle at N=16385
(16384^2 cells) on MI355X, plus the finest-level pass's HBM roofline fraction.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--reps R] [--n 16385]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

`--gpus N` with N > 1 outside a launcher (no WORLD_SIZE in the environment) starts N rank
processes itself -- `python -m torch.distributed.run --nnodes=1 --nproc-per-node N
--master-addr 127.0.0.1` as a CHILD of this process, before anything touches the GPU -- and
exits with its status.  Under a launcher, --gpus must equal WORLD_SIZE, and each rank needs its
own device (LOCAL_RANK < the device count) unless PGMG_BENCH_SOLO=1 or
PGMG_BENCH_TRANSPORT=host (harness tests on a one-GPU box); otherwise the run exits non-zero.

A "step" is one V-cycle of the reference's mg_cpu_exec semantics (2+2 Jacobi sweeps with
the per-sweep residual-norm early exit, full-weighting restriction, the reference
prolongation, recursion to N=5) on the synthetic problem the reference itself solves:
phi0 = 0, f = analytic RHS.  Inputs are resident in HBM before the timed region.

Each of R repetitions (default 5) restarts from phi0 = 0 (set_problem, outside the timed
region), runs W untimed warmup cycles, then times exactly K cycles in ONE call, bracketed
by barrier + device sync on both sides, max over ranks.  `value` = K / the median time.
After every repetition phi's FNV-64 hash (pgmg_solution_hash) is compared with the
reference's hash after W+K cycles (tests/golden/cycles.json, a fixture of the compiled
reference's own runs): `parity` is true only when every repetition matched.

Kernel durations for `roofline` come from one more repetition with hipEvents around every
finest-level pass (PGMG_FLAG_TIME_FINE; the events cost ~2-4 % of the cycle, so the clean
repetitions give `value`).  `roofline.traffic` is the HBM traffic of the same kernel from
two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over a short child run of this very
build, made before this process touches the GPU (--pmc off: null).  Kernel symbols and
algorithmic bytes per launch of the timed passes come from the library (pgmg_fine_pass_info).  With N GPUs the same grid is split into row strips (strong
scaling, RCCL halo exchange); value = V-cycles of the whole job per second.

Prints ONE JSON line on rank 0.  See DESIGN.md "Measurement" for every field.
"""
import argparse
import json
import os
import pathlib
import platform
import shutil
import statistics
import subprocess
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
TRACE_PREWARM = 4         # pre-warm calls before the kernel-trace child's timed call
INST_REPS = 3             # repetitions with per-pass events (the roofline's event-timed median)
PASSES = (0, 1, 2, 3, 4, 5)  # finest-level passes: sweep, k_pre, k_post, k_postpre, carry pass,
                             # recompute form
METRIC = "V-cycles/sec + fine-grid stencil HBM GB/s, 2D Poisson N=16384², fp64"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5, help="timed repetitions (median reported)")
    ap.add_argument("--n", "--N", dest="n", type=int, default=16385,
                    help="points per side (2^k+1); --N under torch.distributed.run")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-n", type=int, default=0, help="grid for the CPU sample (default = --n)")
    ap.add_argument("--cycle", choices=["V", "W", "F"], default="V",
                    help="V (the headline), W (alpha=3 recursions) or F (full multigrid) cycles")
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64",
                    help="f64: the reference's precision (the headline); f32: the fp32 variant")
    ap.add_argument("--general-rhs", choices=["auto", "off"], default="auto",
                    help="also measure the stored-f path (a user RHS streamed, 24 B/pt)")
    ap.add_argument("--pmc", choices=["auto", "off"], default="auto",
                    help="auto: HBM traffic of the finest-level passes from two rocprofv3 --pmc "
                         "passes (FETCH_SIZE, WRITE_SIZE) over a short child run of this build, "
                         "before this process touches the GPU")
    ap.add_argument("--other-configs", choices=["auto", "off"], default="auto",
                    help="auto (the default headline run only: one GPU, V, f64, N = 16385): also "
                         "time BASELINE.json's other GPU configs on this GPU, each hash-checked")
    ap.add_argument("--big-grid", choices=["auto", "off"], default="auto",
                    help="auto (N > 1 GPUs, V, f64, N = 16385): also time BASELINE configs[3]'s "
                         "N = 32769 on the same ranks (1 + 5 cycles, median of 3, hash-checked)")
    ap.add_argument("--fast-mode", choices=["auto", "off"], default="auto",
                    help="auto (one GPU, V, f64): also time PGMG_FLAG_FAST (FMA / shared "
                         "neighbour sums in the finest pass; not bitwise) and report its "
                         "difference from the EXACT result")
    ap.add_argument("--dropin", choices=["auto", "off"], default="auto",
                    help="auto (one GPU, V, f64): also time the reference's own entry point -- "
                         "ParallelMultiGridSolver::v_cycle called once per cycle through the C++ "
                         "mirror (host/gpu_exec, device arrays in place) -- and the context API's "
                         "one-cycle calls it is measured against")
    ap.add_argument("--ops", choices=["auto", "off"], default="auto",
                    help="auto (one GPU, V, f64): the per-op study at --n -- pgmg_jacobi / "
                         "residual / restrict / prolong on reference-layout arrays (the "
                         "Parallel::Compute* entries), GB/s and roofline fraction per op")
    ap.add_argument("--trace", choices=["auto", "off"], default="auto",
                    help="auto: a rocprofv3 --kernel-trace --stats pass over a child run of the "
                         "timed call (warmup + steps cycles), before this process touches the "
                         "GPU: the dominant kernel's rocprof average beside the event timing")
    ap.add_argument("--save-profiles", default="",
                    help="directory to keep the rocprofv3 summaries of the trace and PMC passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--trace-child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or ""


def _cpu_exe():
    ref = ROOT / "oracle" / "_ref" / "ref_harness"
    port = ROOT / "oracle" / "mg_cpu_exec_port"
    if ref.exists():
        return ref, "reference"
    if not port.exists():
        subprocess.run(["make", "-C", str(ROOT / "oracle"), "-s", str(port)], check=True,
                       capture_output=True)
    return port, "port"


def cpu_baseline(n, cycles=1, kind="V", skip=0):
    """The reference's own CPU multigrid (MultigridSolver of mg_cpu_exec, compiled from its
    sources by oracle/Makefile into oracle/_ref/ref_harness, 1 thread, taskset -c 0) on
    the host: a bounded sample of the same workload; the first `skip` cycles are warmup,
    the median of the rest is reported.  Without that binary: the oracle (our C
    restatement, oracle/mg_cpu_exec_port)."""
    exe, what = _cpu_exe()
    cmd = [str(exe), kind, str(n), str(cycles), "1e-7"]
    if shutil.which("taskset"):
        cmd = ["taskset", "-c", "0"] + cmd
    out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
    secs = [float(l.split("seconds")[1].split()[0]) for l in out.splitlines() if "seconds" in l]
    t = statistics.median(secs[skip:])
    src = ("the reference's MultigridSolver (2_part_MG/MultiGrid.hpp) via oracle/_ref/ref_harness"
           if what == "reference" else "oracle/mg_cpu_exec_port (our C restatement)")
    timed = secs[skip:]
    return {"value": round(1.0 / t, 6), "unit": f"{kind}-cycles/s", "cores": 1, "kind": what,
            "N": n, "s_per_cycle": [round(x, 5) for x in timed],
            "spread_pct": round(100 * (max(timed) - min(timed)) / t, 2) if len(timed) > 1 else None,
            "sample": f"{kind}-cycles at N={n} from phi0=0, analytic f: {skip} warmup + median of "
                      f"{len(timed)} timed; {src}, g++/gcc -O2 single thread (taskset -c 0); "
                      f"{t:.4f} s per {kind}-cycle; host {_cpu_model()}, {os.cpu_count()} CPUs"}


def build_sources():
    """Which sources the loaded libpgmg.so was built from (its pgmg_source_hash stamp) against
    the sources of this tree (_pkgload.source_hash): a prebuilt library that travelled with the
    tree is shown to match it, or not."""
    try:
        import _pkgload
        pg = _pkgload.load()
        lib = pg.load().pgmg_source_hash().decode()
        tree = _pkgload.source_hash()
        return {"library": lib, "tree": tree, "match": lib == tree}
    except Exception as e:  # reported, never fatal
        return {"error": str(e)[:200]}


def lib_build_id():
    """sha256 prefix of the libpgmg.so this run loads (names the build a profile measured)."""
    import hashlib
    import _pkgload
    p = pathlib.Path(_pkgload.PKG_DIR) / "libpgmg.so"
    try:
        return "libpgmg.so sha256:" + hashlib.sha256(p.read_bytes()).hexdigest()[:16]
    except OSError:
        return None


def kernel_key(name):
    """rocprofv3 kernel name -> the symbol key bench.py uses: 'k_pre<double,false,...>'."""
    name = name.split("(")[0].replace("void ", "").replace("pgmg::", "")
    return name.replace(" ", "").strip()


def pmc_child(args):
    """The program the live PMC passes profile: the timed call's kernels (a 3-cycle call:
    first k_pre, two cross-cycle k_postpre, the carry pass; then a 2-cycle call that takes the
    carry: the recompute form and another carry pass) of every leg and the per-op study's
    calls, then exit."""
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    legs = [0]
    if args.cycle == "V" and args.general_rhs == "auto":
        legs.append(pg.PGMG_FLAG_STORED_RHS)
    if args.cycle == "V" and args.dtype == "f64" and args.fast_mode == "auto":
        legs.append(pg.PGMG_FLAG_FAST)
    for flags in legs:
        with pg.Solver(args.n, flags=flags, dtype=args.dtype) as s:
            s.set_problem()
            {"V": s.vcycle, "W": s.wcycle, "F": s.fcycle}[args.cycle](3 if args.cycle != "W" else 1)
            if args.cycle == "V":
                s.vcycle(2)
            s.sync()
    if args.ops == "auto" and args.cycle == "V" and args.dtype == "f64":
        import torch
        cases, keep = op_cases(pg, args.n)
        for case in cases:
            for _ in range(2):
                case[1]()
        torch.cuda.synchronize()
        del keep


# algorithmic bytes per interior point of each op (fine grid n = (N-2)^2,
# coarse nc = (Nc-2)^2): Jacobi sweep 24 (read x, f; write x_new), residual 24, restriction
# 8 per fine + 8 per coarse point, prolongation 16 per fine (RMW) + 8 per coarse point
def op_cases(pg, n, device="cuda:0"):
    """The per-op study (ParallelTestRunner.cu:231-468 times ComputeJacobi(v = 100),
    ComputeResidual, ComputeRestriction, ComputeProlungator) on reference-layout device arrays
    at grid n: [(name, call, bytes per call, kernel keys, sweeps)], and the arrays."""
    import torch
    dev = torch.device(device)
    h = 1.0 / (n - 1)
    nc = (n - 1) // 2 + 1
    fine, coarse = float((n - 2) ** 2), float((nc - 2) ** 2)
    x = torch.zeros((n, n), dtype=torch.float64, device=dev)
    f = torch.empty_like(x)
    pg.ops.rhs(f, h)
    tmp = torch.empty_like(x)
    r = torch.zeros_like(x)
    c = torch.zeros((nc, nc), dtype=torch.float64, device=dev)
    e = torch.ones((nc, nc), dtype=torch.float64, device=dev)
    def sweep(check, pair=None):
        # trace keys: k_op_sweep<U,CHECK,SEED,NT> (the checked smoother's ping-pong sweeps),
        # k_op_sweep_ip<U,NT> / k_op_sweep2_ip<U,NT> (the in-place single / paired sweeps), and
        # k_op_defer_scatter (every in-place pass's deferred tile edges: part of the op's cost,
        # counted as 0 sweeps)
        def m(k):
            if not check:
                return (k.startswith("k_op_sweep2_ip") if pair is True else
                        k.startswith("k_op_sweep_ip") if pair is False else
                        k.startswith("k_op_sweep_ip") or k.startswith("k_op_sweep2_ip")) or \
                    k.startswith("k_op_defer_scatter")
            return k.startswith("k_op_sweep<")   # v = 1 checked: two ping-pong sweeps
        return m

    def named(prefix):
        return lambda k: k.startswith(prefix)

    # (name, call, bytes per call counted per sweep, trace-key matcher, sweeps,
    # passes over the grid per call: a paired in-place pass reads x and f and writes x ONCE for
    # two sweeps, so its one-pass bytes are 24 B per point, not 48)
    cases = [
        ("jacobi v=0 (one sweep in place on x: k_op_sweep_ip + the scatter of its deferred "
         "tile edges)",
         lambda: pg.ops.jacobi(x, f, h, 0, eps=-1.0, tmp=tmp, count=False), 24 * fine, sweep(False, False), 1, 1),
        ("jacobi v=1 (2 sweeps, no early exit: Parallel::ComputeJacobi's call in the V-cycle; "
         "one paired pass in place, k_op_sweep2_ip + the scatter)",
         lambda: pg.ops.jacobi(x, f, h, 1, eps=-1.0, tmp=tmp, count=False), 2 * 24 * fine, sweep(False, True), 2, 1),
        ("jacobi v=100 (101 sweeps, no early exit: the per-op study's ComputeJacobi call; one "
         "single and 50 paired passes)",
         lambda: pg.ops.jacobi(x, f, h, 100, eps=-1.0, tmp=tmp, count=False), 101 * 24 * fine, sweep(False),
         101, 51),
        ("jacobi v=1 with the smoother's early-exit checks (JacobiSmoother::smooth)",
         lambda: pg.ops.jacobi(x, f, h, 1, eps=1e-7, tmp=tmp, count=False), 2 * 24 * fine,
         sweep(True), 2, 2),
        ("residual (ComputeResidual)", lambda: pg.ops.residual(r, x, f, h), 24 * fine,
         named("k_op_residual"), 0, 1),
        ("restriction (ComputeRestriction)", lambda: pg.ops.restrict(r, c), 8 * fine + 8 * coarse,
         named("k_op_restrict"), 0, 1),
        ("prolongation, symmetric over the reference's launch grid (ComputeProlungator, "
         "num_thread 32)",
         lambda: pg.ops.prolong(e, r, mode=pg.PGMG_PROLONG_SYMMETRIC, num_thread=32),
         16 * fine + 8 * coarse, named("k_op_prolong<1>"), 0, 1),
        ("prolongation, the CPU path's (MultiGrid.hpp:208-226)",
         lambda: pg.ops.prolong(e, r, mode=pg.PGMG_PROLONG_REFERENCE), 16 * fine + 8 * coarse,
         named("k_op_prolong<0>"), 0, 1),
    ]
    return cases, (x, f, tmp, r, c, e)


def op_row(name, nbytes, keys, sweeps, passes, ms, trace, pmc, pmc_source):
    """One row of the per-op table.  `frac` is the one-pass roofline fraction: the call's
    passes x the bytes one pass moves (24 B per point for a sweep, single or paired) over its
    time -- physically bounded by the copy ceiling.  A multi-sweep call also gets
    `sweep_equiv_frac` (SURVEY §8(d)'s 24 B per SWEEP over the same time; above 1 when two
    sweeps share one pass).  rocprof: the kernels' average from the trace pass (the scatter of
    the in-place passes' deferred edges included, as 0 sweeps); PMC: `traffic_ratio` of the
    call's main kernel, HBM bytes per launch (live rocprofv3 passes of this build) over its
    one-pass algorithmic bytes."""
    per_pass = nbytes / sweeps if sweeps else nbytes
    one = passes * per_pass
    row = {"op": name, "ms_per_call": round(ms, 5), "bytes_per_call": nbytes,
           "passes_per_call": passes, "one_pass_bytes": per_pass,
           "achieved_gbps": round(one / (ms * 1e-3) / 1e9, 1),
           "frac": round(one / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
    if sweeps:
        row["ms_per_sweep"] = round(ms / sweeps, 5)
        if sweeps > passes:
            row["sweep_equiv_gbps"] = round(nbytes / (ms * 1e-3) / 1e9, 1)
            row["sweep_equiv_frac"] = round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
    # rocprof: the case's main kernels (the trace pass ran every case 3 times, so a key shared
    # by several cases -- the in-place single sweep, the scatter -- averages over them)
    tk = [(k, v) for k, v in (trace or {}).items() if keys(k) and not k.startswith("k_op_defer_scatter")]
    if tk:
        n = sum(v[0] for _, v in tk)
        avg = sum(v[0] * v[1] for _, v in tk) / n
        row["kernel_rocprof"] = {k: {"launches": v[0], "ms_per_launch": round(v[1], 5)} for k, v in tk}
        row["ms_per_launch_rocprof"] = round(avg, 5)
        row["frac_rocprof"] = round(per_pass / (avg * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
        sc = [v for k, v in (trace or {}).items() if keys(k) and k.startswith("k_op_defer_scatter")]
        if sc:
            row["scatter_ms_per_launch_rocprof"] = round(sc[0][1], 5)
    if pmc:
        mk = [k for k in pmc if keys(k) and not k.startswith("k_op_defer_scatter")]
        if mk:
            k = max(mk, key=lambda q: pmc[q])
            row.update({"pmc_kernel": k, "traffic": pmc[k],
                        "traffic_ratio": round(pmc[k] / per_pass, 4), "traffic_source": pmc_source})
    return row


def op_study(pg, n, trace, pmc=None, pmc_source=None, reps=5):
    """Each op of op_cases called `reps` times after one warmup call on the null stream,
    timed with events around each call (median); beside it the op's kernels' rocprof average
    from the trace pass and their HBM traffic from the PMC passes (same box, same build)."""
    import torch
    cases, keep = op_cases(pg, n)
    out = []
    for name, call, nbytes, keys, sweeps, passes in cases:
        call()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            call()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        out.append(op_row(name, nbytes, keys, sweeps, passes, statistics.median(ts), trace, pmc,
                          pmc_source))
    del keep
    torch.cuda.empty_cache()
    return out


def trace_child(args):
    """The program the kernel-trace pass profiles: the timed call of the main leg (a fresh
    problem, warmup cycles, then `steps` cycles in one call), then exit."""
    import torch  # noqa: F401
    import _pkgload
    pg = _pkgload.load()
    with pg.Solver(args.n, dtype=args.dtype) as s:
        run = {"V": s.vcycle, "W": s.wcycle, "F": s.fcycle}[args.cycle]
        # TRACE_PREWARM pre-warm calls (clocks ramp up on a GPU that sat idle during the CPU
        # baselines; one call of ~35 ms left the r04 final3 box's trace 5% slower than the
        # event-timed run), then the timed call's shape: a fresh problem, warmup cycles, `steps`
        for _ in range(TRACE_PREWARM):
            s.set_problem()
            run(args.steps)
            s.sync()
        s.set_problem()
        run(max(args.warmup, 0))
        s.sync()
        run(args.steps)
        s.sync()
    if args.ops == "auto" and args.cycle == "V" and args.dtype == "f64":
        import torch
        cases, keep = op_cases(pg, args.n)
        for case in cases:
            for _ in range(3):
                case[1]()
        torch.cuda.synchronize()
        del keep


def _keep_profile(args, src, name):
    if args.save_profiles and src:
        d = pathlib.Path(args.save_profiles)
        d.mkdir(parents=True, exist_ok=True)
        shutil.copy(src, d / name)


def live_trace(args):
    """rocprofv3 --kernel-trace --stats over trace_child on THIS box, before this process
    touches the GPU: {kernel key: (calls, average ms)} from its kernel_stats.csv, or
    (None, reason)."""
    import csv
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    d = tempfile.mkdtemp(prefix="pgmg_trace_")
    cmd = ["timeout", "-s", "KILL", "300", prof, "--kernel-trace", "--stats", "--output-format",
           "csv", "-d", d, "-o", "run", "--", sys.executable, str(ROOT / "bench.py"),
           "--trace-child", "--n", str(args.n), "--dtype", args.dtype, "--cycle", args.cycle,
           "--steps", str(args.steps), "--warmup", str(args.warmup), "--ops", args.ops]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=330)
        files = list(pathlib.Path(d).rglob("*kernel_stats.csv"))
        if r.returncode != 0 or not files:
            return None, f"rocprofv3 --kernel-trace failed (rc={r.returncode})"
        _keep_profile(args, files[0], "trace_kernel_stats.csv")
        out = {}
        for row in csv.DictReader(open(files[0])):
            out[kernel_key(row["Name"])] = (int(row["Calls"]), float(row["AverageNs"]) / 1e6, None, None)
        # the timed call's own launches of the finest-level cross-cycle pass: the last steps - 1
        # in start order (the timed call is the child's last; the fresh-problem calls before it
        # launch fewer, their early check cycles being unfused): the launches the event timing
        # averages
        traces = list(pathlib.Path(d).rglob("*kernel_trace.csv"))
        if traces and args.cycle == "V":
            per = {}
            for row in csv.DictReader(open(traces[0])):
                dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                per.setdefault(kernel_key(row["Kernel_Name"]), []).append(
                    (int(row["Start_Timestamp"]), dur))
                # per launch grid too: the levels table (levels_table) tells the levels apart
                GRID["trace"].setdefault((kernel_key(row["Kernel_Name"]), grid_total(row)), []).append(dur)
            last = args.steps - 1
            for k, v in per.items():
                if k.startswith("k_postpre_lds") and last > 0 and len(v) > last:
                    v.sort()
                    t = [x[1] for x in v[-last:]]
                    out[k] = out[k][:2] + (sum(t) / len(t) / 1e6, len(t))
        return out, ("rocprofv3 --kernel-trace --stats of a child run of the timed call "
                     f"({args.warmup} + {args.steps} cycles, one call each, main leg, after "
                     f"{TRACE_PREWARM} pre-warm calls of {args.steps}) on this box; the dominant "
                     f"kernel's time is the mean over the timed call's own launches")
    except (subprocess.SubprocessError, OSError, KeyError, ValueError) as e:
        return None, f"rocprofv3 --kernel-trace failed: {e}"
    finally:
        shutil.rmtree(d, ignore_errors=True)


# per (kernel key, launch grid): trace durations (ns) and PMC counters, for the levels table
GRID = {"trace": {}, "pmc": {}}


def grid_total(row):
    """Work-items of a launch from a rocprofv3 CSV row."""
    if "Grid_Size" in row:
        return int(row["Grid_Size"])
    return int(row.get("Grid_Size_X", 1)) * int(row.get("Grid_Size_Y", 1)) * int(row.get("Grid_Size_Z", 1))


def fused_grid(N):
    """Work-items of a coarse level's k_pre / k_post launch on one GPU (fused_geometry of
    pgmg_fused.hip restated: the levels table tells the levels apart by it)."""
    rows = (N - 1) // 2
    pts = 2 * rows * N
    target = min(3072, max(512, pts // 21845)) if pts > (1 << 23) else max(256, pts // 8192)
    waves = (N - 2 + 119) // 120
    wpb = min(waves, 4)
    gx = (waves + wpb - 1) // wpb
    gymax = max(1, target // gx)
    r = max(2, (rows + gymax - 1) // gymax)
    r = max(1, min(r, rows))
    gy = (rows + r - 1) // r
    return gx * 64 * wpb * gy


def levels_table(n, grid, fine_bytes):
    """Per bulk level and pass of a V-cycle at grid n: mean duration (us, all launches of the
    trace child), algorithmic GB/s and the HBM traffic ratio (2 x FETCH_SIZE + WRITE_SIZE of
    the PMC child over the algorithmic bytes).  Levels below the finest enter with x0 = 0:
    k_pre reads f, writes rc (8 B per point + 8 per coarse point), k_post reads f and the
    correction and writes x2 (16 + 8); the finest passes' bytes come from the library
    (fine_bytes: {kernel key: bytes per launch}).  The small levels' 2D tile passes (N <= 513)
    are launch-bound and listed by kernel only."""
    lv = {}
    N = n // 2 + 1
    while N >= 129:
        lv[fused_grid(N)] = N
        N = N // 2 + 1
    rows = []
    for (key, g), ds in sorted(grid["trace"].items(), key=lambda kv: (-sum(kv[1]) / len(kv[1]))):
        if key in fine_bytes:
            Nl, alg, what = n, fine_bytes[key], key.split("<")[0]
        elif (key.startswith("k_pre<") or key.startswith("k_post<")) and g in lv:
            Nl = lv[g]
            Nc = Nl // 2 + 1
            fp, cp = float((Nl - 2) ** 2), float((Nc - 2) ** 2)
            alg = 8 * fp + 8 * cp if key.startswith("k_pre<") else 16 * fp + 8 * cp
            what = key.split("<")[0]
        elif key.startswith("k_pre_tile") or key.startswith("k_post_tile"):
            Nl, alg, what = None, None, key.split("<")[0]
        else:
            continue
        us = sum(ds) / len(ds) / 1e3
        c = grid["pmc"].get((key, g), {})
        hbm = None
        if c.get("FETCH_SIZE") and c.get("WRITE_SIZE"):
            hbm = (2 * sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"]) +
                   sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])) * 1024.0
        rows.append({"N": Nl, "pass": what, "kernel": key, "launches": len(ds), "us": round(us, 2),
                     "alg_gbps": round(alg / us * 1e-3, 1) if alg else None,
                     "traffic_ratio": round(hbm / alg, 3) if (hbm and alg) else None})
    rows.sort(key=lambda r: (-(r["N"] or 0), r["pass"]))
    return rows


def launch_ranks(args):
    """--gpus N > 1 without a launcher: N rank processes under torch.distributed.run, started
    as a child process (never an exec) before this process touches the GPU; returns its exit
    status.  The ranks' stdout is this process's: rank 0 prints the JSON line."""
    import socket
    harness = (os.environ.get("PGMG_BENCH_SOLO") == "1" or
               os.environ.get("PGMG_BENCH_TRANSPORT") == "host")
    stub = os.environ.get("PGMG_BENCH_LAUNCH_STUB") == "1"
    if not (harness or stub):
        import torch   # device_count does not initialise the GPU (hipGetDeviceCount only)
        n = torch.cuda.device_count()
        if n < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, this box has {n} "
                  "(PGMG_BENCH_SOLO=1 or PGMG_BENCH_TRANSPORT=host run the ranks on one GPU as a "
                  "harness test)", file=sys.stderr)
            return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    # torch.distributed.run's parser rejects a script argument that abbreviates one of its own
    # options ("--n" could be --nnodes / --nproc-per-node ...): pass the grid as --N
    fwd = ["--N" if a == "--n" else ("--N=" + a[4:] if a.startswith("--n=") else a)
           for a in sys.argv[1:]]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={port}", str(ROOT / "bench.py")] + fwd
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def live_pmc(args):
    """HBM bytes per launch of every kernel of a short child run of THIS build on THIS box:
    one rocprofv3 pass per counter (FETCH_SIZE, WRITE_SIZE; they do not fit one pass), bytes =
    2 x FETCH_SIZE + WRITE_SIZE (KiB; MI355X_MICROARCH.md's gfx950 corrections: FETCH_SIZE
    counts half of a 16 B/lane streaming read, WRITE_SIZE is exact).  Runs before this
    process touches the GPU; returns ({key: bytes}, note) or (None, reason)."""
    import csv
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="pgmg_pmc_")
        cmd = ["timeout", "-s", "KILL", "150", prof, "--pmc", ctr, "--output-format", "csv",
               "-d", d, "-o", "run", "--", sys.executable, str(ROOT / "bench.py"), "--pmc-child",
               "--n", str(args.n), "--dtype", args.dtype, "--cycle", args.cycle,
               "--general-rhs", args.general_rhs, "--fast-mode", args.fast_mode, "--ops", args.ops]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=180)
            files = list(pathlib.Path(d).rglob("*counter_collection.csv"))
            if r.returncode != 0 or not files:
                return None, f"rocprofv3 --pmc {ctr} failed (rc={r.returncode})"
            _keep_profile(args, files[0], f"pmc_{ctr}.csv")
            for row in csv.DictReader(open(files[0])):
                if row.get("Counter_Name") == ctr:
                    vals.setdefault(kernel_key(row["Kernel_Name"]), {}).setdefault(ctr, []).append(
                        float(row["Counter_Value"]))
                    GRID["pmc"].setdefault((kernel_key(row["Kernel_Name"]), grid_total(row)), {}).setdefault(
                        ctr, []).append(float(row["Counter_Value"]))
        except (subprocess.SubprocessError, OSError, KeyError, ValueError) as e:
            return None, f"rocprofv3 --pmc {ctr} failed: {e}"
        finally:
            shutil.rmtree(d, ignore_errors=True)
    out = {}
    for k, v in vals.items():
        if v.get("FETCH_SIZE") and v.get("WRITE_SIZE"):
            fetch = sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"])
            write = sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"])
            out[k] = (2 * fetch + write) * 1024.0
    return out, "live rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this build (bench.py --pmc)"


def golden_hash(kind, n, cycles):
    """The reference's FNV-64 of phi after `cycles` cycles from phi0 = 0 (fixture data:
    tests/golden/cycles.json, generated by tests/golden/make_golden.py), or None."""
    p = ROOT / "tests" / "golden" / "cycles.json"
    if not p.exists():
        return None
    for c in json.loads(p.read_text()):
        if c["kind"] == kind and c["N"] == n and c["eps"] == 1e-7 and len(c["cycles"]) >= cycles:
            return c["cycles"][cycles - 1]["hash"]
    return None


def rank_split_summary(allr, inst_dt, steps):
    """Per-rank (device ms per cycle, ms inside collective groups per cycle, groups per cycle),
    rank order -> the line's rank_split: compute vs RCCL time, median and max over ranks."""
    comp = [r[0] - r[1] for r in allr]
    comm = [r[1] for r in allr]
    return {
        "what": "per rank, per cycle of the instrumented repetitions (hipEvents around every "
                "collective group on the rank's stream, PGMG_FLAG_TIME_COMM): compute = the "
                "call's device time minus the time inside collectives (RCCL transfer + waiting "
                "for a peer)",
        "compute_ms": {"median": round(statistics.median(comp), 4), "max": round(max(comp), 4),
                       "per_rank": [round(x, 4) for x in comp]},
        "rccl_ms": {"median": round(statistics.median(comm), 4), "max": round(max(comm), 4),
                    "per_rank": [round(x, 4) for x in comm]},
        "groups_per_cycle": round(allr[0][2], 2),
        "instrumented_ms_per_step": round(inst_dt * 1e3 / steps, 4)}


PASS_NAMES = {
    0: "k_sweep (finest-level Jacobi sweep, unfused path)",
    1: "k_pre (finest level: 2 Jacobi sweeps + residual + restriction, fused)",
    2: "k_post (finest level: prolongation + 2 Jacobi sweeps, fused)",
    3: "k_postpre (finest level, between cycles: prolongation + 2+2 Jacobi sweeps + residual + "
       "restriction, fused)",
    4: "carry pass (the call's last finest pass: k_postpre that stores the call's result instead "
       "of the next pre-smooth, whose restriction is carried to the next call)",
    5: "recompute form (the first finest pass of a call that took the carry: k_postpre that "
       "recomputes the carried pre-smooth from phi in registers)",
}


def roofline_rows(leg, pmc, pmc_source, trace, trace_note):
    """One roofline row per finest-level pass timed in the instrumented repetitions, the
    dominant (largest total time) first.  Kernel symbol and algorithmic bytes per launch come
    from the library (pgmg_fine_pass_info: the variant that ran and what it read and wrote);
    `traffic` is the same symbol's HBM bytes per launch from the live PMC passes of this build
    (null without them: never another build's); rocprof columns from the trace pass."""
    roof = []
    for w, cnt, ms in leg["passes"]:
        if not cnt or ms <= 0:
            continue
        sym, nb = leg.get("info", {}).get(w, ("", 0.0))
        key = kernel_key(sym) if sym else None
        nbytes = nb if nb > 0 else leg["bytes"][w]
        ach = nbytes / (ms * 1e-3) / 1e9
        traffic = pmc.get(key) if (pmc is not None and key) else None
        name = PASS_NAMES[w] + ("; f regenerated in-kernel" if leg.get("gen") else "; f streamed")
        if leg.get("fast"):
            name += " — FAST mode"
        roof.append({"bound": "hbm", "kernel": name, "symbol": key,
                     "symbol_source": "pgmg_fine_pass_info (the launched kernel)" if key else
                                      "unavailable (hipKernelNameRefByPtr returned nothing)",
                     "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBPS, 4),
                     "traffic": traffic,
                     "traffic_source": pmc_source if traffic else None,
                     "traffic_ratio": round(traffic / nbytes, 4) if traffic else None,
                     "bytes_per_launch": nbytes, "launches_timed": cnt,
                     "ms_per_launch": round(ms, 5),
                     "ms_per_launch_reps": [round(x, 5) for x in leg["passes_reps"][w]]})
        tr = trace.get(key) if (trace is not None and key) else None
        if tr is not None:
            tms = tr[2] if tr[2] is not None else tr[1]
            ach_r = nbytes / (tms * 1e-3) / 1e9
            roof[-1].update({"ms_per_launch_rocprof": round(tms, 5),
                             "ms_per_launch_rocprof_all_launches": round(tr[1], 5),
                             "launches_rocprof": tr[0],
                             "launches_rocprof_timed": tr[3],
                             "frac_rocprof": round(ach_r / HBM_PEAK_GBPS, 4),
                             "event_vs_rocprof": round(ms / tms, 4),
                             "rocprof_source": trace_note})
    roof.sort(key=lambda r: -r["ms_per_launch"] * r["launches_timed"])
    return roof


# the measured copy ceiling (MI355X_MICROARCH.md: 6.29 TB/s float4 copy = 0.79 of 8 TB/s); an
# algorithmic fraction above it means a mis-charged kernel, not a fast one
FRAC_CEILING = 0.79


def implausible_fracs(obj, path="line"):
    """Every roofline-fraction field above the copy ceiling (keys named frac*, except the
    op table's sweep_equiv_frac, which counts two sweeps of one pass) and every traffic source
    that does not name this build: [(path, what)]."""
    bad = []
    if isinstance(obj, dict):
        for k, v in obj.items():
            p = f"{path}.{k}"
            if isinstance(v, (int, float)) and k.startswith("frac") and v > FRAC_CEILING:
                bad.append((p, f"{v} > {FRAC_CEILING}"))
            if k == "traffic_source" and v is not None and "sha256:" not in str(v):
                bad.append((p, f"does not name this build: {v}"))
            bad += implausible_fracs(v, p)
    elif isinstance(obj, list):
        for i, v in enumerate(obj):
            bad += implausible_fracs(v, f"{path}[{i}]")
    return bad


def main():
    args = parse()
    if args.pmc_child:
        return pmc_child(args)
    if args.trace_child:
        return trace_child(args)
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch N ranks for "
                 f"--gpus N (or run plain `python bench.py --gpus N`, which launches them)")
    if os.environ.get("PGMG_BENCH_LAUNCH_STUB") == "1":
        # CPU test of the launcher (tests/test_bench_cpu.py): report the rank, touch no GPU
        # one write(2) per line: the ranks share the launcher's stdout, and print()'s separate
        # writes of the text and the newline can interleave two ranks' lines
        os.write(1, (json.dumps({"stub_rank": rank, "world": world, "local_rank": local_rank,
                                 "n": args.n}) + "\n").encode())
        return None
    # CPU baselines first, before this process touches the GPU (child processes)
    cpu = cpu1 = cpu4 = None
    if world == 1 and rank == 0 and args.cpu_baseline == "auto" and args.dtype == "f64":
        try:
            # two timed cycles (~2 x 8-10 s at N = 16385 for the reference): a spread
            cpu = cpu_baseline(args.cpu_n or args.n, cycles=2, kind=args.cycle)
        except Exception as e:  # reported, not fatal
            cpu = {"value": None, "unit": f"{args.cycle}-cycles/s", "cores": 1, "kind": "port",
                   "sample": f"failed: {e}"}
        try:   # BASELINE config 1: mg_cpu_exec's own size, N = 513 (1 warmup + median of 5)
            cpu1 = cpu_baseline(513, cycles=6, kind="V", skip=1)
        except Exception as e:
            cpu1 = {"value": None, "unit": "V-cycles/s", "cores": 1, "kind": "port",
                    "sample": f"failed: {e}"}
        if args.cycle == "V" and args.n != 4097:
            try:   # BASELINE.md §2's middle size, N = 4097 (1 warmup + median of 3, ~5 s)
                cpu4 = cpu_baseline(4097, cycles=4, kind="V", skip=1)
            except Exception as e:
                cpu4 = {"value": None, "unit": "V-cycles/s", "cores": 1, "kind": "port",
                        "sample": f"failed: {e}"}
    pmc, pmc_note = None, "off"
    if world == 1 and rank == 0 and args.pmc == "auto":
        pmc, pmc_note = live_pmc(args)
    pmc_source = f"{pmc_note}; {lib_build_id()}" if pmc is not None else None
    trace, trace_note = None, "off"
    if world == 1 and rank == 0 and args.trace == "auto":
        trace, trace_note = live_trace(args)
    import torch  # noqa: F401  (loads the ROCm runtime first; see _capi.load)
    import _pkgload
    pg = _pkgload.load()

    dist = None
    # PGMG_BENCH_SOLO=1 (harness test on a one-GPU box only): every rank on device 0 with the
    # null transport (PGMG_FLAG_SOLO: no messages, results meaningless); the line says so
    solo = world > 1 and os.environ.get("PGMG_BENCH_SOLO") == "1"
    # PGMG_BENCH_TRANSPORT=host (harness test on a one-GPU box): every rank on device 0, the
    # strips' messages through the host-staged transport over the gloo group
    # (PGMG_FLAG_HOST_TRANSPORT): a real multi-process solve, parity-checked, not a timing
    host_tp = world > 1 and not solo and os.environ.get("PGMG_BENCH_TRANSPORT") == "host"
    device = 0 if (world == 1 or solo or host_tp) else local_rank
    if world > 1 and device >= torch.cuda.device_count():
        sys.exit(f"bench.py: rank {rank} needs GPU {device}, this box has "
                 f"{torch.cuda.device_count()} (PGMG_BENCH_SOLO=1 or PGMG_BENCH_TRANSPORT=host "
                 f"for a one-GPU harness test)")
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(device)
        dist.init_process_group("gloo")

    def barrier():
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x):
        if dist is None:
            return x
        tt = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    want = golden_hash(args.cycle, args.n, args.warmup + args.steps) if args.dtype == "f64" else None
    # the latency floor of the strips' collectives on this device (world-1 RCCL communicator,
    # rank 0 only): what DESIGN §5 prices a dependent exchange group at
    rccl_floor = None
    if rank == 0 and not (solo or host_tp):
        try:
            rccl_floor = dict(pg.rccl_latency(device, 200), what=(
                "world-1 RCCL communicator on this GPU, hipEvents over 200 calls: a grouped "
                "send+recv of the finest halo at 16385 (2 rows, 262 KB) to itself, allreduce(sum, "
                "3 doubles), allreduce(min, 9 u32); a lower bound of one exchange group between "
                "ranks (no xGMI hop, no peer to wait for)"))
            rccl_floor = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in rccl_floor.items()}
        except Exception as e:  # reported, not fatal
            rccl_floor = {"error": str(e)[:200]}

    def new_solver(flags, n=None):
        kw = dict(device=device, dtype=args.dtype)
        if host_tp:
            kw.update(transport=pg.HostTransport(), rank=rank, world=world)
        elif world > 1:   # a fresh RCCL communicator per context
            t = torch.tensor(list(pg.unique_id()) if rank == 0 else [0] * 128, dtype=torch.uint8)
            dist.broadcast(t, 0)
            kw.update(rank=rank, world=world, uid=bytes(t.tolist()))
        return pg.Solver(args.n if n is None else n,
                         flags=flags | (pg.PGMG_FLAG_SOLO if solo else 0), **kw)

    def parity_of(leg):
        p = leg["parity"]
        if not p or any(x is None for x in p):
            return None
        return all(p)

    def gather(x):
        """x from every rank (rank order); [x] on one rank"""
        if dist is None:
            return [x]
        out = [None] * world
        dist.all_gather_object(out, x)
        return out

    def run_leg(extra_flags, reps, n=None, warm=None, steps=None, want_hash=None,
                inst_reps=INST_REPS):
        """`reps` clean repetitions on one context (set_problem restarts each from phi0 = 0)
        + inst_reps repetitions with per-pass events on a second (per pass, the median over
        them; on row strips also events around every collective group: per-rank compute vs
        RCCL time); returns times, parity, passes"""
        warm = max(args.warmup, 0) if warm is None else warm
        steps = args.steps if steps is None else steps
        want_hash = want if want_hash is None else want_hash
        out = {"times": [], "parity": [], "passes": [], "inst_dt": None, "split": []}
        inst_dt, inst_passes = [], []
        for inst in (False, True):
            fl = extra_flags
            if inst:
                fl |= pg.PGMG_FLAG_TIME_FINE | (pg.PGMG_FLAG_TIME_COMM if world > 1 else 0)
            s = new_solver(fl, n=n)
            run = {"V": s.vcycle, "W": s.wcycle, "F": s.fcycle}[args.cycle]
            for _ in range(inst_reps if inst else reps):
                s.set_problem()
                run(warm)
                s.sync()
                for w in PASSES:  # drop warmup events
                    s.fine_pass_time(w)
                s.comm_stats()
                barrier()
                s.sync()
                t0 = time.perf_counter()
                run(steps)
                t_enq = time.perf_counter()
                s.sync()
                barrier()
                t1 = time.perf_counter()
                dt = max_over_ranks(t1 - t0)
                if inst:
                    inst_dt.append(dt)
                    inst_passes.append([tuple(s.fine_pass_time(w)) for w in PASSES])
                    # what those launches were: kernel symbol and algorithmic bytes per launch,
                    # from the library (the variant that ran, not one named from flags here)
                    out["info"] = {w: s.fine_pass_info(w) for w in PASSES}
                    out["bytes"] = {w: s.fine_pass_bytes(w) for w in PASSES}
                    if world > 1:   # this rank's device time of the call, its collectives' time
                        groups, cms = s.comm_stats()
                        out["split"].append((s.last_elapsed_ms(), cms, groups))
                else:
                    out["times"].append(dt)
                    out["enq"] = t_enq - t0
                    out["dev_ms"] = s.last_elapsed_ms()
                    if not solo:
                        h = s.solution_hash(0)
                        out["parity"].append(None if want_hash is None or h is None else h == want_hash)
                    out["spec"] = (s.dist_info(), s.spec_levels())
                    out["carry"] = s.carry_info()
            out["vbytes"] = s.vcycle_bytes()
            out["fused"] = s.fused
            out["levels"] = s.levels()
            out["gen"] = s.fused and s.fine_pass_bytes(3) < s.fine_pass_bytes(0)
            out["r2"] = world > 1 and not s.dist_info()[0]
            out["comm_ranks"] = s.comm_ranks()
            s.close()
        out["inst_dt"] = statistics.median(inst_dt)
        out["passes"] = [(w, inst_passes[0][i][0], statistics.median(r[i][1] for r in inst_passes))
                         for i, w in enumerate(PASSES)]
        out["passes_reps"] = {w: [r[i][1] for r in inst_passes] for i, w in enumerate(PASSES)}
        if world > 1:
            # per rank (median over the instrumented repetitions): device ms of the timed call
            # per cycle, of which inside collective groups (transfer + waiting for a peer)
            mine = (statistics.median(x[0] for x in out["split"]) / steps,
                    statistics.median(x[1] for x in out["split"]) / steps,
                    statistics.median(x[2] for x in out["split"]) / steps)
            out["rank_split"] = rank_split_summary(gather(mine), out["inst_dt"], steps)
        return out

    main_leg = run_leg(0, max(1, args.reps))
    # BASELINE configs[3]'s grid (N = 32769) on the same N ranks: SURVEY §8(e) asks for
    # V-cycles/s at 1, 2, 4 and 8 GPUs at 16385 AND 32769; the N = 1 number is other_configs'
    # "configs[3]'s grid on ONE MI355X" (1 + 5 cycles, median of 3, the same shape)
    big_leg = None
    # (the host-staged transport runs it too: the harness test of this leg on a one-GPU box)
    if (world > 1 and not solo and args.cycle == "V" and args.dtype == "f64"
            and args.n == 16385 and args.big_grid == "auto"):
        bl = run_leg(0, 3, n=32769, warm=1, steps=5, want_hash=golden_hash("V", 32769, 6),
                     inst_reps=1)
        dt = statistics.median(bl["times"])
        broof = roofline_rows(bl, None, None, None, None)
        big_leg = {"config": "BASELINE configs[3]: V-cycle N=32768^2 on the same row strips "
                             f"x{world} ({'host-staged transport, every rank on GPU 0: harness test, not a measurement' if host_tp else 'RCCL halos'}); "
                             "its one-GPU number: other_configs of the N = 1 line",
                   "value": round(5 / dt, 3), "unit": "V-cycles/s", "n_gpus": world,
                   "ms_per_step": round(dt * 1e3 / 5, 4), "timed": "1 + 5 cycles, median of 3",
                   "parity": parity_of(bl),
                   "roofline": broof[0] if broof else None,
                   "rank_split": bl.get("rank_split")}
    gen_leg = None
    if (world == 1 and args.cycle == "V" and args.general_rhs == "auto" and main_leg["fused"]
            and main_leg["gen"]):
        gen_leg = run_leg(pg.PGMG_FLAG_STORED_RHS, 3)
        gen_leg["stored"] = True

    # BASELINE.json's other GPU configs on this one GPU (timed after the headline legs, each
    # with the reference's hash of its result; the 8-GPU configs' grids as one GPU's run)
    others = None
    if (world == 1 and args.other_configs == "auto" and args.cycle == "V" and args.dtype == "f64"
            and args.n == 16385):
        others = []

        def timed(s, run, warm, k, reps):
            ts = []
            for _ in range(reps):
                s.set_problem()
                run(warm)
                s.sync()
                t0 = time.perf_counter()
                run(k)
                s.sync()
                ts.append(time.perf_counter() - t0)
            return statistics.median(ts)

        with pg.Solver(4097, device=device) as s:   # configs[1]
            dt = timed(s, s.vcycle, 3, 40, 3)
            # the timed call's own result: phi after the last repetition's 3 + 40 cycles
            w43, h43 = golden_hash("V", 4097, 43), s.solution_hash(0)
            others.append({"config": "BASELINE configs[1]: 1xMI355X V-cycle, N=4096^2, 2+2 Jacobi, "
                                     "6 bulk levels, fp64",
                           "value": round(40 / dt, 2), "unit": "V-cycles/s",
                           "ms_per_step": round(dt * 1e3 / 40, 4), "timed": "3 + 40 cycles, median of 3",
                           "parity": None if w43 is None or h43 is None else h43 == w43,
                           "parity_detail": "FNV-64 of phi after the timed repetitions' 3 + 40 cycles "
                                            "against the reference's (tests/golden/cycles.json)"})
        with pg.Solver(32769, device=device) as s:  # configs[3]'s grid on one GPU
            dt = timed(s, s.vcycle, 1, 5, 3)
            w6, h6 = golden_hash("V", 32769, 6), s.solution_hash(0)
            others.append({"config": "BASELINE configs[3]'s grid (N=32768^2) on ONE MI355X: V-cycle, fp64 "
                                     "(the row-strip runs on N GPUs report it as big_grid)",
                           "value": round(5 / dt, 3), "unit": "V-cycles/s",
                           "ms_per_step": round(dt * 1e3 / 5, 4), "timed": "1 + 5 cycles, median of 3",
                           "parity": None if w6 is None or h6 is None else h6 == w6,
                           "parity_detail": "FNV-64 of phi after the timed repetitions' 1 + 5 cycles "
                                            "against the reference's (tests/golden/cycles.json: generated by "
                                            "oracle/mg_cpu_exec_port, confirmed by the reference's own "
                                            "MultigridSolver, profiles/r06/ref32769/)"})
            # configs[4]'s cycle: the FMG start (one F-cycle) then one W-cycle, fp64
            s.set_problem()
            t0 = time.perf_counter()
            s.fcycle(1)
            s.sync()
            t1 = time.perf_counter()
            s.wcycle(1)
            s.sync()
            t2 = time.perf_counter()
            w = golden_hash("G", 32769, 2)
            h = s.solution_hash(0)
            others.append({"config": "BASELINE configs[4]'s cycle (N=32768^2) on ONE MI355X: FMG start "
                                     "(one F-cycle) + one W-cycle, fp64 (fp32-vs-fp64 sweep: "
                                     "profiles/r02_fp32/)",
                           "f_cycle_s": round(t1 - t0, 4), "w_cycle_s": round(t2 - t1, 4),
                           "parity": None if w is None or h is None else h == w})

    # The reference's entry point as its harness drives it (ParallelTestRunner::run_v_cycle ->
    # ParallelMultiGridSolver::v_cycle once per cycle, ParallelTestRunner.cu:171-175): the C++
    # mirror host/gpu_exec on device arrays (phi updated in place, f regenerated), W untimed
    # + K timed one-cycle calls, its own wall clock ("Elapsed Time"); beside it the context
    # API with one-cycle calls (pgmg_vcycle(ctx, 1), no cross-cycle fusion between calls)
    dropin = None
    if world == 1 and args.cycle == "V" and args.dtype == "f64" and args.dropin == "auto":
        def single_calls(flags):
            """3 repetitions of W + K one-cycle calls on a fresh problem; K timed (median)"""
            ts = []
            s = new_solver(flags)
            for _ in range(3):
                s.set_problem()
                for _ in range(max(args.warmup, 0)):
                    s.vcycle(1)
                s.sync()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    s.vcycle(1)
                s.sync()
                ts.append(time.perf_counter() - t0)
            h = s.solution_hash(0)
            carry = s.carry_info()
            s.close()
            return statistics.median(ts), h, carry
        ctx_dt, h_ctx, ctx_carry = single_calls(0)
        nc_dt, h_nc, _ = single_calls(pg.PGMG_FLAG_NO_CARRY)
        exe = pathlib.Path(_pkgload.PKG_DIR) / "host" / "gpu_exec"
        runs = []
        for _ in range(3):
            r = subprocess.run([str(exe), "--n", str(args.n), "--cycles", str(args.steps),
                                "--warmup", str(max(args.warmup, 0)), "--v-only", "--hash"],
                               capture_output=True, text=True, timeout=600)
            out = r.stdout
            secs = [float(l.split("Elapsed Time:")[1].split()[0]) for l in out.splitlines()
                    if "Elapsed Time:" in l]
            hsh = [l.split("FNV-64:")[1].strip() for l in out.splitlines() if "FNV-64:" in l]
            mode = [l.split("phi arrays:")[1].strip() for l in out.splitlines() if "phi arrays:" in l]
            runs.append((r.returncode, secs[0] if secs else None, hsh[0] if hsh else None,
                         mode[0] if mode else None))
        ok = [x for x in runs if x[0] == 0 and x[1]]
        if ok:
            d_dt = statistics.median([x[1] for x in ok])
            dropin = {
                "what": "the reference's entry point: ParallelMultiGridSolver::v_cycle(phi, f, N, h) "
                        "called once per cycle by ParallelTestRunner::run_v_cycle (C++ mirror "
                        "host/gpu_exec --v-only), phi and f device arrays (pgmg_alloc_grid), phi "
                        "updated in place, f regenerated; timed by the harness's own wall clock",
                "value": round(args.steps / d_dt, 4), "unit": "V-cycles/s",
                "ms_per_step": round(d_dt * 1e3 / args.steps, 4),
                "timed": f"{max(args.warmup, 0)} warmup + {args.steps} calls, median of {len(ok)} runs",
                "phi_arrays": ok[0][3],
                "parity": None if want is None else all(x[2] == want for x in ok),
                "context_single_calls": {
                    "what": "pgmg_vcycle(ctx, 1) called once per cycle on the context's own grids "
                            "(each call after the first starts from the carry: the previous "
                            "call's last pass ran its pre-smooth)",
                    "value": round(args.steps / ctx_dt, 4), "unit": "V-cycles/s",
                    "ms_per_step": round(ctx_dt * 1e3 / args.steps, 4),
                    "parity": None if want is None or h_ctx is None else h_ctx == want,
                    "carry_took_made_dropped": list(ctx_carry),
                    "no_carry": {"what": "the same calls with PGMG_FLAG_NO_CARRY (k_pre + k_post "
                                         "at level 0 in every call)",
                                 "value": round(args.steps / nc_dt, 4), "unit": "V-cycles/s",
                                 "ms_per_step": round(nc_dt * 1e3 / args.steps, 4),
                                 "parity": None if want is None or h_nc is None else h_nc == want}},
                "dropin_over_context_time": round(d_dt / ctx_dt, 4),
            }
        else:
            dropin = {"what": "gpu_exec drop-in leg", "failed": [x[0] for x in runs]}

    # FAST mode (PGMG_FLAG_FAST): its rate, and phi after 10 cycles (SURVEY §8(c)'s window:
    # later, near convergence, a borderline early-exit check may decide differently) against
    # the EXACT default's (relative L2 and max-abs; tolerance in tests/test_gpu_fast.py)
    fast_leg = fast_cmp = None
    if (world == 1 and args.cycle == "V" and args.dtype == "f64" and args.fast_mode == "auto"
            and main_leg["fused"]):
        import numpy as np
        fast_leg = run_leg(pg.PGMG_FLAG_FAST, 3)
        sols = []
        for fl in (0, pg.PGMG_FLAG_FAST):
            s = new_solver(fl)
            s.set_problem()
            s.vcycle(10)
            sols.append((s.solution(), s.stats()[0]))
            s.close()
        (ref_phi, ref_sw), (got_phi, got_sw) = sols
        d = got_phi - ref_phi
        fast_cmp = {"cycles": 10, "tolerance": "tests/test_gpu_fast.py (3e-11 at N = 16385)",
                    "rel_l2_vs_exact": float(np.linalg.norm(d) / np.linalg.norm(ref_phi)),
                    "max_abs_vs_exact": float(np.max(np.abs(d))),
                    "sweep_counts_equal": ref_sw == got_sw}
        del sols, ref_phi, got_phi, d

    # the per-op study (Parallel::Compute* on reference-layout arrays), VERDICT r03 #3
    op_rows = None
    if world == 1 and args.cycle == "V" and args.dtype == "f64" and args.ops == "auto":
        op_rows = op_study(pg, args.n, trace, pmc, pmc_source)
        if args.save_profiles:
            pathlib.Path(args.save_profiles).mkdir(parents=True, exist_ok=True)
            (pathlib.Path(args.save_profiles) / "ops_table.json").write_text(
                json.dumps({"N": args.n, "build": lib_build_id(), "ops": op_rows}, indent=1))

    def roofline(leg):
        return roofline_rows(leg, pmc, pmc_source, trace, trace_note)

    if rank == 0:
        med = statistics.median(main_leg["times"])
        value = args.steps / med
        roof = roofline(main_leg)
        metric = METRIC if args.dtype == "f64" else METRIC.replace(", fp64", ", fp32 variant")
        if args.cycle != "V":
            metric = metric.replace("V-cycles/sec", f"{args.cycle}-cycles/sec")
        if args.n != 16385:
            metric = metric.replace("16384²", f"{args.n - 1}²")
        bulk, tail_top = main_leg["levels"]
        spec_info, spec_mask = main_leg["spec"]
        n = args.n
        line = {
            "metric": metric,
            "value": round(value, 4),
            "unit": f"{args.cycle}-cycles/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(med * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic: the reference's own problem, phi0=0, f=2*pi^2*sin(pi x)sin(pi y)",
            "config": {
                "workload": f"{args.cycle}-cycle N={n} ({n - 1}^2 cells), 2+2 Jacobi (v1=v2=1), "
                            f"11 coarsest sweeps, eps=1e-7 early exit, {bulk} bulk levels + "
                            f"one-workgroup LDS tail from N={tail_top} to N=5",
                "N": n, "bulk_levels": bulk, "tail_top": tail_top,
                "parallelism": "single-gpu" if world == 1 else (
                    f"row-strips x{world} (SOLO null transport on one GPU: harness test, "
                    f"not a measurement)" if solo else
                    f"row-strips x{world} (host-staged transport over gloo, every rank on "
                    f"GPU 0: harness test of the multi-process solve, not a measurement)"
                    if host_tp else f"row-strips x{world} (RCCL halos)"),
            },
            "repetitions": {"count": len(main_leg["times"]),
                            "ms_per_step": [round(t * 1e3 / args.steps, 4) for t in main_leg["times"]],
                            "median_ms_per_step": round(med * 1e3 / args.steps, 4),
                            "spread_pct": round(100 * (max(main_leg["times"]) - min(main_leg["times"]))
                                                / med, 2)},
            # the reference's own hash of phi after warmup + steps cycles from phi0 = 0, checked
            # after every repetition (null: no fixture for this N / cycle count)
            "parity": parity_of(main_leg),
            "parity_detail": {"expected_fnv64": want, "checked": main_leg["parity"],
                              "fixture": "tests/golden/cycles.json"},
            "roofline": roof[0] if roof else None,
            "roofline_other": roof[1:],
            "instrumented_ms_per_step": round(main_leg["inst_dt"] * 1e3 / args.steps, 4),
            "vcycle_algorithmic_gbps": round(main_leg["vbytes"] / med * args.steps / 1e9, 2),
            "vcycle_device_ms": round(main_leg["dev_ms"] / args.steps, 4),
            "host_enqueue_ms_per_step": round(main_leg["enq"] * 1e3 / args.steps, 4),
            # early-exit checks recorded and validated after each call (DESIGN.md §3 point 8)
            "speculative_checks": {"enabled": spec_info[0], "rollbacks": spec_info[1],
                                   "in_stream_level_mask": spec_mask},
            # the carry (pgmg_ctx.hip "carry"): the timed call starts from the warmup call's
            # carried pre-smooth and ends with the carry pass (19 k_postpre + 1 carry pass)
            "carry": {"took_made_dropped": list(main_leg.get("carry", ())),
                      "what": "calls that started from the previous call's carried pre-smooth, "
                              "carries made, carries dropped (check could fire), on the clean "
                              "repetitions' context"},
            "rccl_ranks": main_leg.get("comm_ranks"),
            "rccl_floor": rccl_floor,
            "cpu_baseline": cpu,
            "cpu_baseline_config1": cpu1,
            "cpu_baseline_4097": cpu4,
            # the host the CPU samples ran on: every sample uses ONE core (taskset -c 0); the
            # reference CPU rate moves ~2x from host to host of the pool, so
            # each sample carries its per-cycle times and their spread
            "cpu_host": {"model": _cpu_model(), "nproc": os.cpu_count(), "cores_used": 1},
            "pmc": pmc_note,
            "trace": trace_note,
            "build": lib_build_id(),
            "build_sources": build_sources(),
        }
        if others is not None:
            line["other_configs"] = others
        if big_leg is not None:
            line["big_grid"] = big_leg
        if dropin is not None:
            line["dropin"] = dropin
        if op_rows is not None:
            line["ops"] = {"what": "the per-op study at N = %d: the reference's op-level GPU "
                                   "entries (Parallel::Compute*, Parallel_Method.cu:144-199) on "
                                   "reference-layout device arrays; bytes per SURVEY §8(d) over "
                                   "the interior points; event time per call (median of 5) and "
                                   "the kernels' rocprofv3 average from the trace pass" % args.n,
                           "table": op_rows}
        if fast_leg is not None:
            fast_leg["fast"] = True
            fmed = statistics.median(fast_leg["times"])
            froof = roofline(fast_leg)
            line["fast_mode"] = {
                "what": "PGMG_FLAG_FAST: the finest cross-cycle pass with shared neighbour sums "
                        "and FMA residuals (not the reference's expression order: a tolerance, "
                        "not bitwise; SURVEY §8(c) FAST mode)",
                "value": round(args.steps / fmed, 4), "unit": "V-cycles/s",
                "ms_per_step": round(fmed * 1e3 / args.steps, 4),
                "repetitions": len(fast_leg["times"]),
                "vs_exact": fast_cmp,
                "roofline": froof[0] if froof else None,
            }
        if gen_leg is not None:
            gmed = statistics.median(gen_leg["times"])
            groof = roofline(gen_leg)
            line["general_rhs"] = {
                "what": "the same V-cycles with f streamed from HBM (PGMG_FLAG_STORED_RHS: the "
                        "rate a caller with its own right-hand side gets; 24 B per fine point in "
                        "the finest-level passes instead of 16)",
                "value": round(args.steps / gmed, 4), "unit": "V-cycles/s",
                "ms_per_step": round(gmed * 1e3 / args.steps, 4),
                "repetitions": len(gen_leg["times"]),
                "parity": parity_of(gen_leg),
                "roofline": groof[0] if groof else None,
            }
        if "rank_split" in main_leg:
            line["rank_split"] = main_leg["rank_split"]
        # every fraction physically possible (below the measured copy ceiling) and every
        # traffic figure from this build: an empty list
        if GRID["trace"] and world == 1 and args.cycle == "V":
            fine_bytes = {kernel_key(sym): b for sym, b in main_leg.get("info", {}).values() if sym}
            line["levels"] = {
                "what": "per bulk level and pass (rocprofv3 trace + PMC children of this build, "
                        "all their launches): mean us, algorithmic GB/s, HBM traffic ratio "
                        "(2 x FETCH_SIZE + WRITE_SIZE over the algorithmic bytes)",
                "table": levels_table(args.n, GRID, fine_bytes)}
        line["implausible"] = implausible_fracs(line)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and not line["build_sources"].get("match", False):
        # a library that does not carry this tree's source hash measured something else
        print("bench.py: libpgmg.so was not built from this tree's sources "
              f"({line['build_sources']}): rebuild (make -C "
              "parallel-geometric-multigrid-for-poisson-problem_amd)", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
