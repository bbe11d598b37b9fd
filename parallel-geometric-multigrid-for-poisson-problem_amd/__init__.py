"""MI355X-native geometric multigrid for the 2D Poisson problem (fp64; fp32 variant).

The hot path (Jacobi smoother, residual + norm, full-weighting restriction,
prolongation, V/W-cycles) is hand-written HIP for gfx950 in ``csrc/`` behind the C ABI
of ``include/pgmg.h`` (libpgmg.so).  This Python package is plumbing: a ctypes
wrapper used by the tests, ``bench.py`` and ``__graft_entry__``.  The C++ mirror of
the reference's own entry points (``Parallel``, ``ParallelMultiGridSolver``,
``ParallelTestRunner``, ``gpu_exec``) lives in ``host/``.

Import name: the directory name is not a Python identifier, so load it with
``_pkgload.load()`` from the repository root (registers it as ``pgmg_amd``).
"""
import ctypes as C
import pathlib
import contextlib
import subprocess

import numpy as np

from ._capi import (PGMG_FLAG_LOOPBACK, PGMG_FLAG_NO_CROSS, PGMG_FLAG_NO_GRAPH,
                    PGMG_FLAG_STORED_RHS, PGMG_FLAG_EXACT_DIST, PGMG_FLAG_SOLO,
                    PGMG_FLAG_TIME_FINE, PGMG_PRECISION_FP32, PGMG_PRECISION_FP64,
                    PGMG_FLAG_UNFUSED, PGMG_FLAG_NO_RECOMPUTE, PGMG_FLAG_NO_PIN,
                    PGMG_FLAG_NO_R2, PGMG_FLAG_HOST_TRANSPORT, PGMG_FLAG_FAST,
                    PGMG_FLAG_NO_SPEC_FIRE, PGMG_FLAG_NO_CTILE, PGMG_FLAG_NO_CARRY, PGMG_FLAG_TIME_COMM, PGMG_FLAG_NO_SHUFFLE, PGMG_FLAG_NO_SPIN,
                    PGMG_PROLONG_REFERENCE,
                    PGMG_PROLONG_SYMMETRIC, PGMG_OK, PGMG_ERR_STATE, PgmgConfig, PgmgError,
                    check, load)

PKG_DIR = pathlib.Path(__file__).resolve().parent

__all__ = [
    "build", "load", "Solver", "PgmgConfig", "PgmgError", "ops", "config_overrides",
    "PGMG_FLAG_NO_GRAPH", "PGMG_FLAG_TIME_FINE", "PGMG_FLAG_UNFUSED", "PGMG_FLAG_LOOPBACK", "PGMG_FLAG_NO_CROSS",
    "PGMG_PROLONG_REFERENCE", "plan_strips", "LoopbackHub", "unique_id", "rccl_latency",
    "PGMG_PROLONG_SYMMETRIC", "PGMG_PRECISION_FP64", "PGMG_PRECISION_FP32",
    "PGMG_FLAG_STORED_RHS", "PGMG_FLAG_EXACT_DIST", "PGMG_FLAG_SOLO",
    "PGMG_FLAG_NO_RECOMPUTE", "PGMG_FLAG_NO_PIN", "PGMG_FLAG_NO_R2", "PGMG_FLAG_FAST", "PGMG_FLAG_NO_SPEC_FIRE", "PGMG_FLAG_NO_CTILE", "PGMG_FLAG_NO_CARRY", "PGMG_FLAG_TIME_COMM", "PGMG_FLAG_NO_SHUFFLE", "PGMG_FLAG_NO_SPIN",
    "PGMG_FLAG_HOST_TRANSPORT", "HostTransport", "DeviceGrid",
]


def build(jobs=8, verbose=False):
    """Compile libpgmg.so (and host/gpu_exec) for gfx950 in-tree."""
    cmd = ["make", "-C", str(PKG_DIR), f"-j{jobs}", "all"]
    r = subprocess.run(cmd, capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise PgmgError(f"build failed:\n{r.stdout}\n{r.stderr}")
    return PKG_DIR / "libpgmg.so"


# Config fields applied to every Solver created inside `with config_overrides(...)`
# (flags are OR-ed in).  Tests use it to run the default plan's building blocks on small
# grids (cross_min_n, spec_segment) or an alternative plan (PGMG_FLAG_NO_RECOMPUTE, ...)
# through helpers that build their own Solvers.  Everything goes through pgmg_config.
_overrides = {}


@contextlib.contextmanager
def config_overrides(**kw):
    saved = dict(_overrides)
    for k, v in kw.items():
        if k == "flags":
            _overrides["flags"] = _overrides.get("flags", 0) | int(v)
        else:
            _overrides[k] = v
    try:
        yield
    finally:
        _overrides.clear()
        _overrides.update(saved)


def default_config(N, **kw):
    cfg = PgmgConfig()
    check(load().pgmg_config_default(C.byref(cfg), int(N)), "pgmg_config_default")
    kw = dict(kw)
    for k, v in _overrides.items():
        if k == "flags":
            kw["flags"] = kw.get("flags", 0) | v
        else:
            kw.setdefault(k, v)
    for k, v in kw.items():
        if not hasattr(cfg, k):
            raise TypeError(f"unknown config field {k}")
        setattr(cfg, k, v)
    return cfg


def plan_strips(N, world, rank, tail_n=65, gather_n=1025):
    """Finest-level rows [lo, hi) owned by `rank` and the number of strip-distributed
    levels (host arithmetic of the row-strip decomposition; no GPU needed)."""
    lo, hi, nd = C.c_int(), C.c_int(), C.c_int()
    check(load().pgmg_plan_strips(int(N), int(world), int(rank), int(tail_n), int(gather_n),
                                  C.byref(lo), C.byref(hi), C.byref(nd)), "pgmg_plan_strips")
    return lo.value, hi.value, nd.value


def unique_id():
    """A fresh 128-byte RCCL unique id (rank 0 creates it, then broadcasts it)."""
    buf = (C.c_ubyte * 128)()
    check(load().pgmg_comm_unique_id(buf), "pgmg_comm_unique_id")
    return bytes(buf)


def rccl_latency(device=0, reps=200):
    """Latency floor of the strips' collectives on this device (world-1 RCCL communicator):
    {"halo_group_us", "allreduce_sum_us", "allreduce_min_us"} (pgmg_rccl_latency)."""
    us = (C.c_double * 3)()
    uid = (C.c_ubyte * 128).from_buffer_copy(unique_id())
    check(load().pgmg_rccl_latency(uid, int(device), int(reps), us), "pgmg_rccl_latency")
    return {"halo_group_us": us[0], "allreduce_sum_us": us[1], "allreduce_min_us": us[2]}


from .hostcomm import HostTransport  # noqa: E402


class LoopbackHub:
    """In-process rank hub: `world` Solvers in threads of one process share one GPU
    (test transport for the strip decomposition; RCCL refuses two ranks per device)."""

    def __init__(self, world):
        h = C.c_void_p()
        check(load().pgmg_loopback_create(int(world), C.byref(h)), "pgmg_loopback_create")
        self.h = h
        self.world = world

    def fail(self, rank, at_group):
        """Test hook: rank's at_group-th transport group from now on fails (0: never)."""
        check(load().pgmg_loopback_fail(self.h, int(rank), int(at_group)), "pgmg_loopback_fail")

    def close(self):
        if self.h:
            load().pgmg_loopback_destroy(self.h)
            self.h = None


class Solver:
    """A multigrid context: level pyramid resident in HBM, cycles on a HIP stream.

    Mirrors ParallelTestRunner::run_v_cycle / ParallelMultiGridSolver::v_cycle
    (3_part_parallel/ParallelTestRunner.cu:152-186, Parallel_Mg.cu:21-60) with the
    numerics of MultigridSolver (2_part_MG/MultiGrid.hpp:57-136).
    """

    def __init__(self, N, hub=None, uid=None, dtype="f64", transport=None, **cfg):
        """hub: LoopbackHub (ranks as threads on one GPU); uid: 128-byte RCCL unique id;
        transport: a HostTransport (ranks as processes, messages through the caller's
        torch.distributed group, staged in host memory);
        dtype: "f64" (bit-exact to mg_cpu_exec) or "f32" (PGMG_PRECISION_FP32)."""
        self.lib = load()
        if dtype not in ("f64", "f32"):
            raise ValueError(f"dtype must be 'f64' or 'f32', not {dtype!r}")
        cfg.setdefault("precision", PGMG_PRECISION_FP32 if dtype == "f32" else PGMG_PRECISION_FP64)
        if hub is not None:
            cfg["flags"] = cfg.get("flags", 0) | PGMG_FLAG_LOOPBACK
            cfg["world"] = hub.world
            cfg["nccl_unique_id"] = hub.h
        elif transport is not None:
            self._transport = transport   # the callbacks must outlive the context
            cfg["flags"] = cfg.get("flags", 0) | PGMG_FLAG_HOST_TRANSPORT
            cfg.setdefault("world", transport.world)
            cfg.setdefault("rank", transport.rank)
            cfg["nccl_unique_id"] = C.cast(C.pointer(transport.struct), C.c_void_p)
        elif uid is not None:
            self._uid = (C.c_ubyte * 128)(*uid)
            cfg["nccl_unique_id"] = C.cast(self._uid, C.c_void_p)
        self.cfg = default_config(N, **cfg)
        h = C.c_void_p()
        check(self.lib.pgmg_create(C.byref(h), C.byref(self.cfg)), "pgmg_create")
        self.h = h
        self.N = int(N)

    def close(self):
        if getattr(self, "h", None):
            self.lib.pgmg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_problem(self, phi0=None, f=None):
        N = self.N
        args = []
        for a in (phi0, f):
            if a is None:
                args.append(None)
            else:
                a = np.ascontiguousarray(a, dtype=np.float64)
                assert a.shape == (N, N), a.shape
                args.append(a)
        p = [None if a is None else a.ctypes.data_as(C.c_void_p) for a in args]
        check(self.lib.pgmg_set_problem(self.h, p[0], p[1]), "pgmg_set_problem")

    def set_problem_device(self, phi, f=None):
        """Bind device arrays (DeviceGrid, torch tensors or raw device pointers; N*N float64
        in the reference layout) as the problem: phi is updated in place by every following
        cycle call; f None = the analytic RHS (pgmg_set_problem_device)."""
        check(self.lib.pgmg_set_problem_device(self.h, _dptr(phi), _dptr(f)),
              "pgmg_set_problem_device")

    def device_info(self):
        """(a device problem is bound, its calls run in place)"""
        b, i = C.c_int(), C.c_int()
        check(self.lib.pgmg_problem_device_info(self.h, C.byref(b), C.byref(i)),
              "pgmg_problem_device_info")
        return bool(b.value), bool(i.value)

    def vcycle(self, n=1):
        check(self.lib.pgmg_vcycle(self.h, int(n)), "pgmg_vcycle")

    def wcycle(self, n=1):
        check(self.lib.pgmg_wcycle(self.h, int(n)), "pgmg_wcycle")

    def fcycle(self, n=1):
        check(self.lib.pgmg_fcycle(self.h, int(n)), "pgmg_fcycle")

    def sync(self):
        check(self.lib.pgmg_sync(self.h), "pgmg_sync")

    def solution(self):
        out = np.empty((self.N, self.N), dtype=np.float64)
        check(self.lib.pgmg_get_solution(self.h, out.ctypes.data_as(C.c_void_p)),
              "pgmg_get_solution")
        return out

    def solution_hash(self, root=0):
        """FNV-64 of phi (hex string, the golden fixtures' format) on rank `root`; collective
        on row strips (other ranks get None)."""
        v = C.c_ulonglong()
        check(self.lib.pgmg_solution_hash(self.h, int(root), C.byref(v)), "pgmg_solution_hash")
        mine = self.cfg.world <= 1 or root < 0 or self.cfg.rank == root
        return "%016x" % v.value if mine else None

    def gather_solution(self, root, want):
        """Collective: phi gathered to rank `root` only; returns it where `want`, else None
        (row strips of a large grid without a full host copy per rank)."""
        out = np.empty((self.N, self.N), dtype=np.float64) if want else None
        ptr = out.ctypes.data_as(C.c_void_p) if want else None
        check(self.lib.pgmg_gather_solution(self.h, int(root), ptr), "pgmg_gather_solution")
        return out

    def residual_norm(self):
        v = C.c_double()
        check(self.lib.pgmg_residual_norm(self.h, C.byref(v)), "pgmg_residual_norm")
        return v.value

    def stats(self):
        s, e = C.c_longlong(), C.c_longlong()
        check(self.lib.pgmg_stats(self.h, C.byref(s), C.byref(e)), "pgmg_stats")
        return s.value, e.value

    def stats_detail(self):
        """[sweeps, early exits, k_postpre post-check rare paths (-1: not cross-fused),
        k_postpre pre-check rare paths]"""
        v = (C.c_longlong * 4)()
        check(self.lib.pgmg_stats_detail(self.h, v), "pgmg_stats_detail")
        return list(v)

    def last_elapsed_ms(self):
        v = C.c_double()
        check(self.lib.pgmg_last_elapsed_ms(self.h, C.byref(v)), "pgmg_last_elapsed_ms")
        return v.value

    def levels(self):
        b, t = C.c_int(), C.c_int()
        check(self.lib.pgmg_levels(self.h, C.byref(b), C.byref(t)), "pgmg_levels")
        return b.value, t.value

    def vcycle_bytes(self):
        v = C.c_double()
        check(self.lib.pgmg_vcycle_bytes(self.h, C.byref(v)), "pgmg_vcycle_bytes")
        return v.value

    def fine_sweep_time(self):
        n, m = C.c_int(), C.c_double()
        check(self.lib.pgmg_fine_sweep_time(self.h, C.byref(n), C.byref(m)),
              "pgmg_fine_sweep_time")
        return n.value, m.value

    def fine_pass_time(self, which):
        """(count, mean ms) of finest-level kernels: 0 plain sweep, 1 k_pre, 2 k_post,
        3 k_postpre, 4 the carry pass."""
        n, m = C.c_int(), C.c_double()
        check(self.lib.pgmg_fine_pass_time(self.h, int(which), C.byref(n), C.byref(m)),
              "pgmg_fine_pass_time")
        return n.value, m.value

    @property
    def fused(self):
        v = C.c_int()
        check(self.lib.pgmg_fused(self.h, C.byref(v)), "pgmg_fused")
        return bool(v.value)

    def fine_pass_info(self, which):
        """(kernel symbol, algorithmic bytes per launch) of the launches the last
        fine_pass_time(which) averaged ("" / 0 when none was timed)."""
        buf = C.create_string_buffer(512)
        b = C.c_double()
        check(self.lib.pgmg_fine_pass_info(self.h, int(which), buf, 512, C.byref(b)),
              "pgmg_fine_pass_info")
        return buf.value.decode(errors="replace"), b.value

    def carry_info(self):
        """(calls that started from a carried pre-smooth, carries made, carries dropped)."""
        a = (C.c_longlong * 3)()
        check(self.lib.pgmg_carry_info(self.h, a), "pgmg_carry_info")
        return tuple(a)

    def comm_stats(self):
        """(collective groups since the last call, ms inside them with PGMG_FLAG_TIME_COMM else
        -1); synchronous, resets."""
        g, m = C.c_longlong(), C.c_double()
        check(self.lib.pgmg_comm_stats(self.h, C.byref(g), C.byref(m)), "pgmg_comm_stats")
        return g.value, m.value

    def comm_ranks(self):
        """Ranks of the communicator (RCCL: ncclCommCount); 1 without strips."""
        n = C.c_int()
        check(self.lib.pgmg_comm_ranks(self.h, C.byref(n)), "pgmg_comm_ranks")
        return n.value

    def set_eps(self, eps):
        """A new early-exit threshold for the following calls (drops the carry)."""
        check(self.lib.pgmg_set_eps(self.h, float(eps)), "pgmg_set_eps")

    def fine_pass_bytes(self, which):
        """Algorithmic HBM bytes of one launch of finest-level pass `which` on this rank."""
        v = C.c_double()
        check(self.lib.pgmg_fine_pass_bytes(self.h, int(which), C.byref(v)), "pgmg_fine_pass_bytes")
        return v.value

    def dist_info(self):
        """(speculative early-exit checks (recorded, validated after the call)?, calls
        rolled back and rerun with in-stream decisions)"""
        sp, rb = C.c_int(), C.c_longlong()
        check(self.lib.pgmg_dist_info(self.h, C.byref(sp), C.byref(rb)), "pgmg_dist_info")
        return bool(sp.value), rb.value

    def spec_levels(self):
        """Bit mask: bit l = bulk level l's checks are not speculated "does not fire" (decided
        in-stream, or predicted to fire); bit 0 = no speculation at all."""
        m = C.c_ulonglong()
        check(self.lib.pgmg_spec_levels(self.h, C.byref(m)), "pgmg_spec_levels")
        return m.value

    def spec_fire_levels(self):
        """Bit mask: bit l = bulk level l's checks are predicted to fire (one-sweep passes,
        confirmed by the validation)."""
        m = C.c_ulonglong()
        check(self.lib.pgmg_spec_fire_levels(self.h, C.byref(m)), "pgmg_spec_fire_levels")
        return m.value

    def spec_visit_modes(self):
        """W-cycle plans: (does not fire, predicted to fire, in-stream) visit counts of the last
        speculative W call's bulk levels."""
        a = (C.c_longlong * 3)()
        check(self.lib.pgmg_spec_visit_modes(self.h, a), "pgmg_spec_visit_modes")
        return tuple(a)

    @property
    def elem_bytes(self):
        """8 (fp64) or 4 (fp32): bytes per grid element on the device."""
        p, e = C.c_int(), C.c_int()
        check(self.lib.pgmg_precision(self.h, C.byref(p), C.byref(e)), "pgmg_precision")
        return e.value

    def bench_sweep(self, reps):
        m = C.c_double()
        check(self.lib.pgmg_bench_sweep(self.h, int(reps), C.byref(m)), "pgmg_bench_sweep")
        return m.value


def _dptr(t):
    if t is None:
        return None
    if isinstance(t, int):
        return C.c_void_p(t)
    if isinstance(t, DeviceGrid):
        return C.c_void_p(t.ptr)
    return C.c_void_p(t.data_ptr())


class DeviceGrid:
    """An N*N float64 device grid in the reference layout with guard rows
    (pgmg_alloc_grid): what ParallelTestRunner allocates with cudaMallocManaged
    (3_part_parallel/ParallelTestRunner.cu:162-163), here device memory."""

    def __init__(self, N, host=None):
        self.lib = load()
        self.N = int(N)
        p = C.c_void_p()
        check(self.lib.pgmg_alloc_grid(C.byref(p), self.N), "pgmg_alloc_grid")
        self.ptr = p.value
        if host is not None:
            self.upload(host)

    def upload(self, host):
        a = np.ascontiguousarray(host, dtype=np.float64)
        assert a.shape == (self.N, self.N), a.shape
        check(self.lib.pgmg_memcpy_h2d(C.c_void_p(self.ptr), a.ctypes.data_as(C.c_void_p),
                                       a.nbytes), "pgmg_memcpy_h2d")

    def download(self):
        out = np.empty((self.N, self.N), dtype=np.float64)
        check(self.lib.pgmg_memcpy_d2h(out.ctypes.data_as(C.c_void_p), C.c_void_p(self.ptr),
                                       out.nbytes), "pgmg_memcpy_d2h")
        return out

    def close(self):
        if getattr(self, "ptr", None):
            self.lib.pgmg_free_grid(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class _Ops:
    """Op-level entries on caller-owned device buffers (torch tensors or raw pointers),
    mirroring Parallel::Compute* (3_part_parallel/Parallel_Method.cu:144-199)."""

    @staticmethod
    def _ptr(t):
        if t is None:
            return None
        if isinstance(t, int):
            return C.c_void_p(t)
        return C.c_void_p(t.data_ptr())

    def jacobi(self, x, f, h, v, eps=1e-7, tmp=None, stream=None, count=True):
        """count=False: the reference's void ComputeJacobi shape -- no sweep count returned,
        so no device-to-host readback (the call stays asynchronous on `stream`)."""
        H, W = x.shape
        done = C.c_int()
        check(load().pgmg_jacobi(self._ptr(x), self._ptr(tmp), self._ptr(f), H, W, float(h),
                                 int(v), float(eps), C.byref(done) if count else None, stream),
              "pgmg_jacobi")
        return done.value if count else None

    def residual(self, r, x, f, h, stream=None):
        H, W = x.shape
        check(load().pgmg_residual(self._ptr(r), self._ptr(x), self._ptr(f), H, W, float(h),
                                   stream), "pgmg_residual")

    def restrict(self, fine, coarse, stream=None):
        check(load().pgmg_restrict(self._ptr(fine), self._ptr(coarse), fine.shape[0],
                                   coarse.shape[0], stream), "pgmg_restrict")

    def prolong(self, coarse, fine, mode=PGMG_PROLONG_REFERENCE, num_thread=0, stream=None):
        """num_thread > 0: the reference's launch grid (max(1, Nf // num_thread) *
        num_thread rows and columns touched, Parallel_Method.cu:191-197); 0: all of it."""
        check(load().pgmg_prolong_grid(self._ptr(coarse), self._ptr(fine), coarse.shape[0],
                                       fine.shape[0], int(mode), int(num_thread), stream),
              "pgmg_prolong_grid")

    def norm(self, v, stream=None):
        out = C.c_double()
        check(load().pgmg_norm(self._ptr(v), v.numel(), C.byref(out), stream), "pgmg_norm")
        return out.value

    def rhs(self, f, h, a=1.0, p=1.0, q=1.0, stream=None):
        H, W = f.shape
        check(load().pgmg_rhs(self._ptr(f), W, H, float(h), float(a), float(p), float(q),
                              stream), "pgmg_rhs")


ops = _Ops()
