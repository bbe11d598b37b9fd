"""ctypes declarations for libpgmg.so (the C ABI in include/pgmg.h).

Plumbing only: the product is the HIP library; this module lets tests, bench.py and
__graft_entry__ call it.  Loading fails loudly if the shared library is missing —
there is no CPU fallback anywhere in the product path.
"""
import ctypes as C
import os
import pathlib

PKG_DIR = pathlib.Path(__file__).resolve().parent
# PGMG_LIB: another build of the library (A/B measurements of compile-time variants)
LIB_PATH = pathlib.Path(os.environ["PGMG_LIB"]) if os.environ.get("PGMG_LIB") else PKG_DIR / "libpgmg.so"

PGMG_OK = 0
PGMG_ERR_ARG = -1
PGMG_ERR_HIP = -2
PGMG_ERR_NOMEM = -3
PGMG_ERR_COMM = -4
PGMG_ERR_STATE = -5

PGMG_PROLONG_REFERENCE = 0
PGMG_PROLONG_SYMMETRIC = 1

PGMG_FLAG_NO_GRAPH = 1
PGMG_FLAG_TIME_FINE = 2
PGMG_FLAG_UNFUSED = 4
PGMG_FLAG_LOOPBACK = 8
PGMG_FLAG_NO_CROSS = 16
PGMG_FLAG_STORED_RHS = 32
PGMG_FLAG_EXACT_DIST = 64
PGMG_FLAG_SOLO = 128
PGMG_FLAG_NO_RECOMPUTE = 256
PGMG_FLAG_NO_PIN = 512
PGMG_FLAG_NO_R2 = 1024
PGMG_FLAG_HOST_TRANSPORT = 2048
PGMG_FLAG_FAST = 4096
PGMG_FLAG_NO_SPEC_FIRE = 32768
PGMG_FLAGS_RETIRED = 8192 | 16384
PGMG_FLAG_NO_CTILE = 65536
PGMG_FLAG_NO_CARRY = 131072
PGMG_FLAG_TIME_COMM = 262144
PGMG_FLAG_NO_SHUFFLE = 524288
PGMG_FLAG_NO_SPIN = 1048576

PGMG_PRECISION_FP64 = 0
PGMG_PRECISION_FP32 = 1


# pgmg_host_transport (include/pgmg.h): the caller's message functions
HT_EXCHANGE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_void_p),
                          C.POINTER(C.c_ulonglong), C.c_int, C.POINTER(C.c_int),
                          C.POINTER(C.c_void_p), C.POINTER(C.c_ulonglong))
HT_SUM_F64 = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int)
HT_MIN_U32 = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint), C.c_int)


class PgmgHostTransport(C.Structure):
    _fields_ = [("user", C.c_void_p), ("exchange", HT_EXCHANGE),
                ("allreduce_sum_f64", HT_SUM_F64), ("allreduce_min_u32", HT_MIN_U32)]


class PgmgConfig(C.Structure):
    _fields_ = [
        ("N", C.c_int),
        ("v1", C.c_int),
        ("v2", C.c_int),
        ("coarse_iter", C.c_int),
        ("n_coarse", C.c_int),
        ("alpha", C.c_int),
        ("eps", C.c_double),
        ("a", C.c_double),
        ("p", C.c_double),
        ("q", C.c_double),
        ("tail_n", C.c_int),
        ("device", C.c_int),
        ("flags", C.c_uint),
        ("rank", C.c_int),
        ("world", C.c_int),
        ("nccl_unique_id", C.c_void_p),
        ("gather_n", C.c_int),
        ("precision", C.c_int),
        ("cross_min_n", C.c_int),
        ("spec_segment", C.c_int),
        ("comm_timeout_s", C.c_double),
        ("h0", C.c_double),
    ]


# (name, restype, argtypes) for every symbol include/pgmg.h declares
_P = C.c_void_p
_DP = C.POINTER(C.c_double)
SIGNATURES = [
    ("pgmg_config_default", C.c_int, [C.POINTER(PgmgConfig), C.c_int]),
    ("pgmg_create", C.c_int, [C.POINTER(_P), C.POINTER(PgmgConfig)]),
    ("pgmg_destroy", C.c_int, [_P]),
    ("pgmg_set_problem", C.c_int, [_P, _P, _P]),
    ("pgmg_set_problem_device", C.c_int, [_P, _P, _P]),
    ("pgmg_problem_device_info", C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("pgmg_alloc_grid", C.c_int, [C.POINTER(_P), C.c_int]),
    ("pgmg_free_grid", C.c_int, [_P]),
    ("pgmg_grid_serial", C.c_int, [_P, C.POINTER(C.c_ulonglong)]),
    ("pgmg_pointer_is_device", C.c_int, [_P, C.POINTER(C.c_int)]),
    ("pgmg_vcycle", C.c_int, [_P, C.c_int]),
    ("pgmg_wcycle", C.c_int, [_P, C.c_int]),
    ("pgmg_fcycle", C.c_int, [_P, C.c_int]),
    ("pgmg_sync", C.c_int, [_P]),
    ("pgmg_get_solution", C.c_int, [_P, _P]),
    ("pgmg_gather_solution", C.c_int, [_P, C.c_int, _P]),
    ("pgmg_solution_hash", C.c_int, [_P, C.c_int, C.POINTER(C.c_ulonglong)]),
    ("pgmg_residual_norm", C.c_int, [_P, _DP]),
    ("pgmg_stats", C.c_int, [_P, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
    ("pgmg_stats_detail", C.c_int, [_P, C.POINTER(C.c_longlong)]),
    ("pgmg_last_elapsed_ms", C.c_int, [_P, _DP]),
    ("pgmg_levels", C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("pgmg_vcycle_bytes", C.c_int, [_P, _DP]),
    ("pgmg_check_span", C.c_int, [_P, C.c_longlong, C.c_int, C.c_longlong, C.c_longlong,
                                  C.c_longlong, C.c_longlong]),
    ("pgmg_phi_device", C.c_int, [_P, C.POINTER(_P), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                  C.POINTER(C.c_int)]),
    ("pgmg_fine_sweep_time", C.c_int, [_P, C.POINTER(C.c_int), _DP]),
    ("pgmg_fine_pass_time", C.c_int, [_P, C.c_int, C.POINTER(C.c_int), _DP]),
    ("pgmg_fine_pass_info", C.c_int, [_P, C.c_int, C.c_char_p, C.c_int, _DP]),
    ("pgmg_fused", C.c_int, [_P, C.POINTER(C.c_int)]),
    ("pgmg_precision", C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("pgmg_fine_pass_bytes", C.c_int, [_P, C.c_int, _DP]),
    ("pgmg_dist_info", C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_longlong)]),
    ("pgmg_spec_levels", C.c_int, [_P, C.POINTER(C.c_ulonglong)]),
    ("pgmg_spec_fire_levels", C.c_int, [_P, C.POINTER(C.c_ulonglong)]),
    ("pgmg_spec_visit_modes", C.c_int, [_P, C.POINTER(C.c_longlong)]),
    ("pgmg_carry_info", C.c_int, [_P, C.POINTER(C.c_longlong)]),
    ("pgmg_comm_stats", C.c_int, [_P, C.POINTER(C.c_longlong), _DP]),
    ("pgmg_comm_ranks", C.c_int, [_P, C.POINTER(C.c_int)]),
    ("pgmg_set_eps", C.c_int, [_P, C.c_double]),
    ("pgmg_bench_sweep", C.c_int, [_P, C.c_int, _DP]),
    ("pgmg_jacobi", C.c_int, [_P, _P, _P, C.c_int, C.c_int, C.c_double, C.c_int, C.c_double,
                              C.POINTER(C.c_int), _P]),
    ("pgmg_residual", C.c_int, [_P, _P, _P, C.c_int, C.c_int, C.c_double, _P]),
    ("pgmg_restrict", C.c_int, [_P, _P, C.c_int, C.c_int, _P]),
    ("pgmg_prolong", C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, _P]),
    ("pgmg_prolong_grid", C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, _P]),
    ("pgmg_norm", C.c_int, [_P, C.c_longlong, _DP, _P]),
    ("pgmg_rhs", C.c_int, [_P, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, C.c_double,
                           _P]),
    ("pgmg_ops_release", C.c_int, [_P]),
    ("pgmg_device_alloc", C.c_int, [C.POINTER(_P), C.c_size_t]),
    ("pgmg_device_free", C.c_int, [_P]),
    ("pgmg_memcpy_h2d", C.c_int, [_P, _P, C.c_size_t]),
    ("pgmg_memcpy_d2h", C.c_int, [_P, _P, C.c_size_t]),
    ("pgmg_device_sync", C.c_int, []),
    ("pgmg_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("pgmg_comm_unique_id", C.c_int, [_P]),
    ("pgmg_rccl_selftest", C.c_int, [_P, C.c_int]),
    ("pgmg_rccl_latency", C.c_int, [_P, C.c_int, C.c_int, _DP]),
    ("pgmg_tail_prof", C.c_int, [C.POINTER(C.c_ulonglong), C.c_int]),
    ("pgmg_loopback_create", C.c_int, [C.c_int, C.POINTER(_P)]),
    ("pgmg_loopback_destroy", C.c_int, [_P]),
    ("pgmg_loopback_fail", C.c_int, [_P, C.c_int, C.c_longlong]),
    ("pgmg_plan_strips", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("pgmg_last_error", C.c_char_p, []),
    ("pgmg_version", C.c_char_p, []),
    ("pgmg_source_hash", C.c_char_p, []),
]

_lib = None


class PgmgError(RuntimeError):
    pass


def load(path=None):
    """Load libpgmg.so and attach the signatures.  Raises if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = pathlib.Path(path) if path else LIB_PATH
    # torch bundles its own ROCm runtime (libamdhip64.so.7, libhsa-runtime64.so.1, ...)
    # under the same sonames as /opt/rocm.  Whichever loads first is shared by both;
    # torch's C++ breaks (heap corruption at exit) on the /opt/rocm copies, while our
    # library only uses the stable HIP C API.  So let torch's runtime win.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not p.exists():
        raise PgmgError(f"{p} not built: run `make -C {PKG_DIR} lib` (or __graft_entry__.build())")
    lib = C.CDLL(str(p), mode=os.RTLD_NOW | C.RTLD_GLOBAL)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(rc, what=""):
    if rc != PGMG_OK:
        msg = load().pgmg_last_error()
        raise PgmgError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc
