"""ctypes binding of oracle/liboracle.so — the CPU restatement of mg_cpu_exec.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker.  The product (libpgmg.so) never loads it.
"""
import ctypes as C
import pathlib
import subprocess

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
LIB_F32 = HERE / "liboracle_f32.so"   # -DORC_REAL=float: checker of the fp32 variant


class OrcCtx(C.Structure):
    _fields_ = [
        ("eps", C.c_double),
        ("n_coarse", C.c_int),
        ("v1", C.c_int),
        ("v2", C.c_int),
        ("coarse_iter", C.c_int),
        ("alpha", C.c_int),
        ("a", C.c_double),
        ("p", C.c_double),
        ("q", C.c_double),
        ("sweeps", C.c_longlong),
        ("early_exits", C.c_longlong),
        ("smooth_calls", C.c_longlong),
    ]


_libs = {}
_DP = C.POINTER(C.c_double)


def build():
    subprocess.run(["make", "-C", str(HERE), "-s", "all"], check=True)


def _np_dtype(dtype):
    return np.float32 if dtype in ("f32", np.float32) else np.float64


def lib(dtype="f64"):
    """liboracle.so (fp64, pinned to the reference) or liboracle_f32.so (dtype="f32")."""
    key = "f32" if _np_dtype(dtype) is np.float32 else "f64"
    if key not in _libs:
        path = LIB_F32 if key == "f32" else LIB
        if not path.exists():
            build()
        L = C.CDLL(str(path))
        P = C.c_void_p
        sig = {
            "orc_ctx_init": (None, [P]),
            "orc_ctx_size": (C.c_int, []),
            "orc_norm": (C.c_double, [P, C.c_longlong]),
            "orc_residual": (None, [P, P, P, C.c_int, C.c_int, C.c_double]),
            "orc_rhs": (None, [P, P, C.c_int, C.c_int, C.c_double]),
            "orc_exact": (None, [P, P, C.c_double, C.c_int, C.c_int]),
            "orc_jacobi_smooth": (C.c_int, [P, P, P, C.c_int, C.c_int, C.c_double, C.c_int, P]),
            "orc_restrict": (None, [P, P, C.c_int, C.c_int]),
            "orc_prolong": (None, [P, P, C.c_int, C.c_int]),
            "orc_prolong_sym": (None, [P, P] + [C.c_int] * 6),
            "orc_v_cycle": (None, [P, P, P, C.c_int, C.c_double]),
            "orc_w_cycle": (None, [P, P, P, C.c_int, C.c_double]),
            "orc_f_cycle_outer": (None, [P, P, C.c_int]),
            "orc_rel_error": (C.c_double, [P, P, C.c_int]),
            "orc_residual_norm": (C.c_double, [P, P, C.c_int, C.c_double]),
            "orc_hash": (C.c_uint64, [P, C.c_longlong]),
            "orc_real_size": (C.c_int, []),
            "orc_mt64_nth": (C.c_uint64, [C.c_uint64, C.c_longlong]),
            "orc_rhs_mt64": (None, [P, C.c_int, C.c_uint64]),
        }
        for k, (r, a) in sig.items():
            fn = getattr(L, k)
            fn.restype = r
            fn.argtypes = a
        assert L.orc_ctx_size() == C.sizeof(OrcCtx), "OrcCtx layout mismatch"
        assert L.orc_real_size() == (4 if key == "f32" else 8), "oracle element type"
        _libs[key] = L
    return _libs[key]


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class Oracle:
    """Sequential CPU multigrid with the reference's exact semantics."""

    def __init__(self, eps=1e-7, dtype="f64", **kw):
        self.dt = _np_dtype(dtype)
        self.L = lib(dtype)
        self.c = OrcCtx()
        self.L.orc_ctx_init(C.byref(self.c))
        self.c.eps = eps
        for k, v in kw.items():
            setattr(self.c, k, v)

    @property
    def sweeps(self):
        return self.c.sweeps

    @property
    def early_exits(self):
        return self.c.early_exits

    def rhs(self, N, h=None):
        h = 1.0 / (N - 1) * self.c.a if h is None else h
        f = np.zeros((N, N), dtype=self.dt)
        self.L.orc_rhs(C.byref(self.c), _p(f), N, N, h)
        return f

    def exact(self, N):
        u = np.zeros((N, N))
        self.L.orc_exact(C.byref(self.c), _p(u), self.c.a / (N - 1), N, N)
        return u

    def v_cycle(self, phi, f, h=None):
        N = phi.shape[0]
        h = self.c.a / (N - 1) if h is None else h
        self._chk(phi, f)
        self.L.orc_v_cycle(C.byref(self.c), _p(phi), _p(f), N, h)

    def w_cycle(self, phi, f, h=None):
        N = phi.shape[0]
        h = self.c.a / (N - 1) if h is None else h
        self._chk(phi, f)
        self.L.orc_w_cycle(C.byref(self.c), _p(phi), _p(f), N, h)

    def f_cycle_outer(self, phi):
        self._chk(phi)
        self.L.orc_f_cycle_outer(C.byref(self.c), _p(phi), phi.shape[0])

    def smooth(self, x, f, h, num_iter):
        N = x.shape[0]
        self._chk(x, f)
        work = np.zeros(2 * N * N, dtype=self.dt)
        return self.L.orc_jacobi_smooth(C.byref(self.c), _p(x), _p(f), N, N, h, num_iter,
                                        _p(work))

    def rel_error(self, phi):
        phi = np.ascontiguousarray(phi, dtype=self.dt)
        return self.L.orc_rel_error(C.byref(self.c), _p(phi), phi.shape[0])

    def _chk(self, *arrays):
        for a in arrays:
            assert a.dtype == self.dt and a.flags.c_contiguous, (a.dtype, self.dt)


def rhs_mt64(N, seed=12345, dtype="f64"):
    """SURVEY §8(d)'s robustness RHS: std::uniform_real_distribution<double>(-1, 1) over
    std::mt19937_64(seed), one draw per point in row-major order, boundary 0
    (orc_rhs_mt64; pinned to libstdc++ by tests/golden/mt_rhs.json)."""
    f = np.zeros((N, N), dtype=_np_dtype(dtype))
    lib(dtype).orc_rhs_mt64(_p(f), N, seed)
    return f


def residual(x, f, h):
    r = np.zeros_like(x)
    N = x.shape[0]
    lib().orc_residual(_p(r), _p(x), _p(f), x.shape[1], N, h)
    return r


def restrict(fine):
    Nf = fine.shape[0]
    Nc = (Nf - 1) // 2 + 1
    c = np.zeros((Nc, Nc))
    lib().orc_restrict(_p(fine), _p(c), Nf, Nc)
    return c


def prolong(fine, coarse):
    out = np.array(fine, dtype=np.float64, copy=True)
    lib().orc_prolong(_p(out), _p(coarse), out.shape[0], coarse.shape[0])
    return out


def prolong_sym(fine, coarse, num_thread=None):
    """fine += P_sym coarse as prolungator_kernel (Parallel_Method.cu:79-138) computes it.
    num_thread=None: the thread grid covers the whole fine grid; otherwise the grid of
    Parallel::ComputeProlungator (:188-199), max(1, Nf // num_thread) * num_thread wide."""
    out = np.array(fine, dtype=np.float64, copy=True)
    coarse = np.ascontiguousarray(coarse, dtype=np.float64)
    Hf, Wf = out.shape
    Hc, Wc = coarse.shape
    if num_thread is None:
        ey, ex = Hf, Wf
    else:
        ey = max(1, Hf // num_thread) * num_thread
        ex = max(1, Hf // num_thread) * num_thread   # the launch is square in fine_N
    lib().orc_prolong_sym(_p(out), _p(coarse), Hc, Wc, Hf, Wf, ey, ex)
    return out


def norm(v):
    v = np.ascontiguousarray(v, dtype=np.float64)
    return lib().orc_norm(_p(v), v.size)


def fnv_hash(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return "%016x" % lib().orc_hash(_p(a), a.size)


def run_cycles(kind, N, cycles, eps=1e-7, dtype="f64"):
    """phi after `cycles` cycles from phi=0, f=analytic RHS (mg_cpu_exec's setup).
    dtype="f32": the fp32 restatement (float grids and arithmetic)."""
    o = Oracle(eps=eps, dtype=dtype)
    f = o.rhs(N)
    phi = np.zeros((N, N), dtype=o.dt)
    for _ in range(cycles):
        if kind == "V":
            o.v_cycle(phi, f)
        elif kind == "W":
            o.w_cycle(phi, f)
        else:
            o.f_cycle_outer(phi)
    return phi, o
