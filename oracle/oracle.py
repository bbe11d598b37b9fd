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


_lib = None
_DP = C.POINTER(C.c_double)


def build():
    subprocess.run(["make", "-C", str(HERE), "-s", "all"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
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
            "orc_v_cycle": (None, [P, P, P, C.c_int, C.c_double]),
            "orc_w_cycle": (None, [P, P, P, C.c_int, C.c_double]),
            "orc_f_cycle_outer": (None, [P, P, C.c_int]),
            "orc_rel_error": (C.c_double, [P, P, C.c_int]),
            "orc_residual_norm": (C.c_double, [P, P, C.c_int, C.c_double]),
            "orc_hash": (C.c_uint64, [P, C.c_longlong]),
        }
        for k, (r, a) in sig.items():
            fn = getattr(L, k)
            fn.restype = r
            fn.argtypes = a
        assert L.orc_ctx_size() == C.sizeof(OrcCtx), "OrcCtx layout mismatch"
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class Oracle:
    """Sequential CPU multigrid with the reference's exact semantics."""

    def __init__(self, eps=1e-7, **kw):
        self.c = OrcCtx()
        lib().orc_ctx_init(C.byref(self.c))
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
        f = np.zeros((N, N))
        lib().orc_rhs(C.byref(self.c), _p(f), N, N, h)
        return f

    def exact(self, N):
        u = np.zeros((N, N))
        lib().orc_exact(C.byref(self.c), _p(u), self.c.a / (N - 1), N, N)
        return u

    def v_cycle(self, phi, f, h=None):
        N = phi.shape[0]
        h = self.c.a / (N - 1) if h is None else h
        lib().orc_v_cycle(C.byref(self.c), _p(phi), _p(f), N, h)

    def w_cycle(self, phi, f, h=None):
        N = phi.shape[0]
        h = self.c.a / (N - 1) if h is None else h
        lib().orc_w_cycle(C.byref(self.c), _p(phi), _p(f), N, h)

    def f_cycle_outer(self, phi):
        lib().orc_f_cycle_outer(C.byref(self.c), _p(phi), phi.shape[0])

    def smooth(self, x, f, h, num_iter):
        N = x.shape[0]
        work = np.zeros(2 * N * N)
        return lib().orc_jacobi_smooth(C.byref(self.c), _p(x), _p(f), N, N, h, num_iter, _p(work))

    def rel_error(self, phi):
        return lib().orc_rel_error(C.byref(self.c), _p(phi), phi.shape[0])


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


def norm(v):
    v = np.ascontiguousarray(v, dtype=np.float64)
    return lib().orc_norm(_p(v), v.size)


def fnv_hash(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return "%016x" % lib().orc_hash(_p(a), a.size)


def run_cycles(kind, N, cycles, eps=1e-7):
    """phi after `cycles` cycles from phi=0, f=analytic RHS (mg_cpu_exec's setup)."""
    o = Oracle(eps=eps)
    f = o.rhs(N)
    phi = np.zeros((N, N))
    for _ in range(cycles):
        if kind == "V":
            o.v_cycle(phi, f)
        elif kind == "W":
            o.w_cycle(phi, f)
        else:
            o.f_cycle_outer(phi)
    return phi, o
