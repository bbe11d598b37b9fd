// pgmg_tail.hip — the coarse end of the hierarchy in ONE workgroup, all in LDS.
//
// Below N ~ 129 every level is launch/latency-bound: a level of the multi-kernel
// path costs ~9 dependent launches (~1.5-2 us each) for a few microseconds of
// data.  The tail instead runs the complete gamma-cycle (gamma = 1: V, 3: W) for
// the tail's top level and everything below it inside one 1024-thread workgroup:
// the level pyramid (solution E, right-hand side F) plus one scratch grid T live
// in LDS (N_top = 65: 125 KiB of the CU's 160 KiB), separated by __syncthreads.
//
// Semantics are exactly MultigridSolver::v_cycle / w_cycle (MultiGrid.hpp:57-136)
// with JacobiSmoother::smooth (Smoother.hpp:38-116), including the per-sweep
// residual-norm early exit, evaluated sequentially (no speculation needed here).
#include "pgmg_internal.h"

namespace pgmg {

constexpr int kTailMaxLevels = 8;
constexpr int kTailRed = kTailThreads / 64 + 2;  // doubles of reduction scratch at the LDS base

template <class Real>
struct TailLevel {
    int N;
    int off;         // offset of this level's E and F grids (pitch N, no padding)
    Real hh, ih;     // h*h and 1.0/(h*h) rounded on the host
};

template <class Real>
struct TailArgsDev {
    TailArgsT<Real> a;
    int nl;
    int S;           // elements per pyramid
    TailLevel<Real> lv[kTailMaxLevels];
    int gamma;
};

__device__ __forceinline__ double tail_sum(double v, double *red)
{
    #pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        #pragma unroll
        for (int i = 0; i < kTailThreads / 64; ++i) s += red[i];
        red[kTailThreads / 64] = s;
    }
    __syncthreads();
    const double s = red[kTailThreads / 64];
    __syncthreads();
    return s;
}

// out = J(cur) on all points (boundary copied); optionally sum r(cur)^2
template <class Real, bool NORM>
__device__ __forceinline__ double tail_jacobi(const Real *cur, Real *out, const Real *f, int N,
                                              Real hh, Real ih)
{
    double acc = 0.0;
    const int n = N * N;
    for (int k = threadIdx.x; k < n; k += kTailThreads) {
        const int j = k / N;
        const int i = k - j * N;
        if (i == 0 || j == 0 || i == N - 1 || j == N - 1) {
            out[k] = cur[k];
            continue;
        }
        out[k] = Real(0.25) * ((hh * f[k]) + cur[k - 1] + cur[k + 1] + cur[k - N] + cur[k + N]);
        if (NORM) {
            const Real r =
                f[k] - ih * (Real(4) * cur[k] - cur[k - 1] - cur[k + 1] - cur[k - N] - cur[k + N]);
            acc += sq(r);
        }
    }
    return acc;
}

// JacobiSmoother::smooth(x, f, N, N, h, num_iter): num_iter+1 sweeps, break as
// soon as ||r(x_k)|| < eps.  The check of x_k is fused into sweep k+1 (which
// reads the same neighbourhood); when it fires, sweep k+1's output is dropped.
template <class Real>
__device__ void tail_smooth(Real *x, const Real *f, const TailLevel<Real> &L, int num_iter,
                            double eps, Real *T, double *red, long long &sweeps,
                            long long &exits)
{
    Real *cur = x, *oth = T;
    tail_jacobi<Real, false>(cur, oth, f, L.N, L.hh, L.ih);
    __syncthreads();
    Real *tmp = cur;
    cur = oth;
    oth = tmp;
    ++sweeps;
    for (int k = 2; k <= num_iter + 1; ++k) {
        const double acc = tail_jacobi<Real, true>(cur, oth, f, L.N, L.hh, L.ih);
        const double s = tail_sum(acc, red);   // also orders the writes of oth
        if (sqrt(s) < eps) {
            ++exits;
            break;
        }
        tmp = cur;
        cur = oth;
        oth = tmp;
        ++sweeps;
    }
    if (cur != x) {
        const int n = L.N * L.N;
        for (int k = threadIdx.x; k < n; k += kTailThreads) x[k] = cur[k];
    }
    __syncthreads();
}

// T = r(x) on the interior, 0 on the boundary; then fc = R T (MultiGrid.hpp:70-78)
template <class Real>
__device__ void tail_res_restrict(const Real *x, const Real *f, const TailLevel<Real> &Lf, Real *fc,
                                  Real *ec, const TailLevel<Real> &Lc, Real *T)
{
    const int N = Lf.N, n = N * N;
    for (int k = threadIdx.x; k < n; k += kTailThreads) {
        const int j = k / N;
        const int i = k - j * N;
        if (i == 0 || j == 0 || i == N - 1 || j == N - 1) {
            T[k] = Real(0);
            continue;
        }
        T[k] = f[k] - Lf.ih * (Real(4) * x[k] - x[k - 1] - x[k + 1] - x[k - N] - x[k + N]);
    }
    __syncthreads();
    const int Nc = Lc.N, nc = Nc * Nc;
    for (int q = threadIdx.x; q < nc; q += kTailThreads) {
        const int jc = q / Nc;
        const int ic = q - jc * Nc;
        ec[q] = Real(0);  // MultiGrid.hpp:81-82 e_coarse = 0
        if (ic == 0 || jc == 0 || ic == Nc - 1 || jc == Nc - 1) continue;
        const int k = (2 * jc) * N + 2 * ic;
        fc[q] = Real(0.25) * T[k] + Real(0.125) * (T[k + 1] + T[k - 1] + T[k + N] + T[k - N]) +
                Real(0.0625) * (T[k - N - 1] + T[k - N + 1] + T[k + N - 1] + T[k + N + 1]);
    }
    __syncthreads();
}

// x += P e (MultiGrid.hpp:208-226): fine points in [2, Nf-2]^2 only
template <class Real>
__device__ void tail_prolong(Real *x, const TailLevel<Real> &Lf, const Real *e,
                             const TailLevel<Real> &Lc)
{
    const int N = Lf.N, Nc = Lc.N, n = N * N;
    for (int k = threadIdx.x; k < n; k += kTailThreads) {
        const int j = k / N;
        const int i = k - j * N;
        if (i < 2 || j < 2 || i > N - 2 || j > N - 2) continue;
        const int jc = j >> 1, ic = i >> 1;
        const Real *C0 = e + jc * Nc;
        Real v;
        if ((j & 1) == 0) {
            v = ((i & 1) == 0) ? C0[ic] : Real(0.5) * (C0[ic] + C0[ic + 1]);
        } else {
            const Real *C1 = C0 + Nc;
            v = ((i & 1) == 0) ? Real(0.5) * (C0[ic] + C1[ic])
                               : Real(0.25) * (C0[ic] + C0[ic + 1] + C1[ic] + C1[ic + 1]);
        }
        x[k] = x[k] + v;
    }
    __syncthreads();
}

// gamma-cycle (MultiGrid.hpp:57-136) whose top is tail level `top`; levels top.. last
template <class Real>
__device__ void tail_gcycle(const TailArgsDev<Real> &d, int top, Real *E, Real *F, Real *T,
                            double *red, long long &sweeps, long long &exits)
{
    const TailArgsT<Real> &a = d.a;
    int visits[kTailMaxLevels];
    for (int i = 0; i < kTailMaxLevels; ++i) visits[i] = 0;
    int l = top;
    bool descending = true;
    const int last = d.nl - 1;
    for (;;) {
        if (descending) {
            if (l == last) {
                tail_smooth(E + d.lv[l].off, F + d.lv[l].off, d.lv[l], a.coarse_iter, a.eps, T,
                            red, sweeps, exits);
                descending = false;
            } else {
                tail_smooth(E + d.lv[l].off, F + d.lv[l].off, d.lv[l], a.v1, a.eps, T, red,
                            sweeps, exits);
                tail_res_restrict(E + d.lv[l].off, F + d.lv[l].off, d.lv[l], F + d.lv[l + 1].off,
                                  E + d.lv[l + 1].off, d.lv[l + 1], T);
                visits[l + 1] = 0;
                ++l;
            }
        } else {
            if (l == top) break;
            const int p = l - 1;
            if (++visits[l] < d.gamma) {
                descending = true;   // call the cycle on level l again
            } else {
                tail_prolong(E + d.lv[p].off, d.lv[p], E + d.lv[l].off, d.lv[l]);
                tail_smooth(E + d.lv[p].off, F + d.lv[p].off, d.lv[p], a.v2, a.eps, T, red,
                            sweeps, exits);
                l = p;
            }
        }
    }
}

// analytic right-hand side of tail level t from host sine tables (DynamicGridUtils.hpp:111-124)
template <class Real>
__device__ void tail_rhs(const TailArgsDev<Real> &d, int t, Real *F)
{
    const int N = d.lv[t].N, n = N * N;
    const double *sx = d.a.fmg_tab + d.a.fmg_tab_off[t];
    const double *sy = sx + N;
    for (int k = threadIdx.x; k < n; k += kTailThreads) {
        const int j = k / N;
        const int i = k - j * N;
        F[k] = (Real)(d.a.fmg_factor * sx[i] * sy[j]);
    }
}

// values restriction (compute_coarsest_grid) fine level t -> t+1, coarse boundary 0
template <class Real>
__device__ void tail_restrict_values(const Real *x, const TailLevel<Real> &Lf, Real *xc,
                                     const TailLevel<Real> &Lc)
{
    const int N = Lf.N, Nc = Lc.N, nc = Nc * Nc;
    for (int q = threadIdx.x; q < nc; q += kTailThreads) {
        const int jc = q / Nc;
        const int ic = q - jc * Nc;
        if (ic == 0 || jc == 0 || ic == Nc - 1 || jc == Nc - 1) {
            xc[q] = Real(0);
            continue;
        }
        const int k = (2 * jc) * N + 2 * ic;
        xc[q] = Real(0.25) * x[k] + Real(0.125) * (x[k + 1] + x[k - 1] + x[k + N] + x[k - N]) +
                Real(0.0625) * (x[k - N - 1] + x[k - N + 1] + x[k + N - 1] + x[k + N + 1]);
    }
    __syncthreads();
}

template <class Real>
__global__ __launch_bounds__(kTailThreads) void k_tail(TailArgsDev<Real> d)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const TailArgsT<Real> &a = d.a;
    const int S = d.S;
    double *red = lds;                                   // kTailThreads / 64 + 1 partial sums
    Real *E = reinterpret_cast<Real *>(lds + kTailRed);
    Real *F = E + S;
    Real *T = E + 2 * S;

    for (int k = threadIdx.x; k < 2 * S; k += kTailThreads) E[k] = Real(0);
    __syncthreads();
    {
        const int N = d.lv[0].N, n = N * N;
        const long long P = a.P_top;
        for (int k = threadIdx.x; k < n; k += kTailThreads) {
            const int j = k / N;
            const int i = k - j * N;
            if (!a.fmg) F[k] = a.f_top[j * P + i];
            if (a.x0_from_global || a.fmg) E[k] = a.e_top[j * P + i];
        }
    }
    __syncthreads();

    long long sweeps = 0, exits = 0;
    const int last = d.nl - 1;
    if (!a.fmg) {
        tail_gcycle(d, 0, E, F, T, red, sweeps, exits);
    } else {
        // compute_coarsest_grid: restrict phi down to the coarsest level
        for (int t = 0; t < last; ++t)
            tail_restrict_values(E + d.lv[t].off, d.lv[t], E + d.lv[t + 1].off, d.lv[t + 1]);
        for (int t = last; t >= 0; --t) {
            Real *Et = E + d.lv[t].off;
            Real *Ft = F + d.lv[t].off;
            tail_rhs(d, t, Ft);                      // f_fine = compute_rhs (MultiGrid.hpp:162)
            if (t < last) {
                const int n = d.lv[t].N * d.lv[t].N;
                for (int k = threadIdx.x; k < n; k += kTailThreads) Et[k] = Real(0);
                __syncthreads();
                tail_prolong(Et, d.lv[t], E + d.lv[t + 1].off, d.lv[t + 1]);   // :164
                tail_gcycle(d, t, E, F, T, red, sweeps, exits);              // :167 v_cycle
            } else {
                __syncthreads();
            }
            if (t > 0 || a.fmg_smooth_top)                                   // :153 smooth(3)
                tail_smooth(Et, Ft, d.lv[t], 3, a.eps, T, red, sweeps, exits);
        }
    }

    {
        const int N = d.lv[0].N, n = N * N;
        const long long P = a.P_top;
        for (int k = threadIdx.x; k < n; k += kTailThreads) {
            const int j = k / N;
            const int i = k - j * N;
            a.e_top[j * P + i] = E[k];
        }
    }
    if (threadIdx.x == 0 && a.stats != nullptr) {
        atomicAdd(&a.stats[0], (unsigned long long)sweeps);
        atomicAdd(&a.stats[1], (unsigned long long)exits);
    }
}

template <class Real>
size_t tail_lds_bytes(int N_top, int n_coarse)
{
    size_t S = 0;
    int N = N_top;
    for (int l = 0; l < kTailMaxLevels; ++l) {
        S += (size_t)N * N;
        if (N <= n_coarse) break;
        N = (N - 1) / 2 + 1;
    }
    return kTailRed * sizeof(double) + (2 * S + (size_t)N_top * N_top) * sizeof(Real);
}

template <class Real>
hipError_t launch_tail_gamma(const TailArgsT<Real> &a, int gamma, hipStream_t s)
{
    static bool attr_set = false;
    TailArgsDev<Real> d;
    d.a = a;
    d.gamma = gamma;
    int N = a.N_top;
    double h = a.h_top;
    int off = 0, nl = 0;
    for (; nl < kTailMaxLevels; ++nl) {
        d.lv[nl].N = N;
        d.lv[nl].off = off;
        d.lv[nl].hh = (Real)(h * h);
        d.lv[nl].ih = (Real)(1.0 / (h * h));
        off += N * N;
        if (N <= a.n_coarse) {
            ++nl;
            break;
        }
        N = (N - 1) / 2 + 1;
        h = 2 * h;  // MultiGrid.hpp:83 v_cycle(e_coarse, res_coarse, Nc, 2 * h)
    }
    d.nl = nl;
    d.S = off;
    const size_t bytes = tail_lds_bytes<Real>(a.N_top, a.n_coarse);
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void *)k_tail<Real>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    k_tail<Real><<<dim3(1), dim3(kTailThreads), bytes, s>>>(d);
    return hipGetLastError();
}

template hipError_t launch_tail_gamma<double>(const TailArgsT<double> &, int, hipStream_t);
template hipError_t launch_tail_gamma<float>(const TailArgsT<float> &, int, hipStream_t);
template size_t tail_lds_bytes<double>(int, int);
template size_t tail_lds_bytes<float>(int, int);

}  // namespace pgmg
