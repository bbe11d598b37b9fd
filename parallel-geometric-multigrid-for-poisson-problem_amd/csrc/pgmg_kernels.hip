// pgmg_kernels.hip — CDNA4 (gfx950) stencil kernels of the multigrid V-cycle.
//
// Every kernel is a bandwidth-bound fp64 stencil (≈0.25 flop/byte), so the design
// goal is HBM streaming efficiency, not arithmetic:
//   * lane t of a wave owns the aligned column pair (1+2t, 2+2t): one 16-byte
//     load/store per row per array (global_load/store_dwordx4), 1 KiB per wave;
//   * blocks march down a segment of rows keeping the x rows above/below in
//     registers, so each x element crosses HBM once per sweep (plus one halo row
//     per segment);
//   * horizontal neighbours come from the adjacent lane through DPP
//     (wave_shr:1 / wave_shl:1, full-rate VALU moves); only lanes 0 and 63 load a
//     halo column;
//   * U rows are loaded before any is used so every wave keeps 2·U 16-B loads
//     in flight.
// Expression order follows the reference exactly (file:line at each kernel) and
// the build uses -ffp-contract=off, so every value is bit-identical to mg_cpu_exec.
#include "pgmg_internal.h"

namespace pgmg {

// deterministic block sum (fixed tree) of one double per thread; result valid in thread 0
template <int NT>
__device__ __forceinline__ double block_sum(double v, double *red)
{
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0) {
        #pragma unroll
        for (int i = 0; i < NT / 64; ++i) s += red[i];
    }
    return s;
}

// ---------------------------------------------------------------------------
// Jacobi sweep.  Reference: JacobiSmoother::smooth, Smoother.hpp:59-69
//   out[i] = 0.25 * ((h*h*f[i]) + x[i-1] + x[i+1] + x[i-W] + x[i+W])
// NORM: residual of x_in at the same points, DynamicGridUtils.hpp:59-69
//   r[i] = f[i] - (1.0/(h*h)) * (4*x[i] - x[i-1] - x[i+1] - x[i-W] - x[i+W])
// ---------------------------------------------------------------------------
constexpr int kU = 4;  // rows in flight per wave

template <class T, bool X0_ZERO, bool NORM, bool FINE>
__global__ __launch_bounds__(kBlock) void k_sweep(SweepArgsT<T> a)
{
    __shared__ double red[kBlock / 64];
    if (a.skip != nullptr && *a.skip != 0u) return;  // smoother already exited (uniform)
    const bool leader = blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0;
    if (leader) {
        if (a.reset != nullptr) *a.reset = 0u;
        if (a.stats != nullptr) atomicAdd(&a.stats[0], 1ull);
    }
    const int lane = threadIdx.x & 63;
    const int npairs = (a.W - 1) >> 1;
    const int t_raw = blockIdx.x * kBlock + threadIdx.x;
    const bool act = t_raw < npairs;
    const int t = act ? t_raw : npairs - 1;      // idle lanes shadow the last pair
    const int c = 1 + 2 * t;
    const bool second = (c + 1) <= a.W - 2;      // else column c+1 is the right boundary
    const int jb = a.row0 + blockIdx.y * a.rows_per_block;
    const int je = min(jb + a.rows_per_block, a.row1);
    const long long P = a.P;
    using D2 = V2<T>;
    const T *__restrict__ X = a.xin;
    const T *__restrict__ F = a.f;
    T *__restrict__ O = a.xout;
    const T hh = a.hh, ih = a.inv_hh;
    double acc = 0.0;

    D2 w0 = zero2<T>(), w1 = zero2<T>();
    if (!X0_ZERO) {
        w0 = ldv(X + (jb - 1) * P + c);
        w1 = ldv(X + jb * P + c);
    }
    for (int j = jb; j < je; j += kU) {
        D2 xn[kU], fv[kU];
        T el[kU], er[kU];
        #pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int r = min(j + u, je - 1);
            fv[u] = ldv(F + r * P + c);
            el[u] = T(0);
            er[u] = T(0);
            if (!X0_ZERO) {
                xn[u] = ldv(X + (r + 1) * P + c);
                if (lane == 0) el[u] = X[r * P + c - 1];
                if (lane == 63) er[u] = X[r * P + c + 2];
            } else {
                xn[u] = zero2<T>();
            }
        }
        #pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int r = j + u;
            const D2 up = (u == 0) ? w0 : (u == 1 ? w1 : xn[u - 2]);
            const D2 ce = (u == 0) ? w1 : xn[u - 1];
            const D2 dn = xn[u];
            T left = dpp_shr(ce.y);
            T right = dpp_shl(ce.x);
            if (lane == 0) left = el[u];
            if (lane == 63) right = er[u];
            D2 o;
            o.x = T(0.25) * ((hh * fv[u].x) + left + ce.y + up.x + dn.x);
            o.y = second ? T(0.25) * ((hh * fv[u].y) + ce.x + right + up.y + dn.y) : ce.y;
            const bool live = act && r < je;
            if (NORM) {
                const T r0 = fv[u].x - ih * (T(4) * ce.x - left - ce.y - up.x - dn.x);
                const T r1 = fv[u].y - ih * (T(4) * ce.y - ce.x - right - up.y - dn.y);
                if (live) {
                    acc += sq(r0);
                    if (second) acc += sq(r1);
                }
            }
            if (live) stv(O + r * P + c, o);
        }
        w0 = xn[kU - 2];
        w1 = xn[kU - 1];
    }
    if (NORM) {
        const double s = block_sum<kBlock>(acc, red);
        if (threadIdx.x == 0) a.partials[blockIdx.y * gridDim.x + blockIdx.x] = s;
    }
}

int sweep_blocks(int W, int row0, int row1, int *rows_per_block, int *gx, int *gy)
{
    const int npairs = (W - 1) / 2;
    const int bx = (npairs + kBlock - 1) / kBlock;
    const int rows = row1 - row0;
    // aim for >= ~4096 blocks on big grids (16/CU), >= 4 rows per block
    int rpb = (int)(((long long)rows * bx + 4095) / 4096);
    rpb = rpb < 4 ? 4 : (rpb > 64 ? 64 : rpb);
    rpb = (rpb + kU - 1) / kU * kU;
    const int by = (rows + rpb - 1) / rpb;
    *rows_per_block = rpb;
    *gx = bx;
    *gy = by;
    return bx * by;
}

template <class T>
void launch_sweep(const SweepArgsT<T> &a, bool x0_zero, bool fine, hipStream_t s)
{
    int rpb, gx, gy;
    sweep_blocks(a.W, a.row0, a.row1, &rpb, &gx, &gy);
    SweepArgsT<T> b = a;
    b.rows_per_block = rpb;
    const dim3 grid(gx, gy), blk(kBlock);
    const bool norm = a.partials != nullptr;
    if (fine) {
        if (x0_zero) launchk(k_sweep<T, true, false, true>, grid, blk, s, b);
        else if (norm) launchk(k_sweep<T, false, true, true>, grid, blk, s, b);
        else launchk(k_sweep<T, false, false, true>, grid, blk, s, b);
    } else {
        if (x0_zero) launchk(k_sweep<T, true, false, false>, grid, blk, s, b);
        else if (norm) launchk(k_sweep<T, false, true, false>, grid, blk, s, b);
        else launchk(k_sweep<T, false, false, false>, grid, blk, s, b);
    }
    // x (unless x0 = 0), f in; x out
    g_last_launch.bytes = (x0_zero ? 16.0 : 24.0) * row_pts(a.row0, a.row1, a.W) * sizeof(T) / 8.0;
}

// ---------------------------------------------------------------------------
// Fused residual + full-weighting restriction.
// Reference: MultiGrid.hpp:70-78 (compute_residual then restrict_full_weighting)
//   C[c] = 0.25*F[k] + 0.125*(F[k+1] + F[k-1] + F[k+Nf] + F[k-Nf])
//        + 0.0625*(F[k-Nf-1] + F[k-Nf+1] + F[k+Nf-1] + F[k+Nf+1])   (:199-202)
// with F = r computed on the fly (never written to HBM).  Lane t produces coarse
// column ic = t+1, whose fine centre column is c+1 (c = 2t+1).
// ---------------------------------------------------------------------------
template <class T>
struct XRow {
    V2<T> own;   // x at (c, c+1)
    V2<T> nxt;   // x at (c+2, c+3)
    T lft;       // x at c-1
};

template <class T>
__device__ __forceinline__ XRow<T> load_xrow(const T *X, long long off, int c, int lane)
{
    XRow<T> r;
    r.own = ldv(X + off + c);
    r.nxt.x = dpp_shl(r.own.x);
    r.nxt.y = dpp_shl(r.own.y);
    r.lft = dpp_shr(r.own.y);
    if (lane == 63) r.nxt = ldv(X + off + c + 2);
    if (lane == 0) r.lft = X[off + c - 1];
    return r;
}

template <class T>
struct RTriple {
    T r0, r1, r2;  // residual at columns c, c+1, c+2
};

template <class T>
__device__ __forceinline__ RTriple<T> resid3(const XRow<T> &u, const XRow<T> &m, const XRow<T> &d,
                                             V2<T> fo, T fn, T ih)
{
    RTriple<T> r;
    r.r0 = fo.x - ih * (T(4) * m.own.x - m.lft - m.own.y - u.own.x - d.own.x);
    r.r1 = fo.y - ih * (T(4) * m.own.y - m.own.x - m.nxt.x - u.own.y - d.own.y);
    r.r2 = fn - ih * (T(4) * m.nxt.x - m.own.y - m.nxt.y - u.nxt.x - d.nxt.x);
    return r;
}

template <class T>
__global__ __launch_bounds__(kBlock) void k_res_restrict(ResRestrictArgsT<T> a)
{
    const int lane = threadIdx.x & 63;
    const int nact = a.Wc - 2;                   // coarse interior columns
    const int t_raw = blockIdx.x * kBlock + threadIdx.x;
    const bool act = t_raw < nact;
    const int t = min(t_raw, a.Wc - 2);          // last fine pair index is Wc-2
    const int c = 1 + 2 * t;
    const int jcb = a.jc0 + blockIdx.y * a.rows_per_block;
    const int jce = min(jcb + a.rows_per_block, a.jc1);
    if (jcb >= jce) return;
    const long long Pf = a.Pf, Pc = a.Pc;
    const T *__restrict__ X = a.x;
    const T *__restrict__ F = a.f;
    const T ih = a.inv_hh;

    // window: x rows 2jc-1 (A) and 2jc (B); r row 2jc-1 (up)
    XRow<T> xz = load_xrow(X, (2LL * jcb - 2) * Pf, c, lane);
    XRow<T> xa = load_xrow(X, (2LL * jcb - 1) * Pf, c, lane);
    XRow<T> xb = load_xrow(X, (2LL * jcb) * Pf, c, lane);
    V2<T> fo = ldv(F + (2LL * jcb - 1) * Pf + c);
    T fn = dpp_shl(fo.x);
    if (lane == 63) fn = F[(2LL * jcb - 1) * Pf + c + 2];
    RTriple<T> up = resid3(xz, xa, xb, fo, fn, ih);

    for (int jc = jcb; jc < jce; ++jc) {
        const long long rm = 2LL * jc, rd = rm + 1;
        const XRow<T> xc = load_xrow(X, rd * Pf, c, lane);
        const XRow<T> xd = load_xrow(X, (rd + 1) * Pf, c, lane);
        const V2<T> fm = ldv(F + rm * Pf + c);
        const V2<T> fd = ldv(F + rd * Pf + c);
        T fmn = dpp_shl(fm.x), fdn = dpp_shl(fd.x);
        if (lane == 63) {
            fmn = F[rm * Pf + c + 2];
            fdn = F[rd * Pf + c + 2];
        }
        const RTriple<T> mid = resid3(xa, xb, xc, fm, fmn, ih);
        const RTriple<T> dn = resid3(xb, xc, xd, fd, fdn, ih);
        const T v = T(0.25) * mid.r1 + T(0.125) * (mid.r2 + mid.r0 + dn.r1 + up.r1) +
                    T(0.0625) * (up.r0 + up.r2 + dn.r0 + dn.r2);
        if (act) a.rc[jc * Pc + (t + 1)] = v;
        up = dn;
        xa = xc;
        xb = xd;
    }
}

int res_restrict_rows_per_block(int Wc, int nrows)
{
    const int bx = (Wc - 2 + kBlock - 1) / kBlock;
    int rpb = (int)(((long long)nrows * bx + 4095) / 4096);
    return rpb < 2 ? 2 : (rpb > 32 ? 32 : rpb);
}

template <class T>
void launch_res_restrict(const ResRestrictArgsT<T> &a, hipStream_t s)
{
    const int bx = (a.Wc - 2 + kBlock - 1) / kBlock;
    const int rows = a.jc1 - a.jc0;
    ResRestrictArgsT<T> b = a;
    b.rows_per_block = res_restrict_rows_per_block(a.Wc, rows);
    const int by = (rows + b.rows_per_block - 1) / b.rows_per_block;
    k_res_restrict<T><<<dim3(bx, by), dim3(kBlock), 0, s>>>(b);
}

// ---------------------------------------------------------------------------
// Prolongation fine += P coarse, reference flavour (MultiGrid.hpp:208-226):
//   F[J,I]     += C[c]
//   F[J+1,I]   += 0.5*(C[c] + C[c+Nc])
//   F[J,I+1]   += 0.5*(C[c] + C[c+1])
//   F[J+1,I+1] += 0.25*(C[c] + C[c+1] + C[c+Nc] + C[c+Nc+1])
// for ic, jc in [1, Nc-2]: every fine point in [2, Nf-2]^2 is written exactly
// once, fine row/col 1 never.  Each lane gathers its own value.
// ---------------------------------------------------------------------------
template <class T>
__global__ __launch_bounds__(kBlock) void k_prolong(ProlongArgsT<T> a)
{
    const int npairs = (a.Wf - 1) >> 1;
    const int t_raw = blockIdx.x * kBlock + threadIdx.x;
    const bool act = t_raw < npairs;
    const int t = act ? t_raw : npairs - 1;
    const int c = 1 + 2 * t;
    const bool okx = t >= 1;                 // odd column c: coarse ic = t
    const bool oky = (t + 1) <= a.Wc - 2;    // even column c+1: coarse ic = t+1
    const int jb = a.row0 + blockIdx.y * a.rows_per_block;
    const int je = min(jb + a.rows_per_block, a.row1);
    const long long Pf = a.Pf, Pc = a.Pc;
    for (int j = jb; j < je; ++j) {
        const int jc = j >> 1;
        const T *C0 = a.c + jc * Pc;
        const T c00 = C0[t], c01 = C0[t + 1];
        // assign: start from +0.0 — the same additions as into a zeroed grid
        V2<T> v = a.assign ? zero2<T>() : ldv(a.fine + j * Pf + c);
        if ((j & 1) == 0) {
            if (okx) v.x = v.x + T(0.5) * (c00 + c01);
            if (oky) v.y = v.y + c01;
        } else {
            const T *C1 = C0 + Pc;
            const T c10 = C1[t], c11 = C1[t + 1];
            if (okx) v.x = v.x + T(0.25) * (c00 + c01 + c10 + c11);
            if (oky) v.y = v.y + T(0.5) * (c01 + c11);
        }
        if (act) stv(a.fine + j * Pf + c, v);
    }
}

template <class T>
void launch_prolong(const ProlongArgsT<T> &a, hipStream_t s)
{
    const int npairs = (a.Wf - 1) / 2;
    const int bx = (npairs + kBlock - 1) / kBlock;
    const int rows = a.row1 - a.row0;
    int rpb = (int)(((long long)rows * bx + 4095) / 4096);
    rpb = rpb < 2 ? 2 : (rpb > 32 ? 32 : rpb);
    ProlongArgsT<T> b = a;
    b.rows_per_block = rpb;
    const int by = (rows + rpb - 1) / rpb;
    k_prolong<T><<<dim3(bx, by), dim3(kBlock), 0, s>>>(b);
}

// ---------------------------------------------------------------------------
// Early-exit fix-up (Smoother.hpp:75-88 `if (res_norm < epsilon) break;`).
// Sweep k ran speculatively and left sum r(x_{k-1})^2 per block in `partials`.
// Every block re-reduces the partials in the same fixed order (no atomics, so
// the decision is identical everywhere and run-to-run); on trigger the
// smoother's result is x_{k-1}: copy it over the speculative x_k.
// ---------------------------------------------------------------------------
constexpr int kFixBlocks = 256;

template <class T>
__global__ __launch_bounds__(kBlock) void k_fixup(FixupArgsT<T> a)
{
    __shared__ double red[kBlock / 64];
    __shared__ int trig;
    const bool leader = blockIdx.x == 0 && threadIdx.x == 0;
    if (*a.done_prev != 0u) {
        if (leader) *a.done_next = 1u;
        return;
    }
    double s = 0.0;
    for (int k = threadIdx.x; k < a.np; k += kBlock) s += a.partials[k];
    s = block_sum<kBlock>(s, red);
    if (threadIdx.x == 0) {
        const double tot = a.global_sum != nullptr ? *a.global_sum : s;
        trig = (sqrt(tot) < a.eps) ? 1 : 0;
    }
    __syncthreads();
    if (leader) {
        *a.done_next = trig ? 1u : 0u;
        if (trig && a.stats != nullptr) {
            atomicAdd(&a.stats[0], (unsigned long long)-1LL);  // speculative sweep undone
            atomicAdd(&a.stats[1], 1ull);
        }
    }
    if (!trig) return;
    const int npairs = (a.W - 1) >> 1;
    const long long P = a.P;
    const long long total = (long long)(a.row1 - a.row0) * npairs;
    for (long long k = (long long)blockIdx.x * kBlock + threadIdx.x; k < total;
         k += (long long)gridDim.x * kBlock) {
        const int r = a.row0 + (int)(k / npairs);
        const int t = (int)(k % npairs);
        const int c = 1 + 2 * t;
        stv(a.dst + r * P + c, ldv(a.src + r * P + c));
    }
}

template <class T>
void launch_fixup(const FixupArgsT<T> &a, hipStream_t s)
{
    k_fixup<T><<<dim3(kFixBlocks), dim3(kBlock), 0, s>>>(a);
}

template <class T>
__global__ __launch_bounds__(kBlock) void k_copy_rows(const T *src, T *dst, int W, long long P,
                                                      int row0, int row1)
{
    const int npairs = (W - 1) >> 1;
    const long long total = (long long)(row1 - row0) * npairs;
    for (long long k = (long long)blockIdx.x * kBlock + threadIdx.x; k < total;
         k += (long long)gridDim.x * kBlock) {
        const int r = row0 + (int)(k / npairs);
        const int c = 1 + 2 * (int)(k % npairs);
        stv(dst + r * P + c, ldv(src + r * P + c));
    }
}

template <class T>
void launch_copy_rows(const T *src, T *dst, int W, int P, int row0, int row1, hipStream_t s)
{
    const long long total = (long long)(row1 - row0) * ((W - 1) / 2);
    long long nb = (total + kBlock - 1) / kBlock;
    if (nb > 4096) nb = 4096;
    if (nb < 1) nb = 1;
    k_copy_rows<T><<<dim3((unsigned)nb), dim3(kBlock), 0, s>>>(src, dst, W, P, row0, row1);
}

// ---------------------------------------------------------------------------
// RHS from separable host sine tables: f = factor * sin(p*pi*x/a) * sin(q*pi*y/a)
// (DynamicGridUtils.hpp:111-124) = (factor * sx[i]) * sy[j], same IEEE ops.
// ---------------------------------------------------------------------------
template <class T>
__global__ void k_rhs(T *f, const double *sx, const double *sy, double factor, int W,
                      long long P, int row0, int row1)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = row0 + blockIdx.y;
    if (i >= W || j >= row1) return;
    f[j * P + i] = (T)(factor * sx[i] * sy[j]);
}

template <class T>
void launch_rhs(T *f, const double *sx, const double *sy, double factor, int W, int P, int row0,
                int row1, hipStream_t s)
{
    k_rhs<T><<<dim3((W + 255) / 256, row1 - row0), dim3(256), 0, s>>>(f, sx, sy, factor, W, P,
                                                                  row0, row1);
}

// MultiGrid.hpp:187-205 applied to values (compute_coarsest_grid, MultiGrid.hpp:28-55).
// A lane owns coarse column ic and marches down a band of coarse rows; per fine row it
// loads the aligned pair (2ic-1, 2ic) (one 16-byte load) and takes 2ic+1 from the next
// lane by DPP (the wave's last lane loads it), so every fine row is read once, whole.
// Fine row 2jc+1 is kept for the next coarse row.
// wave_shl:1 with the wave's last lane keeping `last` (bound_ctrl off: a lane without a
// source lane is not written).  One instruction per dword and no select, so it cannot
// be sunk into a branch that disables the source lane.
__device__ __forceinline__ double shl_or_last(double v, double last)
{
    const long long b = __double_as_longlong(v), o = __double_as_longlong(last);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, 0x130, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), 0x130, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ float shl_or_last(float v, float last)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(last), __float_as_int(v), 0x130,
                                                      0xF, 0xF, false));
}

template <class T>
__global__ __launch_bounds__(256) void k_restrict_values(const T *Fn, long long Pf, T *C, int Nc,
                                                         long long Pc, int jc0, int jc1, int rpb)
{
    const int jb = jc0 + blockIdx.y * rpb;
    const int je = min(jb + rpb, jc1);
    if (jb >= je) return;   // uniform over the block
    const int lane = threadIdx.x & 63;
    const int ic = 1 + blockIdx.x * 256 + threadIdx.x;
    const bool own = ic <= Nc - 2;
    // lanes past the last coarse column load the boundary pair (in range) and store nothing;
    // lane Nc-1's pair.x is the east column of lane Nc-2
    const T *__restrict__ q = Fn + 2 * min(ic, Nc - 1) - 1;
    T uw, uc, ue;
    {
        const T *p = q + (long long)(2 * jb - 1) * Pf;
        const V2<T> v = ldv(p);
        const T x = lane == 63 ? p[2] : T(0);
        uw = v.x;
        uc = v.y;
        ue = shl_or_last(v.x, x);
    }
    // coarse row jc from fine rows 2jc (m) and 2jc+1 (d) and the kept row 2jc-1
    auto emit = [&](int jc, V2<T> vm, V2<T> vd, T xm, T xd) {
        const T me = shl_or_last(vm.x, xm), de = shl_or_last(vd.x, xd);
        if (own)
            C[(long long)jc * Pc + ic] = T(0.25) * vm.y + T(0.125) * (me + vm.x + vd.y + uc) +
                                         T(0.0625) * (uw + ue + vd.x + de);
        uw = vd.x;
        uc = vd.y;
        ue = de;
    };
    // RB coarse rows (2 RB fine-row loads in flight per lane) per step
    constexpr int RB = 4;
    int jc = jb;
    for (; jc + RB <= je; jc += RB) {
        const T *m = q + (long long)(2 * jc) * Pf;
        V2<T> v[2 * RB];
        T x[2 * RB];
        #pragma unroll
        for (int k = 0; k < 2 * RB; ++k) {
            v[k] = ldv(m + k * Pf);
            x[k] = T(0);
        }
        if (lane == 63) {
            #pragma unroll
            for (int k = 0; k < 2 * RB; ++k) x[k] = m[k * Pf + 2];
        }
        #pragma unroll
        for (int r = 0; r < RB; ++r) emit(jc + r, v[2 * r], v[2 * r + 1], x[2 * r], x[2 * r + 1]);
    }
    for (; jc < je; ++jc) {
        const T *m = q + (long long)(2 * jc) * Pf, *d = m + Pf;
        const V2<T> vm = ldv(m), vd = ldv(d);
        T xm = T(0), xd = T(0);
        if (lane == 63) {
            xm = m[2];
            xd = d[2];
        }
        emit(jc, vm, vd, xm, xd);
    }
}

template <class T>
void launch_restrict_values(const T *fine, int Nf, int Pf, T *coarse, int Nc, int Pc, hipStream_t s,
                            int jc0, int jc1)
{
    (void)Nf;
    jc0 = jc0 < 1 ? 1 : jc0;
    jc1 = jc1 > Nc - 1 ? Nc - 1 : jc1;
    if (jc1 <= jc0) return;
    const int gx = (Nc - 2 + 255) / 256;
    // ~2048 workgroups (8 rounds of the resident ones), bands of at least 8 coarse rows
    const int rows = jc1 - jc0;
    int rpb = (rows * gx + 2047) / 2048;
    rpb = rpb < 8 ? 8 : rpb;
    const int gy = (rows + rpb - 1) / rpb;
    k_restrict_values<T><<<dim3(gx, gy), dim3(256), 0, s>>>(fine, Pf, coarse, Nc, Pc, jc0, jc1, rpb);
}

// Two full-weighting steps in one pass: level l+2 = R R (level l) on its interior points,
// the intermediate level's values computed in registers, never stored (compute_coarsest_grid,
// MultiGrid.hpp:28-55, restricts level by level; a level-(l+2) interior point reads only
// interior points of level l+1, so the intermediate grid's frame never matters).  Lane t of
// a wave owns level-(l+2) column i (63 per wave; lane 63 only supplies its neighbour's east
// values); per lane and fine row: the two aligned pairs of columns 4i-3 .. 4i, the east
// column 4i+1 from the next lane; per level-(l+2) row, four fine rows are loaded and two
// level-(l+1) rows computed.  Every value goes through the reference's expression in the
// reference's order, so the result is bitwise the two-step one.
template <class T>
__device__ __forceinline__ T rfw(T u_w, T u_c, T u_e, T m_w, T m_c, T m_e, T d_w, T d_c, T d_e)
{
    return T(0.25) * m_c + T(0.125) * (m_e + m_w + d_c + u_c) + T(0.0625) * (u_w + u_e + d_w + d_e);
}

template <class T> struct Row4 {   // a lane's fine columns 4i-3 .. 4i and 4i+1
    T a, b, c, d, e;
};

template <class T>
__global__ __launch_bounds__(256) void k_restrict2_values(const T *Fn, long long Pf, T *C, int Nc,
                                                          long long Pc, int jc0, int jc1, int rpb)
{
    const int jb = jc0 + blockIdx.y * rpb;
    const int je = min(jb + rpb, jc1);
    if (jb >= je) return;   // uniform over the block
    const int lane = threadIdx.x & 63;
    const int i = 1 + blockIdx.x * 252 + (int)(threadIdx.x >> 6) * 63 + lane;
    const bool own = lane < 63 && i <= Nc - 2;
    const T *__restrict__ q = Fn + 4 * min(i, Nc - 1) - 3;   // in range (see k_restrict_values)
    auto ld = [&](int r) {
        const T *p = q + (long long)r * Pf;
        const V2<T> v0 = ldv(p), v1 = ldv(p + 2);
        const T x = lane == 63 ? p[4] : T(0);
        Row4<T> o;
        o.a = v0.x;
        o.b = v0.y;
        o.c = v1.x;
        o.d = v1.y;
        o.e = shl_or_last(v0.x, x);
        return o;
    };
    // the two intermediate values of a lane (columns 2i-1 and 2i) from fine rows u, m, d
    auto mid = [&](const Row4<T> &u, const Row4<T> &m, const Row4<T> &d, T &A, T &B) {
        A = rfw(u.a, u.b, u.c, m.a, m.b, m.c, d.a, d.b, d.c);
        B = rfw(u.c, u.d, u.e, m.c, m.d, m.e, d.c, d.d, d.e);
    };
    Row4<T> f3 = ld(4 * jb - 1);   // fine row 4j-1 of the step j
    T pA, pB;                       // intermediate row 2j-1
    {
        const Row4<T> u = ld(4 * jb - 3), m = ld(4 * jb - 2);
        mid(u, m, f3, pA, pB);
    }
    for (int j = jb; j < je; ++j) {
        const Row4<T> r0 = ld(4 * j), r1 = ld(4 * j + 1), r2 = ld(4 * j + 2), r3 = ld(4 * j + 3);
        T mA, mB, dA, dB;
        mid(f3, r0, r1, mA, mB);   // intermediate row 2j
        mid(r1, r2, r3, dA, dB);   // intermediate row 2j+1
        const T pE = dpp_shl(pA), mE = dpp_shl(mA), dE = dpp_shl(dA);
        if (own) C[(long long)j * Pc + i] = rfw(pA, pB, pE, mA, mB, mE, dA, dB, dE);
        f3 = r3;
        pA = dA;
        pB = dB;
    }
}

template <class T>
void launch_restrict2_values(const T *fine, int Pf, T *coarse, int Nc, int Pc, hipStream_t s)
{
    const int jc0 = 1, jc1 = Nc - 1;
    if (jc1 <= jc0) return;
    const int gx = (Nc - 2 + 251) / 252;
    const int rows = jc1 - jc0;
    int rpb = (rows * gx + 2047) / 2048;
    rpb = rpb < 4 ? 4 : rpb;
    const int gy = (rows + rpb - 1) / rpb;
    k_restrict2_values<T><<<dim3(gx, gy), dim3(256), 0, s>>>(fine, Pf, coarse, Nc, Pc, jc0, jc1, rpb);
}

template <class T>
__global__ void k_fill_rows(T *o, long long P, int row0, int row1)
{
    const long long n = (long long)(row1 - row0) * P;
    T *base = o + (long long)row0 * P;
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (long long)gridDim.x * blockDim.x)
        base[k] = T(0);
}

template <class T>
void launch_fill_rows(T *o, int P, int row0, int row1, hipStream_t s)
{
    long long nb = ((long long)(row1 - row0) * P + 255) / 256;
    if (nb > 8192) nb = 8192;
    if (nb < 1) nb = 1;
    k_fill_rows<T><<<dim3((unsigned)nb), dim3(256), 0, s>>>(o, P, row0, row1);
}

template <class T>
__global__ void k_zero_frame(T *o, long long P, int N, int r0, int r1)
{
    // rows 0, 1, N-1 whole; columns 0, N-1 of rows 2..N-2; only rows in [r0, r1)
    const int a = r0 > 2 ? r0 : 2, b = r1 < N - 1 ? r1 : N - 1;
    const int nmid = b > a ? b - a : 0;
    const int n = 3 * N + 2 * nmid;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        if (k < 3 * N) {
            const int j = k < N ? 0 : (k < 2 * N ? 1 : N - 1);
            if (j >= r0 && j < r1) o[(long long)j * P + (k % N)] = T(0);
        } else {
            const int r = k - 3 * N;
            o[(long long)(a + (r >> 1)) * P + ((r & 1) ? N - 1 : 0)] = T(0);
        }
    }
}

template <class T>
void launch_zero_frame(T *o, int P, int N, hipStream_t s, int r0, int r1)
{
    r0 = r0 < 0 ? 0 : r0;
    r1 = r1 > N ? N : r1;
    if (r1 <= r0) return;
    const int n = 3 * N + 2 * (r1 - r0);
    k_zero_frame<T><<<dim3((n + 255) / 256), dim3(256), 0, s>>>(o, P, N, r0, r1);
}

// rows 0 and N-1 and columns 0 and N-1 of a double grid (pitch Ps: the caller's array in the
// reference layout) into a level grid (pitch Pd) — the boundary the passes pass through
template <class T>
__global__ void k_copy_frame(const double *src, long long Ps, T *dst, long long Pd, int N)
{
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < 4 * N; k += gridDim.x * blockDim.x) {
        const int q = k % N, w = k / N;
        const int j = w == 0 ? 0 : (w == 1 ? N - 1 : q);
        const int i = w < 2 ? q : (w == 2 ? 0 : N - 1);
        dst[(long long)j * Pd + i] = (T)src[(long long)j * Ps + i];
    }
}

template <class T>
void launch_copy_frame(const double *src, long long Ps, T *dst, long long Pd, int N, hipStream_t s)
{
    k_copy_frame<T><<<dim3((4 * N + 255) / 256), dim3(256), 0, s>>>(src, Ps, dst, Pd, N);
}

// sum r(x)^2 over rows [row0,row1), interior columns — reporting only
template <class T>
__global__ __launch_bounds__(kBlock) void k_resnorm(const T *x, const T *f, double *partials,
                                                    T ih, int W, long long P, int row0, int row1)
{
    __shared__ double red[kBlock / 64];
    const long long n = (long long)(row1 - row0) * (W - 2);
    double acc = 0.0;
    for (long long k = (long long)blockIdx.x * kBlock + threadIdx.x; k < n;
         k += (long long)gridDim.x * kBlock) {
        const int j = row0 + (int)(k / (W - 2));
        const int i = 1 + (int)(k % (W - 2));
        const long long q = j * P + i;
        const T r = f[q] - ih * (T(4) * x[q] - x[q - 1] - x[q + 1] - x[q - P] - x[q + P]);
        acc += sq(r);
    }
    const double s = block_sum<kBlock>(acc, red);
    if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

template <class T>
void launch_resnorm_partials(const T *x, const T *f, double *partials, T inv_hh, int W, int P,
                             int row0, int row1, int nblocks, hipStream_t s)
{
    k_resnorm<T><<<dim3(nblocks), dim3(kBlock), 0, s>>>(x, f, partials, inv_hh, W, P, row0, row1);
}

__global__ __launch_bounds__(kBlock) void k_sum_partials(const double *partials, int np,
                                                         double *out)
{
    __shared__ double red[kBlock / 64];
    double s = 0.0;
    for (int k = threadIdx.x; k < np; k += kBlock) s += partials[k];
    s = block_sum<kBlock>(s, red);
    if (threadIdx.x == 0) *out = s;
}

void launch_sum_partials(const double *partials, int np, double *out, hipStream_t s)
{
    k_sum_partials<<<dim3(1), dim3(kBlock), 0, s>>>(partials, np, out);
}

// widen / narrow rows between T storage (pitch P) and a dense double array (pitch N)
template <class T>
__global__ void k_to_double(const T *src, long long P, double *dst, int N, int row0, int row1)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = row0 + blockIdx.y;
    if (i >= N || j >= row1) return;
    dst[(long long)j * N + i] = (double)src[j * P + i];
}

template <class T>
__global__ void k_from_double(const double *src, int N, T *dst, long long P, int row0, int row1)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = row0 + blockIdx.y;
    if (i >= N || j >= row1) return;
    dst[j * P + i] = (T)src[(long long)j * N + i];
}

template <class T>
void launch_to_double(const T *src, int P, double *dst, int N, int row0, int row1, hipStream_t s)
{
    if (row1 > row0)
        k_to_double<T><<<dim3((N + 255) / 256, row1 - row0), dim3(256), 0, s>>>(src, P, dst, N, row0, row1);
}

template <class T>
void launch_from_double(const double *src, int N, T *dst, int P, int row0, int row1, hipStream_t s)
{
    if (row1 > row0)
        k_from_double<T><<<dim3((N + 255) / 256, row1 - row0), dim3(256), 0, s>>>(src, N, dst, P, row0, row1);
}

#define PGMG_INSTANTIATE(T)                                                                        \
    template void launch_sweep<T>(const SweepArgsT<T> &, bool, bool, hipStream_t);                \
    template void launch_res_restrict<T>(const ResRestrictArgsT<T> &, hipStream_t);                \
    template void launch_prolong<T>(const ProlongArgsT<T> &, hipStream_t);                         \
    template void launch_fixup<T>(const FixupArgsT<T> &, hipStream_t);                             \
    template void launch_copy_rows<T>(const T *, T *, int, int, int, int, hipStream_t);            \
    template void launch_rhs<T>(T *, const double *, const double *, double, int, int, int, int,   \
                                hipStream_t);                                                      \
    template void launch_restrict_values<T>(const T *, int, int, T *, int, int, hipStream_t, int, int); \
    template void launch_restrict2_values<T>(const T *, int, T *, int, int, hipStream_t);            \
    template void launch_fill_rows<T>(T *, int, int, int, hipStream_t);                            \
    template void launch_zero_frame<T>(T *, int, int, hipStream_t, int, int);                      \
    template void launch_copy_frame<T>(const double *, long long, T *, long long, int, hipStream_t); \
    template void launch_resnorm_partials<T>(const T *, const T *, double *, T, int, int, int, int, \
                                             int, hipStream_t);                                    \
    template void launch_to_double<T>(const T *, int, double *, int, int, int, hipStream_t);      \
    template void launch_from_double<T>(const double *, int, T *, int, int, int, hipStream_t);
PGMG_INSTANTIATE(double)
PGMG_INSTANTIATE(float)
#undef PGMG_INSTANTIATE

}  // namespace pgmg
