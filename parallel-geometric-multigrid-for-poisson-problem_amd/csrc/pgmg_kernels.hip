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

// ---------------------------------------------------------------------------
// lane exchange: wave64 DPP moves on the two dword halves of a double
// ---------------------------------------------------------------------------
__device__ __forceinline__ double dpp_prev(double v)  // lane i <- lane i-1 (wave_shr:1)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x138, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x138, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double dpp_next(double v)  // lane i <- lane i+1 (wave_shl:1)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x130, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x130, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double2 ld2(const double *p) { return *reinterpret_cast<const double2 *>(p); }
__device__ __forceinline__ void st2(double *p, double2 v) { *reinterpret_cast<double2 *>(p) = v; }

// deterministic block sum (fixed tree) of one double per thread; result valid in thread 0
template <int NT>
__device__ __forceinline__ double block_sum(double v, double *red)
{
    #pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
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

template <bool X0_ZERO, bool NORM, bool FINE>
__global__ __launch_bounds__(kBlock) void k_sweep(SweepArgs a)
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
    const double *__restrict__ X = a.xin;
    const double *__restrict__ F = a.f;
    double *__restrict__ O = a.xout;
    const double hh = a.hh, ih = a.inv_hh;
    double acc = 0.0;

    double2 w0 = make_double2(0.0, 0.0), w1 = make_double2(0.0, 0.0);
    if (!X0_ZERO) {
        w0 = ld2(X + (jb - 1) * P + c);
        w1 = ld2(X + jb * P + c);
    }
    for (int j = jb; j < je; j += kU) {
        double2 xn[kU], fv[kU];
        double el[kU], er[kU];
        #pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int r = min(j + u, je - 1);
            fv[u] = ld2(F + r * P + c);
            el[u] = 0.0;
            er[u] = 0.0;
            if (!X0_ZERO) {
                xn[u] = ld2(X + (r + 1) * P + c);
                if (lane == 0) el[u] = X[r * P + c - 1];
                if (lane == 63) er[u] = X[r * P + c + 2];
            } else {
                xn[u] = make_double2(0.0, 0.0);
            }
        }
        #pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int r = j + u;
            const double2 up = (u == 0) ? w0 : (u == 1 ? w1 : xn[u - 2]);
            const double2 ce = (u == 0) ? w1 : xn[u - 1];
            const double2 dn = xn[u];
            double left = dpp_prev(ce.y);
            double right = dpp_next(ce.x);
            if (lane == 0) left = el[u];
            if (lane == 63) right = er[u];
            double2 o;
            o.x = 0.25 * ((hh * fv[u].x) + left + ce.y + up.x + dn.x);
            o.y = second ? 0.25 * ((hh * fv[u].y) + ce.x + right + up.y + dn.y) : ce.y;
            const bool live = act && r < je;
            if (NORM) {
                const double r0 = fv[u].x - ih * (4 * ce.x - left - ce.y - up.x - dn.x);
                const double r1 = fv[u].y - ih * (4 * ce.y - ce.x - right - up.y - dn.y);
                if (live) {
                    acc += r0 * r0;
                    if (second) acc += r1 * r1;
                }
            }
            if (live) st2(O + r * P + c, o);
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

void launch_sweep(const SweepArgs &a, bool x0_zero, bool fine, hipStream_t s)
{
    int rpb, gx, gy;
    sweep_blocks(a.W, a.row0, a.row1, &rpb, &gx, &gy);
    SweepArgs b = a;
    b.rows_per_block = rpb;
    const dim3 grid(gx, gy), blk(kBlock);
    const bool norm = a.partials != nullptr;
    if (fine) {
        if (x0_zero) k_sweep<true, false, true><<<grid, blk, 0, s>>>(b);
        else if (norm) k_sweep<false, true, true><<<grid, blk, 0, s>>>(b);
        else k_sweep<false, false, true><<<grid, blk, 0, s>>>(b);
    } else {
        if (x0_zero) k_sweep<true, false, false><<<grid, blk, 0, s>>>(b);
        else if (norm) k_sweep<false, true, false><<<grid, blk, 0, s>>>(b);
        else k_sweep<false, false, false><<<grid, blk, 0, s>>>(b);
    }
}

// ---------------------------------------------------------------------------
// Fused residual + full-weighting restriction.
// Reference: MultiGrid.hpp:70-78 (compute_residual then restrict_full_weighting)
//   C[c] = 0.25*F[k] + 0.125*(F[k+1] + F[k-1] + F[k+Nf] + F[k-Nf])
//        + 0.0625*(F[k-Nf-1] + F[k-Nf+1] + F[k+Nf-1] + F[k+Nf+1])   (:199-202)
// with F = r computed on the fly (never written to HBM).  Lane t produces coarse
// column ic = t+1, whose fine centre column is c+1 (c = 2t+1).
// ---------------------------------------------------------------------------
struct XRow {
    double2 own;   // x at (c, c+1)
    double2 nxt;   // x at (c+2, c+3)
    double lft;    // x at c-1
};

__device__ __forceinline__ XRow load_xrow(const double *X, long long off, int c, int lane)
{
    XRow r;
    r.own = ld2(X + off + c);
    r.nxt.x = dpp_next(r.own.x);
    r.nxt.y = dpp_next(r.own.y);
    r.lft = dpp_prev(r.own.y);
    if (lane == 63) r.nxt = ld2(X + off + c + 2);
    if (lane == 0) r.lft = X[off + c - 1];
    return r;
}

struct RTriple {
    double r0, r1, r2;  // residual at columns c, c+1, c+2
};

__device__ __forceinline__ RTriple resid3(const XRow &u, const XRow &m, const XRow &d, double2 fo,
                                          double fn, double ih)
{
    RTriple r;
    r.r0 = fo.x - ih * (4 * m.own.x - m.lft - m.own.y - u.own.x - d.own.x);
    r.r1 = fo.y - ih * (4 * m.own.y - m.own.x - m.nxt.x - u.own.y - d.own.y);
    r.r2 = fn - ih * (4 * m.nxt.x - m.own.y - m.nxt.y - u.nxt.x - d.nxt.x);
    return r;
}

__global__ __launch_bounds__(kBlock) void k_res_restrict(ResRestrictArgs a)
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
    const double *__restrict__ X = a.x;
    const double *__restrict__ F = a.f;
    const double ih = a.inv_hh;

    // window: x rows 2jc-1 (A) and 2jc (B); r row 2jc-1 (up)
    XRow xz = load_xrow(X, (2LL * jcb - 2) * Pf, c, lane);
    XRow xa = load_xrow(X, (2LL * jcb - 1) * Pf, c, lane);
    XRow xb = load_xrow(X, (2LL * jcb) * Pf, c, lane);
    double2 fo = ld2(F + (2LL * jcb - 1) * Pf + c);
    double fn = dpp_next(fo.x);
    if (lane == 63) fn = F[(2LL * jcb - 1) * Pf + c + 2];
    RTriple up = resid3(xz, xa, xb, fo, fn, ih);

    for (int jc = jcb; jc < jce; ++jc) {
        const long long rm = 2LL * jc, rd = rm + 1;
        const XRow xc = load_xrow(X, rd * Pf, c, lane);
        const XRow xd = load_xrow(X, (rd + 1) * Pf, c, lane);
        const double2 fm = ld2(F + rm * Pf + c);
        const double2 fd = ld2(F + rd * Pf + c);
        double fmn = dpp_next(fm.x), fdn = dpp_next(fd.x);
        if (lane == 63) {
            fmn = F[rm * Pf + c + 2];
            fdn = F[rd * Pf + c + 2];
        }
        const RTriple mid = resid3(xa, xb, xc, fm, fmn, ih);
        const RTriple dn = resid3(xb, xc, xd, fd, fdn, ih);
        const double v = 0.25 * mid.r1 + 0.125 * (mid.r2 + mid.r0 + dn.r1 + up.r1) +
                         0.0625 * (up.r0 + up.r2 + dn.r0 + dn.r2);
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

void launch_res_restrict(const ResRestrictArgs &a, hipStream_t s)
{
    const int bx = (a.Wc - 2 + kBlock - 1) / kBlock;
    const int rows = a.jc1 - a.jc0;
    ResRestrictArgs b = a;
    b.rows_per_block = res_restrict_rows_per_block(a.Wc, rows);
    const int by = (rows + b.rows_per_block - 1) / b.rows_per_block;
    k_res_restrict<<<dim3(bx, by), dim3(kBlock), 0, s>>>(b);
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
__global__ __launch_bounds__(kBlock) void k_prolong(ProlongArgs a)
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
        const double *C0 = a.c + jc * Pc;
        const double c00 = C0[t], c01 = C0[t + 1];
        double2 v = ld2(a.fine + j * Pf + c);
        if ((j & 1) == 0) {
            if (okx) v.x = v.x + 0.5 * (c00 + c01);
            if (oky) v.y = v.y + c01;
        } else {
            const double *C1 = C0 + Pc;
            const double c10 = C1[t], c11 = C1[t + 1];
            if (okx) v.x = v.x + 0.25 * (c00 + c01 + c10 + c11);
            if (oky) v.y = v.y + 0.5 * (c01 + c11);
        }
        if (act) st2(a.fine + j * Pf + c, v);
    }
}

void launch_prolong(const ProlongArgs &a, hipStream_t s)
{
    const int npairs = (a.Wf - 1) / 2;
    const int bx = (npairs + kBlock - 1) / kBlock;
    const int rows = a.row1 - a.row0;
    int rpb = (int)(((long long)rows * bx + 4095) / 4096);
    rpb = rpb < 2 ? 2 : (rpb > 32 ? 32 : rpb);
    ProlongArgs b = a;
    b.rows_per_block = rpb;
    const int by = (rows + rpb - 1) / rpb;
    k_prolong<<<dim3(bx, by), dim3(kBlock), 0, s>>>(b);
}

// ---------------------------------------------------------------------------
// Early-exit fix-up (Smoother.hpp:75-88 `if (res_norm < epsilon) break;`).
// Sweep k ran speculatively and left sum r(x_{k-1})^2 per block in `partials`.
// Every block re-reduces the partials in the same fixed order (no atomics, so
// the decision is identical everywhere and run-to-run); on trigger the
// smoother's result is x_{k-1}: copy it over the speculative x_k.
// ---------------------------------------------------------------------------
constexpr int kFixBlocks = 256;

__global__ __launch_bounds__(kBlock) void k_fixup(FixupArgs a)
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
        st2(a.dst + r * P + c, ld2(a.src + r * P + c));
    }
}

void launch_fixup(const FixupArgs &a, hipStream_t s)
{
    k_fixup<<<dim3(kFixBlocks), dim3(kBlock), 0, s>>>(a);
}

__global__ __launch_bounds__(kBlock) void k_copy_rows(const double *src, double *dst, int W,
                                                      long long P, int row0, int row1)
{
    const int npairs = (W - 1) >> 1;
    const long long total = (long long)(row1 - row0) * npairs;
    for (long long k = (long long)blockIdx.x * kBlock + threadIdx.x; k < total;
         k += (long long)gridDim.x * kBlock) {
        const int r = row0 + (int)(k / npairs);
        const int c = 1 + 2 * (int)(k % npairs);
        st2(dst + r * P + c, ld2(src + r * P + c));
    }
}

void launch_copy_rows(const double *src, double *dst, int W, int P, int row0, int row1,
                      hipStream_t s)
{
    const long long total = (long long)(row1 - row0) * ((W - 1) / 2);
    long long nb = (total + kBlock - 1) / kBlock;
    if (nb > 4096) nb = 4096;
    if (nb < 1) nb = 1;
    k_copy_rows<<<dim3((unsigned)nb), dim3(kBlock), 0, s>>>(src, dst, W, P, row0, row1);
}

// ---------------------------------------------------------------------------
// RHS from separable host sine tables: f = factor * sin(p*pi*x/a) * sin(q*pi*y/a)
// (DynamicGridUtils.hpp:111-124) = (factor * sx[i]) * sy[j], same IEEE ops.
// ---------------------------------------------------------------------------
__global__ void k_rhs(double *f, const double *sx, const double *sy, double factor, int W,
                      long long P, int row0, int row1)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = row0 + blockIdx.y;
    if (i >= W || j >= row1) return;
    f[j * P + i] = factor * sx[i] * sy[j];
}

void launch_rhs(double *f, const double *sx, const double *sy, double factor, int W, int P,
                int row0, int row1, hipStream_t s)
{
    k_rhs<<<dim3((W + 255) / 256, row1 - row0), dim3(256), 0, s>>>(f, sx, sy, factor, W, P,
                                                                  row0, row1);
}

// MultiGrid.hpp:187-205 applied to values (compute_coarsest_grid, MultiGrid.hpp:28-55)
__global__ void k_restrict_values(const double *Fn, int Nf, long long Pf, double *C, int Nc,
                                  long long Pc)
{
    const long long n = (long long)(Nc - 2) * (Nc - 2);
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (long long)gridDim.x * blockDim.x) {
        const long long jc = 1 + k / (Nc - 2), ic = 1 + k % (Nc - 2);
        const long long q = (2 * jc) * Pf + 2 * ic;
        C[jc * Pc + ic] = 0.25 * Fn[q] + 0.125 * (Fn[q + 1] + Fn[q - 1] + Fn[q + Pf] + Fn[q - Pf]) +
                          0.0625 * (Fn[q - Pf - 1] + Fn[q - Pf + 1] + Fn[q + Pf - 1] + Fn[q + Pf + 1]);
    }
}

void launch_restrict_values(const double *fine, int Nf, int Pf, double *coarse, int Nc, int Pc,
                            hipStream_t s)
{
    long long nb = ((long long)(Nc - 2) * (Nc - 2) + 255) / 256;
    if (nb > 4096) nb = 4096;
    if (nb < 1) nb = 1;
    k_restrict_values<<<dim3((unsigned)nb), dim3(256), 0, s>>>(fine, Nf, Pf, coarse, Nc, Pc);
}

__global__ void k_fill_rows(double *o, long long P, int row0, int row1, double v)
{
    const long long n = (long long)(row1 - row0) * P;
    double *base = o + (long long)row0 * P;
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (long long)gridDim.x * blockDim.x)
        base[k] = v;
}

void launch_fill_rows(double *o, int P, int row0, int row1, double v, hipStream_t s)
{
    long long nb = ((long long)(row1 - row0) * P + 255) / 256;
    if (nb > 8192) nb = 8192;
    if (nb < 1) nb = 1;
    k_fill_rows<<<dim3((unsigned)nb), dim3(256), 0, s>>>(o, P, row0, row1, v);
}

// sum r(x)^2 over rows [row0,row1), interior columns — reporting only
__global__ __launch_bounds__(kBlock) void k_resnorm(const double *x, const double *f,
                                                    double *partials, double ih, int W,
                                                    long long P, int row0, int row1)
{
    __shared__ double red[kBlock / 64];
    const long long n = (long long)(row1 - row0) * (W - 2);
    double acc = 0.0;
    for (long long k = (long long)blockIdx.x * kBlock + threadIdx.x; k < n;
         k += (long long)gridDim.x * kBlock) {
        const int j = row0 + (int)(k / (W - 2));
        const int i = 1 + (int)(k % (W - 2));
        const long long q = j * P + i;
        const double r = f[q] - ih * (4 * x[q] - x[q - 1] - x[q + 1] - x[q - P] - x[q + P]);
        acc += r * r;
    }
    const double s = block_sum<kBlock>(acc, red);
    if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

void launch_resnorm_partials(const double *x, const double *f, double *partials, double inv_hh,
                             int W, int P, int row0, int row1, int nblocks, hipStream_t s)
{
    k_resnorm<<<dim3(nblocks), dim3(kBlock), 0, s>>>(x, f, partials, inv_hh, W, P, row0, row1);
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

}  // namespace pgmg
