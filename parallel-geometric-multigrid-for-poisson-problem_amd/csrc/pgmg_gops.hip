// pgmg_gops.hip — op-level kernels on caller-owned arrays in the reference layout
// (row-major, pitch = W, no padding, no alignment guarantee).  These back the C-ABI entries
// that mirror Parallel::ComputeJacobi / ComputeResidual / ComputeRestriction /
// ComputeProlungator (3_part_parallel/Parallel_Method.cu:144-199) and the per-op study that
// times them (ParallelTestRunner.cu:231-468); the V-cycle itself uses the aligned, fused
// passes of pgmg_fused.hip.
//
// Same streaming scheme as the level kernels (pgmg_kernels.hip), adapted to the caller's
// layout:
//   * lane t of a wave owns the column pair (c, c+1), c = 1 + 2t: one 16-byte load per row
//     and array.  With an odd pitch (every reference grid: W = 2^k + 1) every other row's
//     pairs are only 8-byte aligned; gfx950 runs in unaligned-access mode, so they are still
//     one global_load/store_dwordx4 each (ldvu / stvu, pgmg_real.h), a wave's 1 KiB row
//     segment spanning 9 cache lines instead of 8;
//   * workgroups march down bands of rows keeping the rows above and below in registers, U
//     rows of loads issued before any is used, so each input element crosses HBM once per
//     op (plus one halo row per band);
//   * horizontal neighbours come from the adjacent lane by DPP (wave_shr / wave_shl); only
//     a wave's edge lanes load a halo column;
//   * no 64-bit division in the index path (the r03 kernels were one thread per point with a
//     k / (W - 2), k % (W - 2) per point).
// Expressions and their order are the reference's, file:line at each kernel; the build uses
// -ffp-contract=off, so every value is bit-identical to the CPU reference (the KATs in
// tests/test_gpu_parity.py).  Per-block partial sums use a fixed grid, so early-exit
// decisions are deterministic run to run.
#include <algorithm>

#include "pgmg_internal.h"

namespace pgmg {

template <int NT>
__device__ __forceinline__ double gblock_sum(double v, double *red)
{
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0) {
        #pragma unroll
        for (int i = 0; i < NT / 64; ++i) s += red[i];
    }
    return s;
}

__device__ __forceinline__ void st_nt1(double *p, double v) { __builtin_nontemporal_store(v, p); }
// a column pair's 16-byte store (8-byte alignment promised: one global_store_dwordx4 either
// way; NT: non-temporal, the output is read again only a whole pass later)
typedef double dpair_u __attribute__((ext_vector_type(2), aligned(8)));
template <bool NT>
__device__ __forceinline__ void st2(double *p, double2 v)
{
    if (NT) {
        dpair_u w;
        w.x = v.x;
        w.y = v.y;
        __builtin_nontemporal_store(w, reinterpret_cast<dpair_u *>(p));
    } else {
        stvu<double>(p, v);
    }
}

// Geometry of a row-marching op over `rows` rows of `pairs` lane pairs: gx column blocks of
// kBlock lanes, gy bands of rpb rows (a multiple of U), about `target` workgroups in all.
struct OpGeom {
    int gx, gy, rpb;
};
static OpGeom op_geom(int pairs, int rows, int U, int target)
{
    OpGeom g;
    g.gx = (pairs + kBlock - 1) / kBlock;
    long long rpb = ((long long)rows * g.gx + target - 1) / target;
    if (rpb < U) rpb = U;
    rpb = (rpb + U - 1) / U * U;
    if (rows < 1) rows = 1;
    g.rpb = (int)rpb;
    g.gy = (int)((rows + rpb - 1) / rpb);
    if (g.gy < 1) g.gy = 1;
    return g;
}

// ---------------------------------------------------------------------------
// One Jacobi sweep, out-of-place.  Smoother.hpp:63-70 (JacobiSmoother::smooth):
//   out[i] = 0.25 * ((h*h*f[i]) + x[i-1] + x[i+1] + x[i-W] + x[i+W])
// CHECK: per-block partial sums of r(x)^2 of the INPUT x (the early-exit check of the
// previous sweep's result, DynamicGridUtils.hpp:59-69 + norm; decided by k_g_fixup):
//   r[i] = f[i] - (1.0/(h*h)) * (4*x[i] - x[i-1] - x[i+1] - x[i-W] - x[i+W])
// SEED: also copy x's boundary (rows 0, H-1; columns 0, W-1) into out, so a ping-pong buffer
// needs no full seed copy (the next sweep reads the boundary as neighbours).
// ---------------------------------------------------------------------------
template <int U, bool CHECK, bool SEED, bool NT>
__global__ __launch_bounds__(kBlock) void k_op_sweep(const double *__restrict__ X,
                                                     const double *__restrict__ F,
                                                     double *__restrict__ O, double *partials,
                                                     const unsigned *skip, unsigned *reset,
                                                     unsigned long long *stats, double hh,
                                                     double ih, int H, int W, int rpb)
{
    __shared__ double red[kBlock / 64];
    if (skip != nullptr && *skip != 0u) return;  // the smoother already exited (uniform)
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        if (reset != nullptr) *reset = 0u;
        if (stats != nullptr) atomicAdd(&stats[0], 1ull);
    }
    const int lane = threadIdx.x & 63;
    const int npairs = (W - 1) >> 1;
    const int t_raw = blockIdx.x * kBlock + threadIdx.x;
    const bool act = t_raw < npairs;
    const int t = act ? t_raw : npairs - 1;  // idle lanes shadow the last pair
    const int c = 1 + 2 * t;
    const bool second = c + 1 <= W - 2;      // else column c+1 is the right boundary
    const bool lastp = t == npairs - 1;
    const bool ld_l = lane == 0;
    // the right neighbour of column c+1: the next lane's column, loaded by a wave's last lane
    // and by the last pair (W even: its next lane shadows it)
    const bool ld_r = (lane == 63 || lastp) && second;
    const int jb = 1 + blockIdx.y * rpb;
    const int je = min(jb + rpb, H - 1);
    const long long Wl = W;
    double acc = 0.0;

    double2 w0 = ldvu<double>(X + (long long)(jb - 1) * Wl + c);
    double2 w1 = ldvu<double>(X + (long long)jb * Wl + c);
    if (SEED && jb == 1 && act) st2<false>(O + c, w0);
    for (int j = jb; j < je; j += U) {
        double2 xn[U], fv[U];
        double el[U], er[U];
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long r = min(j + u, je - 1);
            fv[u] = ldvu<double>(F + r * Wl + c);
            xn[u] = ldvu<double>(X + (r + 1) * Wl + c);
            el[u] = ld_l ? X[r * Wl + c - 1] : 0.0;
            er[u] = ld_r ? X[r * Wl + c + 2] : 0.0;
        }
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = j + u;
            const double2 up = (u == 0) ? w0 : (u == 1 ? w1 : xn[u - 2]);
            const double2 ce = (u == 0) ? w1 : xn[u - 1];
            const double2 dn = xn[u];
            double left = dpp_shr(ce.y);
            double right = dpp_shl(ce.x);
            if (ld_l) left = el[u];
            if (ld_r) right = er[u];
            double2 o;
            o.x = 0.25 * ((hh * fv[u].x) + left + ce.y + up.x + dn.x);
            o.y = second ? 0.25 * ((hh * fv[u].y) + ce.x + right + up.y + dn.y) : ce.y;
            const bool live = act && r < je;
            if (CHECK) {
                const double r0 = fv[u].x - ih * (4 * ce.x - left - ce.y - up.x - dn.x);
                const double r1 = fv[u].y - ih * (4 * ce.y - ce.x - right - up.y - dn.y);
                if (live) {
                    acc += r0 * r0;
                    if (second) acc += r1 * r1;
                }
            }
            if (live) {
                double *q = O + (long long)r * Wl + c;
                st2<NT>(q, o);
                if (SEED) {
                    if (t == 0) q[-1] = el[u];
                    if (lastp && second) q[2] = er[u];
                }
            }
        }
        w0 = xn[U - 2];
        w1 = xn[U - 1];
    }
    if (SEED && je == H - 1 && act) st2<false>(O + (long long)(H - 1) * Wl + c, w1);
    if (CHECK) {
        const double s = gblock_sum<kBlock>(acc, red);
        if (threadIdx.x == 0) partials[blockIdx.y * gridDim.x + blockIdx.x] = s;
    }
}

// Lane t's column pair (c, c+1) of a row; a pair that leaves the row loads element-wise.
__device__ __forceinline__ double2 ld_pair(const double *row, int c, int W)
{
    if (c >= 0 && c + 1 <= W - 1) return ldvu<double>(row + c);
    double2 v;
    v.x = (c >= 0 && c <= W - 1) ? row[c] : 0.0;
    v.y = (c + 1 >= 0 && c + 1 <= W - 1) ? row[c + 1] : 0.0;
    return v;
}

template <bool NT>
__device__ __forceinline__ void st_owned(double *q, double2 o, bool ox, bool oy)
{
    if (ox && oy) st2<NT>(q, o);
    else if (ox) q[0] = o.x;
    else if (oy) q[1] = o.y;
}

// ---------------------------------------------------------------------------
// Geometry of the paired sweep (k_op_sweep2_ip below): wave tiles load 128 columns and own
// the 120 of lanes 2..61 (two stencil levels shrink the valid columns by one per side each).
// ---------------------------------------------------------------------------
constexpr int kOv2Stride = 120;

static OpGeom sweep2_geom(int H, int W, int U, int target)
{
    const int waves = (W - 2 + kOv2Stride - 1) / kOv2Stride;
    return op_geom(waves * 64, H - 2, U, target);
}

constexpr int kOpTarget = 4096;   // workgroups per op launch (16 per CU)

// Measured at N = 16385 (scripts/op_ab.py, profiles/r04_ops/): one round of resident
// workgroups (1024 of 4 waves on 256 CUs) and non-temporal stores beat 2048-8192 workgroups,
// 4 rows, default stores or overlapping wave tiles (r04, kept in git history); r04 (op_ab.py
// --rows, profiles/r04_ops/op_rows.jsonl): 16 rows in flight (214 VGPRs: 2 waves per SIMD, the
// 1024 workgroups in two rounds) 1.390-1.393 ms against 1.403-1.405 for 8 rows on the same box
static OpGeom sweep_geom(int H, int W)
{
    return op_geom((W - 1) / 2, H - 2, 16, tuning_int("PGMG_OP_BLOCKS", 1024));
}

int g_blocks(int H, int W)
{
    const OpGeom g = sweep_geom(H, W);
    return g.gx * g.gy;
}

void launch_g_sweep(const double *xin, const double *f, double *xout, double *partials,
                    const unsigned *skip, unsigned *reset, unsigned long long *stats, double hh,
                    double inv_hh, int H, int W, bool seed, hipStream_t s)
{
    const OpGeom g = sweep_geom(H, W);
    const dim3 grid(g.gx, g.gy);
    const bool chk = partials != nullptr;
#define PGMG_K(CH, SD) k_op_sweep<16, CH, SD, true><<<grid, kBlock, 0, s>>>(xin, f, xout, partials, skip, reset, stats, hh, inv_hh, H, W, g.rpb)
    if (chk && seed) PGMG_K(true, true);
    else if (chk) PGMG_K(true, false);
    else if (seed) PGMG_K(false, true);
    else PGMG_K(false, false);
#undef PGMG_K
}

// ---------------------------------------------------------------------------
// Early-exit decision after a checked sweep (Smoother.hpp:75-80): re-reduce the partials in a
// fixed order; when sqrt(sum) < eps the sweep that followed the check is undone (out := in on
// the interior) and every later sweep of the call skips.  Rare path: only when a check fires.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_g_fixup(const double *partials, int np, double eps,
                                                    const unsigned *done_prev, unsigned *done_next,
                                                    const double *src, double *dst,
                                                    unsigned long long *stats, int H, int W)
{
    __shared__ double red[kBlock / 64];
    __shared__ int trig;
    const bool leader = blockIdx.x == 0 && threadIdx.x == 0;
    if (*done_prev != 0u) {
        if (leader) *done_next = 1u;
        return;
    }
    double s = 0.0;
    for (int k = threadIdx.x; k < np; k += kBlock) s += partials[k];
    s = gblock_sum<kBlock>(s, red);
    if (threadIdx.x == 0) trig = (sqrt(s) < eps) ? 1 : 0;
    __syncthreads();
    if (leader) {
        *done_next = trig ? 1u : 0u;
        if (trig && stats != nullptr) {
            atomicAdd(&stats[0], (unsigned long long)-1LL);
            atomicAdd(&stats[1], 1ull);
        }
    }
    if (!trig) return;
    // rows of the interior over the blocks, columns over the threads
    const long long Wl = W;
    for (int r = 1 + blockIdx.x; r < H - 1; r += gridDim.x)
        for (int i = 1 + threadIdx.x; i < W - 1; i += kBlock) dst[r * Wl + i] = src[r * Wl + i];
}

void launch_g_fixup(const double *partials, int np, double eps, const unsigned *done_prev,
                    unsigned *done_next, const double *src, double *dst,
                    unsigned long long *stats, int H, int W, hipStream_t s)
{
    k_g_fixup<<<dim3(256), dim3(kBlock), 0, s>>>(partials, np, eps, done_prev, done_next, src,
                                                  dst, stats, H, W);
}

// ---------------------------------------------------------------------------
// In-place sweeps (r05): Parallel::ComputeJacobi updates the caller's one array d_x
// (Parallel_Method.cu:144-160, jacobi_kernel :6-24, which races -- SURVEY Q3); these passes
// write x in place and still compute exactly the out-of-place sweep J(x), with no ping-pong
// buffer and no interior copy-back.
//
// A workgroup owns a tile: a band of rows [jb, je) by its column range.  Inside the tile it
// marches the rows as the out-of-place kernels do (each row's old values are read before the
// row is written, and are kept in registers for the next row); an output that ANOTHER
// workgroup reads as an input is never written in place, it is deferred to a side buffer:
//   * the band's edge rows (the band above reads row jb, the one below row je-1; two rows per
//     side for the paired sweeps, which read two rows of halo) -> SR, one row per slot;
//   * the columns at the boundary between column blocks e and e+1 -> SC[(e*H + row)*K + k]:
//     the single sweep's 2 (block e's last column, block e+1's first), the paired pass's 4
//     (two per side: an owned output two columns from the boundary reads x two columns
//     across it; the next two columns the neighbour's edge lanes load reach only lanes that
//     own nothing, so their values may be old or new).
// The waves of one workgroup read each other's edge columns.  BAR: a barrier between an
// iteration's loads (waited for) and its stores orders them (iteration i stores rows that no
// wave loads in iteration i+1 or later), and only the workgroup boundaries are deferred;
// !BAR: no barrier, every WAVE boundary is deferred instead (2 of 128 columns for the single
// sweep, 8 of 120 for the paired pass).  launch_g_defer_scatter then writes the deferred
// values into x (after the pass, in stream order).
// No wave leaves early (lanes past the grid shadow or load zeros), so every barrier is met.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wait_loads_then_barrier()
{
    __builtin_amdgcn_s_waitcnt(0);   // this wave's loads have returned
    __syncthreads();
}

template <int U, bool NT, bool BAR, int NTH = kBlock>
__global__ __launch_bounds__(NTH) void k_op_sweep_ip(double *X, const double *__restrict__ F,
                                                        double *__restrict__ SR,
                                                        double *__restrict__ SC, unsigned *reset,
                                                        unsigned long long *stats, double hh,
                                                        int H, int W, int rpb)
{
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        if (reset != nullptr) *reset = 0u;
        if (stats != nullptr) atomicAdd(&stats[0], 1ull);
    }
    const int lane = threadIdx.x & 63;
    const int npairs = (W - 1) >> 1;
    const int t_raw = blockIdx.x * NTH + threadIdx.x;
    const bool act = t_raw < npairs;
    const int t = act ? t_raw : npairs - 1;  // idle lanes shadow the last pair (no stores)
    const int c = 1 + 2 * t;
    const bool second = c + 1 <= W - 2;
    const bool lastp = t == npairs - 1;
    const bool ld_l = lane == 0;
    const bool ld_r = (lane == 63 || lastp) && second;
    const int jb = 1 + blockIdx.y * rpb;
    const int je = min(jb + rpb, H - 1);
    const bool def_top = jb > 1, def_bot = je < H - 1;
    // boundaries (BAR: of column blocks, else of waves) e: unit e's last lane (.y) and unit
    // e+1's first lane (.x); a next unit exists iff its first pair is in the row
    const int gw = t_raw >> 6;   // the wave's index along the row
    const bool def_l = BAR ? (threadIdx.x == 0 && blockIdx.x > 0) : (lane == 0 && gw > 0);
    const bool def_r = BAR ? (threadIdx.x == NTH - 1 && blockIdx.x + 1 < gridDim.x)
                           : (lane == 63 && 64 * (gw + 1) < npairs);
    const long long ue = BAR ? (long long)blockIdx.x : (long long)gw;   // this lane's unit
    const long long Wl = W;
    double2 w0 = ldvu<double>(X + (long long)(jb - 1) * Wl + c);
    double2 w1 = ldvu<double>(X + (long long)jb * Wl + c);
    for (int j = jb; j < je; j += U) {
        double2 xn[U], fv[U];
        double el[U], er[U];
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long r = min(j + u, je - 1);
            fv[u] = ldvu<double>(F + r * Wl + c);
            xn[u] = ldvu<double>(X + (r + 1) * Wl + c);
            el[u] = ld_l ? X[r * Wl + c - 1] : 0.0;
            er[u] = ld_r ? X[r * Wl + c + 2] : 0.0;
        }
        if (BAR) wait_loads_then_barrier();
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = j + u;
            const double2 up = (u == 0) ? w0 : (u == 1 ? w1 : xn[u - 2]);
            const double2 ce = (u == 0) ? w1 : xn[u - 1];
            const double2 dn = xn[u];
            double left = dpp_shr(ce.y);
            double right = dpp_shl(ce.x);
            if (ld_l) left = el[u];
            if (ld_r) right = er[u];
            double2 o;
            o.x = 0.25 * ((hh * fv[u].x) + left + ce.y + up.x + dn.x);
            o.y = second ? 0.25 * ((hh * fv[u].y) + ce.x + right + up.y + dn.y) : ce.y;
            if (act && r < je) {
                const bool dt = def_top && r == jb, db = def_bot && r == je - 1;
                if (dt) stvu<double>(SR + (long long)(2 * blockIdx.y) * Wl + c, o);
                if (db) stvu<double>(SR + (long long)(2 * blockIdx.y + 1) * Wl + c, o);
                if (def_l) SC[((ue - 1) * H + r) * 2 + 1] = o.x;
                if (def_r) SC[(ue * H + r) * 2] = o.y;
                if (!dt && !db) {
                    double *q = X + (long long)r * Wl + c;
                    if (def_l) q[1] = o.y;
                    else if (def_r) q[0] = o.x;
                    else st2<NT>(q, o);
                }
            }
        }
        w0 = xn[U - 2];
        w1 = xn[U - 1];
    }
}

// Two sweeps in one pass, in place: k_op_sweep2's wave tiles (128 columns loaded, the 120 of
// lanes 2..61 owned); the boundary columns are block e's last wave's lane 61 and block e+1's
// first wave's lane 2 (4 contiguous columns), the deferred rows two per band side.
template <int U, bool NT, bool BAR, int NTH = kBlock>
__global__ __launch_bounds__(NTH) void k_op_sweep2_ip(double *X, const double *__restrict__ F,
                                                         double *__restrict__ SR,
                                                         double *__restrict__ SC,
                                                         unsigned long long *stats, double hh,
                                                         int H, int W, int rpb)
{
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && stats != nullptr)
        atomicAdd(&stats[0], 2ull);
    constexpr int kWaves = NTH / 64;
    const int lane = threadIdx.x & 63;
    const int wib = threadIdx.x >> 6;
    const int wave = (blockIdx.x * NTH + threadIdx.x) >> 6;
    const int c = kOv2Stride * wave - 3 + 2 * lane;
    const bool inx = c >= 1 && c <= W - 2, iny = c + 1 >= 1 && c + 1 <= W - 2;
    const bool mid = lane >= 2 && lane <= 61;
    const bool ox = mid && inx, oy = mid && iny;
    // this lane's slot in the boundary buffer (-1: not a boundary column)
    int kc = -1;
    long long eb = 0;
    if (BAR) {   // column-block boundaries
        if (wib == kWaves - 1 && lane == 61 && blockIdx.x + 1 < gridDim.x) {
            kc = 0;
            eb = blockIdx.x;
        } else if (wib == 0 && lane == 2 && blockIdx.x > 0) {
            kc = 2;
            eb = blockIdx.x - 1;
        }
    } else {     // wave boundaries (a next wave exists iff its first owned column is in the row)
        const int nwaves = (W - 2 + kOv2Stride - 1) / kOv2Stride;
        if (lane == 61 && wave + 1 < nwaves) {
            kc = 0;
            eb = wave;
        } else if (lane == 2 && wave > 0 && wave < nwaves) {
            kc = 2;
            eb = wave - 1;
        }
    }
    const int jb = 1 + blockIdx.y * rpb;
    const int je = min(jb + rpb, H - 1);   // x2 rows [jb, je)
    const bool def_top = jb > 1, def_bot = je < H - 1;
    const long long Wl = W;
    auto ldrow = [&](const double *A, int r) {
        return (r >= 0 && r <= H - 1) ? ld_pair(A + (long long)r * Wl, c, W) : make_double2(0.0, 0.0);
    };
    auto jrow = [&](double2 up, double2 ce, double2 dn, double2 f) {
        const double l = dpp_shr(ce.y);
        const double r = dpp_shl(ce.x);
        double2 o;
        o.x = inx ? 0.25 * ((hh * f.x) + l + ce.y + up.x + dn.x) : ce.x;
        o.y = iny ? 0.25 * ((hh * f.y) + ce.x + r + up.y + dn.y) : ce.y;
        return o;
    };
    double2 xa = ldrow(X, jb - 2), xb = ldrow(X, jb - 1);
    double2 fa = make_double2(0.0, 0.0), fb = ldrow(F, jb - 1);
    double2 ya = make_double2(0.0, 0.0), yb = make_double2(0.0, 0.0);
    const int iend = je + 2;   // new rows i = jb .. je+1
    for (int i = jb; i < iend; i += U) {
        double2 xn[U], fn[U];
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = min(i + u, iend - 1);
            xn[u] = ldrow(X, r);
            fn[u] = ldrow(F, r);
        }
        if (BAR) wait_loads_then_barrier();
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            const int ii = i + u;
            if (ii < iend) {
                const int r1 = ii - 1;
                double2 y1 = jrow(xa, xb, xn[u], fb);
                if (r1 < 1 || r1 > H - 2) y1 = xb;
                const int r2 = ii - 2;
                if (r2 >= jb) {
                    const double2 z = jrow(ya, yb, y1, fa);
                    const bool dt = def_top && r2 < jb + 2, db = def_bot && r2 >= je - 2;
                    if (dt) st_owned<false>(SR + (long long)(4 * blockIdx.y + (r2 - jb)) * Wl + c, z, ox, oy);
                    if (db) st_owned<false>(SR + (long long)(4 * blockIdx.y + 2 + r2 - (je - 2)) * Wl + c, z, ox, oy);
                    if (kc >= 0) stvu<double>(SC + (eb * H + r2) * 4 + kc, z);
                    else if (!dt && !db) st_owned<NT>(X + (long long)r2 * Wl + c, z, ox, oy);
                }
                xa = xb;
                xb = xn[u];
                fa = fb;
                fb = fn[u];
                ya = yb;
                yb = y1;
            }
        }
    }
}

// The deferred outputs into x.  blockIdx.y < nslot (= gy * 2R): one band-row slot (the first R
// rows of band by when a band lies above it, the last R when one lies below), the x blocks
// striding over its columns; blockIdx.y >= nslot: one column-block boundary e (K columns from
// col0(e) = ca*e + cb), the x blocks striding over rows 1 .. H-2.  No division in the loops.
__global__ __launch_bounds__(kBlock) void k_op_defer_scatter(double *X, const double *SR,
                                                             const double *SC, int H, int W,
                                                             int rpb, int gy, int R, int K,
                                                             int ca, int cb)
{
    const long long Wl = W;
    const int nslot = gy * 2 * R;
    const int tid = blockIdx.x * kBlock + threadIdx.x, nthr = gridDim.x * kBlock;
    if ((int)blockIdx.y < nslot) {
        const int slot = blockIdx.y;
        const int by = slot / (2 * R), sl = slot - by * 2 * R;
        const int jb = 1 + by * rpb, je = min(jb + rpb, H - 1);
        int row;
        bool ok;
        if (sl < R) {
            row = jb + sl;
            ok = jb > 1 && row < je;
        } else {
            row = je - R + (sl - R);
            ok = je < H - 1 && row >= jb;
        }
        if (!ok) return;
        const double *src = SR + (long long)slot * Wl;
        double *dst = X + row * Wl;
        for (int col = 1 + tid; col <= W - 2; col += nthr) dst[col] = src[col];
    } else {
        const int e = blockIdx.y - nslot;
        const int c0 = ca * e + cb;
        for (int row = 1 + tid; row <= H - 2; row += nthr) {
            const double *src = SC + ((long long)e * H + row) * K;
            double *dst = X + row * Wl + c0;
            for (int q = 0; q < K; q += 2) {
                const double2 v = ldvu<double>(src + q);
                if (c0 + q >= 1 && c0 + q + 1 <= W - 2) {
                    stvu<double>(dst + q, v);
                } else {
                    if (c0 + q >= 1 && c0 + q <= W - 2) dst[q] = v.x;
                    if (c0 + q + 1 >= 1 && c0 + q + 1 <= W - 2) dst[q + 1] = v.y;
                }
            }
        }
    }
}

// The single in-place sweep: 512-thread workgroups (8 waves; half the column-block boundaries
// to defer of 256) and 512 of them (one per CU at 217 VGPRs), 16 rows in flight, non-temporal
// stores, tile edges deferred per column block.  Measured at 16385 (r05, scripts/op_ip_ab.py
// --nth, profiles/r05_ops/op_ip_nth.jsonl, 3 interleaved rounds): one-sweep call 1.320-1.329 ms
// against 1.382-1.398 with 256 threads x 1024 (1.333-1.336 at 512 x 1024, 1.359-1.364 with 8
// rows in flight); the forms measured against it are in git history (r05).
constexpr int kIpNth = 512, kIpRows = 16;
static OpGeom sweep_ip_geom(int H, int W)
{
    // op_geom counts columns in workgroups of kBlock lanes: scale the pair count
    OpGeom g = op_geom(((W - 1) / 2 + kIpNth / kBlock - 1) / (kIpNth / kBlock), H - 2, kIpRows,
                       tuning_int("PGMG_OPIP_BLOCKS", 512));
    g.gx = ((W - 1) / 2 + kIpNth - 1) / kIpNth;
    return g;
}
// the paired pass: 256-thread workgroups, 8 rows in flight (512 threads measured slower, r05,
// op_ip_nth.jsonl: two sweeps 1.44-1.48 ms at 512 / 1024 workgroups, 1.41-1.42 at 2048,
// against 1.377-1.389)
constexpr int kIp2Rows = 8;
static OpGeom sweep2_ip_geom(int H, int W)
{
    return sweep2_geom(H, W, kIp2Rows, tuning_int("PGMG_OP2IP_BLOCKS", 1024));
}

// boundaries between deferral units along a row: the column blocks
static int ip_bounds(const OpGeom &g) { return g.gx > 1 ? g.gx - 1 : 0; }

// side buffer elements of either in-place pass
size_t g_defer_elems(int H, int W)
{
    const OpGeom a = sweep_ip_geom(H, W), b = sweep2_ip_geom(H, W);
    const size_t m1 = (size_t)a.gy * 2 * W + (size_t)ip_bounds(a) * H * 2;
    const size_t m2 = (size_t)b.gy * 4 * W + (size_t)ip_bounds(b) * H * 4;
    return std::max(m1, m2) + 64;
}

static void defer_scatter(double *x, const double *SR, const double *SC, const OpGeom &g, int R,
                          int nbound, int K, int ca, int cb, int H, int W, hipStream_t s)
{
    const int nslot = g.gy * 2 * R;
    // x blocks per slot / boundary: ~16 elements (rows) per thread.  Measured (r05,
    // profiles/r05_ops/scatter_ab.txt, kernel trace at 16385): 16 per thread 26.6 / 36.2 us for
    // the single / paired pass's scatter against 28.2 / 60.0 with 4 and 42 / 74 with 64 -- the
    // boundary columns' scattered 16-byte writes (one row each) go faster with fewer writers in
    // flight; writing whole 64-byte segments (merged with the pass's in-place values) instead:
    // 63-153 / 99-208 us, not kept
    constexpr int per = 16;
    int bx = (std::max(W, H) + per * kBlock - 1) / (per * kBlock);
    if (bx < 1) bx = 1;
    k_op_defer_scatter<<<dim3(bx, nslot + nbound), kBlock, 0, s>>>(x, SR, SC, H, W, g.rpb, g.gy, R,
                                                                   K, ca, cb);
}

void launch_g_sweep_ip(double *x, const double *f, double *side, unsigned *reset,
                       unsigned long long *stats, double hh, int H, int W, hipStream_t s)
{
    const OpGeom g = sweep_ip_geom(H, W);
    double *SR = side, *SC = side + (size_t)g.gy * 2 * W;
    k_op_sweep_ip<kIpRows, true, true, kIpNth><<<dim3(g.gx, g.gy), kIpNth, 0, s>>>(
        x, f, SR, SC, reset, stats, hh, H, W, g.rpb);
    // boundary e: columns 2 kIpNth (e+1) and the next
    defer_scatter(x, SR, SC, g, 1, ip_bounds(g), 2, 2 * kIpNth, 2 * kIpNth, H, W, s);
}

void launch_g_sweep2_ip(double *x, const double *f, double *side, unsigned long long *stats,
                        double hh, int H, int W, hipStream_t s)
{
    const OpGeom g = sweep2_ip_geom(H, W);
    double *SR = side, *SC = side + (size_t)g.gy * 4 * W;
    k_op_sweep2_ip<kIp2Rows, true, true><<<dim3(g.gx, g.gy), kBlock, 0, s>>>(x, f, SR, SC, stats, hh,
                                                                             H, W, g.rpb);
    // boundary e: block e's last wave w = kWaves (e+1) - 1, lane 61 -> columns kOv2Stride w +
    // 119 ...; 4 columns
    constexpr int kWaves = kBlock / 64;
    defer_scatter(x, SR, SC, g, 2, ip_bounds(g), 4, kOv2Stride * kWaves,
                  kOv2Stride * (kWaves - 1) + 119, H, W, s);
}

// ---------------------------------------------------------------------------
// Residual on the interior, DynamicGridUtils.hpp:59-69 (= Parallel_Method.cu:29-49's
// device_compute_residual); the boundary of r is untouched:
//   r[i] = f[i] - (1.0/(h*h)) * (4*x[i] - x[i-1] - x[i+1] - x[i-W] - x[i+W])
// ---------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(kBlock) void k_op_residual(double *__restrict__ R,
                                                        const double *__restrict__ X,
                                                        const double *__restrict__ F, double ih,
                                                        int H, int W, int rpb)
{
    const int lane = threadIdx.x & 63;
    const int npairs = (W - 1) >> 1;
    const int t_raw = blockIdx.x * kBlock + threadIdx.x;
    const bool act = t_raw < npairs;
    const int t = act ? t_raw : npairs - 1;
    const int c = 1 + 2 * t;
    const bool second = c + 1 <= W - 2;
    const bool ld_l = lane == 0;
    const bool ld_r = (lane == 63 || t == npairs - 1) && second;
    const int jb = 1 + blockIdx.y * rpb;
    const int je = min(jb + rpb, H - 1);
    const long long Wl = W;
    double2 w0 = ldvu<double>(X + (long long)(jb - 1) * Wl + c);
    double2 w1 = ldvu<double>(X + (long long)jb * Wl + c);
    for (int j = jb; j < je; j += U) {
        double2 xn[U], fv[U];
        double el[U], er[U];
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long r = min(j + u, je - 1);
            fv[u] = ldvu<double>(F + r * Wl + c);
            xn[u] = ldvu<double>(X + (r + 1) * Wl + c);
            el[u] = ld_l ? X[r * Wl + c - 1] : 0.0;
            er[u] = ld_r ? X[r * Wl + c + 2] : 0.0;
        }
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            const double2 up = (u == 0) ? w0 : (u == 1 ? w1 : xn[u - 2]);
            const double2 ce = (u == 0) ? w1 : xn[u - 1];
            const double2 dn = xn[u];
            double left = dpp_shr(ce.y);
            double right = dpp_shl(ce.x);
            if (ld_l) left = el[u];
            if (ld_r) right = er[u];
            double2 o;
            o.x = fv[u].x - ih * (4 * ce.x - left - ce.y - up.x - dn.x);
            o.y = fv[u].y - ih * (4 * ce.y - ce.x - right - up.y - dn.y);
            if (act && j + u < je) {
                double *q = R + (long long)(j + u) * Wl + c;
                if (second) st2<true>(q, o);
                else st_nt1(q, o.x);
            }
        }
        w0 = xn[U - 2];
        w1 = xn[U - 1];
    }
}

void launch_g_residual(double *r, const double *x, const double *f, double inv_hh, int H, int W,
                       hipStream_t s)
{
    // the sweep's pattern (2 reads, 1 write): its geometry (1024 workgroups)
    // 16 rows in flight, as the sweep (r04, scripts/op_ru_ab.py, profiles/r04_ops/op_ru.jsonl:
    // 1.344-1.351 ms against 1.360-1.362 for 8 rows, 3 interleaved rounds; 2048 workgroups
    // 1.362-1.382)
    // (r05: 512-thread workgroups x 512 / 1024 measured the same or slower, 1.357-1.378 ms
    // against 1.358-1.363; profiles/r05_ops/op_misc_ab.jsonl)
    const OpGeom g = op_geom((W - 1) / 2, H - 2, 16, tuning_int("PGMG_OPR_BLOCKS", 1024));
    k_op_residual<16><<<dim3(g.gx, g.gy), kBlock, 0, s>>>(r, x, f, inv_hh, H, W, g.rpb);
}

// ---------------------------------------------------------------------------
// Full-weighting restriction, MultiGrid.hpp:187-205 (= Parallel_Method.cu:51-77's
// restriction_kernel_full_weighting); the coarse boundary is untouched:
//   C[jc][ic] = 0.25*F[k] + 0.125*(F[k+1] + F[k-1] + F[k+Nf] + F[k-Nf])
//             + 0.0625*(F[k-Nf-1] + F[k-Nf+1] + F[k+Nf-1] + F[k+Nf+1]),  k = 2jc*Nf + 2ic
// Lane t owns coarse column ic = 1 + t and loads the fine pair (2ic, 2ic+1) of each fine row;
// column 2ic-1 is the previous lane's second element (DPP), a wave's lane 0 loads it.  A band
// of coarse rows marches down the fine rows 2jc-1 .. 2jc+1, carrying the shared row 2jc+1.
// ---------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(kBlock) void k_op_restrict(const double *__restrict__ Fn,
                                                        double *__restrict__ C, int Nf, int Nc,
                                                        int rpb)
{
    const int lane = threadIdx.x & 63;
    const int nic = Nc - 2;
    const int t_raw = blockIdx.x * kBlock + threadIdx.x;
    const bool act = t_raw < nic;
    const int ic = 1 + (act ? t_raw : nic - 1);
    const int jb = 1 + blockIdx.y * rpb;
    const int je = min(jb + rpb, Nc - 1);
    const long long Wf = Nf;
    const int col = 2 * ic;
    // fine row 2jb - 1, carried
    double2 top = ldvu<double>(Fn + (long long)(2 * jb - 1) * Wf + col);
    double tl = lane == 0 ? Fn[(long long)(2 * jb - 1) * Wf + col - 1] : 0.0;
    for (int jc = jb; jc < je; jc += U) {
        double2 mid[U], bot[U];
        double ml[U], bl[U];
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long j = min(jc + u, je - 1);
            const double *m = Fn + (2 * j) * Wf + col;
            mid[u] = ldvu<double>(m);
            bot[u] = ldvu<double>(m + Wf);
            ml[u] = lane == 0 ? m[-1] : 0.0;
            bl[u] = lane == 0 ? m[Wf - 1] : 0.0;
        }
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            const double2 tp = u == 0 ? top : bot[u - 1];
            const double tlu = u == 0 ? tl : bl[u - 1];
            // column 2ic - 1 of each row: the previous lane's .y
            double tL = dpp_shr(tp.y), mL = dpp_shr(mid[u].y), bL = dpp_shr(bot[u].y);
            if (lane == 0) {
                tL = tlu;
                mL = ml[u];
                bL = bl[u];
            }
            // F[k] = mid.x; F[k+1] = mid.y; F[k-1] = mL; F[k+Nf] = bot.x; F[k-Nf] = tp.x;
            // F[k-Nf-1] = tL; F[k-Nf+1] = tp.y; F[k+Nf-1] = bL; F[k+Nf+1] = bot.y
            const double v = 0.25 * mid[u].x + 0.125 * (mid[u].y + mL + bot[u].x + tp.x) +
                             0.0625 * (tL + tp.y + bL + bot[u].y);
            if (act && jc + u < je) C[(long long)(jc + u) * Nc + ic] = v;
        }
        top = bot[U - 1];
        tl = bl[U - 1];
    }
}

void launch_g_restrict(const double *fine, double *coarse, int Nf, int Nc, hipStream_t s)
{
    // 8 coarse rows of loads in flight (r04, scripts/op_ru_ab.py --restrict-prolong,
    // profiles/r04_ops/op_rp.jsonl: 0.561-0.566 ms against 0.573-0.577 for 4, 3 interleaved
    // rounds)
    const OpGeom g = op_geom(Nc - 2, Nc - 2, 8, tuning_int("PGMG_OPRS_BLOCKS", kOpTarget));
    k_op_restrict<8><<<dim3(g.gx, g.gy), kBlock, 0, s>>>(fine, coarse, Nf, Nc, g.rpb);
}

// ---------------------------------------------------------------------------
// Prolongation, fine += P coarse, over the fine points (y, x) with y, x < ext only: the
// reference's thread grid (ComputeProlungator, Parallel_Method.cu:191-197) covers
// max(1, Nf / num_thread) * num_thread rows and columns, so for Nf = 2^k + 1 its last fine
// row and column are never written (ext = Nf: everything).
// Lane t owns coarse column ic = t and the fine pair (2ic, 2ic+1); C[ic+1] is the next lane's
// coarse value (DPP), a wave's last lane loads it.  Fine rows march in pairs (2jc, 2jc+1)
// reading coarse rows jc and jc+1 (carried).
//  MODE 0: MultiGrid.hpp:208-226 (the CPU path): rows and columns 2 .. Nf-2 only (fine row /
//          column 1 never corrected), Fn = Fn + v with
//          v = C0[ic] | 0.5*(C0[ic] + C0[ic+1]) | 0.5*(C0[ic] + C1[ic])
//            | 0.25*(C0[ic] + C0[ic+1] + C1[ic] + C1[ic+1])   (even/even, even/odd, odd/even,
//                                                              odd/odd row/column)
//  MODE 1: prolungator_kernel, Parallel_Method.cu:79-138 (the GPU reference's symmetric
//          form): the fine boundary := 0, every interior point (rows / columns 1 .. Nf-2)
//          Fn += v with the same four cases.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_op_prolong(const double *__restrict__ C,
                                                       double *__restrict__ Fn, int Nc, int Nf,
                                                       int ext, int rpb)
{
    const int lane = threadIdx.x & 63;
    const int t_raw = blockIdx.x * kBlock + threadIdx.x;
    const bool act = t_raw < Nc;
    const int ic = act ? t_raw : Nc - 1;
    const int E = ext < Nf ? ext : Nf;
    const int x0 = 2 * ic, x1 = 2 * ic + 1;
    const bool has1 = x1 < Nf;                        // the last coarse column has no odd fine
    const bool ld_n = (lane == 63 || ic == Nc - 1) ? false : false;
    (void)ld_n;
    const long long Wf = Nf, Wc = Nc;
    // fine rows [yb, ye) of this band, in whole pairs starting at an even row
    const int yb = 2 * (blockIdx.y * rpb);
    const int ye = min(yb + 2 * rpb, Nf);
    // coarse row jc = yb / 2 and its right neighbour column
    const bool nxt_ok = ic + 1 < Nc;
    double c0 = C[(long long)(yb >> 1) * Wc + ic];
    double c0n = (lane == 63 && nxt_ok) ? C[(long long)(yb >> 1) * Wc + ic + 1] : 0.0;
    for (int y = yb; y < ye; y += 2) {
        const int jc = y >> 1;
        const bool has_c1 = jc + 1 < Nc;
        const double c1 = has_c1 ? C[(long long)(jc + 1) * Wc + ic] : 0.0;
        const double c1n = (lane == 63 && nxt_ok && has_c1) ? C[(long long)(jc + 1) * Wc + ic + 1] : 0.0;
        double *p0 = Fn + (long long)y * Wf + x0;
        double *p1 = p0 + Wf;
        const bool row1 = y + 1 < ye;
        double2 f0, f1;
        if (has1) {
            f0 = ldvu<double>(p0);
            f1 = row1 ? ldvu<double>(p1) : f0;
        } else {
            f0.x = p0[0];
            f0.y = 0.0;
            f1.x = row1 ? p1[0] : 0.0;
            f1.y = 0.0;
        }
        // next coarse column by DPP (lane 63: its own load)
        double a_n = dpp_shl(c0), b_n = dpp_shl(c1);
        if (lane == 63) {
            a_n = c0n;
            b_n = c1n;
        }
        // even fine row y: (y, x0) = c0; (y, x1) = 0.5*(c0 + a_n)
        // odd fine row y+1: (y+1, x0) = 0.5*(c0 + c1); (y+1, x1) = 0.25*(c0 + a_n + c1 + b_n)
        const double v00 = c0;
        const double v01 = 0.5 * (c0 + a_n);
        const double v10 = 0.5 * (c0 + c1);
        const double v11 = 0.25 * (c0 + a_n + c1 + b_n);
        double2 o0 = f0, o1 = f1;
        if (MODE == 0) {
            // rows / columns 2 .. Nf-2
            const bool cx0 = x0 >= 2 && x0 <= Nf - 2, cx1 = x1 >= 2 && x1 <= Nf - 2;
            const bool ry0 = y >= 2 && y <= Nf - 2, ry1 = y + 1 >= 2 && y + 1 <= Nf - 2;
            if (ry0 && cx0) o0.x = f0.x + v00;
            if (ry0 && cx1) o0.y = f0.y + v01;
            if (ry1 && cx0) o1.x = f1.x + v10;
            if (ry1 && cx1) o1.y = f1.y + v11;
        } else {
            const bool b0 = x0 == 0 || x0 == Nf - 1, b1 = x1 == Nf - 1;
            const bool yb0 = y == 0 || y == Nf - 1, yb1 = y + 1 == Nf - 1;
            o0.x = (yb0 || b0) ? 0.0 : f0.x + v00;
            o0.y = (yb0 || b1) ? 0.0 : f0.y + v01;
            o1.x = (yb1 || b0) ? 0.0 : f1.x + v10;
            o1.y = (yb1 || b1) ? 0.0 : f1.y + v11;
        }
        // write only the points inside the reference's launch extent
        if (act && y < E) {
            if (has1 && x1 < E) stvu<double>(p0, o0);
            else if (x0 < E) p0[0] = o0.x;
        }
        if (act && row1 && y + 1 < E) {
            if (has1 && x1 < E) stvu<double>(p1, o1);
            else if (x0 < E) p1[0] = o1.x;
        }
        c0 = c1;
        c0n = c1n;
    }
}

void launch_g_prolong(const double *coarse, double *fine, int Nc, int Nf, int mode, int ext,
                      hipStream_t s)
{
    // one band = rpb coarse rows = 2 rpb fine rows
    // (r04: 4 row pairs of loads in flight per step measured slower, 1.07-1.09 ms against
    // 1.006-1.016, profiles/r04_ops/op_rp.jsonl)
    const OpGeom g = op_geom(Nc, (Nf + 1) / 2, 1, tuning_int("PGMG_OPP_BLOCKS", kOpTarget));
    const dim3 grid(g.gx, g.gy);
    if (mode == 1) k_op_prolong<1><<<grid, kBlock, 0, s>>>(coarse, fine, Nc, Nf, ext, g.rpb);
    else k_op_prolong<0><<<grid, kBlock, 0, s>>>(coarse, fine, Nc, Nf, ext, g.rpb);
}

// ---------------------------------------------------------------------------
// sum of squares (DynamicGridUtils::norm's sum, DynamicGridUtils.hpp:71-80): per-block
// partials over a flat array, 16-byte loads where the array allows
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_g_sumsq(const double *v, long long n, double *partials)
{
    __shared__ double red[kBlock / 64];
    double acc = 0.0;
    for (long long k = (long long)blockIdx.x * kBlock + threadIdx.x; k < n;
         k += (long long)gridDim.x * kBlock)
        acc += v[k] * v[k];
    const double s = gblock_sum<kBlock>(acc, red);
    if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

void launch_g_sumsq(const double *v, long long n, double *partials, int nblocks, hipStream_t s)
{
    k_g_sumsq<<<dim3(nblocks), dim3(kBlock), 0, s>>>(v, n, partials);
}

// compute_rhs, DynamicGridUtils.hpp:111-124: f[j][i] = factor * sx[i] * sy[j] (the host's
// sine tables, so bitwise the CPU's values); a block per row band, a thread per column
__global__ void k_g_rhs(double *f, const double *sx, const double *sy, double factor, int W, int H)
{
    const long long Wl = W;
    for (int j = blockIdx.y; j < H; j += gridDim.y) {
        const double syj = sy[j];
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < W; i += gridDim.x * blockDim.x)
            f[j * Wl + i] = factor * sx[i] * syj;
    }
}

void launch_g_rhs(double *f, const double *sx, const double *sy, double factor, int W, int H,
                  hipStream_t s)
{
    const int gx = (W + 255) / 256;
    int gy = 4096 / gx;
    if (gy < 1) gy = 1;
    if (gy > H) gy = H;
    k_g_rhs<<<dim3(gx, gy), dim3(256), 0, s>>>(f, sx, sy, factor, W, H);
}

}  // namespace pgmg
