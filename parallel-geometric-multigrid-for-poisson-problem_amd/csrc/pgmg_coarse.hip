// pgmg_coarse.hip — the latency-bound coarse levels' two passes as 2D LDS tiles.
//
// A level entered with x0 = 0 (every level below the finest in a V/W-cycle, RECOMP) costs
// two fused passes: k_pre (x1 = J(0), the check ||r(x1)||, x2 = J(x1), rc = R r(x2)) and
// k_post (the pre-smoothed iterate recomputed from f, + P ec, two sweeps with the check
// ||r(x1)||).  pgmg_fused.hip runs them as row-marching bands: right for the bulk levels,
// where HBM streaming is what counts, but on the small levels (N <= 513: 0.02-0.26 M points)
// the launch spends its ~6 µs in ONE wave's serial chain -- a band of 2 coarse rows marches
// 12 fine rows (3x redundant) with four stencil stages per row, ~1000 VALU + 700 SALU
// instructions per wave, one wave per SIMD, nothing to hide the latency behind
// (profiles/r03_final/levels: k_pre at 129 7.4 µs, 64 waves, wait 47 % / issue 51 %).
//
// Here a workgroup owns a TC x TC tile of coarse points and the fine points around it:
// it loads its f window (+ halo) once, then every stencil stage is one point per thread over
// the window in LDS, a barrier between stages -- ~5 short stages instead of a 12-row chain.
// The halo is recomputed by neighbouring tiles (~1.7x redundant points at TC = 8), spread
// over 256 threads instead of serialised in one wave.
//
// Semantics are exactly k_pre / k_post's (pgmg_fused.hip pre_body / post_body with
// X0_ZERO, RECOMP, no strips, no regenerated f), every value through the reference's
// expression in its order (MultiGrid.hpp:57-94, Smoother.hpp:59-88, DynamicGridUtils.hpp:
// 59-69, MultiGrid.hpp:187-226), so the results are bitwise those of the row-marching
// passes; only the check's per-block partial sums are grouped differently (their order is
// not part of the contract; the count goes with them into the check's record).
#include "pgmg.h"
#include "pgmg_coarse.h"

namespace pgmg {

constexpr int kCT = 256;   // threads per tile workgroup

template <class T> __device__ __forceinline__ double csq(double acc, T r)
{
    return __builtin_fma((double)r, (double)r, acc);
}

__device__ __forceinline__ double ctile_block_sum(double v, double *red)
{
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0)
        for (int i = 0; i < kCT / 64; ++i) s += red[i];
    return s;
}

// Early-exit decision of an in-stream check (MODE 2): every workgroup re-reduces the
// check's partials in the same order (pgmg_fused.hip rare_decide's semantics); workgroup
// (0,0) books the exit (one sweep less, one exit more) when it fired.
__device__ __forceinline__ bool ctile_decide(const double *partials, int np, double eps,
                                             const double *global_sum,
                                             unsigned long long *stats, double *red, int *trig)
{
    double v = 0.0;
    for (int k = threadIdx.x; k < np; k += kCT) v += partials[k];
    v = ctile_block_sum(v, red);
    if (threadIdx.x == 0) *trig = (sqrt(global_sum != nullptr ? *global_sum : v) < eps) ? 1 : 0;
    __syncthreads();
    const bool t = *trig != 0;
    if (t && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && stats != nullptr) {
        atomicAdd(&stats[0], (unsigned long long)-1LL);
        atomicAdd(&stats[1], 1ull);
    }
    return t;
}

// MODE 0: the pass (two sweeps, the check's partials).  MODE 1: the check predicted to fire
// (k_pre1 / k_post1): one sweep is the result, the check's partials written, one sweep and one
// exit booked.  MODE 2: the in-stream rare path (k_pre_rare / k_post_rare): decide the check
// from the MODE 0 pass's partials; when it fired, redo the pass with one sweep.
// ---------------------------------------------------------------------------
// pre: coarse tile rows [jca, jcb) x columns [ica, icb) of rc; window of fine points
// (2 jca - 3 + i, 2 ica - 3 + j), i, j in [0, W): rc at (jc, ic) needs r at fine points
// 2jc-1 .. 2jc+1, r(x2) needs x2 one further, x2 needs x1 one further (x1 = J(0) pointwise)
// ---------------------------------------------------------------------------
template <class T, int TC, int MODE>
__global__ __launch_bounds__(kCT) void k_pre_tile(CoarseArgsT<T> a)
{
    constexpr int W = 2 * TC + 5;
    constexpr int W2 = W - 2, W4 = W - 4;
    __shared__ T sF[W * W], sX1[W * W], sX2[W2 * W2], sR[W4 * W4];
    __shared__ double red[kCT / 64];
    __shared__ int trig;
    const bool lead = blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0;
    if constexpr (MODE == 2) {
        const bool t = ctile_decide(a.dec_partials, a.dec_np, a.eps, a.global_sum, a.stats, red, &trig);
        if (lead && a.fired != nullptr) *a.fired = t ? 1u : 0u;
        if (!t) return;
    }
    const int N = a.N, Nc = a.Nc;
    const long long P = a.P, Pc = a.Pc;
    const T hh = a.hh, ih = a.ih;
    const int jca = a.jt0 + blockIdx.y * TC, jcb = min(jca + TC, a.jt1);
    const int ica = 1 + blockIdx.x * TC, icb = min(ica + TC, Nc - 1);
    const int y0 = 2 * jca - 3, x0 = 2 * ica - 3;
    // the check's fine points owned by this tile (a partition of the rank's interior rows):
    // rows [2 jca, 2 jcb), the first tile from own_lo, the last up to own_hi; columns likewise
    const int oy0 = blockIdx.y == 0 ? a.own_lo : 2 * jca;
    const int oy1 = jcb == a.jt1 ? a.own_hi : 2 * jcb;
    const int ox0 = ica == 1 ? 1 : 2 * ica, ox1 = icb == Nc - 1 ? N - 1 : 2 * icb;
    // f rows read: x1 on [2 jca - 3, 2 jcb + 1] (a strip holds them: its halo; the window's
    // rows past them are not loaded)
    const int fy0 = max(1, 2 * jca - 3), fy1 = min(N - 2, 2 * jcb + 1);
    if (lead) {
        if (MODE == 0) {
            if (a.stats != nullptr) atomicAdd(&a.stats[0], 2ull);
            if (a.fired != nullptr) *a.fired = 0u;   // the pre check's outcome for k_post RECOMP
        } else if (MODE == 1) {
            if (a.fired != nullptr) *a.fired = 1u;
            if (a.stats != nullptr) {
                atomicAdd(&a.stats[0], 1ull);
                atomicAdd(&a.stats[1], 1ull);
            }
        }
    }
    // x1 = J(0) = 0.25 * ((hh*f) + 0) on the interior, 0 on and outside the boundary
    for (int q = threadIdx.x; q < W * W; q += kCT) {
        const int i = q / W, j = q - (q / W) * W;
        const int y = y0 + i, x = x0 + j;
        const bool in = y >= 1 && y <= N - 2 && x >= 1 && x <= N - 2;
        const T fv = (in && y >= fy0 && y <= fy1) ? a.f[y * P + x] : T(0);
        sF[q] = fv;
        sX1[q] = in ? T(0.25) * ((hh * fv) + T(0)) : T(0);
    }
    __syncthreads();
    // x2 = J(x1) (MODE 0) or r(x1) (one sweep: the residual the restriction reads); the
    // check's r(x1) on the owned points
    double acc = 0.0;
    for (int q = threadIdx.x; q < W2 * W2; q += kCT) {
        const int i = 1 + q / W2, j = 1 + (q - (q / W2) * W2);
        const int y = y0 + i, x = x0 + j;
        const bool in = y >= 1 && y <= N - 2 && x >= 1 && x <= N - 2;
        const int k = i * W + j;
        const T c = sX1[k], l = sX1[k - 1], r = sX1[k + 1], u = sX1[k - W], d = sX1[k + W];
        const T fv = sF[k];
        const T r1 = fv - ih * (T(4) * c - l - r - u - d);
        if (MODE == 0) sX2[q] = in ? T(0.25) * ((hh * fv) + l + r + u + d) : c;
        else sX2[q] = r1;
        if (MODE != 2 && in && y >= oy0 && y < oy1 && x >= ox0 && x < ox1) acc = csq(acc, r1);
    }
    __syncthreads();
    if (MODE == 0) {
        // r(x2) on the window's inner points (only interior points feed rc)
        for (int q = threadIdx.x; q < W4 * W4; q += kCT) {
            const int i = 2 + q / W4, j = 2 + (q - (q / W4) * W4);
            const int k = (i - 1) * W2 + (j - 1);
            const T c = sX2[k], l = sX2[k - 1], r = sX2[k + 1], u = sX2[k - W2], d = sX2[k + W2];
            sR[q] = sF[i * W + j] - ih * (T(4) * c - l - r - u - d);
        }
        __syncthreads();
    }
    // full-weighting restriction, MultiGrid.hpp:199-202: centre fine point (2jc, 2ic) is window
    // point (2 (jc - jca) + 3, 2 (ic - ica) + 3): sR point (2 (jc - jca) + 1, ..), sX2 point
    // (2 (jc - jca) + 2, ..)
    const T *R = MODE == 0 ? sR : sX2;
    constexpr int RW = MODE == 0 ? W4 : W2;
    constexpr int RO = MODE == 0 ? 1 : 2;
    for (int q = threadIdx.x; q < TC * TC; q += kCT) {
        const int jc = jca + q / TC, ic = ica + (q - (q / TC) * TC);
        if (jc < jcb && ic < icb) {
            const int k = (2 * (jc - jca) + RO) * RW + 2 * (ic - ica) + RO;
            const T v = T(0.25) * R[k] + T(0.125) * (R[k + 1] + R[k - 1] + R[k + RW] + R[k - RW]) +
                        T(0.0625) * (R[k - RW - 1] + R[k - RW + 1] + R[k + RW - 1] + R[k + RW + 1]);
            a.rc[jc * Pc + ic] = v;
        }
    }
    if (MODE != 2) {
        const double s = ctile_block_sum(acc, red);
        if (threadIdx.x == 0) a.partials[blockIdx.y * gridDim.x + blockIdx.x] = s;
    }
}

// ---------------------------------------------------------------------------
// post: the fine points of rows [ya, yb) x columns [xa, xb) -- the tile's coarse rows'
// fine rows 2jc-1, 2jc (the last tile down to N-2; the first / last tile column also writes
// boundary column 0 / N-1, as k_post does); window (2 jca - 4 + i, 2 ica - 4 + j)
//   g1 = J(0) -> ph = J(g1) (or g1 if the pre check fired) -> xe = ph + P ec -> x1 = J(xe)
//   -> x2 = J(x1) (one sweep: x1 is the result), the check r(x1) on the owned interior points
// ---------------------------------------------------------------------------
template <class T, int TC, int MODE>
__global__ __launch_bounds__(kCT) void k_post_tile(CoarseArgsT<T> a)
{
    constexpr int W = 2 * TC + 8;
    constexpr int W2 = W - 2, W4 = W - 4;
    constexpr int CW = TC + 6;   // coarse rows jca-2 .. jca+TC+3 (xe's prolongation reads)
    __shared__ T sF[W * W], sG[W * W], sXE[W2 * W2], sX1[W4 * W4], sC[CW * CW];
    __shared__ double red[kCT / 64];
    __shared__ int trig;
    const bool lead = blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0;
    if constexpr (MODE == 2) {
        if (!ctile_decide(a.dec_partials, a.dec_np, a.eps, a.global_sum, a.stats, red, &trig)) return;
    }
    const int N = a.N, Nc = a.Nc;
    const long long P = a.P, Pc = a.Pc;
    const T hh = a.hh, ih = a.ih;
    const int jca = a.jt0 + blockIdx.y * TC, jcb = min(jca + TC, a.jt1);
    const int ica = 1 + blockIdx.x * TC, icb = min(ica + TC, Nc - 1);
    const int y0 = 2 * jca - 4, x0 = 2 * ica - 4;
    const int cy0 = jca - 2, cx0 = ica - 2;
    // the fine points written by this tile: rows [2 jca, 2 jcb) (the first tile from own_lo, the
    // last up to own_hi), columns [2 ica, 2 icb) (the first from the boundary column 0, the last
    // up to N - 1)
    const int ya = blockIdx.y == 0 ? a.own_lo : 2 * jca;
    const int yb = jcb == a.jt1 ? a.own_hi : 2 * jcb;
    const int xa = ica == 1 ? 0 : 2 * ica, xb = icb == Nc - 1 ? N : 2 * icb;
    // rows read: f on [ya - 3, yb + 2], the correction's coarse rows of xe on [ya - 2, yb + 1]
    const int fy0 = max(1, ya - 3), fy1 = min(N - 2, yb + 2);
    const int cm0 = max(0, (ya - 2) >> 1), cm1 = min(Nc - 1, ((yb + 1) >> 1) + 1);
    if (lead && a.stats != nullptr) {
        if (MODE == 0) atomicAdd(&a.stats[0], 2ull);
        if (MODE == 1) {
            atomicAdd(&a.stats[0], 1ull);
            atomicAdd(&a.stats[1], 1ull);
        }
    }
    const bool pfired = *a.pre_fired != 0u;
    for (int q = threadIdx.x; q < W * W; q += kCT) {
        const int i = q / W, j = q - (q / W) * W;
        const int y = y0 + i, x = x0 + j;
        const bool in = y >= 1 && y <= N - 2 && x >= 1 && x <= N - 2;
        const T fv = (in && y >= fy0 && y <= fy1) ? a.f[y * P + x] : T(0);
        sF[q] = fv;
        sG[q] = in ? T(0.25) * ((hh * fv) + T(0)) : T(0);
    }
    for (int q = threadIdx.x; q < CW * CW; q += kCT) {
        const int m = cy0 + q / CW, n = cx0 + (q - (q / CW) * CW);
        sC[q] = (m >= cm0 && m <= cm1 && n >= 0 && n <= Nc - 1) ? a.ec[m * Pc + n] : T(0);
    }
    __syncthreads();
    // ph = J(g1) (or g1), then + P ec on rows / columns 2 .. N-2 (MultiGrid.hpp:208-226)
    for (int q = threadIdx.x; q < W2 * W2; q += kCT) {
        const int i = 1 + q / W2, j = 1 + (q - (q / W2) * W2);
        const int y = y0 + i, x = x0 + j;
        const bool in = y >= 1 && y <= N - 2 && x >= 1 && x <= N - 2;
        const int k = i * W + j;
        const T c = sG[k];
        T ph = c;
        if (in && !pfired) ph = T(0.25) * ((hh * sF[k]) + sG[k - 1] + sG[k + 1] + sG[k - W] + sG[k + W]);
        if (y >= 2 && y <= N - 2 && x >= 2 && x <= N - 2) {
            const int m = (y >> 1) - cy0, n = (x >> 1) - cx0;
            const int kc = m * CW + n;
            const T c00 = sC[kc], c01 = sC[kc + 1], c10 = sC[kc + CW], c11 = sC[kc + CW + 1];
            T v;
            if ((y & 1) == 0) v = (x & 1) == 0 ? c00 : T(0.5) * (c00 + c01);
            else v = (x & 1) == 0 ? T(0.5) * (c00 + c10) : T(0.25) * (c00 + c01 + c10 + c11);
            ph = ph + v;
        }
        sXE[q] = ph;
    }
    __syncthreads();
    // x1 = J(xe)
    for (int q = threadIdx.x; q < W4 * W4; q += kCT) {
        const int i = 2 + q / W4, j = 2 + (q - (q / W4) * W4);
        const int y = y0 + i, x = x0 + j;
        const bool in = y >= 1 && y <= N - 2 && x >= 1 && x <= N - 2;
        const int k = (i - 1) * W2 + (j - 1);
        const T c = sXE[k];
        sX1[q] = in ? T(0.25) * ((hh * sF[i * W + j]) + sXE[k - 1] + sXE[k + 1] + sXE[k - W2] + sXE[k + W2]) : c;
    }
    __syncthreads();
    // x2 = J(x1) (x1 itself with one sweep) on the owned points, written; the check's r(x1)
    // on the owned interior
    double acc = 0.0;
    const int wc = xb - xa, npts = (yb - ya) * wc;
    for (int q = threadIdx.x; q < npts; q += kCT) {
        const int y = ya + q / wc, x = xa + (q - (q / wc) * wc);
        T out = T(0);   // boundary columns: the passthrough of x1's boundary, 0
        if (x >= 1 && x <= N - 2) {
            const int k = (y - y0 - 2) * W4 + (x - x0 - 2);
            const T c = sX1[k], l = sX1[k - 1], r = sX1[k + 1], u = sX1[k - W4], d = sX1[k + W4];
            const T fv = sF[(y - y0) * W + (x - x0)];
            if (MODE != 2 && y >= a.sum_lo && y < a.sum_hi) {
                const T r1 = fv - ih * (T(4) * c - l - r - u - d);
                acc = csq(acc, r1);
            }
            out = MODE == 0 ? T(0.25) * ((hh * fv) + l + r + u + d) : c;
        }
        a.x2[y * P + x] = out;
    }
    if (MODE != 2) {
        const double s = ctile_block_sum(acc, red);
        if (threadIdx.x == 0) a.partials[blockIdx.y * gridDim.x + blockIdx.x] = s;
    }
}

// TC = 8 on every level (profiles/r04_ctile/ab_tc_maxn_tail.jsonl, 3 interleaved rounds): TC = 16
// at 1025 (1024 workgroups of 51 KiB LDS, 3 resident per CU) ran its k_post_tile in 20 us
// against 15 us row-marching; TC = 8 there is on par with the row-marching passes
static int ctile_tc(int N) { return tuning_int("PGMG_CTILE_TC", 8) == 16 ? 16 : 8; }

// N <= 513 (profiles/r04_ctile/, profiles/r04_final/coarse/): at 1025 the row-marching passes
// are as fast or faster (26 vs 29 us per V-cycle at TC = 8, 20 us for k_post_tile alone at
// TC = 16); on row strips the 2049 / 4097 levels' thin strips ran 0-5 % slower per rank with
// tiles (profiles/r04_strips/)
bool coarse_tile_ok(int N, bool dist)
{
    return N >= 9 && N <= (dist ? tuning_int("PGMG_CTILE_DIST_MAXN", 513)
                                : tuning_int("PGMG_CTILE_MAXN", 513));
}

int coarse_tile_blocks_rows(int N, int jt0, int jt1)
{
    if (N < 9 || jt1 <= jt0) return 0;
    const int tc = ctile_tc(N);
    const int nx = (N / 2 - 1 + tc - 1) / tc;   // interior coarse columns (Nc - 2)
    return nx * ((jt1 - jt0 + tc - 1) / tc);
}

int coarse_tile_blocks(int N) { return coarse_tile_blocks_rows(N, 1, N / 2); }

template <class T>
void launch_pre_tile(const CoarseArgsT<T> &a, int mode, hipStream_t s)
{
    const int tc = ctile_tc(a.N);
    const dim3 g((a.Nc - 2 + tc - 1) / tc, (a.jt1 - a.jt0 + tc - 1) / tc);
#define PGMG_PT(TCV)                                                                  \
    do {                                                                              \
        if (mode == 1) k_pre_tile<T, TCV, 1><<<g, kCT, 0, s>>>(a);                   \
        else if (mode == 2) k_pre_tile<T, TCV, 2><<<g, kCT, 0, s>>>(a);              \
        else k_pre_tile<T, TCV, 0><<<g, kCT, 0, s>>>(a);                             \
    } while (0)
    if (tc == 16) PGMG_PT(16);
    else PGMG_PT(8);
#undef PGMG_PT
}

template <class T>
void launch_post_tile(const CoarseArgsT<T> &a, int mode, hipStream_t s)
{
    const int tc = ctile_tc(a.N);
    const dim3 g((a.Nc - 2 + tc - 1) / tc, (a.jt1 - a.jt0 + tc - 1) / tc);
#define PGMG_PT(TCV)                                                                  \
    do {                                                                              \
        if (mode == 1) k_post_tile<T, TCV, 1><<<g, kCT, 0, s>>>(a);                  \
        else if (mode == 2) k_post_tile<T, TCV, 2><<<g, kCT, 0, s>>>(a);             \
        else k_post_tile<T, TCV, 0><<<g, kCT, 0, s>>>(a);                            \
    } while (0)
    if (tc == 16) PGMG_PT(16);
    else PGMG_PT(8);
#undef PGMG_PT
}

template void launch_pre_tile<double>(const CoarseArgsT<double> &, int, hipStream_t);
template void launch_pre_tile<float>(const CoarseArgsT<float> &, int, hipStream_t);
template void launch_post_tile<double>(const CoarseArgsT<double> &, int, hipStream_t);
template void launch_post_tile<float>(const CoarseArgsT<float> &, int, hipStream_t);

}  // namespace pgmg
