// pgmg_fused.hip — temporally fused smoother passes for the default cycle (v1 = v2 = 1).
//
// With v = 1 the reference smoother runs two sweeps and checks ||r(x1)|| < eps after
// the first (the check after the last sweep cannot change the result).  Instead of
// six HBM passes per level (2 sweeps, residual+restriction, prolongation, 2 sweeps)
// a level now costs two:
//
//   k_pre : x0, f  -> x1 = J(x0) -> x2 = J(x1) -> r = f - A x2 -> rc = R r
//           writes x2 (into the ping-pong buffer) and rc; sum r(x1)^2 per block
//           (MultiGrid.hpp:66-78 + Smoother.hpp:59-88)
//   k_post: phi, ec, f -> x_eff = phi + P ec -> x1 = J(x_eff) -> x2 = J(x1)
//           writes x2 (back into the level's solution buffer); sum r(x1)^2
//           (MultiGrid.hpp:86-89 + Smoother.hpp:59-88)
//
// 26 B/point instead of 64 (pre) and 24+2 instead of 64 (post).  Both are
// speculative in the early exit: when ||r(x1)|| < eps fires (rare; never on fine
// levels in practice) the fix-up kernels recompute the exact reference result
// (x1 instead of x2, and rc from r(x1)) from the still-intact inputs.
//
// Tiling: a wave owns 120 columns but loads 128 (4-column overlap each side), so
// every stencil level's horizontal neighbours come from the adjacent lane by DPP
// and the validity shrinks one column per level: x0 [c0, c0+127] -> x1 [+1,-1] ->
// x2 [+2,-2] -> r [+3,-3] -> rc centres [+4,-4] = the owned columns.  Rows march
// down a segment with every stage lagging one row behind the previous one; the
// pipeline needs 4 rows of x0 above and below the segment (the halo rows are
// re-read by the neighbouring segment, mostly from L2 / Infinity Cache).
//
// Every expression keeps the reference's left-to-right order; built with
// -ffp-contract=off, so the results are bit-identical to the unfused path.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "pgmg.h"
#include "pgmg_fused.h"

namespace pgmg {

struct Cols {
    int c;          // odd column of this lane's pair (c, c+1)
    bool bx, by;    // column c / c+1 is a boundary (or outside) column: passthrough
    bool own;       // lane owns its pair (lanes 2..61 of the wave tile)
    bool edge;      // wave-uniform: some lane of this wave has a boundary/outside column
};

// fp32 stencil stages as packed 2-vector arithmetic (pgmg_real.h pf2); 0 = the scalar
// expressions (measurement builds: scripts/build_variant.sh NAME -DPGMG_F32_PK=0)
#ifndef PGMG_F32_PK
#define PGMG_F32_PK 1
#endif
// One Jacobi stage on a row: J(ce) with boundary passthrough.  EDGE = false: the caller
// guarantees that neither the row nor any column of the wave is a boundary (no selects).
template <class T, bool EDGE = true>
__device__ __forceinline__ V2<T> jstage(V2<T> up, V2<T> ce, V2<T> dn, V2<T> f, T hh,
                                          const Cols &k, bool brow)
{
    const T l = dpp_shr(ce.y);
    const T r = dpp_shl(ce.x);
    V2<T> o;
    if constexpr (sizeof(T) == 4 && PGMG_F32_PK) {   // packed: L = (l, c), R = (c+1, r)
        const pf2 L = {l, ce.x}, R = {ce.y, r};
        o = unpk(0.25f * (((((hh * pk(f)) + L) + R) + pk(up)) + pk(dn)));
    } else {
        o.x = T(0.25) * ((hh * f.x) + l + ce.y + up.x + dn.x);
        o.y = T(0.25) * ((hh * f.y) + ce.x + r + up.y + dn.y);
    }
    if constexpr (EDGE) {
        if (brow || k.bx) o.x = ce.x;
        if (brow || k.by) o.y = ce.y;
    }
    return o;
}

// J(0): the Jacobi stage of an all-zero iterate, 0.25 * ((hh*f) + 0 + 0 + 0 + 0).  The first
// +0 turns a -0 into +0 and the other three change nothing, so ONE add of +0 gives the same
// IEEE result (the compiler may not drop x + 0 itself: it is not an identity for x = -0)
template <class T, bool EDGE = true>
__device__ __forceinline__ V2<T> j0stage(V2<T> f, T hh, const Cols &k, bool brow)
{
    V2<T> o;
    o.x = T(0.25) * ((hh * f.x) + T(0));
    o.y = T(0.25) * ((hh * f.y) + T(0));
    if constexpr (EDGE) {
        if (brow || k.bx) o.x = T(0);
        if (brow || k.by) o.y = T(0);
    }
    return o;
}

// Residual r = f - (1/h^2)(4x - xl - xr - xu - xd) on a row (DynamicGridUtils.hpp:59-69)
template <class T>
__device__ __forceinline__ V2<T> rstage(V2<T> up, V2<T> ce, V2<T> dn, V2<T> f, T ih)
{
    const T l = dpp_shr(ce.y);
    const T r = dpp_shl(ce.x);
    V2<T> o;
    if constexpr (sizeof(T) == 4 && PGMG_F32_PK) {
        const pf2 L = {l, ce.x}, R = {ce.y, r};
        o = unpk(pk(f) - ih * ((((4.0f * pk(ce) - L) - R) - pk(up)) - pk(dn)));
    } else {
        o.x = f.x - ih * (T(4) * ce.x - l - ce.y - up.x - dn.x);
        o.y = f.y - ih * (T(4) * ce.y - ce.x - r - up.y - dn.y);
    }
    return o;
}

// Check sums of k_postpre_lds: acc + r.x^2 (+ r.y^2 unless column c+1 is a boundary) on an
// owned pair of a band row.  PGMG_CHK_SEL (r05): as selects instead of a branch around the
// residual (0: neither type, 1: fp32 only, 2: both, 3: fp64 only) -- a skipped term adds
// (+0)^2, which leaves the sum (>= +0) bitwise unchanged, and the residual's dependent chain,
// no longer in a branch of its own, can interleave with the sweeps around it.  Measured at
// 16385 (scripts/pp_ab.py, profiles/r05_fp32/chk_sel_*.jsonl, 3-4 interleaved rounds on two
// boxes): fp64 0.4-0.6 % faster (1.0687 -> 1.0646 ms); fp32 6 % slower although its packed
// chains lose their s_nops (92 -> 12 per 6 rows): 118 -> 161 VGPRs, 4 -> 3 waves per SIMD
// (and at 2 register sets of loads, 109 VGPRs, still 4.6 % slower) -- so fp64 only.
#ifndef PGMG_CHK_SEL
#define PGMG_CHK_SEL 3
#endif
template <int M, class T> constexpr bool chk_sel_m() { return M == 2 || (M == 1 && sizeof(T) == 4) || (M == 3 && sizeof(T) == 8); }
template <class T> constexpr bool chk_sel() { return chk_sel_m<PGMG_CHK_SEL, T>(); }
// the same choice for the check sums of k_post_r2 (the F-cycle's finest post pass; same
// values).  Measured (scripts/pp_ab.py, profiles/r05_fp32/chk_sel_post_*.jsonl, 3 interleaved
// rounds): selects in every k_post -- F at 16385 4.449 -> 4.408 ms per cycle (-0.9 %), V at
// 16385 1.7875 -> 1.7917 (+0.2 %, level 1's k_post), V at 4097 equal; in k_post_r2 alone
// (chk_sel_r2only_*.jsonl) F 4.470 -> 4.421 (-1.1 %), V unchanged -- so k_post_r2 only.
// In k_pre the select form raises most instantiations' VGPRs by 14-100, several from 3 to 2
// waves per SIMD: not used there.
#ifndef PGMG_CHK_SEL_LV
#define PGMG_CHK_SEL_LV 3
#endif
template <class T> constexpr bool chk_sel_lv() { return chk_sel_m<PGMG_CHK_SEL_LV, T>(); }
template <class T>
__device__ __forceinline__ double chk_acc(double acc, V2<T> r, bool in, bool by)
{
    const T rx = in ? r.x : T(0);
    const T ry = (in && !by) ? r.y : T(0);
    return sqacc(sqacc(acc, rx), ry);
}

// Row factor of the regenerated RHS through the constant address space: a scalar load
// (the table is read-only), not a per-row vector load the row loop would wait on
__device__ __forceinline__ double gsy_s(const double *gsy, int row)
{
    return ((const __attribute__((address_space(4))) double *)gsy)[row];
}

__device__ __forceinline__ bool boundary_row(int row, int N) { return row <= 0 || row >= N - 1; }

// Wave tile: STRIDE owned columns, loaded window starts MARGIN columns to the left;
// lanes [MARGIN/2, 63 - (64*2 - STRIDE - MARGIN)/2] own their pair.
template <int STRIDE, int MARGIN>
__device__ __forceinline__ Cols lane_cols_t(int N, int bx = -1)
{
    if (bx < 0) bx = blockIdx.x;
    const int wave = (bx * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    Cols k;
    k.c = STRIDE * wave + 1 - MARGIN + 2 * lane;
    k.bx = k.c <= 0 || k.c >= N - 1;
    k.by = k.c + 1 <= 0 || k.c + 1 >= N - 1;
    k.own = lane >= MARGIN / 2 && lane < MARGIN / 2 + STRIDE / 2 && k.c <= N - 2;
    // the wave's columns are [c0, c0 + 127]: uniform, kept in a scalar register
    const int c0 = __builtin_amdgcn_readfirstlane(STRIDE * wave + 1 - MARGIN);
    k.edge = c0 <= 0 || c0 + 127 >= N - 1;
    return k;
}

__device__ __forceinline__ Cols lane_cols(int N, int bx = -1) { return lane_cols_t<120, 4>(N, bx); }

// Logical (column block, band) of this workgroup.  xcd: XCD-aware order -- the hardware
// deals linear workgroup ids round-robin to the 8 XCDs (id mod 8), so XCD x takes the ids
// x, x+8, ...; those get one contiguous run of tiles, and tiles that share halo columns run
// side by side behind the same L2 (k_postpre: 1.1 % per V-cycle)
__device__ __forceinline__ void xcd_tile(int &bx, int &by)
{
    const int nb = (int)(gridDim.x * gridDim.y), id = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    const int q = nb >> 3, r = nb & 7, x = id & 7;
    const int t = x * q + min(x, r) + (id >> 3);
    bx = t % (int)gridDim.x;
    by = t / (int)gridDim.x;
}
__device__ __forceinline__ void fused_block(int &bx, int &by, bool xcd = false)
{
    bx = blockIdx.x;
    by = blockIdx.y;
    if (xcd) xcd_tile(bx, by);
}

// deterministic sum over the block (fixed tree) -> thread 0
__device__ __forceinline__ double fused_block_sum(double v, double *red)
{
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0)
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
    return s;
}

struct ProlongCols {
    bool vx, vy;   // column c / c+1 receives a correction
    int ic;        // coarse column of the odd fine column c: (c-1)/2
};

// EDGE = false: the caller guarantees row in [2, Nf-2] and both columns in [2, Nf-2]
// (interior bands and wave tiles), so no masks
template <class T, bool EDGE = true>
__device__ __forceinline__ V2<T> add_prolong(V2<T> p, int row, T ca, T cb, T da, T db, const ProlongCols &pc, int Nc)
{
    // MultiGrid.hpp:219-223; row in [2, Nf-2] <=> its coarse row m in [1, Nc-2]
    const int m = row >> 1;
    if (EDGE && (m < 1 || m > Nc - 2)) return p;
    if ((row & 1) == 0) {
        if (!EDGE || pc.vx) p.x = p.x + T(0.5) * (ca + cb);
        if (!EDGE || pc.vy) p.y = p.y + cb;
    } else {
        if (!EDGE || pc.vx) p.x = p.x + T(0.25) * (ca + cb + da + db);
        if (!EDGE || pc.vy) p.y = p.y + T(0.5) * (cb + db);
    }
    return p;
}

// The row loop of k_pre / k_post: iterations of R rows at i = i_begin, i_begin + R, ..,
// < i_end; full_at(i) holds on one contiguous run of them.  The run is executed three
// iterations (3R = 12 rows) at a time with no branch inside: the row windows (two carried
// rows and the new one: period 3; f in k_pre: period 4) come back to their registers after
// 12 rows, and no merge of the FULL and general paths forces copies of every window.
template <int R, int U, class FullAt, class Iter>
__device__ __forceinline__ void row_loop(int i_begin, int i_end, const FullAt &full_at, const Iter &iter)
{
    int i = i_begin;
    if constexpr (U == 0) {   // one loop, the path chosen per iteration
        for (; i < i_end; i += R) {
            if (full_at(i)) iter(i, std::true_type{});
            else iter(i, std::false_type{});
        }
        return;
    }
    for (; i < i_end && !full_at(i); i += R) iter(i, std::false_type{});
    if constexpr (U == 3) {
        for (; i + 3 * R <= i_end && full_at(i + 2 * R); i += 3 * R) {
            iter(i, std::true_type{});
            iter(i + R, std::true_type{});
            iter(i + 2 * R, std::true_type{});
        }
    } else {
        for (; i < i_end && full_at(i); i += R) iter(i, std::true_type{});
    }
    for (; i < i_end; i += R) {
        if (full_at(i)) iter(i, std::true_type{});
        else iter(i, std::false_type{});
    }
}

// ---------------------------------------------------------------------------
// k_pre
// ---------------------------------------------------------------------------
// GENF: f is the analytic RHS, regenerated per row from the gfx/gsy tables (see k_postpre_lds)
// PIN (F-cycle): x0 = (+0) + P ec (a.pin_ec), computed per row from the coarse rows
// (2 B/point read instead of 8, and the prolongation pass into the zeroed grid is gone)
// S1 (rare path of an in-stream check, k_pre_rare): the check after the first sweep fired,
// so the pass is redone with ONE sweep — x1 stored instead of x2, rc = R r(x1) — and
// writes no partial sums and no sweep count (the decision kernel's job)
// S1P (a pre check predicted to fire, k_pre1): the S1 pass that also writes the per-block
// partials of the check's r(x1)^2 (the same terms, rows and order as the full pass), so the
// speculative call's validation can confirm the prediction
template <class T, bool X0_ZERO, bool FINE, int PAIRS, bool GENF, bool PIN, bool S1, bool S1P = false>
__device__ __forceinline__ void pre_body(const PreArgsT<T> &a, double *red)
{
    constexpr int R = 2 * PAIRS;  // rows loaded per iteration (and prefetched ahead)
    if (a.cond != nullptr && *a.cond == 0u) return;  // conditional (rare-path) launch
    int lbx, lby;
    fused_block(lbx, lby, (a.nt & 16) != 0);
    const Cols k = lane_cols(a.N, lbx);
    const int N = a.N;
    const long long P = a.P;
    const int jcb = a.jc0 + lby * a.rows_per_block;
    const int jce = min(jcb + a.rows_per_block, a.jc1);
    const int olo = max(2 * jcb, a.row_lo), ohi = min(2 * jce, a.row_hi);  // x2 rows written
    const int clo = max(jcb, max(1, a.rc_lo)), chi = min(jce, min(N / 2, a.rc_hi));  // rc rows
    if (!S1 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        if (a.stats != nullptr) atomicAdd(&a.stats[0], 2ull);
        // the pre check's outcome for k_post RECOMP: "did not fire" unless a rare path or the
        // predicted-to-fire pass says otherwise (a level's visits share the flag: a W-cycle's
        // visit recorded "does not fire" may follow one predicted to fire)
        if (a.fired != nullptr) *a.fired = 0u;
    }
    const T *__restrict__ X = a.x0 + k.c;
    const long long Px = a.Px != 0 ? a.Px : P;   // x0's pitch (the caller's array: N)
    const T *__restrict__ F = a.f + k.c;
    const double fxa = GENF ? a.gfx[k.c] : 0.0, fxb = GENF ? a.gfx[k.c + 1] : 0.0;
    const bool store = a.x2 != nullptr;
    T *__restrict__ O = a.x2 + k.c;
    const T hh = a.hh, ih = a.ih;
    const V2<T> z = zero2<T>();
    // windows: x0 rows i-2,i-1 ; x1 rows i-3,i-2 ; x2 rows i-4,i-3 ; r rows i-5,i-4 ;
    //          f rows i-3,i-2,i-1
    V2<T> a0 = z, a1 = z, b0 = z, b1 = z, c0 = z, c1 = z, d0 = z, d1 = z, f0 = z, f1 = z, f2 = z;
    V2<T> q0 = z, q1 = z;   // S1: r(x1) rows ii-4, ii-3
    double acc = 0.0;
    // steps [i_begin, i_end): rows 2jcb-4 .. 2jce+3, rounded up to whole iterations
    // (the extra rows are computed but never stored; kHalo covers their loads)
    const int i_begin = 2 * jcb - 4;
    // a wave whose owned columns all lie past the grid (the last block's spare
    // waves) streams nothing; it still joins the block reduction below
    // (c0w: the wave's first column, wave-uniform, so the row loop is scalar-controlled)
    const int c0w = __builtin_amdgcn_readfirstlane(k.c - 2 * (int)(threadIdx.x & 63));
    const bool idle = c0w + 4 > N - 2;
    // wave-uniform: no lane has a boundary column and every prolongation column pair is
    // corrected (c0 >= 3, c0 + 127 <= N - 3)
    const bool inner = c0w >= 3 && c0w + 127 <= N - 3;
    const int i_end = idle ? i_begin
                           : i_begin + ((2 * (jce - jcb) + 8 + R - 1) / R) * R;
    V2<T> nx[R], nf[R];
    // PIN: coarse rows (i >> 1) .. (i >> 1) + PAIRS of an iteration starting at row i
    ProlongCols pc;
    pc.ic = (k.c - 1) >> 1;
    pc.vx = k.c >= 3 && k.c <= N - 2;
    pc.vy = k.c + 1 >= 2 && k.c + 1 <= N - 3;
    const T *__restrict__ E = PIN ? a.pin_ec + pc.ic : nullptr;
    const long long Pc = a.Pc;
    // both coarse columns ic and ic+1 are loaded (no DPP for ic+1): the wave's last lane
    // needs column ic+1 too, since k_pre's four stencil levels after x0 use the whole
    // 4-column margin of the 128-column tile
    T ncr[PAIRS + 1], ncrn[PAIRS + 1];
    #pragma unroll
    for (int q = 0; q < R; ++q) {
        nx[q] = (X0_ZERO || PIN || idle) ? z : ldvu(X + (i_begin + q) * Px);
        if constexpr (!GENF) nf[q] = idle ? z : ldv(F + (i_begin + q) * P);
    }
    if constexpr (PIN) {
        #pragma unroll
        for (int q = 0; q <= PAIRS; ++q) {
            ncr[q] = idle ? T(0) : E[(long long)((i_begin >> 1) + q) * Pc];
            ncrn[q] = idle ? T(0) : E[(long long)((i_begin >> 1) + q) * Pc + 1];
        }
    }
    // FULL: every row of the iteration is interior to the band, the grid and the restriction
    // range, and the wave's columns are all interior (no boundary column, every prolongation
    // column corrected): the per-row range checks and the boundary selects drop out.  The
    // condition holds on one contiguous run of iterations (each clause bounds i from one side)
    auto full_at = [&](int i) {
        return !S1 && inner && i >= 3 && i + R <= N && i - 2 >= olo && i + R - 3 < ohi &&
               ((i - 4) >> 1) >= clo && ((i + R - 6) >> 1) < chi &&
               (!PIN || ((i >> 1) >= 1 && ((i + R - 1) >> 1) <= a.Nc - 2));
    };
    auto iter = [&](int i, auto full_t) {
        V2<T> cx[R], cf[R];
        T cr[PAIRS + 1], crn[PAIRS + 1];
        #pragma unroll
        for (int q = 0; q < R; ++q) {
            cx[q] = nx[q];
            if constexpr (!GENF) cf[q] = nf[q];
        }
        if constexpr (PIN) {
            #pragma unroll
            for (int q = 0; q <= PAIRS; ++q) {
                cr[q] = ncr[q];
                crn[q] = ncrn[q];
            }
        }
        if (i + R < i_end) {  // prefetch the next R rows
            #pragma unroll
            for (int q = 0; q < R; ++q) {
                if (!X0_ZERO && !PIN) nx[q] = ldvu(X + (i + R + q) * Px);
                if constexpr (!GENF) nf[q] = ldv(F + (i + R + q) * P);
            }
            if constexpr (PIN) {
                #pragma unroll
                for (int q = 0; q <= PAIRS; ++q) {
                    ncr[q] = E[(long long)(((i + R) >> 1) + q) * Pc];
                    ncrn[q] = E[(long long)(((i + R) >> 1) + q) * Pc + 1];
                }
            }
        }
        double gy[R];   // GENF row factors of the iteration, loaded together up front
        if constexpr (GENF) {
            #pragma unroll
            for (int q = 0; q < R; ++q) gy[q] = gsy_s(a.gsy, i + q);
        }
        {
            constexpr bool FULL = decltype(full_t)::value;
            #pragma unroll
            for (int s = 0; s < R; ++s) {
                const int ii = i + s;
                V2<T> a2 = cx[s];
                if constexpr (PIN) {
                    const int pq = s >> 1;
                    a2 = add_prolong<T, !FULL>(z, ii, cr[pq], crn[pq], cr[pq + 1], crn[pq + 1], pc, a.Nc);
                }
                V2<T> f3;
                if constexpr (GENF) {
                    f3 = mk2<T>((T)(fxa * gy[s]), (T)(fxb * gy[s]));
                } else {
                    f3 = cf[s];
                }
                // x1 row ii-1
                const V2<T> b2 = (X0_ZERO && !PIN) ? j0stage<T, !FULL>(f2, hh, k, boundary_row(ii - 1, N))
                                                   : jstage<T, !FULL>(a0, a1, a2, f2, hh, k, boundary_row(ii - 1, N));
                // r(x1) and x2 on row ii-2
                const V2<T> r1 = rstage(b0, b1, b2, f1, ih);
                if constexpr (S1) {
                    // x1 row ii-1 is the result; restriction of r(x1): rows ii-4, ii-3, ii-2 =
                    // 2jc-1, 2jc, 2jc+1 when ii is odd
                    if (store && ii - 1 >= olo && ii - 1 < ohi && k.own) stv(O + (ii - 1) * P, b2);
                    if constexpr (S1P) {   // the check's terms: r(x1) on row ii-2
                        const int row = ii - 2;
                        if (row >= olo && row < ohi && k.own) {
                            acc = sqacc(acc, r1.x);
                            if (!k.by) acc = sqacc(acc, r1.y);
                        }
                    }
                    if ((s & 1) == 1) {
                        const int jc = (ii - 3) >> 1;
                        const T m2 = dpp_shl(q1.x);
                        const T u2 = dpp_shl(q0.x);
                        const T e2 = dpp_shl(r1.x);
                        const int ic = (k.c + 1) >> 1;
                        if (jc >= clo && jc < chi && k.own && ic <= a.Nc - 2) {
                            const T v = T(0.25) * q1.y + T(0.125) * (m2 + q1.x + r1.y + q0.y) +
                                        T(0.0625) * (q0.x + u2 + r1.x + e2);
                            a.rc[(long long)jc * a.Pc + ic] = v;
                        }
                    }
                    q0 = q1;
                    q1 = r1;
                    a0 = a1;
                    a1 = a2;
                    b0 = b1;
                    b1 = b2;
                    f0 = f1;
                    f1 = f2;
                    f2 = f3;
                    continue;
                }
                {
                    const int row = ii - 2;
                    if ((FULL || (row >= olo && row < ohi)) && k.own) {
                        acc = sqacc(acc, r1.x);
                        if (FULL || !k.by) acc = sqacc(acc, r1.y);
                    }
                }
                const V2<T> c2 = jstage<T, !FULL>(b0, b1, b2, f1, hh, k, boundary_row(ii - 2, N));
                if (store && (FULL || (ii - 2 >= olo && ii - 2 < ohi)) && k.own) {
                    if (a.nt & 1) stv_nt(O + (ii - 2) * P, c2);
                    else stv(O + (ii - 2) * P, c2);
                }
                // r(x2) on row ii-3 (garbage on boundary rows; never used there)
                const V2<T> d2 = rstage(c0, c1, c2, f0, ih);
                // restriction: rows ii-5, ii-4, ii-3 = 2jc-1, 2jc, 2jc+1 when ii is even
                if ((s & 1) == 0) {
                    const int jc = (ii - 4) >> 1;
                    const T m2 = dpp_shl(d1.x);
                    const T u2 = dpp_shl(d0.x);
                    const T e2 = dpp_shl(d2.x);
                    const int ic = (k.c + 1) >> 1;
                    if ((FULL || (jc >= clo && jc < chi && ic <= a.Nc - 2)) && k.own) {
                        const T v = T(0.25) * d1.y + T(0.125) * (m2 + d1.x + d2.y + d0.y) +
                                         T(0.0625) * (d0.x + u2 + d2.x + e2);
                        if (a.nt & 2) __builtin_nontemporal_store(v, &a.rc[(long long)jc * a.Pc + ic]);
                        else a.rc[(long long)jc * a.Pc + ic] = v;
                    }
                }
                a0 = a1;
                a1 = a2;
                b0 = b1;
                b1 = b2;
                c0 = c1;
                c1 = c2;
                d0 = d1;
                d1 = d2;
                f0 = f1;
                f1 = f2;
                f2 = f3;
            }
        }
    };
    // (PIN: the 12-row form needs 170 VGPRs, past the 168 of 3 waves per SIMD)
    row_loop<R, PIN ? 0 : 3>(i_begin, i_end, full_at, iter);
    if constexpr (!S1 || S1P) {
        const double sum = fused_block_sum(acc, red);
        if (threadIdx.x == 0) a.partials[lby * gridDim.x + lbx] = sum;
    }
}

template <class T, bool X0_ZERO, bool FINE, int PAIRS, bool GENF = false, bool PIN = false>
__global__ __launch_bounds__(256) void k_pre(PreArgsT<T> a)
{
    __shared__ double red[4];
    pre_body<T, X0_ZERO, FINE, PAIRS, GENF, PIN, false>(a, red);
}

// A coarse level's pre-smooth whose check is predicted to fire (speculative calls, levels that
// converged: pgmg_ctx.hip "predicted to fire"): x1 = J(x0) (J(0) on a level entered with
// x0 = 0) is the result, rc = R r(x1), one sweep and one exit booked, the "pre fired" flag the
// level's RECOMP k_post reads set -- what k_pre + k_pre_rare compute when the check fires, in
// one launch; the partials confirm it afterwards
template <class T, bool X0_ZERO, int PAIRS>
__global__ __launch_bounds__(256) void k_pre1(PreArgsT<T> a)
{
    __shared__ double red[4];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        if (a.fired != nullptr) *a.fired = 1u;
        if (a.stats != nullptr) {
            atomicAdd(&a.stats[0], 1ull);
            atomicAdd(&a.stats[1], 1ull);
        }
    }
    pre_body<T, X0_ZERO, false, PAIRS, false, false, true, true>(a, red);
}

// Decision of an in-stream early-exit check from the partial sums of the pass just run
// (every block re-reduces them in the same order; a row strip's all-rank sum comes in
// f.global_sum); block (0,0) books the exit.  Blocks that find it did not fire return.
__device__ __forceinline__ bool rare_decide(const FixArgsF &f, double *red, int *trig)
{
    double v = 0.0;
    for (int k = threadIdx.x; k < f.np; k += blockDim.x) v += f.partials[k];
    v = fused_block_sum(v, red);
    if (threadIdx.x == 0) {
        const double tot = f.global_sum != nullptr ? *f.global_sum : v;
        *trig = (sqrt(tot) < f.eps) ? 1 : 0;
    }
    __syncthreads();
    const bool t = *trig != 0;
    if (t && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && f.stats != nullptr) {
        atomicAdd(&f.stats[0], (unsigned long long)-1LL);
        atomicAdd(&f.stats[1], 1ull);
    }
    return t;
}

// rare path of k_pre's check (replaces the scalar k_pre_fixup on in-stream levels): when it
// fired, the same fused pass with one sweep; a.fired records the decision for k_post RECOMP
template <class T, bool X0_ZERO, int PAIRS, bool PIN>
__global__ __launch_bounds__(256) void k_pre_rare(PreArgsT<T> a, FixArgsF f)
{
    __shared__ double red[4];
    __shared__ int trig;
    const bool t = rare_decide(f, red, &trig);
    if (a.fired != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
        *a.fired = t ? 1u : 0u;
    if (!t) return;
    __syncthreads();
    pre_body<T, X0_ZERO, false, PAIRS, false, PIN, true>(a, red);
}

// ---------------------------------------------------------------------------
// k_post
// ---------------------------------------------------------------------------
// full weighting of one point from its 3x3 neighbourhood (rows u / m / d = above / centre /
// below, columns w / c / e): MultiGrid.hpp:187-205's expression and operand order (the same as
// pgmg_kernels.hip's rfw for k_restrict2_values)
constexpr int kR2Stride = 116;   // k_post_r2's wave-tile stride (6-column margin)

template <class T>
__device__ __forceinline__ T rfw_post(T u_w, T u_c, T u_e, T m_w, T m_c, T m_e, T d_w, T d_c, T d_e)
{
    return T(0.25) * m_c + T(0.125) * (m_e + m_w + d_c + u_c) + T(0.0625) * (u_w + u_e + d_w + d_e);
}

// R2 (k_post_r2, the finest level's last pass of an F-cycle that another one follows): the next
// F-cycle starts by restricting this pass's result twice (compute_coarsest_grid, MultiGrid.hpp:
// 28-55; the level-1 values are dead), so the pass forms level 2 itself from the x2 rows it
// holds.  The band starts 4 rows earlier and ends 6 rows later (x2 valid on fine rows 2jcb-4 ..
// 2jce+1 instead of its own 2jcb .. 2jce-1; only its own rows are stored), the last two x2 rows
// and level-1 rows stay in registers, lane t forms the level-1 value at fine column c+1 (its
// east column from lane t+1 by DPP) and the level-2 centre lanes (level-1 column even) the
// level-2 value from lanes t-1 .. t+1.  A band owns the level-2 rows r2 with 4 r2 in its own
// fine rows; a wave the level-2 columns whose centre fine column it owns.  A level-2 point
// reads x2 three columns past its centre each side, so the wave tiles are 116 columns apart
// with a 6-column margin (lanes 3 .. 60 own, instead of 120 / 4 and lanes 2 .. 61) and lane 63
// loads its own east coarse column (x_eff, x1, x2 then valid on tile columns 0 .. 127, 1 .. 126,
// 2 .. 125): every owned centre's window (at most columns 2t-2 .. 2t+4 of lane t <= 60) is in
// the tile.
// RECOMP (levels entered with x0 = 0): phi is not read.  The loaded row is f[ii+1];
// x1 = J(0) is pointwise, so x1 row ii+1 -> phi row ii = J(x1) (or x1 when the pre
// check fired) -> x_eff row ii: one more row of lag than reading phi, 16 B/point less.
template <class T, bool FINE, int PAIRS, bool RECOMP, bool GENF, bool S1, bool S1P = false,
          bool R2 = false>
__device__ __forceinline__ void post_body(const PostArgsT<T> &a, double *red)
{
    constexpr int R = 2 * PAIRS;
    if (a.cond != nullptr && *a.cond == 0u) return;  // conditional (rare-path) launch
    int lbx, lby;
    fused_block(lbx, lby, (a.nt & 16) != 0);
    // R2: 116-column stride, 6-column margin (kR2Stride): see k_post_r2
    const Cols k = R2 ? lane_cols_t<kR2Stride, 6>(a.N, lbx) : lane_cols(a.N, lbx);
    const int N = a.N, Nc = a.Nc;
    const long long P = a.P, Pc = a.Pc;
    const int jcb = a.jc0 + lby * a.rows_per_block;
    const int jce = min(jcb + a.rows_per_block, a.jc1);
    const int olo = max(2 * jcb, a.row_lo), ohi = min(2 * jce, a.row_hi);
    const int slo = a.sum_hi > a.sum_lo ? max(olo, a.sum_lo) : olo;
    const int shi = a.sum_hi > a.sum_lo ? min(ohi, a.sum_hi) : ohi;
    if (!S1 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && a.stats != nullptr)
        atomicAdd(&a.stats[0], (unsigned long long)(2 + a.sw_adj));
    ProlongCols pc;
    pc.ic = (k.c - 1) >> 1;
    pc.vx = k.c >= 3 && k.c <= N - 2;
    pc.vy = k.c + 1 >= 2 && k.c + 1 <= N - 3;
    const T *__restrict__ F = a.f + k.c;
    const double fxa = GENF ? a.gfx[k.c] : 0.0, fxb = GENF ? a.gfx[k.c + 1] : 0.0;
    // the streamed array: phi, or f one row ahead (RECOMP)
    const T *__restrict__ X = RECOMP ? F + P : a.phi + k.c;
    const T *__restrict__ E = a.ec + pc.ic;
    T *__restrict__ O = a.x2 + k.c;
    const long long Po = a.Po != 0 ? a.Po : P;   // x2's pitch (the caller's array: N)
    const T hh = a.hh, ih = a.ih;
    const V2<T> z = zero2<T>();
    // windows: x_eff rows i-2,i-1 ; x1 rows i-3,i-2 ; f rows i-2,i-1
    V2<T> a0 = z, a1 = z, b0 = z, b1 = z, f1 = z, f2 = z;
    // RECOMP: pre-smooth x1 rows ii-1, ii ; f row ii
    V2<T> g0 = z, g1 = z, fc = z;
    double acc = 0.0;
    const int i_begin = 2 * jcb - 2 - (R2 ? 4 : 0);
    const int c0w = __builtin_amdgcn_readfirstlane(k.c - 2 * (int)(threadIdx.x & 63));
    const bool idle = c0w + 4 > N - 2;  // spare wave (wave-uniform)
    const bool inner = c0w >= 3 && c0w + 127 <= N - 3;   // see pre_body
    const int i_end = idle ? i_begin
                           : i_begin + ((2 * (jce - jcb) + (R2 ? 10 : 4) + R - 1) / R) * R;
    const bool pfired = RECOMP && *a.pre_fired != 0u;
    // R2: x2 rows q-2, q-1 and level-1 rows r1-2, r1-1 of this lane's level-1 column i1
    V2<T> q0 = z, q1 = z;
    T w0 = T(0), w1 = T(0);
    const int i1 = (k.c + 1) >> 1, i2 = i1 >> 1;
    const bool lane63 = (threadIdx.x & 63) == 63;
    const bool eall = R2 && (a.nt & 8) != 0;   // every lane loads its east coarse column
    const bool r2col = R2 && (i1 & 1) == 0 && k.own && i2 >= 1 && i2 <= a.Nr2 - 2;
    if (RECOMP && !idle) {
        const V2<T> fm = ldv(F + (i_begin - 1) * P);
        fc = ldv(F + i_begin * P);
        g0 = j0stage(fm, hh, k, boundary_row(i_begin - 1, N));
        g1 = j0stage(fc, hh, k, boundary_row(i_begin, N));
    }
    // coarse row m = ii/2 of fine row ii; an iteration of R rows uses coarse rows
    // i/2 .. i/2 + PAIRS
    V2<T> np_[R], nf[R];
    T ncr[PAIRS + 1], ncre[PAIRS + 1];   // ncre (R2): lane 63's east coarse column
    #pragma unroll
    for (int q = 0; q < R; ++q) {
        np_[q] = idle ? z : ldv(X + (i_begin + q) * P);
        if (!RECOMP && !GENF) nf[q] = idle ? z : ldv(F + (i_begin + q) * P);
    }
    #pragma unroll
    for (int q = 0; q <= PAIRS; ++q) {
        ncr[q] = idle ? T(0) : E[(long long)((i_begin >> 1) + q) * Pc];
        if (R2) ncre[q] = idle || !(lane63 || eall) ? T(0) : E[(long long)((i_begin >> 1) + q) * Pc + 1];
    }
    // FULL: as in pre_body (rows interior to the band, the sum range and the grid; interior
    // wave columns)
    auto full_at = [&](int i) {
        return !S1 && inner && i >= 3 && i + R <= N - 2 && i - 2 >= slo && i + R - 3 < shi &&
               ((i + R - 1) >> 1) <= Nc - 2;
    };
    auto iter = [&](int i, auto full_t) {
        V2<T> cp[R], cf[R];
        T cr[PAIRS + 1], cre[PAIRS + 1];
        #pragma unroll
        for (int q = 0; q < R; ++q) {
            cp[q] = np_[q];
            if (!RECOMP && !GENF) cf[q] = nf[q];
        }
        #pragma unroll
        for (int q = 0; q <= PAIRS; ++q) {
            cr[q] = ncr[q];
            if (R2) cre[q] = ncre[q];
        }
        if (i + R < i_end) {
            #pragma unroll
            for (int q = 0; q < R; ++q) {
                np_[q] = ldv(X + (i + R + q) * P);
                if (!RECOMP && !GENF) nf[q] = ldv(F + (i + R + q) * P);
            }
            #pragma unroll
            for (int q = 0; q <= PAIRS; ++q) {
                ncr[q] = E[(long long)(((i + R) >> 1) + q) * Pc];
                if (R2 && (lane63 || eall)) ncre[q] = E[(long long)(((i + R) >> 1) + q) * Pc + 1];
            }
        }
        T crn[PAIRS + 1];
        #pragma unroll
        for (int q = 0; q <= PAIRS; ++q) {
            crn[q] = dpp_shl(cr[q]);
            // R2: lane 63's own east column, so x_eff is valid on all 128 columns of the tile
            if (R2 && (lane63 || eall)) crn[q] = cre[q];
        }
        double gy[R];   // GENF row factors of the iteration, loaded together up front
        if constexpr (GENF) {
            #pragma unroll
            for (int q = 0; q < R; ++q) gy[q] = gsy_s(a.gsy, i + q);
        }
        {
            constexpr bool FULL = decltype(full_t)::value;
            #pragma unroll
            for (int s = 0; s < R; ++s) {
                const int ii = i + s;
                const int pq = s >> 1;
                V2<T> ph, f3;
                if (RECOMP) {
                    const V2<T> fn = cp[s];  // f row ii+1
                    const V2<T> g2 = j0stage<T, !FULL>(fn, hh, k, boundary_row(ii + 1, N));
                    ph = pfired ? g1 : jstage<T, !FULL>(g0, g1, g2, fc, hh, k, boundary_row(ii, N));
                    f3 = fc;
                    g0 = g1;
                    g1 = g2;
                    fc = fn;
                } else {
                    ph = cp[s];
                    if constexpr (GENF) {
                        f3 = mk2<T>((T)(fxa * gy[s]), (T)(fxb * gy[s]));
                    } else {
                        f3 = cf[s];
                    }
                }
                const V2<T> a2 = add_prolong<T, !FULL>(ph, ii, cr[pq], crn[pq], cr[pq + 1], crn[pq + 1], pc, Nc);
                const V2<T> b2 = jstage<T, !FULL>(a0, a1, a2, f2, hh, k, boundary_row(ii - 1, N));
                if constexpr (S1) {   // the post check fired: x1 row ii-1 is the result
                    if (ii - 1 >= olo && ii - 1 < ohi && k.own) stvu(O + (ii - 1) * Po, b2);
                    if constexpr (S1P) {   // the check's terms: r(x1) on row ii-2 (k_post1)
                        const int row = ii - 2;
                        const V2<T> r1 = rstage(b0, b1, b2, f1, ih);
                        if constexpr (R2 && chk_sel_lv<T>()) {
                            acc = chk_acc<T>(acc, r1, row >= slo && row < shi && k.own, k.by);
                        } else if (row >= slo && row < shi && k.own) {
                            acc = sqacc(acc, r1.x);
                            if (!k.by) acc = sqacc(acc, r1.y);
                        }
                        b0 = b1;
                        b1 = b2;
                    }
                    a0 = a1;
                    a1 = a2;
                    f1 = f2;
                    f2 = f3;
                    continue;
                }
                {
                    const int row = ii - 2;
                    const V2<T> r1 = rstage(b0, b1, b2, f1, ih);
                    if constexpr (R2 && chk_sel_lv<T>()) {
                        acc = chk_acc<T>(acc, r1, (FULL || (row >= slo && row < shi)) && k.own, !FULL && k.by);
                    } else if ((FULL || (row >= slo && row < shi)) && k.own) {
                        acc = sqacc(acc, r1.x);
                        if (FULL || !k.by) acc = sqacc(acc, r1.y);
                    }
                }
                const V2<T> c2 = jstage<T, !FULL>(b0, b1, b2, f1, hh, k, boundary_row(ii - 2, N));
                if ((FULL || (ii - 2 >= olo && ii - 2 < ohi)) && k.own) {
                    if (a.nt & 4) stv_nt(O + (ii - 2) * Po, c2);
                    else stvu(O + (ii - 2) * Po, c2);
                }
                if constexpr (R2) {
                    // x2 row q = ii - 2 (i is even: q is odd exactly for odd s)
                    if (s & 1) {   // q = 2 r1 + 1: level-1 row r1 from x2 rows q-2, q-1, q
                        const T v1 = rfw_post<T>(q0.x, q0.y, dpp_shl(q0.x), q1.x, q1.y, dpp_shl(q1.x),
                                                 c2.x, c2.y, dpp_shl(c2.x));
                        const int r1 = (ii - 3) >> 1;
                        if (r1 & 1) {   // r1 = 2 r2 + 1 (wave-uniform): level-2 row r2
                            const T v2 = rfw_post<T>(dpp_shr(w0), w0, dpp_shl(w0), dpp_shr(w1), w1,
                                                     dpp_shl(w1), dpp_shr(v1), v1, dpp_shl(v1));
                            const int r2 = r1 >> 1;
                            if (r2col && 4 * r2 >= olo && 4 * r2 < ohi && r2 >= 1 && r2 <= a.Nr2 - 2)
                                a.r2out[(long long)r2 * a.Pr2 + i2] = v2;
                        }
                        w0 = w1;
                        w1 = v1;
                    }
                    q0 = q1;
                    q1 = c2;
                }
                a0 = a1;
                a1 = a2;
                b0 = b1;
                b1 = b2;
                f1 = f2;
                f2 = f3;
            }
        }
    };
    // (one loop with the path chosen per iteration: the 12-row form of k_pre costs k_post
    // 150 -> 210 VGPRs, i.e. 3 -> 2 waves per SIMD, and measured slower; hoisting the pre
    // check's outcome out of the loop measured no gain)
    row_loop<R, 0>(i_begin, i_end, full_at, iter);
    if constexpr (!S1 || S1P) {
        const double sum = fused_block_sum(acc, red);
        if (threadIdx.x == 0) a.partials[lby * gridDim.x + lbx] = sum;
    }
}

template <class T, bool FINE, int PAIRS, bool RECOMP, bool GENF = false>
__global__ __launch_bounds__(256) void k_post(PostArgsT<T> a)
{
    __shared__ double red[4];
    post_body<T, FINE, PAIRS, RECOMP, GENF, false>(a, red);
}

// the finest level's last pass of an F-cycle with the next F-cycle's level-2 restriction
template <class T, bool GENF>
__global__ __launch_bounds__(256) void k_post_r2(PostArgsT<T> a)
{
    __shared__ double red[4];
    post_body<T, true, 2, false, GENF, false, false, true>(a, red);
}

// a coarse level's post-smooth whose check is predicted to fire (see k_pre1): x1 is the
// result (RECOMP: the pre-smoothed iterate recomputed as the pre check decided; otherwise read),
// one sweep and one exit booked, the check's partials written
template <class T, int PAIRS, bool RECOMP>
__global__ __launch_bounds__(256) void k_post1(PostArgsT<T> a)
{
    __shared__ double red[4];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && a.stats != nullptr) {
        atomicAdd(&a.stats[0], 1ull);
        atomicAdd(&a.stats[1], 1ull);
    }
    post_body<T, false, PAIRS, RECOMP, false, true, true>(a, red);
}

// rare path of k_post's check (replaces the scalar k_post_fixup on in-stream levels)
template <class T, int PAIRS, bool RECOMP>
__global__ __launch_bounds__(256) void k_post_rare(PostArgsT<T> a, FixArgsF f)
{
    __shared__ double red[4];
    __shared__ int trig;
    if (!rare_decide(f, red, &trig)) return;
    __syncthreads();
    post_body<T, false, PAIRS, RECOMP, false, true>(a, red);
}


// ---------------------------------------------------------------------------
// k_postpre: the finest level between two consecutive cycles of one call.
//   xe = phi + P ec -> x1 -> x2 (post-smooth of cycle k, never stored)
//   -> x3 -> x4 (pre-smooth of cycle k+1, stored) -> r(x4) -> rc (cycle k+1)
// Checks: ||r(x1)|| (post) and ||r(x3)|| (pre), both speculative (partials1/2).
// Read phi, f, ec; write x4, rc: 24 B per fine point + 16 B per coarse point,
// replacing k_post + k_pre (48 + 16).  Wave tile: 114 owned columns of 128
// (validity shrinks 6 columns per side through 6 stencil levels + restriction).
// Stage lags behind the loaded row i: xe i, x1 i-1, x2 i-2, x3 i-3, x4 i-4,
// r(x4) i-5, rc when i-5 = 2jc+1.
// ---------------------------------------------------------------------------
// 128-column wave tiles owning 116: six stencil levels shrink the validity six columns
// from the left; on the right the prolongation reads coarse column ic+1 from LDS (no DPP),
// so six suffice there too (114 + 6/8 before: 1.13-1.14 -> 1.11-1.13 ms; 112 + 8/8 with
// line-aligned stores: slower, 1.133 ms)
constexpr int kPPStride = 116, kPPMargin = 6;

// Horizontal neighbours of a row's column pair (left of c, right of c+1), shared by the
// stages that use the same centre row (a Jacobi sweep and a residual of the same iterate).
template <class T> struct Nbr {
    T l, r;
};
template <class T> __device__ __forceinline__ Nbr<T> nbr(V2<T> ce)
{
    return Nbr<T>{dpp_shr(ce.y), dpp_shl(ce.x)};
}
template <class T, bool EDGE>
__device__ __forceinline__ V2<T> jsn(V2<T> up, V2<T> ce, V2<T> dn, Nbr<T> n, V2<T> f, T hh,
                                       const Cols &k, bool brow)
{
    V2<T> o;
    if constexpr (sizeof(T) == 4 && PGMG_F32_PK) {   // packed (as jstage)
        const pf2 L = {n.l, ce.x}, R = {ce.y, n.r};
        o = unpk(0.25f * (((((hh * pk(f)) + L) + R) + pk(up)) + pk(dn)));
    } else {
        o.x = T(0.25) * ((hh * f.x) + n.l + ce.y + up.x + dn.x);
        o.y = T(0.25) * ((hh * f.y) + ce.x + n.r + up.y + dn.y);
    }
    if constexpr (EDGE) {
        if (brow || k.bx) o.x = ce.x;
        if (brow || k.by) o.y = ce.y;
    }
    return o;
}
// jsn with the RHS term hh*f precomputed (hf): the same IEEE product, formed once per row
// instead of once per sweep that reads the row
template <class T, bool EDGE>
__device__ __forceinline__ V2<T> jsh(V2<T> up, V2<T> ce, V2<T> dn, Nbr<T> n, V2<T> hf,
                                       const Cols &k, bool brow)
{
    V2<T> o;
    if constexpr (sizeof(T) == 4 && PGMG_F32_PK) {   // packed: L = (l, c), R = (c+1, r), same order per element
        const pf2 L = {n.l, ce.x}, R = {ce.y, n.r};
        o = unpk(0.25f * ((((pk(hf) + L) + R) + pk(up)) + pk(dn)));
    } else {
        o.x = T(0.25) * (hf.x + n.l + ce.y + up.x + dn.x);
        o.y = T(0.25) * (hf.y + ce.x + n.r + up.y + dn.y);
    }
    if constexpr (EDGE) {
        if (brow || k.bx) o.x = ce.x;
        if (brow || k.by) o.y = ce.y;
    }
    return o;
}
// FAST mode (OPT & 16): the neighbour sum of a centre row, S = (l + r) + (u + d), shared by
// its Jacobi stage, 0.25 * (hh*f + S), and its residual, f - ih * (4x - S) as two FMAs
template <class T>
__device__ __forceinline__ V2<T> nsum(V2<T> up, V2<T> ce, V2<T> dn, Nbr<T> n)
{
    V2<T> sm;
    sm.x = (n.l + ce.y) + (up.x + dn.x);
    sm.y = (ce.x + n.r) + (up.y + dn.y);
    return sm;
}
template <class T, bool EDGE>
__device__ __forceinline__ V2<T> jsum(V2<T> sm, V2<T> ce, V2<T> hf, const Cols &k, bool brow)
{
    V2<T> o;
    o.x = T(0.25) * (hf.x + sm.x);
    o.y = T(0.25) * (hf.y + sm.y);
    if constexpr (EDGE) {
        if (brow || k.bx) o.x = ce.x;
        if (brow || k.by) o.y = ce.y;
    }
    return o;
}
template <class T>
__device__ __forceinline__ V2<T> rsum(V2<T> sm, V2<T> ce, V2<T> f, T ih)
{
    V2<T> o;
    o.x = __builtin_fma(-ih, __builtin_fma(T(4), ce.x, -sm.x), f.x);
    o.y = __builtin_fma(-ih, __builtin_fma(T(4), ce.y, -sm.y), f.y);
    return o;
}
template <class T>
__device__ __forceinline__ V2<T> rsn(V2<T> up, V2<T> ce, V2<T> dn, Nbr<T> n, V2<T> f, T ih)
{
    V2<T> o;
    if constexpr (sizeof(T) == 4 && PGMG_F32_PK) {   // packed (as jsh)
        const pf2 L = {n.l, ce.x}, R = {ce.y, n.r};
        o = unpk(pk(f) - ih * ((((4.0f * pk(ce) - L) - R) - pk(up)) - pk(dn)));
    } else {
        o.x = f.x - ih * (T(4) * ce.x - n.l - ce.y - up.x - dn.x);
        o.y = f.y - ih * (T(4) * ce.y - ce.x - n.r - up.y - dn.y);
    }
    return o;
}

// ---------------------------------------------------------------------------
// k_postpre_lds (default): the same pass, but the rows of phi, f and ec are staged
// once per block in LDS.  A block's 4 wave tiles overlap by 12 columns each; loading
// every tile from HBM re-reads 14 of each 128 columns (12 %).  Here the block's
// 256 lanes load its 468-column window (4 x 114 owned + 2 x 6 margin) exactly once
// per row (one 16-byte load per lane), and each wave reads its 128-column window
// (and the coarse correction, with its right neighbour) from LDS.  Double-buffered
// by row pairs: while the waves compute pair g from one slot, the loads of pair g+2
// are in flight in registers and pair g+1 sits in the other slot; one barrier per
// row pair.  Coarse rows live in a ring of 3 (pair g reads coarse rows g and g+1).
// ---------------------------------------------------------------------------
constexpr int kPPWaves = 4;   // waves per k_postpre block (8-wave blocks measured equal, r02)
// The recompute form (OPT 256, the first finest pass of a call that took the carry): two more
// Jacobi stages in front, so two more columns of margin per side (112-column stride) and two
// more lead rows
constexpr int kPPStrideRC = 112, kPPMarginRC = 8;
template <int OPT> constexpr int pp_stride() { return (OPT & 256) ? kPPStrideRC : kPPStride; }
template <int OPT> constexpr int pp_margin() { return (OPT & 256) ? kPPMarginRC : kPPMargin; }
constexpr int kPPLdsRow = kPPWaves * kPPStride + 2 * kPPMargin + 4;          // doubles per row
constexpr int kPPLdsCoarse = kPPWaves * (kPPStride / 2) + kPPMargin + 8;     // per coarse row
static_assert(kPPWaves * kPPStrideRC + 2 * kPPMarginRC + 4 <= kPPLdsRow &&
                  kPPWaves * (kPPStrideRC / 2) + kPPMarginRC + 8 <= kPPLdsCoarse,
              "the recompute form's windows fit the LDS rows");
// fp32 (r05): the rows are staged from 16-byte loads of FOUR columns per lane (8-byte lane
// loads stream at 0.54-0.70x the 16-byte rate, MI355X_MICROARCH.md), starting two columns
// left of the window (column L0 - 2 is 16-byte aligned: column 1 of every row sits on a
// 128-byte boundary), so an fp32 LDS row carries a 2-element shift and 4 more elements; the
// coarse rows likewise from 16-byte loads at cc0 (aligned), rows padded to whole 16 bytes.
// Compile-time A/B knobs of the fp32 form (scripts/build_variant.sh): quad row loads, quad
// coarse loads, quad x4 stores, register sets of loads in flight.  Measured (r05,
// scripts/pp_ab.py --dtype f32, profiles/r05_fp32/pp_f32.jsonl, 3 interleaved rounds at 16385):
// k_postpre_lds<float> 0.636-0.651 ms as built before, 0.644-0.648 with every knob off,
// 0.675-0.687 with quad loads (2 waves of 4 do all the loading, ds_write_b128), 0.647-0.649
// with quad stores only -- the knobs stay off; the pass's cost for fp32 is its per-lane work
// on 2 columns, not the load width.
#ifndef PGMG_PP_CHEAPCHK
#define PGMG_PP_CHEAPCHK 0
#endif
#ifndef PGMG_F32_QLOAD
#define PGMG_F32_QLOAD 0
#endif
#ifndef PGMG_F32_QCOARSE
#define PGMG_F32_QCOARSE 0
#endif
#ifndef PGMG_F32_QSTORE
#define PGMG_F32_QSTORE 0
#endif
#ifndef PGMG_F32_DEPTH
#define PGMG_F32_DEPTH 3
#endif
template <class T> constexpr bool pp_ql() { return sizeof(T) == 4 && PGMG_F32_QLOAD; }
template <class T> constexpr bool pp_qc() { return sizeof(T) == 4 && PGMG_F32_QCOARSE; }
template <class T> constexpr bool pp_qs() { return sizeof(T) == 4 && PGMG_F32_QSTORE; }
template <class T> constexpr int pp_sh() { return pp_ql<T>() ? 2 : 0; }
template <class T> constexpr int pp_lds_row() { return kPPLdsRow + (pp_ql<T>() ? 4 : 0); }
template <class T> constexpr int pp_lds_coarse()
{
    return pp_qc<T>() ? (kPPLdsCoarse + 3) / 4 * 4 : kPPLdsCoarse;
}
// the register type of one row's staging load: a column pair (fp64), a column quad (fp32)
template <class T> using PPV = typename std::conditional<pp_ql<T>(), float4, V2<T>>::type;
template <class T> using PPC = typename std::conditional<pp_qc<T>(), float4, V2<T>>::type;

// R2 (row strips): also sum r(x2)^2 into partials3.  When the post check fires the
// pre-smooth restarts from x1 and its first check is ||r(J(x1))|| = ||r(x2)||; having it
// here lets one allreduce of three sums decide every rare path.
// GENF (the problem's f is the analytic RHS of compute_rhs): f is not streamed from HBM
// but regenerated per point as (T)(fx[i] * sy[j]) with fx[i] = factor*sin(p pi x_i / a)
// (per lane, in registers) and sy[j] = sin(q pi y_j / a) (per row, a scalar load) — the
// same IEEE operations as k_rhs, so the values are identical to the stored f.  One
// multiply per point replaces 8 bytes per point of the pass (28 -> 20 B/pt).
// OPT (compile-time, result-identical): 2 non-temporal x4 stores, 4 non-temporal rc
// stores, 64 the F-cycle's smooth(3) (no correction, no restriction), 128 the carry pass
// (the last pass of a call that hands the next call its pre-smooth: x2 -- the call's result --
// is stored INSTEAD of x4; the next call recomputes x4 from it), 256 the recompute form
// (the first pass of a call that took the carry: the input is the previous call's x2, whose
// pre-smooth -- two Jacobi stages, the carry pass's own expressions, bitwise its x4 -- runs in
// front of the correction; the pipeline's rows lag two more).
// Logical block of the 2D grid (x: column block, y: band).
struct Blk {
    int x, y;
};

constexpr int kPPR = 2;   // rows per LDS slot (a row pair)

// Row pairs of loads in flight per wave (register sets).  3 also makes the guard-free loop
// body 6 rows, the period of the row windows (no window copies: 141 -> 129 VALU per row);
// the fp64 instantiations with more live state (streamed f, the strips' third sum, the
// F-cycle's four-sweep form, the recompute form) keep 2, which fits 256 VGPRs without spilling.
template <class T, bool R2, bool GENF, int OPT>
constexpr int pp_depth()
{
    return sizeof(T) == 4 ? PGMG_F32_DEPTH : ((GENF && !R2 && !(OPT & (64 | 32 | 256))) ? 3 : 2);
}
// Lane t's 16-byte (fp32: 8-byte) column pair of a row segment starting at `base`; lanes
// t >= n read 0 (descriptor range check).  The descriptor is built from wave-uniform values.
template <class T, int NT>
__device__ __forceinline__ V2<T> buf_row(const T *base, int n, int t)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T *>(base), (short)0, n * (int)sizeof(V2<T>), 0x00020000);
    if constexpr (sizeof(T) == 8) {
        return __builtin_bit_cast(V2<T>, __builtin_amdgcn_raw_buffer_load_b128(
                                             r, t * 16, 0, NT ? 2 : 0));
    } else {
        return __builtin_bit_cast(V2<T>, __builtin_amdgcn_raw_buffer_load_b64(
                                             r, t * 8, 0, NT ? 2 : 0));
    }
}
template <class T, int NT>
__device__ __forceinline__ void buf_store_row(T *base, int bytes, int off, V2<T> v)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);
    if constexpr (sizeof(T) == 8) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, off, 0, NT ? 2 : 0);
    } else {
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, off, 0, NT ? 2 : 0);
    }
}
template <class T>
__device__ __forceinline__ void buf_store_one(T *base, int bytes, int off, T v)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);
    if constexpr (sizeof(T) == 8) {
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, off, 0, 0);
    } else {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, 0);
    }
}
// fp32: lane t's 16-byte column quad of a row segment of n quads starting at `base`
__device__ __forceinline__ float4 buf_quad(const float *base, int n, int t)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(base), (short)0, n * 16, 0x00020000);
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, t * 16, 0, 0));
}
template <int NT>
__device__ __forceinline__ void buf_store_quad(float *base, int bytes, int off, float4 v)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, off, 0, NT ? 2 : 0);
}
template <class T>
__device__ __forceinline__ T buf_one(const T *base, int n, int t)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T *>(base), (short)0, n * (int)sizeof(T), 0x00020000);
    if constexpr (sizeof(T) == 8)
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, t * 8, 0, 0));
    else
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, t * 4, 0, 0));
}

// The body of k_postpre_lds for one block.  EDGE = false: no row of the block's band and
// no column of this wave is a boundary, so the Jacobi stages carry no passthrough selects.
template <class T, bool R2, bool GENF, bool EDGE, int OPT>
__device__ __forceinline__ void postpre_lds_run(const PostPreArgsT<T> &a, const Cols &k,
                                                double *red, T (&sx)[2][kPPR][pp_lds_row<T>()],
                                                T (&sf)[2][kPPR][GENF ? 1 : pp_lds_row<T>()],
                                                T (&se)[3][pp_lds_coarse<T>()], const Blk bk)
{
    constexpr bool Q = pp_ql<T>();   // fp32: 16-byte column quads (above)
    constexpr bool QC = pp_qc<T>(), QS = pp_qs<T>();
    constexpr int SH = pp_sh<T>();
    constexpr int R = kPPR;
    constexpr bool RC = (OPT & 256) != 0;           // the recompute form
    constexpr bool CARRY = (OPT & 128) != 0;        // the carry pass
    constexpr int ST = pp_stride<OPT>(), MG = pp_margin<OPT>();
    constexpr int LAG = RC ? 2 : 0;                 // rows the correction lags the input
    const int N = a.N, Nc = a.Nc;
    const long long P = a.P, Pc = a.Pc;
    const int jcb = a.jc0 + bk.y * a.rows_per_block;
    const int jce = min(jcb + a.rows_per_block, a.jc1);
    const int olo = max(2 * jcb, a.row_lo), ohi = min(2 * jce, a.row_hi);
    const int clo = max(jcb, max(1, a.rc_lo)), chi = min(jce, min(N / 2, a.rc_hi));
    if (bk.x == 0 && bk.y == 0 && threadIdx.x == 0 && a.stats != nullptr)
        atomicAdd(&a.stats[0], (unsigned long long)(4 + a.sw_adj));
    ProlongCols pc;
    pc.ic = (k.c - 1) >> 1;
    pc.vx = k.c >= 3 && k.c <= N - 2;
    pc.vy = k.c + 1 >= 2 && k.c + 1 <= N - 3;
    const T hh = a.hh, ih = a.ih;
    const V2<T> z = zero2<T>();

    // loader geometry: the block window starts at column L0 (odd: 16-byte aligned pairs)
    const int wpb = blockDim.x >> 6;
    const int t = threadIdx.x;
    const int L0 = ST * wpb * bk.x + 1 - MG;
    const int npairs = (ST * wpb + 2 * MG) / 2;
    const int cc0 = (L0 - 1) >> 1;                               // first coarse column
    const int ncc = (ST / 2) * wpb + MG + 2;
    // OPT & 64 (F-cycle smooth(3)): no coarse correction, no restriction
    // Row loads through buffer descriptors (one per row, built from wave-uniform values):
    // VMEM-only loads whose out-of-range lanes (past the window or the grid's last column)
    // read 0 from the descriptor's range check.  A `ldr ? load : 0` select compiles to a
    // FLAT load, which also counts on lgkmcnt, so the LDS wait before every barrier drained
    // the row pairs prefetched for later steps.
    // lanes that load (columns >= N never matter)
    const int nvx = max(0, min(npairs, (N - 1 - L0) / 2 + 1));
    const int nve = (OPT & 64) ? 0 : max(0, min(ncc, Nc - cc0));
    // stores: x4 row segment of the block window (lanes that own their pair), rc (lanes
    // owning a coarse column <= Nc-2); anything else gets an out-of-range offset
    constexpr int kOOB = 1 << 30;
    const int xbytes = (2 * npairs + 8) * (int)sizeof(T);
    const int xoff = k.own ? (k.c - L0) * (int)sizeof(T) : kOOB;
    const int cbytes = (ncc + 8) * (int)sizeof(T);
    const int coff = (k.own && ((k.c + 1) >> 1) <= Nc - 2) ? (((k.c + 1) >> 1) - cc0) * (int)sizeof(T) : kOOB;
    // GENF: this lane's columns of fx (tables padded: valid for columns/rows -8 ..)
    const double fxa = GENF ? a.gfx[k.c] : 0.0, fxb = GENF ? a.gfx[k.c + 1] : 0.0;
    // land them before the row loop: a load still in flight at the loop entry makes the
    // loop's first use of fxa wait for every outstanding load (vmcnt(0)) in every iteration
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    // this wave's window in the LDS rows
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int xo = ST * w + 2 * lane;
    const int co = (ST / 2) * w + lane;
    // fp32 quads: the window's 2 * npairs columns from L0 - 2 (nq4 quads; nvq of them inside
    // the loaded range, the rest read 0); coarse: ncc columns from cc0 (ncq quads, nveq valid).
    // A quad past the old pair/element range loads columns past the grid's last one or the
    // window: they reach only lanes that own nothing (the margins), as before.
    const int nq4 = (2 * npairs + 2 + 3) / 4, nvq = (2 * nvx + 2 + 3) / 4;
    const int ncq = (ncc + 3) / 4, nveq = (nve + 3) / 4;
    // fp32 x4 stores: odd lane l (16-byte aligned column) stores its pair and lane l+1's as
    // one quad when both own theirs; an owning odd lane without an owning partner (the grid's
    // right edge) stores its pair alone
    const bool own_next = lane + 1 < MG / 2 + ST / 2 && k.c + 2 <= N - 2;
    const int xoff16 = (QS && (lane & 1) && k.own && own_next) ? xoff : kOOB;
    const int xoff8 = QS ? (((lane & 1) && k.own && !own_next) ? xoff : kOOB) : xoff;

    V2<T> e0 = z, e1 = z, b0 = z, b1 = z, c0 = z, c1 = z, g0 = z, g1 = z, h0 = z, h1 = z,
            d0 = z, d1 = z;
    V2<T> f1 = z, f2 = z, f3 = z, f4 = z, f5 = z;  // f[i-1], f[i-2], ..., f[i-5]
    V2<T> q1 = z, q2 = z, q3 = z, q4 = z;          // hh * f[i-1], ..., hh * f[i-4]
    V2<T> f6 = z, f7 = z, q5 = z, q6 = z;          // RC: the windows two rows longer
    V2<T> p0 = z, p1 = z, a0 = z, a1 = z;          // RC: input rows i-2, i-1; stage-1 rows i-3, i-2
    double acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
    const int i_begin = 2 * jcb - 6 - LAG;
    // row pairs (uniform over the block): the input rows 2jcb-6-LAG .. 2jce+4+LAG
    const int ng = (2 * (jce - jcb) + 11 + 2 * LAG + R - 1) / R;
    // coarse row of the first pair (RC: the correction of pair gi's rows lags one pair)
    const int m0 = (i_begin >> 1) - (RC ? 1 : 0);
    auto ring = [](int m) { return (m + 3 * 4096) % 3; };  // m >= -3

    if (t < 2 * R * 4) {   // the 4 pad doubles past the window (read by spare lanes only)
        const int sl = t >> 3, q = (t >> 2) & 1, j = pp_lds_row<T>() - 4 + (t & 3);
        sx[sl][q][j] = T(0);
        if constexpr (!GENF) sf[sl][q][j] = T(0);
    }
    // D register sets: pair p's loads go to set p % D, issued D pairs ahead (D = 2: sets
    // A, B; D = 3: A, B, C)
    constexpr int D = pp_depth<T, R2, GENF, OPT>();
    static_assert(D == 2 || D == 3, "two or three register sets");
    using PV = PPV<T>;
    PV pxA[R], pfA[R], pxB[R], pfB[R], pxC[R], pfC[R];   // C unused (dead) when D = 2
    using PC = PPC<T>;
    const PC cz{};
    PC peA = cz, peB = cz, peC = cz;   // the pair's second coarse row (pairs: in .x)
    auto load_coarse = [&](int m) {
        if constexpr (QC) return buf_quad(reinterpret_cast<const float *>(a.ec) + (long long)m * Pc + cc0, nveq, t);
        else {
            PC v = cz;
            v.x = buf_one<T>(a.ec + (long long)m * Pc + cc0, nve, t);
            return v;
        }
    };
    auto store_coarse = [&](int m, PC v) {
        if constexpr (QC) {
            if (t < ncq) *reinterpret_cast<float4 *>(&se[ring(m)][4 * t]) = v;
        } else {
            if (t < ncc) se[ring(m)][t] = v.x;
        }
    };
    auto load_pair = [&](int p, PV (&px)[R], PV (&pf)[R], PC &pe) {
        #pragma unroll
        for (int q = 0; q < R; ++q) {
            const long long row = (long long)(i_begin + p * R + q) * P + L0;
            if constexpr (Q) {
                px[q] = buf_quad(reinterpret_cast<const float *>(a.phi) + row - SH, nvq, t);
                if constexpr (!GENF) pf[q] = buf_quad(reinterpret_cast<const float *>(a.f) + row - SH, nvq, t);
            } else {
                px[q] = buf_row<T, 0>(a.phi + row, nvx, t);
                if constexpr (!GENF) pf[q] = buf_row<T, 0>(a.f + row, nvx, t);
            }
        }
        pe = load_coarse(m0 + p + 1);   // 2nd coarse row
    };
    auto store_pair = [&](int p, const PV (&px)[R], const PV (&pf)[R], PC pe) {
        if (t < (Q ? nq4 : npairs)) {
            #pragma unroll
            for (int q = 0; q < R; ++q) {
                *reinterpret_cast<PV *>(&sx[p & 1][q][(Q ? 4 : 2) * t]) = px[q];
                if constexpr (!GENF) *reinterpret_cast<PV *>(&sf[p & 1][q][(Q ? 4 : 2) * t]) = pf[q];
            }
        }
        store_coarse(m0 + p + 1, pe);
    };
    // prologue: pair 0 (+ its first coarse row) into slot 0; pairs 1 .. D in flight
    load_pair(0, pxA, pfA, peA);
    store_coarse(m0, load_coarse(m0));
    store_pair(0, pxA, pfA, peA);
    if (ng > 1) load_pair(1, pxB, pfB, peB);
    if constexpr (D == 3) {
        if (ng > 2) load_pair(2, pxC, pfC, peC);
        if (ng > 3) load_pair(3, pxA, pfA, peA);
    } else {
        if (ng > 2) load_pair(2, pxA, pfA, peA);
    }
    __syncthreads();

    // pair gi: compute from slot gi & 1; pair gi+1 (set (gi+1) & 1) -> the other slot;
    // issue pair gi+3 into the set just freed; one barrier
    T wprev = T(0);   // dpp_shl(d2.x) of the previous restriction row (d0 starts as zero)
    auto step = [&](int gi, PV (&px)[R], PV (&pf)[R], PC &pe) {
        // keep the scheduler inside one pair: interleaving the unrolled pairs only raises
        // the register pressure (the loads of a pair are issued two pairs ahead anyway)
        __builtin_amdgcn_sched_barrier(0);
        const int slot = gi & 1;
        // the other slot's previous readers passed the last barrier: stage pair gi+1 (loaded
        // D steps ago) first and reissue its register set for pair gi+1+D, so the loads in
        // flight are never younger than this step's stores (counted waits stay small)
        if (gi + 1 < ng) store_pair(gi + 1, px, pf, pe);
        if (gi + 1 + D < ng) load_pair(gi + 1 + D, px, pf, pe);
        const int i = i_begin + gi * R;
        const int m = m0 + gi;
        const T *E0 = se[ring(m)], *E1 = se[ring(m + 1)];
        const T cr0 = E0[co], crn0 = E0[co + 1], cr1 = E1[co], crn1 = E1[co + 1];
        #pragma unroll
        for (int s = 0; s < R; ++s) {
            const int ii = i + s;
            const V2<T> xr = ldv(&sx[slot][s][xo + SH]);
            // f[ii]: from LDS, or (GENF) generated once here and carried in the f window
            // (regenerating it at every use instead: fewer VGPRs, 8 more multiplies per
            // row, measured slower in r01)
            V2<T> f0 = z;
            if constexpr (!GENF) f0 = ldv(&sf[slot][s][xo + SH]);
            if constexpr (GENF) {
                const double sy = gsy_s(a.gsy, ii);
                f0 = mk2<T>((T)(fxa * sy), (T)(fxb * sy));
            }
            const V2<T> q0 = mk2<T>(hh * f0.x, hh * f0.y);
            constexpr bool FAST = (OPT & 16) != 0;
            // RC: the carry pass's pre-smooth of the input (its g / h stages, the same
            // expressions on the same values: bitwise its x4), row ii-2; then every stage below
            // runs on row L = ii - 2 with the f windows two rows further back
            V2<T> xin = xr;
            if constexpr (RC) {
                const V2<T> a2 = FAST ? jsum<T, EDGE>(nsum<T>(p0, p1, xr, nbr<T>(p1)), p1, q1, k, boundary_row(ii - 1, N))
                                      : jsh<T, EDGE>(p0, p1, xr, nbr<T>(p1), q1, k, boundary_row(ii - 1, N));
                xin = FAST ? jsum<T, EDGE>(nsum<T>(a0, a1, a2, nbr<T>(a1)), a1, q2, k, boundary_row(ii - 2, N))
                           : jsh<T, EDGE>(a0, a1, a2, nbr<T>(a1), q2, k, boundary_row(ii - 2, N));
                p0 = p1; p1 = xr;
                a0 = a1; a1 = a2;
            }
            const int L = ii - LAG;
            const V2<T> fq2 = RC ? f4 : f2, fq3 = RC ? f5 : f3, fq4 = RC ? f6 : f4, fq5 = RC ? f7 : f5;
            const V2<T> hq1 = RC ? q3 : q1, hq2 = RC ? q4 : q2, hq3 = RC ? q5 : q3, hq4 = RC ? q6 : q4;
            const V2<T> e2 = (OPT & 64) ? xin : add_prolong<T, EDGE>(xin, L, cr0, crn0, cr1, crn1, pc, Nc);
            // post-smooth sweep 1: x1 row ii-1
            const V2<T> b2 = FAST ? jsum<T, EDGE>(nsum<T>(e0, e1, e2, nbr<T>(e1)), e1, hq1, k, boundary_row(L - 1, N))
                                  : jsh<T, EDGE>(e0, e1, e2, nbr<T>(e1), hq1, k, boundary_row(L - 1, N));
            const Nbr<T> nb1 = nbr<T>(b1), nc1 = nbr<T>(c1), ng1 = nbr<T>(g1);
            // FAST: the neighbour sums of x1 row ii-2 and x3 row ii-4, each shared by a sweep
            // and a check
            const V2<T> sb = FAST ? nsum<T>(b0, b1, b2, nb1) : z;
            {   // post check: r(x1) on row ii-2
#if PGMG_PP_CHEAPCHK   // measurement only: what the checks' residuals cost (the sums are wrong)
                const V2<T> r1 = b1;
#else
                const V2<T> r1 = FAST ? rsum<T>(sb, b1, fq2, ih) : rsn<T>(b0, b1, b2, nb1, fq2, ih);
#endif
                const int row = L - 2;
                if constexpr (chk_sel<T>()) {
                    acc1 = chk_acc<T>(acc1, r1, row >= olo && row < ohi && k.own, k.by);
                } else if (row >= olo && row < ohi && k.own) {
                    acc1 = sqacc(acc1, r1.x);
                    if (!k.by) acc1 = sqacc(acc1, r1.y);
                }
            }
            // post-smooth sweep 2: x2 row L-2 (= phi of cycle k+1)
            const V2<T> c2 = FAST ? jsum<T, EDGE>(sb, b1, hq2, k, boundary_row(L - 2, N))
                                  : jsh<T, EDGE>(b0, b1, b2, nb1, hq2, k, boundary_row(L - 2, N));
            if constexpr (CARRY) {   // the carry pass: x2 is the call's result (x4 is not stored)
                const int xb2 = (L - 2 >= olo && L - 2 < ohi) ? xbytes : 0;
                buf_store_row<T, (OPT & 2) ? 1 : 0>(a.x2 + (long long)(L - 2) * P + L0, xb2, xoff, c2);
            }
            if (R2) {   // r(x2) on row ii-3
                const V2<T> r2 = rsn<T>(c0, c1, c2, nc1, fq3, ih);
                const int row = L - 3;
                if constexpr (chk_sel<T>()) {
                    acc3 = chk_acc<T>(acc3, r2, row >= olo && row < ohi && k.own, k.by);
                } else if (row >= olo && row < ohi && k.own) {
                    acc3 = sqacc(acc3, r2.x);
                    if (!k.by) acc3 = sqacc(acc3, r2.y);
                }
            }
            // pre-smooth sweep 1: x3 row ii-3
            const V2<T> g2 = FAST ? jsum<T, EDGE>(nsum<T>(c0, c1, c2, nc1), c1, hq3, k, boundary_row(L - 3, N))
                                  : jsh<T, EDGE>(c0, c1, c2, nc1, hq3, k, boundary_row(L - 3, N));
            const V2<T> sgg = FAST ? nsum<T>(g0, g1, g2, ng1) : z;
            {   // pre check: r(x3) on row ii-4
#if PGMG_PP_CHEAPCHK
                const V2<T> r3 = g1;
#else
                const V2<T> r3 = FAST ? rsum<T>(sgg, g1, fq4, ih) : rsn<T>(g0, g1, g2, ng1, fq4, ih);
#endif
                const int row = L - 4;
                if constexpr (chk_sel<T>()) {
                    acc2 = chk_acc<T>(acc2, r3, row >= olo && row < ohi && k.own, k.by);
                } else if (row >= olo && row < ohi && k.own) {
                    acc2 = sqacc(acc2, r3.x);
                    if (!k.by) acc2 = sqacc(acc2, r3.y);
                }
            }
            // pre-smooth sweep 2: x4 row ii-4 (stored)
            const V2<T> h2 = FAST ? jsum<T, EDGE>(sgg, g1, hq4, k, boundary_row(L - 4, N))
                                  : jsh<T, EDGE>(g0, g1, g2, ng1, hq4, k, boundary_row(L - 4, N));
            // branch-free: rows outside the band get a zero-record descriptor, lanes that do
            // not own their pair an out-of-range offset (every step issues the same memory
            // instructions, so the compiler can count its waits)
            if constexpr (!CARRY) {
                const int xb = (L - 4 >= olo && L - 4 < ohi) ? xbytes : 0;
                T *xrow = a.x4 + (long long)(L - 4) * P + L0;
                if constexpr (QS) {   // lane l+1's pair by DPP; odd lanes store the quad
                    const float4 v4 = make_float4(h2.x, h2.y, dpp_shl(h2.x), dpp_shl(h2.y));
                    buf_store_quad<(OPT & 2) ? 1 : 0>(reinterpret_cast<float *>(xrow), xb, xoff16, v4);
                    if constexpr (EDGE)
                        buf_store_row<T, (OPT & 2) ? 1 : 0>(xrow, xb, xoff8, h2);
                } else {
                    buf_store_row<T, (OPT & 2) ? 1 : 0>(xrow, xb, xoff8, h2);
                }
            }
            // r(x4) on row ii-5
            const V2<T> d2 = FAST ? rsum<T>(nsum<T>(h0, h1, h2, nbr<T>(h1)), h1, fq5, ih)
                                  : rsn<T>(h0, h1, h2, nbr<T>(h1), fq5, ih);
            // restriction: rows L-7, L-6, L-5 = 2jc-1, 2jc, 2jc+1 when L is even
            if (!(OPT & 64) && (s & 1) == 0) {
                const int jc = (L - 6) >> 1;
                const T m2 = dpp_shl(d1.x);
                const T u2 = wprev;               // = dpp_shl(d0.x): row ii-7 was d2 two rows ago
                const T w2 = dpp_shl(d2.x);
                wprev = w2;
                const T v = T(0.25) * d1.y + T(0.125) * (m2 + d1.x + d2.y + d0.y) +
                                 T(0.0625) * (d0.x + u2 + d2.x + w2);
                buf_store_one<T>(a.rc + (long long)jc * Pc + cc0, (jc >= clo && jc < chi) ? cbytes : 0,
                                 coff, v);
            }
            e0 = e1; e1 = e2;
            b0 = b1; b1 = b2;
            c0 = c1; c1 = c2;
            g0 = g1; g1 = g2;
            h0 = h1; h1 = h2;
            d0 = d1; d1 = d2;
            if constexpr (RC) {
                f7 = f6; f6 = f5;
                q6 = q5; q5 = q4;
            }
            f5 = f4; f4 = f3; f3 = f2; f2 = f1; f1 = f0;
            q4 = q3; q3 = q2; q2 = q1; q1 = q0;
        }
        __syncthreads();
    };
    if constexpr (D == 3) {
        // 6 rows per iteration, no guard inside: the row windows rotate with periods 3 (two
        // carried rows and the new one) and 6 (f), so after 6 rows every carried value is
        // back in its register (a guarded step would merge two paths and force copies)
        int gi = 0;
        for (; gi + 3 <= ng; gi += 3) {
            step(gi, pxB, pfB, peB);
            step(gi + 1, pxC, pfC, peC);
            step(gi + 2, pxA, pfA, peA);
        }
        if (gi < ng) step(gi, pxB, pfB, peB);
        if (gi + 1 < ng) step(gi + 1, pxC, pfC, peC);
    } else {
        for (int gi = 0; gi < ng; gi += 2) {
            step(gi, pxB, pfB, peB);
            if (gi + 1 < ng) step(gi + 1, pxA, pfA, peA);
        }
    }
    const int slot = bk.y * gridDim.x + bk.x;
    const double s1 = fused_block_sum(acc1, red);
    __syncthreads();
    const double s2 = fused_block_sum(acc2, red);
    if (R2) {
        __syncthreads();
        const double s3 = fused_block_sum(acc3, red);
        if (threadIdx.x == 0) a.partials3[slot] = s3;
    }
    if (threadIdx.x == 0) {
        a.partials1[slot] = s1;
        a.partials2[slot] = s2;
    }
}


// two waves per SIMD (3 spills and measured slower, r02)
// fp32: the minimum waves per SIMD the register allocation must allow (PGMG_F32_WAVES, r05);
// 2 lets it take up to 256 VGPRs (it uses 118 with the branch-form checks: 4 waves anyway;
// 4 with the select-form checks spills 140 bytes)
#ifndef PGMG_F32_WAVES
#define PGMG_F32_WAVES 2
#endif
template <class T> constexpr int pp_waves() { return sizeof(T) == 4 ? PGMG_F32_WAVES : 2; }
template <class T, bool R2, bool GENF, int OPT>
__global__ __launch_bounds__(64 * kPPWaves) __attribute__((amdgpu_waves_per_eu(pp_waves<T>())))
void k_postpre_lds(PostPreArgsT<T> a)
{
    __shared__ double red[kPPWaves];
    __shared__ __attribute__((aligned(16))) T sx[2][kPPR][pp_lds_row<T>()];
    __shared__ __attribute__((aligned(16))) T sf[2][kPPR][GENF ? 1 : pp_lds_row<T>()];
    __shared__ __attribute__((aligned(16))) T se[3][pp_lds_coarse<T>()];
    Blk bk{(int)blockIdx.x, (int)blockIdx.y};
    if (a.xcd) xcd_tile(bk.x, bk.y);
    const Cols k = lane_cols_t<pp_stride<OPT>(), pp_margin<OPT>()>(a.N, bk.x);
    // the band's rows 2jcb-6 .. 2jce+5 (RC: from 2jcb-8; see postpre_lds_run): does it reach
    // row 0 or N-1?
    const int jcb = a.jc0 + bk.y * a.rows_per_block;
    const int jce = min(jcb + a.rows_per_block, a.jc1);
    constexpr int lag = (OPT & 256) ? 2 : 0;
    const bool edge_rows = 2 * jcb - 6 - lag <= 0 || 2 * jce + 6 + lag >= a.N - 1;
    if (k.edge || edge_rows)
        postpre_lds_run<T, R2, GENF, true, OPT>(a, k, red, sx, sf, se, bk);
    else
        postpre_lds_run<T, R2, GENF, false, OPT>(a, k, red, sx, sf, se, bk);
}

// one block: both decisions, stats, flags for the conditional rare-path kernels
// global != nullptr (row strips): the all-rank sums {post, pre} instead of the partials
__global__ __launch_bounds__(256) void k_postpre_decide(const double *p1, const double *p2, int np,
                                                        const double *global, double eps,
                                                        unsigned *flags,
                                                        unsigned long long *stats)
{
    __shared__ double red[4];
    double s1 = 0.0, s2 = 0.0;
    for (int k = threadIdx.x; k < np; k += blockDim.x) {
        s1 += p1[k];
        s2 += p2[k];
    }
    s1 = fused_block_sum(s1, red);
    __syncthreads();
    s2 = fused_block_sum(s2, red);
    if (threadIdx.x == 0 && global != nullptr) {
        s1 = global[0];
        s2 = global[1];
    }
    if (threadIdx.x == 0) {
        const unsigned t1 = sqrt(s1) < eps ? 1u : 0u;
        const unsigned t2 = (!t1 && sqrt(s2) < eps) ? 1u : 0u;
        flags[0] = t1;
        flags[1] = t2;
        if (stats != nullptr) {
            // t1: the post-smooth stopped after 1 sweep and the pre-smooth is redone from
            //     x1 by the conditional k_pre (which counts its own sweeps): -1 - 2
            // t2: the pre-smooth stopped after 1 sweep: -1
            if (t1) {
                atomicAdd(&stats[0], (unsigned long long)-3LL);
                atomicAdd(&stats[1], 1ull);
                atomicAdd(&stats[2], 1ull);
            }
            if (t2) {
                atomicAdd(&stats[0], (unsigned long long)-1LL);
                atomicAdd(&stats[1], 1ull);
                atomicAdd(&stats[3], 1ull);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// launch geometry
// ---------------------------------------------------------------------------
// Launch geometry.  Blocks march down long row bands: the grid is sized to about
// the number of workgroups resident at once, so the 8 halo rows per band are a small
// fraction and there is no tail wave of blocks.
thread_local LaunchNote g_last_launch;

#ifdef PGMG_TUNING
int tuning_int(const char *name, int dflt)
{
    const char *v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}
#endif

static void fused_geometry(int N, int jc0, int jc1, int *threads, int *gx, int *gy, int *rpb,
                           int stride = 120, int target = 0, int maxw = 4)
{
    const int waves = (N - 2 + stride - 1) / stride;
    const int wpb = waves < maxw ? waves : maxw;
    *threads = 64 * wpb;
    *gx = (waves + wpb - 1) / wpb;
    const int rows = jc1 - jc0;   // coarse rows
    // ~22k fine points per workgroup, 256 .. 3072 workgroups: measured per level at N =
    // 16385 (scripts/level_sweep.sh): 8193 best at 3072, 4097 at 768 (band halos), and
    // the finest level's first/last passes at 3072 (6 rounds of the 512 resident)
    if (target <= 0) {
        const long long pts = 2LL * rows * N;
        if (pts > (1LL << 23)) {
            // ~22k points per workgroup, at least one round of the 512 resident (8193 on 8
            // strips: 37+28 -> 34+24 us), at most 3072
            // (measurement build: PGMG_FUSED_BLOCKS_BIG for the levels of N >= 8193 alone)
            const int dflt = (int)std::min(3072LL, std::max(512LL, pts / 21845));
            target = tuning_int("PGMG_FUSED_BLOCKS", pts >= (1LL << 25) ? tuning_int("PGMG_FUSED_BLOCKS_BIG", dflt) : dflt);
        } else {
            // latency-bound levels (N <= 2049): short bands (~8k points per workgroup);
            // measured at N = 16385: 2049 26+20 -> 23+18 us, 1025 13+11 -> 12+10, 513..129
            // 12+10 -> 7+7
            target = tuning_int("PGMG_FUSED_SMALL_BLOCKS",
                                (int)std::max((long long)tuning_int("PGMG_FUSED_SMALL_MIN", 256),
                                              pts / tuning_int("PGMG_FUSED_SMALL_PTS", 8192)));
        }
    }

    // (no cap on the band height: a cap of 512 coarse rows once turned a one-round target of
    // 504 workgroups at N = 16385 into 576, i.e. 1.125 rounds)
    const int rmin = 2, rmax = 1 << 20;
    // bands so that gx * gy does not exceed the target (a target of whole rounds of the
    // resident workgroups must not spill a few workgroups into one more round: 3096
    // workgroups for a 3072 target cost ~2 % in k_postpre)
    const int gymax = std::max(1, target / *gx);
    int r = (rows + gymax - 1) / gymax;
    r = r < rmin ? rmin : (r > rmax ? rmax : r);
    if (r > rows) r = rows;
    if (r < 1) r = 1;
    *rpb = r;
    *gy = (rows + r - 1) / r;
}

int fused_blocks(int N, int jc0, int jc1)
{
    int t, gx, gy, r;
    fused_geometry(N, jc0, jc1, &t, &gx, &gy, &r);
    return gx * gy;
}

// k_post_r2's workgroups (its 116-column tiles): the partial sums its check writes
// k_post_r2's grid target (0: fused_geometry's default, 3072 at N = 16385 = 4 rounds of the 768
// resident at 3 waves/SIMD); one function for the launch and the log sizing
static int r2_target() { return tuning_int("PGMG_R2_BLOCKS", 0); }

int post_r2_blocks(int N, int jc0, int jc1)
{
    int t, gx, gy, r;
    fused_geometry(N, jc0, jc1, &t, &gx, &gy, &r, kR2Stride, r2_target());
    return gx * gy;
}

// ---------------------------------------------------------------------------
// read/write extents of the fused passes (pgmg_internal.h, check_span)
// ---------------------------------------------------------------------------
// Every span below restates the kernel's own loop bounds: a band of coarse rows
// [jcb, jce) streams fine rows 2jcb - lead .. 2jcb - lead + ceil((2(jce - jcb) + extra) / R)
// * R - 1 (k_pre: lead 4, extra 8, R 4; k_post: 2, 4, 4; k_postpre_lds: 6, 11, 2), and wave w
// of a 120-column tiling reads columns 120w - 3 .. 120w + 124 unless it is idle
// (120w - 3 + 4 > N - 2).
static inline long long fdiv2(long long v) { return v >= 0 ? v / 2 : -((1 - v) / 2); }

struct Span {
    long long r0, r1;   // fine rows (inclusive)
    bool any;
};

static Span band_rows(int jc0, int jc1, int r, int lead, int extra, int R)
{
    Span sp{0, -1, false};
    if (jc1 <= jc0 || r <= 0) return sp;
    const int nb = (jc1 - jc0 + r - 1) / r;
    sp.r0 = 2LL * jc0 - lead;
    for (int b = std::max(0, nb - 2); b < nb; ++b) {   // the last (full or short) bands
        const int jcb = jc0 + b * r, jce = std::min(jcb + r, jc1);
        const long long n = ((2LL * (jce - jcb) + extra + R - 1) / R) * R;
        sp.r1 = std::max(sp.r1, 2LL * jcb - lead + n - 1);
    }
    sp.any = true;
    return sp;
}

// last column read by a non-idle wave of k_pre / k_post (120-column stride, 4-column
// margin: wave w covers 120w - 3 .. 120w + 124); -1 when every wave is idle
static long long tile_col_hi(int N, int waves, int stride = 120, int margin = 4)
{
    // wave w's tile starts at column stride*w + 1 - margin; idle once that + 4 > N - 2
    const int wmax = std::min(waves - 1, (N - 7 + margin) / stride);
    return wmax < 0 ? -1 : (long long)stride * wmax + 1 - margin + 127;
}

#define PGMG_SPAN(o, P, r0, r1, c0, c1, what)                                                  \
    do {                                                                                       \
        const int e_ = check_span((o), (P), (int)sizeof(T), (r0), (r1), (c0), (c1), (what));   \
        if (e_) return e_;                                                                     \
    } while (0)

// k_pre / k_pre_rare: x0 and f over the band rows, the PIN coarse rows, x2 and rc stores
template <class T>
static int pre_spans(const PreArgsT<T> &a, int t, int gx, int r, bool x0_read, bool f_read)
{
    const Span sp = band_rows(a.jc0, a.jc1, r, 4, 8, 4);
    const long long chi = tile_col_hi(a.N, gx * (t / 64));
    if (!sp.any || chi < 0) return PGMG_OK;
    if (x0_read) PGMG_SPAN(a.x0, a.Px != 0 ? a.Px : a.P, sp.r0, sp.r1, -3, chi, "k_pre x0");
    if (f_read) PGMG_SPAN(a.f, a.P, sp.r0, sp.r1, -3, chi, "k_pre f");
    if (a.pin_ec != nullptr)   // coarse rows i/2 .. i/2 + 2 of every 4-row iteration i
        PGMG_SPAN(a.pin_ec, a.Pc, fdiv2(sp.r0), fdiv2(sp.r1 + 1 - 4) + 2, -2,
                  fdiv2(chi - 2) + 1, "k_pre PIN coarse grid");
    const int olo = std::max(2 * a.jc0, a.row_lo), ohi = std::min(2 * a.jc1, a.row_hi);
    if (a.x2 != nullptr) PGMG_SPAN(a.x2, a.P, olo, ohi - 1, 1, a.N - 1, "k_pre x2");
    const int clo = std::max(a.jc0, std::max(1, a.rc_lo));
    const int chi2 = std::min(a.jc1, std::min(a.N / 2, a.rc_hi));
    if (a.rc != nullptr) PGMG_SPAN(a.rc, a.Pc, clo, chi2 - 1, 1, a.Nc - 2, "k_pre rc");
    return PGMG_OK;
}

// k_post / k_post_rare: phi (or f one row ahead, RECOMP), f, the coarse correction, x2
// (r2: k_post_r2's bands start 4 rows earlier and stream 6 rows more)
template <class T>
static int post_spans(const PostArgsT<T> &a, int t, int gx, int r, bool f_read, bool r2 = false)
{
    const Span sp = band_rows(a.jc0, a.jc1, r, r2 ? 6 : 2, r2 ? 10 : 4, 4);
    const int margin = r2 ? 6 : 4;   // k_post_r2: 116-column stride, 6-column margin
    const long long chi = tile_col_hi(a.N, gx * (t / 64), r2 ? kR2Stride : 120, margin);
    const long long clo = 1 - margin;
    if (!sp.any || chi < 0) return PGMG_OK;
    if (a.pre_fired != nullptr) {   // RECOMP: f rows i_begin - 1 .. last + 1, phi not read
        PGMG_SPAN(a.f, a.P, sp.r0 - 1, sp.r1 + 1, clo, chi, "k_post f (recompute)");
    } else {
        PGMG_SPAN(a.phi, a.P, sp.r0, sp.r1, clo, chi, "k_post phi");
        if (f_read) PGMG_SPAN(a.f, a.P, sp.r0, sp.r1, clo, chi, "k_post f");
    }
    PGMG_SPAN(a.ec, a.Pc, fdiv2(sp.r0), fdiv2(sp.r1 + 1 - 4) + 2, fdiv2(clo - 1), fdiv2(chi - 2) + 1,
              "k_post coarse correction");
    const int olo = std::max(2 * a.jc0, a.row_lo), ohi = std::min(2 * a.jc1, a.row_hi);
    if (a.x2 != nullptr) PGMG_SPAN(a.x2, a.Po != 0 ? a.Po : a.P, olo, ohi - 1, 1, a.N - 1, "k_post x2");
    return PGMG_OK;
}

// k_postpre_lds (and its smooth(3) form, coarse = false): each block loads its window of
// row pairs through buffer descriptors (columns L0 .. L0 + 2 nvx - 1, coarse columns
// cc0 .. cc0 + nve - 1; the descriptor range stops them at the grid's last column)
template <class T>
static int postpre_spans(const PostPreArgsT<T> &a, int t, int gx, int r, bool coarse)
{
    const int lag = a.recompute ? 2 : 0;   // the recompute form: 2 more rows each end
    const int ST = a.recompute ? kPPStrideRC : kPPStride, MG = a.recompute ? kPPMarginRC : kPPMargin;
    const Span sp = band_rows(a.jc0, a.jc1, r, 6 + lag, 11 + 2 * lag, kPPR);
    if (!sp.any) return PGMG_OK;
    const int wpb = t / 64;
    const int npairs = (ST * wpb + 2 * MG) / 2;
    const int ncc = (ST / 2) * wpb + MG + 2;
    long long c1 = -1, e0 = 0, e1 = -1;
    bool first = true;
    for (int bx = 0; bx < gx; ++bx) {
        const int L0 = ST * wpb * bx + 1 - MG;
        const int nvx = std::max(0, std::min(npairs, (a.N - 1 - L0) / 2 + 1));
        if (nvx > 0) c1 = std::max(c1, (long long)L0 + 2 * nvx - 1);
        const int cc0 = (L0 - 1) >> 1;
        const int nve = std::max(0, std::min(ncc, a.Nc - cc0));
        if (nve > 0) {
            e0 = first ? cc0 : std::min(e0, (long long)cc0);
            e1 = std::max(e1, (long long)cc0 + nve - 1);
            first = false;
        }
    }
    const long long c0 = 1 - MG;
    if (c1 < c0) return PGMG_OK;
    PGMG_SPAN(a.phi, a.P, sp.r0, sp.r1, c0, c1, "k_postpre phi");
    if (a.gfx == nullptr) PGMG_SPAN(a.f, a.P, sp.r0, sp.r1, c0, c1, "k_postpre f");
    if (coarse && e1 >= e0)   // coarse rows m0 .. m0 + ng of a band (m0 = jcb - 3; RC jcb - 5)
        PGMG_SPAN(a.ec, a.Pc, a.jc0 - 3 - lag, fdiv2(sp.r1 + 1), e0, e1, "k_postpre coarse correction");
    const int olo = std::max(2 * a.jc0, a.row_lo), ohi = std::min(2 * a.jc1, a.row_hi);
    if (a.x4 != nullptr) PGMG_SPAN(a.x4, a.P, olo, ohi - 1, 1, a.N - 1, "k_postpre x4");
    if (a.x2 != nullptr) PGMG_SPAN(a.x2, a.P, olo, ohi - 1, 1, a.N - 1, "k_postpre x2 (carry pass)");
    if (coarse && a.rc != nullptr) {
        const int clo = std::max(a.jc0, std::max(1, a.rc_lo));
        const int chi = std::min(a.jc1, std::min(a.N / 2, a.rc_hi));
        PGMG_SPAN(a.rc, a.Pc, clo, chi - 1, 1, a.Nc - 2, "k_postpre rc");
    }
    return PGMG_OK;
}

// The finest level gets its own kernel symbols (FINE) so rocprofv3 statistics
// isolate the roofline kernels.
template <class T>
int launch_pre(const PreArgsT<T> &a0, bool x0_zero, bool fine, hipStream_t s)
{
    int t, gx, gy, r;
    fused_geometry(a0.N, a0.jc0, a0.jc1, &t, &gx, &gy, &r);
    if (const int e = pre_spans(a0, t, gx, r, !x0_zero && a0.pin_ec == nullptr, a0.gfx == nullptr))
        return e;
    PreArgsT<T> a = a0;
    a.rows_per_block = r;
    // non-temporal stores on the finest level only (its x2 is read again a level-pass later;
    // coarse outputs are re-read while still in the caches): fine k_pre 0.99 -> 0.97 ms
    a.nt = (fine ? 1 : 0) | (tuning_int("PGMG_FUSED_XCD", 1) ? 16 : 0);
    const dim3 g(gx, gy), b(t);
    // two row pairs per iteration (r01 sweeps: on x0 = 0 levels 2 as fast as 3 at 8193 and
    // faster below, 4 slower; one pair slower everywhere)
    if (a.pin_ec != nullptr) {   // F-cycle: x0 = prolongation of the coarse grid
        if (fine && a.gfx != nullptr) launchk(k_pre<T, false, true, 2, true, true>, g, b, s, a);
        else if (fine) launchk(k_pre<T, false, true, 2, false, true>, g, b, s, a);
        else if (a.gfx != nullptr) launchk(k_pre<T, false, false, 2, true, true>, g, b, s, a);
        else launchk(k_pre<T, false, false, 2, false, true>, g, b, s, a);
    } else if (x0_zero) {
        launchk(k_pre<T, true, false, 2>, g, b, s, a);
    } else if (fine && a.gfx != nullptr) {
        launchk(k_pre<T, false, true, 2, true>, g, b, s, a);
    } else if (fine) {
        launchk(k_pre<T, false, true, 2>, g, b, s, a);
    } else if (a.gfx != nullptr) {
        launchk(k_pre<T, false, false, 2, true>, g, b, s, a);
    } else {
        launchk(k_pre<T, false, false, 2>, g, b, s, a);
    }
    // x0 (unless zero or the F-cycle's prolongation, which reads the coarse grid instead), f
    // (unless regenerated) in; x2 (unless recomputed later), rc out
    const double n = row_pts(std::max(2 * a.jc0, a.row_lo), std::min(2 * a.jc1, a.row_hi), a.N);
    const double nc = row_pts(a.rc_lo, a.rc_hi, a.Nc);
    const bool rx0 = !x0_zero && a.pin_ec == nullptr;
    g_last_launch.bytes = (8.0 * n * ((rx0 ? 1 : 0) + (a.gfx == nullptr ? 1 : 0) + (a.x2 != nullptr ? 1 : 0)) +
                           8.0 * nc * (a.pin_ec != nullptr ? 2 : 1)) * sizeof(T) / 8.0;
    return PGMG_OK;
}

// phi (unless recomputed from f), f (unless regenerated), ec in; x2 out
template <class T>
static double post_bytes(const PostArgsT<T> &a)
{
    const double n = row_pts(std::max(2 * a.jc0, a.row_lo), std::min(2 * a.jc1, a.row_hi), a.N);
    const double nc = row_pts(std::max(a.jc0, 1), std::min(a.jc1 + 1, a.Nc - 1), a.Nc);
    return (8.0 * n * ((a.pre_fired == nullptr ? 1 : 0) + (a.gfx == nullptr ? 1 : 0) + 1) + 8.0 * nc) *
           sizeof(T) / 8.0;
}

template <class T>
int launch_post(const PostArgsT<T> &a0, bool fine, hipStream_t s)
{
    int t, gx, gy, r;
    fused_geometry(a0.N, a0.jc0, a0.jc1, &t, &gx, &gy, &r);
    if (const int e = post_spans(a0, t, gx, r, a0.gfx == nullptr)) return e;
    PostArgsT<T> a = a0;
    a.rows_per_block = r;
    // fine k_post: 1.01 -> 0.93 ms with non-temporal stores
    a.nt = (fine ? 4 : 0) | (tuning_int("PGMG_FUSED_XCD", 1) ? 16 : 0);
    const dim3 g(gx, gy), b(t);
    const bool rec = a.pre_fired != nullptr;
    if (fine && a.gfx != nullptr) launchk(k_post<T, true, 2, false, true>, g, b, s, a);
    else if (fine) launchk(k_post<T, true, 2, false>, g, b, s, a);
    else if (rec) launchk(k_post<T, false, 2, true>, g, b, s, a);
    else if (a.gfx != nullptr) launchk(k_post<T, false, 2, false, true>, g, b, s, a);
    else launchk(k_post<T, false, 2, false>, g, b, s, a);
    g_last_launch.bytes = post_bytes(a);
    return PGMG_OK;
}

template <class T>
int launch_post_r2(const PostArgsT<T> &a0, hipStream_t s)
{
    int t, gx, gy, r;
    fused_geometry(a0.N, a0.jc0, a0.jc1, &t, &gx, &gy, &r, kR2Stride, r2_target());
    if (a0.r2out == nullptr || a0.pre_fired != nullptr || a0.Po != 0 || a0.Nr2 < 3 ||
        4 * (a0.Nr2 - 1) != a0.N - 1)
        return PGMG_ERR_ARG;
    if (const int e = post_spans(a0, t, gx, r, a0.gfx == nullptr, true)) return e;
    PGMG_SPAN(a0.r2out, a0.Pr2, 1, a0.Nr2 - 2, 1, a0.Nr2 - 2, "k_post_r2 level-2 restriction");
    PostArgsT<T> a = a0;
    a.rows_per_block = r;
    a.nt = 4 | (tuning_int("PGMG_R2_EALL", 0) ? 8 : 0) | (tuning_int("PGMG_F_XCD", 1) ? 16 : 0);
    const dim3 g(gx, gy), b(t);
    if (a.gfx != nullptr) launchk(k_post_r2<T, true>, g, b, s, a);
    else launchk(k_post_r2<T, false>, g, b, s, a);
    // k_post's, plus the level-2 restriction written
    g_last_launch.bytes = post_bytes(a) + 8.0 * row_pts(1, a.Nr2 - 1, a.Nr2) * sizeof(T) / 8.0;
    return PGMG_OK;
}

// k_postpre's grid target: 3072 workgroups = 6 full rounds of the 512 that are resident
// at once (2 per CU at its ~200 VGPRs); measured r01 against 2048 .. 8192
// (PGMG_PP_BLOCKS): 2048 1.30 ms, 3072 1.18 ms, 4096 1.25 ms, 8192 1.28 ms at N = 16385.
// Workgroups of k_postpre: whole rounds of the 512 resident (2 per CU at 184 VGPRs), about
// one round per ~2700 fine rows: 3072 on the full 16385 grid (r01: 2048 1.30 ms, 3072 1.18,
// 4096 1.25), 512 on strips of 2048 / 4096 rows (scripts/strip_probe.py, per-rank time at
// 8 ranks 0.43 -> 0.39 ms; 768 / 1024, i.e. 1.5 / 2 rounds of short bands, lose)
// (r02: bands of ~190 fine rows are the invariant — on the 32769 grid 12 rounds, 6144
// workgroups, beat 6: 6.79 -> 6.70 ms per V-cycle; 9216 / 12288 the same as 6144)
static int pp_target(int jc0, int jc1)
{
    const int rounds = std::max(1, std::min(12, 6 * (2 * (jc1 - jc0) + 64) / 16384));
    return tuning_int("PGMG_PP_BLOCKS", (2048 / kPPWaves) * rounds);   // 512 resident at 4 waves
}

int postpre_blocks(int N, int jc0, int jc1, bool rc)
{
    int t, gx, gy, r;
    fused_geometry(N, jc0, jc1, &t, &gx, &gy, &r, rc ? kPPStrideRC : kPPStride, pp_target(jc0, jc1),
                   kPPWaves);
    return gx * gy;
}

// The cross-cycle finest-level pass.  OPT 2: non-temporal x4 stores (x4 is read again
// only by the next cycle's pass; r01: 1.18 vs 1.20 ms; non-temporal rc stores no gain).
// Forms (one GPU unless noted): the plain pass; R2 (row strips: the third sum); the carry pass
// (x2 stored instead of x4, OPT 128); the recompute form (OPT 256), alone or as a carry pass
// too (a one-cycle call that took the carry and makes the next); FAST (fp64) of each.
// Every launch path below launches: there is no configuration that returns without the pass.
template <class T, bool GENF, int OPT>
static void launch_pp_form(const PostPreArgsT<T> &a, dim3 g, dim3 b, hipStream_t s)
{
    launchk(k_postpre_lds<T, false, GENF, OPT>, g, b, s, a);
}
template <class T, int OPT>
static void launch_pp_form(const PostPreArgsT<T> &a, bool genf, dim3 g, dim3 b, hipStream_t s)
{
    if (genf) launch_pp_form<T, true, OPT>(a, g, b, s);
    else launch_pp_form<T, false, OPT>(a, g, b, s);
}

template <class T>
int launch_postpre(const PostPreArgsT<T> &a0, hipStream_t s)
{
    const bool rc = a0.recompute != 0, carry = a0.x2 != nullptr;
    int t, gx, gy, r;
    fused_geometry(a0.N, a0.jc0, a0.jc1, &t, &gx, &gy, &r, rc ? kPPStrideRC : kPPStride,
                   pp_target(a0.jc0, a0.jc1), kPPWaves);
    if ((rc || carry) && a0.partials3 != nullptr) return PGMG_ERR_ARG;   // one GPU only
    if (carry == (a0.x4 != nullptr)) return PGMG_ERR_ARG;                // x2 replaces x4
    if (const int e = postpre_spans(a0, t, gx, r, true)) return e;
    PostPreArgsT<T> a = a0;
    a.rows_per_block = r;
    a.xcd = tuning_int("PGMG_PP_XCD", 1);
    const dim3 g(gx, gy), b(t);
    const bool genf = a.gfx != nullptr;
    const bool fast = a.fast && sizeof(T) == 8;   // FAST mode: fp64
    if (a.partials3 != nullptr) {
        if (genf) launchk(k_postpre_lds<T, true, true, 2>, g, b, s, a);
        else launchk(k_postpre_lds<T, true, false, 2>, g, b, s, a);
    } else if constexpr (sizeof(T) == 8) {
        switch ((fast ? 16 : 0) | (carry ? 128 : 0) | (rc ? 256 : 0)) {
        case 0: launch_pp_form<T, 2>(a, genf, g, b, s); break;
        case 16: launch_pp_form<T, 2 | 16>(a, genf, g, b, s); break;
        case 128: launch_pp_form<T, 2 | 128>(a, genf, g, b, s); break;
        case 144: launch_pp_form<T, 2 | 16 | 128>(a, genf, g, b, s); break;
        case 256: launch_pp_form<T, 2 | 256>(a, genf, g, b, s); break;
        case 272: launch_pp_form<T, 2 | 16 | 256>(a, genf, g, b, s); break;
        case 384: launch_pp_form<T, 2 | 128 | 256>(a, genf, g, b, s); break;
        default: launch_pp_form<T, 2 | 16 | 128 | 256>(a, genf, g, b, s); break;
        }
    } else {
        switch ((carry ? 128 : 0) | (rc ? 256 : 0)) {
        case 0: launch_pp_form<T, 2>(a, genf, g, b, s); break;
        case 128: launch_pp_form<T, 2 | 128>(a, genf, g, b, s); break;
        case 256: launch_pp_form<T, 2 | 256>(a, genf, g, b, s); break;
        default: launch_pp_form<T, 2 | 128 | 256>(a, genf, g, b, s); break;
        }
    }
    // phi (x2 of the previous call in the recompute form), f (unless regenerated), ec in; x4
    // (x2 in the carry pass), rc out: the same bytes in every form
    const double n = row_pts(std::max(2 * a.jc0, a.row_lo), std::min(2 * a.jc1, a.row_hi), a.N);
    const double nc = row_pts(a.rc_lo, a.rc_hi, a.Nc);
    g_last_launch.bytes = (8.0 * n * (2 + (genf ? 0 : 1)) + 16.0 * nc) * sizeof(T) / 8.0;
    return PGMG_OK;
}

// ---------------------------------------------------------------------------
// Fused smooth(3) (JacobiSmoother::smooth with num_iter = 3, Smoother.hpp:38-116): four
// sweeps x0 -> x4 in ONE pass of k_postpre_lds (OPT 64: no correction, no restriction)
// with the checks ||r(x1)||, ||r(x2)||, ||r(x3)|| < eps summed speculatively; the decision
// kernel finds the first check that fires and the rare-path kernel recomputes x_k from
// the untouched x0.  Used by the F-cycle climb on the levels below the finest.
// ---------------------------------------------------------------------------
template <class T>
int launch_smooth4(const PostPreArgsT<T> &a0, hipStream_t s)
{
    int t, gx, gy, r;
    fused_geometry(a0.N, a0.jc0, a0.jc1, &t, &gx, &gy, &r, kPPStride, pp_target(a0.jc0, a0.jc1),
                   kPPWaves);
    if (const int e = postpre_spans(a0, t, gx, r, false)) return e;
    PostPreArgsT<T> a = a0;
    a.rows_per_block = r;
    a.xcd = tuning_int("PGMG_F_XCD", 1);
    if (a.gfx != nullptr) k_postpre_lds<T, true, true, 64><<<dim3(gx, gy), dim3(t), 0, s>>>(a);
    else k_postpre_lds<T, true, false, 64><<<dim3(gx, gy), dim3(t), 0, s>>>(a);
    return PGMG_OK;
}

__device__ __forceinline__ double block_sum_strided(const double *p, int n, double *red)
{
    double v = 0.0;
    for (int k = threadIdx.x; k < n; k += blockDim.x) v += p[k];
    return fused_block_sum(v, red);
}

// flags[0] = first k in 1..3 whose check ||r(x_k)|| < eps fires, 0 if none; stats
// [sweeps, exits].  global3 (row strips): all-rank sums {r(x1), r(x3), r(x2)}.
__global__ __launch_bounds__(256) void k_smooth4_decide(const double *p1, const double *p2,
                                                        const double *p3, int np,
                                                        const double *global3, double eps,
                                                        unsigned *flags,
                                                        unsigned long long *stats)
{
    __shared__ double red[4];
    double s1 = block_sum_strided(p1, np, red);
    __syncthreads();
    double s3 = block_sum_strided(p3, np, red);
    __syncthreads();
    double s2 = block_sum_strided(p2, np, red);
    if (threadIdx.x == 0) {
        if (global3 != nullptr) {
            s1 = global3[0];
            s2 = global3[1];
            s3 = global3[2];
        }
        const int k = sqrt(s1) < eps ? 1 : (sqrt(s3) < eps ? 2 : (sqrt(s2) < eps ? 3 : 0));
        flags[0] = (unsigned)k;
        if (stats != nullptr) {
            atomicAdd(&stats[0], (unsigned long long)(k ? k : 4));
            if (k) atomicAdd(&stats[1], 1ull);
        }
    }
}

// x_K = J^K(x0) at one point (boundary points pass through)
template <int K, class T>
__device__ T fxs(const T *x0, const T *f, long long P, int N, T hh, int j, int i)
{
    if constexpr (K == 0) {
        return x0[(long long)j * P + i];
    } else {
        if (j <= 0 || i <= 0 || j >= N - 1 || i >= N - 1) return x0[(long long)j * P + i];
        return T(0.25) * ((hh * f[(long long)j * P + i]) + fxs<K - 1>(x0, f, P, N, hh, j, i - 1) +
                          fxs<K - 1>(x0, f, P, N, hh, j, i + 1) +
                          fxs<K - 1>(x0, f, P, N, hh, j - 1, i) +
                          fxs<K - 1>(x0, f, P, N, hh, j + 1, i));
    }
}

template <class T>
__global__ __launch_bounds__(256) void k_smooth4_fix(const unsigned *flags, const T *x0, const T *f,
                                                     T *out, long long P, int N, T hh, int row_lo,
                                                     int row_hi)
{
    const unsigned k = flags[0];
    if (k == 0) return;   // uniform: the normal case
    const long long W = N - 2;
    const long long n = (long long)(row_hi - row_lo) * W;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += stride) {
        const int j = row_lo + (int)(q / W), i = 1 + (int)(q % W);
        T v;
        if (k == 1) v = fxs<1>(x0, f, P, N, hh, j, i);
        else if (k == 2) v = fxs<2>(x0, f, P, N, hh, j, i);
        else v = fxs<3>(x0, f, P, N, hh, j, i);
        out[(long long)j * P + i] = v;
    }
}

template <class T>
void launch_smooth4_finish(const PostPreArgsT<T> &a, int np, const double *global3, double eps,
                           unsigned *flags, unsigned long long *stats, hipStream_t s)
{
    k_smooth4_decide<<<dim3(1), dim3(256), 0, s>>>(a.partials1, a.partials2, a.partials3, np,
                                                    global3, eps, flags, stats);
    const int blocks = std::max(1, std::min(1024, (int)(((long long)(a.row_hi - a.row_lo) * a.N + 255) / 256)));
    k_smooth4_fix<T><<<dim3(blocks), dim3(256), 0, s>>>(flags, a.phi, a.f, a.x4, a.P, a.N, a.hh,
                                                        a.row_lo, a.row_hi);
}

void launch_postpre_decide(const double *partials1, const double *partials2, unsigned long long *stats,
                           int np, const double *global, double eps, unsigned *flags, hipStream_t s)
{
    k_postpre_decide<<<dim3(1), dim3(256), 0, s>>>(partials1, partials2, np, global, eps, flags,
                                                  stats);
}

// Validation of a speculative call: one workgroup per recorded check re-reduces its
// partials exactly as fix_decide / k_postpre_decide do (256 threads, strided, then the
// block sum) and flags the checks that could fire.  The 1e-12 margin makes the flag a
// superset of "fires" whatever order the exact path sums in (an all-rank sum of row
// strips goes through launch_sum_partials + allreduce: relative differences below
// ~4e-13 for the <= 3072 non-negative terms of one rank).
__global__ __launch_bounds__(256) void k_verify_checks(const CheckRef *checks, double eps,
                                                       unsigned *out, double *norm)
{
    __shared__ double red[4];
    const CheckRef c = checks[blockIdx.x];
    double s = 0.0;
    for (long long k = threadIdx.x; k < c.np; k += blockDim.x) s += c.partials[k];
    s = fused_block_sum(s, red);
    if (threadIdx.x == 0) {
        // flag = the prediction may be wrong: "does not fire" checks that could fire, "fires"
        // checks that could not (same margin the other way); in-stream checks are logged
        // for the norms only
        const bool could_fire = sqrt(s) < eps * (1.0 + 1e-12);
        const bool must_fire = sqrt(s) < eps * (1.0 - 1e-12);
        out[blockIdx.x] = c.expect == 0 ? (could_fire ? 1u : 0u)
                                        : (c.expect == 1 ? (must_fire ? 0u : 1u) : 0u);
        norm[blockIdx.x] = sqrt(s);
    }
}

void launch_verify_checks(const CheckRef *checks, int n, double eps, unsigned *out, double *norm,
                          hipStream_t s)
{
    if (n > 0) k_verify_checks<<<dim3(n), dim3(256), 0, s>>>(checks, eps, out, norm);
}

// The validation's reply (after the all-rank MIN): any = 1 when one of the first n_any checks
// could fire on every rank, then every check's norm and verdict, each stored straight into
// the context's pinned host staging -- the call then waits for the stream once, with no copy
// operations between the kernels and the wait.
__global__ __launch_bounds__(256) void k_spec_reply(const unsigned *f, const double *norm, int n,
                                                    int n_any, unsigned *h_any, double *h_norm,
                                                    unsigned *h_flags, unsigned *h_seq, unsigned seq)
{
    __shared__ unsigned any;
    if (threadIdx.x == 0) any = 0u;
    __syncthreads();
    unsigned v = 0u;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const unsigned fk = f[k];
        if (k < n_any) v |= fk;
        h_flags[k] = fk;
        h_norm[k] = norm[k];
    }
    if (v) atomicOr(&any, 1u);
    __syncthreads();
    if (threadIdx.x == 0) *h_any = any;
    // every store above reaches the host before the sequence word (the host polls it)
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(h_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_spec_reply(const unsigned *flags, const double *norm, int n, int n_any, unsigned *h_any,
                       double *h_norm, unsigned *h_flags, unsigned *h_seq, unsigned seq, hipStream_t s)
{
    k_spec_reply<<<dim3(1), dim3(256), 0, s>>>(flags, norm, n, n_any, h_any, h_norm, h_flags, h_seq,
                                                seq);
}

__global__ __launch_bounds__(256) void k_spec_open(const unsigned long long *stats,
                                                   unsigned long long *stats_bk, unsigned *flags,
                                                   int nflags)
{
    if (threadIdx.x < 4) stats_bk[threadIdx.x] = stats[threadIdx.x];
    for (int k = threadIdx.x; k < nflags; k += blockDim.x) flags[k] = 0u;
}

void launch_spec_open(const unsigned long long *stats, unsigned long long *stats_bk, unsigned *flags,
                      int nflags, hipStream_t s)
{
    k_spec_open<<<dim3(1), dim3(256), 0, s>>>(stats, stats_bk, flags, nflags);
}

// ---------------------------------------------------------------------------
// Fix-ups (rare path): the early-exit check after the first sweep fired.
// Scalar grid-stride code recomputing the reference result from the inputs
// the fused pass left untouched.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool fix_decide(const FixArgsF &a, double *red, int *trig)
{
    if (a.cond != nullptr && *a.cond == 0u) return false;  // uniform
    if (a.force) return true;  // recompute requested by k_postpre_decide (stats done there)
    double s = 0.0;
    for (int k = threadIdx.x; k < a.np; k += blockDim.x) s += a.partials[k];
    s = fused_block_sum(s, red);
    if (threadIdx.x == 0) {
        const double tot = a.global_sum != nullptr ? *a.global_sum : s;
        *trig = (sqrt(tot) < a.eps) ? 1 : 0;
    }
    __syncthreads();
    const bool t = *trig != 0;
    if (t && blockIdx.x == 0 && threadIdx.x == 0 && a.stats != nullptr) {
        atomicAdd(&a.stats[0], (unsigned long long)-1LL);
        atomicAdd(&a.stats[1], 1ull);
    }
    return t;
}

template <class T>
struct FixCtx {
    const T *x0, *f;
    const T *ec;
    int N, Nc;
    long long P, Pc;
    T hh, ih;
    bool x0_zero;
    const unsigned *pre_fired;  // non-null: phi (x0 of fxeff) is recomputed from f
    bool pin;                   // x0 = (+0) + P ec (k_pre PIN, F-cycle)
    long long Px;               // x0's pitch (0: P; the caller's array: N)
};

template <class T>
__device__ T fxpin(const FixCtx<T> &c, int j, int i);

template <class T>
__device__ __forceinline__ T fx0(const FixCtx<T> &c, int j, int i)
{
    if (c.pin) return fxpin(c, j, i);
    return c.x0_zero ? T(0) : c.x0[(long long)j * (c.Px != 0 ? c.Px : c.P) + i];
}

template <bool POST, class T>
__device__ T fx1(const FixCtx<T> &c, int j, int i);

// pre-smoothed iterate of x0 = 0 (k_post RECOMP): x1 = J(0), phi = fired ? x1 : J(x1)
template <class T>
__device__ T fphi0(const FixCtx<T> &c, int j, int i)
{
    FixCtx<T> z = c;
    z.x0_zero = true;
    z.pre_fired = nullptr;
    if (*c.pre_fired != 0u || j <= 0 || i <= 0 || j >= c.N - 1 || i >= c.N - 1)
        return fx1<false>(z, j, i);
    return T(0.25) * ((c.hh * c.f[(long long)j * c.P + i]) + fx1<false>(z, j, i - 1) +
                   fx1<false>(z, j, i + 1) + fx1<false>(z, j - 1, i) + fx1<false>(z, j + 1, i));
}

// x_eff = phi + P ec at one fine point (MultiGrid.hpp:208-226)
template <class T>
__device__ T fxeff(const FixCtx<T> &c, int j, int i)
{
    T v = c.pre_fired != nullptr ? fphi0(c, j, i) : c.x0[(long long)j * c.P + i];
    if (j < 2 || i < 2 || j > c.N - 2 || i > c.N - 2) return v;
    const int jc = j >> 1, ic = i >> 1;
    const T *C0 = c.ec + (long long)jc * c.Pc;
    T w;
    if ((j & 1) == 0) {
        w = ((i & 1) == 0) ? C0[ic] : T(0.5) * (C0[ic] + C0[ic + 1]);
    } else {
        const T *C1 = C0 + c.Pc;
        w = ((i & 1) == 0) ? T(0.5) * (C0[ic] + C1[ic]) : T(0.25) * (C0[ic] + C0[ic + 1] + C1[ic] + C1[ic + 1]);
    }
    return v + w;
}

// x0 of a PIN pre-smooth: the prolongation of ec into a zeroed grid (frame 0)
template <class T>
__device__ T fxpin(const FixCtx<T> &c, int j, int i)
{
    const T v = T(0);
    if (j < 2 || i < 2 || j > c.N - 2 || i > c.N - 2) return v;
    const int jc = j >> 1, ic = i >> 1;
    const T *C0 = c.ec + (long long)jc * c.Pc;
    T w;
    if ((j & 1) == 0) {
        if ((i & 1) == 0) return v + C0[ic];
        w = T(0.5) * (C0[ic] + C0[ic + 1]);
    } else {
        const T *C1 = C0 + c.Pc;
        w = ((i & 1) == 0) ? T(0.5) * (C0[ic] + C1[ic]) : T(0.25) * (C0[ic] + C0[ic + 1] + C1[ic] + C1[ic + 1]);
    }
    return v + w;
}

template <bool POST, class T>
__device__ T fin(const FixCtx<T> &c, int j, int i)
{
    return POST ? fxeff(c, j, i) : fx0(c, j, i);
}

template <bool POST, class T>
__device__ T fx1(const FixCtx<T> &c, int j, int i)
{
    if (j <= 0 || i <= 0 || j >= c.N - 1 || i >= c.N - 1) return fin<POST>(c, j, i);
    return T(0.25) * ((c.hh * c.f[(long long)j * c.P + i]) + fin<POST>(c, j, i - 1) +
                   fin<POST>(c, j, i + 1) + fin<POST>(c, j - 1, i) + fin<POST>(c, j + 1, i));
}

// two post-smooth sweeps from x_eff (row-strip rare path: x2 on rows past the strip)
template <class T>
__device__ T fx2post(const FixCtx<T> &c, int j, int i)
{
    if (j <= 0 || i <= 0 || j >= c.N - 1 || i >= c.N - 1) return fxeff(c, j, i);
    return T(0.25) * ((c.hh * c.f[(long long)j * c.P + i]) + fx1<true>(c, j, i - 1) +
                      fx1<true>(c, j, i + 1) + fx1<true>(c, j - 1, i) + fx1<true>(c, j + 1, i));
}

template <class T>
__device__ T fr1(const FixCtx<T> &c, int j, int i)
{
    return c.f[(long long)j * c.P + i] -
           c.ih * (T(4) * fx1<false>(c, j, i) - fx1<false>(c, j, i - 1) - fx1<false>(c, j, i + 1) -
                   fx1<false>(c, j - 1, i) - fx1<false>(c, j + 1, i));
}

template <class T>
__global__ __launch_bounds__(256) void k_pre_fixup(FixArgsF a, PreArgsT<T> p, int x0_zero)
{
    __shared__ double red[4];
    __shared__ int trig;
    const bool t = fix_decide(a, red, &trig);
    if (p.fired != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *p.fired = t ? 1u : 0u;
    if (!t) return;
    FixCtx<T> c{p.x0, p.f, p.pin_ec, p.N, p.Nc, p.P, p.Pc, p.hh, p.ih, x0_zero != 0, nullptr,
                p.pin_ec != nullptr, p.Px};
    const long long W = p.N - 2;
    const long long nrows = p.x2 != nullptr ? (long long)(p.row_hi - p.row_lo) : 0;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < nrows * W; k += stride) {
        const int j = p.row_lo + (int)(k / W), i = 1 + (int)(k % W);
        p.x2[(long long)j * p.P + i] = fx1<false>(c, j, i);
    }
    const int clo = max(1, p.rc_lo), chi = min(p.Nc - 1, p.rc_hi);
    const long long Wc = p.Nc - 2;
    const long long ncr = chi > clo ? (long long)(chi - clo) : 0;
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < ncr * Wc; k += stride) {
        const int jc = clo + (int)(k / Wc), ic = 1 + (int)(k % Wc);
        const int j = 2 * jc, i = 2 * ic;
        p.rc[(long long)jc * p.Pc + ic] =
            T(0.25) * fr1(c, j, i) + T(0.125) * (fr1(c, j, i + 1) + fr1(c, j, i - 1) + fr1(c, j + 1, i) + fr1(c, j - 1, i)) +
            T(0.0625) * (fr1(c, j - 1, i - 1) + fr1(c, j - 1, i + 1) + fr1(c, j + 1, i - 1) + fr1(c, j + 1, i + 1));
    }
}

template <class T>
__global__ __launch_bounds__(256) void k_post_fixup(FixArgsF a, PostArgsT<T> p)
{
    __shared__ double red[4];
    __shared__ int trig;
    if (!fix_decide(a, red, &trig)) return;
    FixCtx<T> c{p.phi, p.f, p.ec, p.N, p.Nc, p.P, p.Pc, p.hh, p.ih, false, p.pre_fired};
    const long long W = p.N - 2;
    const long long nrows = (long long)(p.row_hi - p.row_lo);
    const long long stride = (long long)gridDim.x * blockDim.x;
    const long long Po = p.Po != 0 ? p.Po : p.P;
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < nrows * W; k += stride) {
        const int j = p.row_lo + (int)(k / W), i = 1 + (int)(k % W);
        p.x2[(long long)j * Po + i] = p.fix_sweeps == 2 ? fx2post(c, j, i) : fx1<true>(c, j, i);
    }
}

// Fix-up grid: every block re-reduces the partials (the decision) and the grid-stride
// recompute only runs when a check fired, so small levels get few blocks (a 256-block
// launch costs ~2 us more than a 1-block one on a latency-bound level); 256 blocks from
// 2^20 points up (a fired recompute on the finest levels then still has the whole chip).
static int fixup_blocks(int N, int row_lo, int row_hi)
{
    // the rare-path recompute is scalar pointwise recursion (tens of loads per point): one
    // thread per point, up to 8192 blocks (was one per 16, at most 256 blocks: a fired
    // coarse-level fix-up cost ~40 us; 200 V-cycles at N = 4097, where the levels above
    // the tail converge and fire every cycle: 1083 -> 2435 V-cycles/s; 100 at 16385:
    // 439 -> 523; scripts/long_run.sh)
    const long long pts = (long long)(row_hi > row_lo ? row_hi - row_lo : 0) * N;
    const long long shift = 8, cap = 8192;
    long long b = pts >> shift;
    return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

// rare paths of the in-stream checks as fused one-sweep passes (decision inside; a launch
// that finds the check did not fire returns at once).  f is streamed (the stored f is
// valid whenever a pass regenerates it in-kernel).
template <class T>
int launch_pre_rare(const FixArgsF &f, const PreArgsT<T> &a0, bool x0_zero, hipStream_t s)
{
    int t, gx, gy, r;
    fused_geometry(a0.N, a0.jc0, a0.jc1, &t, &gx, &gy, &r);
    if (const int e = pre_spans(a0, t, gx, r, !x0_zero && a0.pin_ec == nullptr, true)) return e;
    PreArgsT<T> a = a0;
    a.rows_per_block = r;
    a.gfx = a.gsy = nullptr;
    a.nt = 0;
    const dim3 g(gx, gy), b(t);
    if (x0_zero) k_pre_rare<T, true, 2, false><<<g, b, 0, s>>>(a, f);
    else if (a.pin_ec != nullptr) k_pre_rare<T, false, 2, true><<<g, b, 0, s>>>(a, f);
    else k_pre_rare<T, false, 2, false><<<g, b, 0, s>>>(a, f);
    return PGMG_OK;
}

template <class T>
int launch_post_rare(const FixArgsF &f, const PostArgsT<T> &a0, hipStream_t s)
{
    int t, gx, gy, r;
    fused_geometry(a0.N, a0.jc0, a0.jc1, &t, &gx, &gy, &r);
    if (const int e = post_spans(a0, t, gx, r, true)) return e;
    PostArgsT<T> a = a0;
    a.rows_per_block = r;
    a.gfx = a.gsy = nullptr;
    a.nt = 0;
    const dim3 g(gx, gy), b(t);
    if (a.pre_fired != nullptr) k_post_rare<T, 2, true><<<g, b, 0, s>>>(a, f);
    else k_post_rare<T, 2, false><<<g, b, 0, s>>>(a, f);
    return PGMG_OK;
}

// the predicted-to-fire passes of a coarse level (entered with x0 = 0 and RECOMP, or from the
// previous gamma visit's iterate): the full passes' geometry and spans, f from memory
template <class T>
int launch_pre1(const PreArgsT<T> &a0, bool x0_zero, hipStream_t s)
{
    int t, gx, gy, r;
    fused_geometry(a0.N, a0.jc0, a0.jc1, &t, &gx, &gy, &r);
    if (const int e = pre_spans(a0, t, gx, r, !x0_zero, true)) return e;
    PreArgsT<T> a = a0;
    a.rows_per_block = r;
    a.gfx = a.gsy = nullptr;
    a.nt = 0;
    if (x0_zero) k_pre1<T, true, 2><<<dim3(gx, gy), dim3(t), 0, s>>>(a);
    else k_pre1<T, false, 2><<<dim3(gx, gy), dim3(t), 0, s>>>(a);
    return PGMG_OK;
}

template <class T>
int launch_post1(const PostArgsT<T> &a0, hipStream_t s)
{
    int t, gx, gy, r;
    fused_geometry(a0.N, a0.jc0, a0.jc1, &t, &gx, &gy, &r);
    if (const int e = post_spans(a0, t, gx, r, true)) return e;
    PostArgsT<T> a = a0;
    a.rows_per_block = r;
    a.gfx = a.gsy = nullptr;
    a.nt = 0;
    if (a.pre_fired != nullptr) k_post1<T, 2, true><<<dim3(gx, gy), dim3(t), 0, s>>>(a);
    else k_post1<T, 2, false><<<dim3(gx, gy), dim3(t), 0, s>>>(a);
    return PGMG_OK;
}

template <class T>
void launch_pre_fixup(const FixArgsF &a, const PreArgsT<T> &p, bool x0_zero, hipStream_t s)
{
    k_pre_fixup<T><<<dim3(fixup_blocks(p.N, p.row_lo, p.row_hi)), dim3(256), 0, s>>>(
        a, p, x0_zero ? 1 : 0);
}

template <class T>
void launch_post_fixup(const FixArgsF &a, const PostArgsT<T> &p, hipStream_t s)
{
    k_post_fixup<T><<<dim3(fixup_blocks(p.N, p.row_lo, p.row_hi)), dim3(256), 0, s>>>(a, p);
}

#define PGMG_INSTANTIATE(T)                                                                       \
    template int launch_pre<T>(const PreArgsT<T> &, bool, bool, hipStream_t);                   \
    template int launch_pre1<T>(const PreArgsT<T> &, bool, hipStream_t);                            \
    template int launch_post1<T>(const PostArgsT<T> &, hipStream_t);                            \
    template int launch_post<T>(const PostArgsT<T> &, bool, hipStream_t);                       \
    template int launch_post_r2<T>(const PostArgsT<T> &, hipStream_t);                          \
    template int launch_postpre<T>(const PostPreArgsT<T> &, hipStream_t);                       \
    template int launch_smooth4<T>(const PostPreArgsT<T> &, hipStream_t);                        \
    template void launch_smooth4_finish<T>(const PostPreArgsT<T> &, int, const double *, double, \
                                           unsigned *, unsigned long long *, hipStream_t);       \
    template void launch_pre_fixup<T>(const FixArgsF &, const PreArgsT<T> &, bool, hipStream_t);  \
    template int launch_pre_rare<T>(const FixArgsF &, const PreArgsT<T> &, bool, hipStream_t);   \
    template int launch_post_rare<T>(const FixArgsF &, const PostArgsT<T> &, hipStream_t);       \
    template void launch_post_fixup<T>(const FixArgsF &, const PostArgsT<T> &, hipStream_t);
PGMG_INSTANTIATE(double)
PGMG_INSTANTIATE(float)
#undef PGMG_INSTANTIATE

}  // namespace pgmg
