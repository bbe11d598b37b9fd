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
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "pgmg_internal.h"

namespace pgmg {

constexpr int kTailMaxLevels = 8;
constexpr int kTailWaves = kTailThreads / 64;
constexpr int kTailRed = 2 * kTailWaves + 2;  // doubles of reduction scratch at the LDS base
// The register-resident paths of the tail (r01/r02; each replaced a generic LDS loop and is
// bitwise the same): 3x3-interior smoothing on one wave (tail_smooth_small), the 9x9 + 5x5
// pair by tail_w9, the 17x17 level and below by tail_w17 on wave 0, and the block team's
// 65x65 / 33x33 smoothing with the iterate in registers (tail_smooth_rows).  The 33x33 level
// on wave 0 (16 points a lane) spills and was measured slower (r02): not built.
constexpr bool kTailSmallOff = false;
constexpr bool kTailW9 = true;
constexpr bool kTailW17 = true;
constexpr bool kTailRows = true;

template <class Real>
struct TailLevel {
    int N;
    int off;         // offset of this level's E and F grids (pitch N, no padding)
    Real hh, ih;     // h*h and 1.0/(h*h) rounded on the host
    float rN;        // 1.0f / N: row of a flat index k as int((k + 0.5f) * rN), exact for N <= 65
};

template <class Real>
struct TailArgsDev {
    TailArgsT<Real> a;
    int nl;
    int S;           // elements per pyramid
    TailLevel<Real> lv[kTailMaxLevels];
    int gamma;
    double eps2;     // the early-exit test sqrt(s) < eps as s < eps2 (norm2_threshold)
    int wave_n;      // levels with N <= wave_n run on wave 0 alone (no workgroup barriers)
    // measurement (PGMG_TAIL_PROF=1, pgmg_tail_prof): thread 0 adds shader-clock cycles
    // [0] wave-team hand-offs, [1] block smooth, [2] block res+restrict, [3] block
    // prolong, [4] whole kernel, [5] launches, [6] wave smooth, [7] wave res+restrict+prolong
    unsigned long long *prof;
};

__device__ __forceinline__ unsigned long long tail_clock() { return __builtin_amdgcn_s_memtime(); }

// sweeps and early exits, returned by value up the call chain (counters passed by reference
// ended up in scratch memory: a load + store on the dependent chain of every sweep)
struct Cnt {
    int sweeps = 0, exits = 0;
    __device__ Cnt &operator+=(const Cnt &o)
    {
        sweeps += o.sweeps;
        exits += o.exits;
        return *this;
    }
};

// Two execution teams for the same level code.  BlockTeam: the whole 1024-thread
// workgroup, stages separated by __syncthreads.  WaveTeam: wave 0 alone; LDS operations
// of one wavefront are performed in program order (AMDGPU memory model), so a stage
// boundary only has to stop the compiler from moving LDS accesses across it.  The deep,
// tiny levels of a W-cycle (3^l visits of a few hundred points) run as a WaveTeam: a
// stage there costs a few dozen cycles instead of a 16-wave barrier.
struct BlockTeam {
    static constexpr int size = kTailThreads;
    __device__ static int tid() { return threadIdx.x; }
    __device__ static void sync() { __syncthreads(); }
    // deterministic total of one double per thread (wave sums in wave order), valid in
    // every thread; one barrier, alternating scratch halves (par)
    __device__ static double sum(double v, double *red, int &par)
    {
        v = wave_sum(v);
        double *r = red + par * kTailWaves;
        if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = v;
        __syncthreads();
        double s = 0.0;
        #pragma unroll
        for (int i = 0; i < kTailWaves; ++i) s += r[i];
        par ^= 1;
        return s;
    }
};

struct WaveTeam {
    static constexpr int size = 64;
    __device__ static int tid() { return threadIdx.x & 63; }
    __device__ static void sync()
    {
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_wave_barrier();
    }
    __device__ static double sum(double v, double *, int &)
    {
        v = wave_sum(v);
        return v;
    }
};

__device__ __forceinline__ int tail_row(int k, float rN) { return (int)(((float)k + 0.5f) * rN); }

// out = J(cur) on all points (boundary copied); optionally sum r(cur)^2
template <class Team, class Real, bool NORM>
__device__ __forceinline__ double tail_jacobi(const Real *cur, Real *out, const Real *f,
                                              const TailLevel<Real> &L)
{
    double acc = 0.0;
    const int N = L.N, n = N * N;
    const Real hh = L.hh, ih = L.ih;
    for (int k = Team::tid(); k < n; k += Team::size) {
        const int j = tail_row(k, L.rN);
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

// The smoother of a level whose interior fits one wave ((N-2)^2 <= 64: N = 5, 9), run by
// the wave team: one interior point per lane, its iterate and h*h*f in registers, sweeps
// IN PLACE in LDS (a wave's LDS reads of the old neighbours precede its writes in program
// order; the compiler fence keeps them there), the check of x_k fused into sweep k+1 and,
// when it fires, the lane's register copy of x_k written back — no scratch grid, no
// boundary lanes, no copy pass.  Same expressions and operand order as tail_jacobi.
template <int PP, class Real>
__device__ __forceinline__ Cnt tail_smooth_small(Real *x, const Real *f, const TailLevel<Real> &L,
                                                 int num_iter, double eps)
{
    int sweeps = 0, exits = 0;
    // PP interior points per lane: point q of lane t is interior index t + 64 q
    const int N = L.N, m = N - 2, nin = m * m;
    const int lane = threadIdx.x & 63;
    const int mg = (65536 + m - 1) / m;                 // p / m for p < 256, m <= 15
    bool act[PP];
    int k[PP];
    Real fk[PP], hf[PP], xc[PP];
    const Real hh = L.hh, ih = L.ih;
    #pragma unroll
    for (int q = 0; q < PP; ++q) {
        const int p = lane + 64 * q;
        act[q] = p < nin;
        const int jj = (p * mg) >> 16;
        k[q] = act[q] ? (1 + jj) * N + 1 + (p - jj * m) : N + 1;
        fk[q] = f[k[q]];
        hf[q] = hh * fk[q];
        xc[q] = x[k[q]];
    }
    auto fence = [] {
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_wave_barrier();
    };
    {   // sweep 1 (no check before it)
        Real nx[PP];
        #pragma unroll
        for (int q = 0; q < PP; ++q) {
            const int kk = k[q];
            nx[q] = Real(0.25) * (hf[q] + x[kk - 1] + x[kk + 1] + x[kk - N] + x[kk + N]);
        }
        fence();
        #pragma unroll
        for (int q = 0; q < PP; ++q) {
            if (act[q]) x[k[q]] = nx[q];
            xc[q] = nx[q];
        }
        fence();
        ++sweeps;
    }
    for (int it = 2; it <= num_iter + 1; ++it) {
        Real nx[PP];
        double acc = 0.0;
        #pragma unroll
        for (int q = 0; q < PP; ++q) {
            const int kk = k[q];
            const Real l = x[kk - 1], r = x[kk + 1], u = x[kk - N], d = x[kk + N];
            const Real res = fk[q] - ih * (Real(4) * xc[q] - l - r - u - d);
            if (act[q]) acc += sq(res);
            nx[q] = Real(0.25) * (hf[q] + l + r + u + d);
        }
        fence();
        #pragma unroll
        for (int q = 0; q < PP; ++q)
            if (act[q]) x[k[q]] = nx[q];
        fence();
        const double s = wave_sum(acc);
        if (s < eps) {   // x_{it-1} is the result: the speculative sweep is undone
            #pragma unroll
            for (int q = 0; q < PP; ++q)
                if (act[q]) x[k[q]] = xc[q];
            fence();
            ++exits;
            return Cnt{sweeps, exits};
        }
        #pragma unroll
        for (int q = 0; q < PP; ++q) xc[q] = nx[q];
        ++sweeps;
    }
    return Cnt{sweeps, exits};
}

// Block-team smoother of an NN x NN level (NN = 33, 65) with the iterate in registers.
// Wave w owns the rows j0 = 1 + RPW*w .. j0 + RPW - 1 with RPW = (NN - 1) / waves, so the
// waves cover rows 1 .. NN-1 exactly and the last wave's last row is the boundary row NN-1
// (passed through): every wave holds RPW rows and no register array is indexed at run time.
// Lane l holds column l (NN = 65: column 64, a boundary column, is a per-row register of
// every lane); left/right neighbours are DPP moves across the wave.  The rows above and
// below the wave: for sweep 1 and sweep 2 (with the check of x_1) ghost rows the wave
// computes itself (x_0 rows j0-2 .. j0+RPW read from the grid, x_1 on rows j0-1 and j0+RPW);
// from sweep 3 on, the neighbouring waves' edge rows exchanged through LDS (scratch T,
// double-buffered) in the same barrier that publishes the wave partials of the check.  A
// smoother call with num_iter = 1 (2 sweeps) thus has one barrier for its check and one
// after the write-back (tail_jacobi: two passes over the grid in LDS and a block sum per
// sweep).  Expressions, operand order and the fused check are tail_smooth's.
// R != nullptr (a pre-smooth followed by the residual and restriction): also R = r(x) of the
// result on the interior, from the registers (the final iterate and its neighbour rows are
// at hand: tail_res_restrict's expression and operand order), written after the closing
// barrier -- R may be T, whose edge-row buffers are free by then; the caller syncs
template <class Real, int NN>
__device__ __forceinline__ Cnt tail_smooth_rows(Real *x, const Real *f, const TailLevel<Real> &L,
                                                int num_iter, double eps, Real *T, double *red,
                                                int &par, Real *R = nullptr)
{
    static_assert((NN - 1) % kTailWaves == 0, "waves must tile rows 1 .. NN-1");
    constexpr int RPW = (NN - 1) / kTailWaves;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int j0 = 1 + RPW * w;
    const bool act = lane < NN;                         // lane holds a column of the grid
    const bool bcol = lane == 0 || lane == NN - 1;      // boundary column: passthrough
    const Real hh = L.hh, ih = L.ih;
    const bool first = w == 0, last = w == kTailWaves - 1;
    auto ld = [&](int j) { return (act && j >= 0 && j < NN) ? x[j * NN + lane] : Real(0); };
    // NN = 65: column 64 (right boundary, constant while smoothing) of row j
    auto ldb = [&](int j) { return (NN == 65 && j >= 0 && j < NN) ? x[j * NN + 64] : Real(0); };
    Real xr[RPW], hf[RPW], fr[RPW], xb[RPW];
    bool brow[RPW];   // the grid's last row (last wave only): passed through, not checked
    #pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int j = j0 + r;
        brow[r] = j == NN - 1;
        xr[r] = ld(j);
        fr[r] = act ? f[j * NN + lane] : Real(0);
        hf[r] = hh * fr[r];
        xb[r] = ldb(j);
    }
    // rows j0-2, j0-1 above and j0+RPW, j0+RPW+1 below (rows past the grid are never used:
    // the first wave's row above is the boundary row 0, the last wave's last row is one)
    const Real gu2 = ld(j0 - 2), gu = ld(j0 - 1), gd = ld(j0 + RPW), gd2 = ld(j0 + RPW + 1);
    const Real bu = ldb(j0 - 1), bd = ldb(j0 + RPW);
    const Real fu = (act && !first) ? f[(j0 - 1) * NN + lane] : Real(0);
    const Real fd = (act && !last) ? f[(j0 + RPW) * NN + lane] : Real(0);
    // edge-row exchange buffer: [par][wave][first, last][64] (T holds 4 * kTailWaves * 64,
    // tail_lds_bytes)
    auto hbuf = [&](int pp, int ww, int side) { return T + ((pp * kTailWaves + ww) * 2 + side) * 64; };
    int hp = 0;
    auto put_edges = [&](const Real (&v)[RPW]) {
        hbuf(hp, w, 0)[lane] = v[0];
        hbuf(hp, w, 1)[lane] = v[RPW - 1];
    };
    auto get_edges = [&](Real &up, Real &dn) {
        up = first ? gu : hbuf(hp, max(w - 1, 0), 1)[lane];
        dn = last ? Real(0) : hbuf(hp, min(w + 1, kTailWaves - 1), 0)[lane];
    };
    // J of one row (boundary columns passed through)
    auto jrow = [&](Real c, Real u, Real d, Real hfv, Real rb, Real &lf, Real &rt) {
        lf = dpp_shr(c);
        rt = dpp_shl(c);
        if (NN == 65 && lane == 63) rt = rb;
        const Real o = Real(0.25) * (hfv + lf + rt + u + d);
        return (bcol || !act) ? c : o;
    };
    // one sweep out = J(in) on this wave's rows; NORM: acc = sum r(in)^2 over its interior points
    auto sweep = [&](const Real (&in)[RPW], Real (&out)[RPW], Real up, Real dn, auto norm_t) {
        constexpr bool NORM = decltype(norm_t)::value;
        double acc = 0.0;
        #pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const Real u = r == 0 ? up : in[r - 1];
            const Real d = r + 1 < RPW ? in[r + 1] : dn;
            const Real c = in[r];
            Real lf, rt;
            const Real o = jrow(c, u, d, hf[r], xb[r], lf, rt);
            out[r] = brow[r] ? c : o;
            if (NORM) {
                const Real res = fr[r] - ih * (Real(4) * c - lf - rt - u - d);
                acc += (act && !bcol && !brow[r]) ? sq(res) : 0.0;
            }
        }
        return acc;
    };
    Real nx[RPW];
    sweep(xr, nx, gu, gd, std::false_type{});
    int sweeps = 1, exits = 0;
    // x_1 on the ghost rows j0-1 and j0+RPW (the boundary row 0 stays as it is)
    Real up, dn;
    {
        Real lf, rt;
        const Real u1 = jrow(gu, gu2, xr[0], hh * fu, bu, lf, rt);
        const Real d1 = jrow(gd, xr[RPW - 1], gd2, hh * fd, bd, lf, rt);
        up = first ? gu : u1;
        dn = last ? Real(0) : d1;
    }
    for (int k = 2; k <= num_iter + 1; ++k) {
        // sweep k (x_k = J(x_{k-1})) and the check of x_{k-1}; ONE barrier publishes both
        // the wave partials of the check (BlockTeam::sum's arithmetic) and x_k's edge rows
        Real nn[RPW];
        const double acc = wave_sum(sweep(nx, nn, up, dn, std::true_type{}));
        double *rp = red + par * kTailWaves;
        if (lane == 0) rp[w] = acc;
        hp ^= 1;
        put_edges(nn);
        __syncthreads();
        double sm = 0.0;
        #pragma unroll
        for (int i = 0; i < kTailWaves; ++i) sm += rp[i];
        par ^= 1;
        if (sm < eps) {
            ++exits;
            break;
        }
        get_edges(up, dn);
        #pragma unroll
        for (int r = 0; r < RPW; ++r) nx[r] = nn[r];
        ++sweeps;
    }
    // everyone has read the grid (ghost rows) before anyone writes it: the check's barrier
    // above, or this one when no check ran
    if (num_iter < 1) __syncthreads();
    #pragma unroll
    for (int r = 0; r < RPW; ++r)
        if (act && !brow[r]) x[(j0 + r) * NN + lane] = nx[r];
    __syncthreads();
    if (R != nullptr) {   // up / dn: the final iterate's neighbour rows (x_1's ghost rows,
        #pragma unroll    // the last exchange, or the rows a firing check used)
        for (int r = 0; r < RPW; ++r) {
            const Real u = r == 0 ? up : nx[r - 1];
            const Real d = r + 1 < RPW ? nx[r + 1] : dn;
            const Real c = nx[r];
            const Real lf = dpp_shr(c);
            Real rt = dpp_shl(c);
            if (NN == 65 && lane == 63) rt = xb[r];
            const Real res = fr[r] - ih * (Real(4) * c - lf - rt - u - d);
            if (act && !bcol && !brow[r]) R[(j0 + r) * NN + lane] = res;
        }
    }
    return Cnt{sweeps, exits};
}

// JacobiSmoother::smooth(x, f, N, N, h, num_iter): num_iter+1 sweeps, break as
// soon as ||r(x_k)|| < eps, tested as sum r^2 < eps2 = norm2_threshold(eps) (no sqrt on
// the dependent chain of every sweep; the same decisions, see pgmg_internal.h).  The check of x_k is fused into sweep k+1 (which
// reads the same neighbourhood); when it fires, sweep k+1's output is dropped.
// R: see tail_smooth_rows (only the block team's register levels, tail_rows_level)
template <class Team, class Real>
__device__ __forceinline__ Cnt tail_smooth(Real *x, const Real *f, const TailLevel<Real> &L,
                                           int num_iter, double eps, Real *T, double *red, int &par,
                                           Real *R = nullptr)
{
    if constexpr (Team::size == kTailThreads && kTailRows) {
        if (L.N == 65) return tail_smooth_rows<Real, 65>(x, f, L, num_iter, eps, T, red, par, R);
        if (L.N == 33) return tail_smooth_rows<Real, 33>(x, f, L, num_iter, eps, T, red, par, R);
    }
    if constexpr (Team::size == 64) {
        const int nin = (L.N - 2) * (L.N - 2);
        if (!kTailSmallOff && nin <= 64) return tail_smooth_small<1>(x, f, L, num_iter, eps);
        // (tail_smooth_small<4> for N = 17 on the wave team measured no faster than the
        // block team there: W at 4097 5.98 vs 5.99 /s, wave_n 17 vs 9)
    }
    int sweeps = 0, exits = 0;
    Real *cur = x, *oth = T;
    tail_jacobi<Team, Real, false>(cur, oth, f, L);
    Team::sync();
    Real *tmp = cur;
    cur = oth;
    oth = tmp;
    ++sweeps;
    for (int k = 2; k <= num_iter + 1; ++k) {
        const double acc = tail_jacobi<Team, Real, true>(cur, oth, f, L);
        const double s = Team::sum(acc, red, par);   // also orders the writes of oth
        if (Team::size != kTailThreads) Team::sync();  // (the block sum has its barrier)
        if (s < eps) {
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
        for (int k = Team::tid(); k < n; k += Team::size) x[k] = cur[k];
    }
    Team::sync();
    return Cnt{sweeps, exits};
}

// interior point p of an m x m interior (lane p of the wave team): its flat index
__device__ __forceinline__ int tail_small_index(int p, int m, int N)
{
    const int mg = (65536 + m - 1) / m;
    const int jj = (p * mg) >> 16;
    return (1 + jj) * N + 1 + (p - jj * m);
}

// Bilinear prolongation of one fine point (j, i) of a tail level (MultiGrid.hpp:208-226),
// branch-free: the four parity cases are the one expression s * (((a + b) + c) + d) with the
// unused terms -0.0 (x + (-0) == x for every x, and 1 * x == x), so every case performs the
// reference's operations in its order.  The geometry is computed once per call.
struct PGeo {
    int ob, boff;   // coarse (cj, ci) offset; offset of the second term (1 or NC)
    bool cor;       // the point is corrected: j, i in [2, Nf - 2]
    bool mb, mcd;   // term b is used (i or j odd); terms c, d are used (both odd)
};
__device__ __forceinline__ PGeo pgeo(int j, int i, int Nf, int NC, bool in)
{
    PGeo g;
    const bool jo = (j & 1) != 0, io = (i & 1) != 0;
    g.cor = in && j >= 2 && i >= 2 && j <= Nf - 2 && i <= Nf - 2;
    g.ob = g.cor ? (j >> 1) * NC + (i >> 1) : 0;
    g.boff = io ? 1 : NC;
    g.mb = jo || io;
    g.mcd = jo && io;
    return g;
}
template <class Real>
__device__ __forceinline__ Real pweight(const Real *C, const PGeo &g, int NC)
{
    const Real a = C[g.ob], b = C[g.ob + g.boff], c = C[g.ob + NC], d = C[g.ob + NC + 1];
    const Real nz = -Real(0);
    const Real s = g.mcd ? Real(0.25) : (g.mb ? Real(0.5) : Real(1));
    return s * (((a + (g.mb ? b : nz)) + (g.mcd ? c : nz)) + (g.mcd ? d : nz));
}

// the levels tail_smooth smooths in registers with the block team
template <class Team>
__device__ __forceinline__ bool tail_rows_level(int N)
{
    return Team::size == kTailThreads && kTailRows && (N == 65 || N == 33);
}

// fc = R T, ec = 0 from a residual T already on the interior (MultiGrid.hpp:78-82)
template <class Team, class Real>
__device__ __forceinline__ void tail_restrict_T(const Real *T, const TailLevel<Real> &Lf, Real *fc, Real *ec,
                                                const TailLevel<Real> &Lc)
{
    const int N = Lf.N, Nc = Lc.N, nc = Nc * Nc;
    for (int q = Team::tid(); q < nc; q += Team::size) {
        const int jc = tail_row(q, Lc.rN);
        const int ic = q - jc * Nc;
        ec[q] = Real(0);  // MultiGrid.hpp:81-82 e_coarse = 0
        if (ic == 0 || jc == 0 || ic == Nc - 1 || jc == Nc - 1) continue;
        const int k = (2 * jc) * N + 2 * ic;
        fc[q] = Real(0.25) * T[k] + Real(0.125) * (T[k + 1] + T[k - 1] + T[k + N] + T[k - N]) +
                Real(0.0625) * (T[k - N - 1] + T[k - N + 1] + T[k + N - 1] + T[k + N + 1]);
    }
    Team::sync();
}

// T = r(x) on the interior (its boundary is never read); then fc = R T (MultiGrid.hpp:70-78)
template <class Team, class Real>
__device__ __forceinline__ void tail_res_restrict(const Real *x, const Real *f, const TailLevel<Real> &Lf, Real *fc,
                                  Real *ec, const TailLevel<Real> &Lc, Real *T)
{
    if constexpr (Team::size == 64) {
        // wave team, interior <= 64 points: one residual per lane (the restriction reads
        // only interior fine points, so T's boundary is never needed), then one coarse
        // point per lane
        const int N = Lf.N, m = N - 2;
        if (!kTailSmallOff && m * m <= 64) {
            const int lane = threadIdx.x & 63;
            if (lane < m * m) {
                const int k = tail_small_index(lane, m, N);
                T[k] = f[k] - Lf.ih * (Real(4) * x[k] - x[k - 1] - x[k + 1] - x[k - N] - x[k + N]);
            }
            Team::sync();
            const int Nc = Lc.N;
            if (lane < Nc * Nc) {
                const int jc = tail_row(lane, Lc.rN), ic = lane - jc * Nc;
                ec[lane] = Real(0);  // MultiGrid.hpp:81-82 e_coarse = 0
                if (ic > 0 && jc > 0 && ic < Nc - 1 && jc < Nc - 1) {
                    const int k = (2 * jc) * N + 2 * ic;
                    fc[lane] = Real(0.25) * T[k] + Real(0.125) * (T[k + 1] + T[k - 1] + T[k + N] + T[k - N]) +
                               Real(0.0625) * (T[k - N - 1] + T[k - N + 1] + T[k + N - 1] + T[k + N + 1]);
                }
            }
            Team::sync();
            return;
        }
    }
    // the residual on the interior only: the restriction reads no boundary point of T
    const int N = Lf.N, m = N - 2, mm = m * m;
    const float rm = 1.0f / (float)m;
    for (int p = Team::tid(); p < mm; p += Team::size) {
        const int jj = tail_row(p, rm);
        const int k = (1 + jj) * N + 1 + (p - jj * m);
        T[k] = f[k] - Lf.ih * (Real(4) * x[k] - x[k - 1] - x[k + 1] - x[k - N] - x[k + N]);
    }
    Team::sync();
    tail_restrict_T<Team>(T, Lf, fc, ec, Lc);
}

// x += P e (MultiGrid.hpp:208-226): fine points in [2, Nf-2]^2 only
template <class Team, class Real>
__device__ __forceinline__ void tail_prolong(Real *x, const TailLevel<Real> &Lf, const Real *e,
                             const TailLevel<Real> &Lc)
{
    const int N = Lf.N, Nc = Lc.N, n = N * N;
    // wave team, (N-3)^2 <= 64 corrected points: one per lane, no boundary tests
    const bool small = Team::size == 64 && !kTailSmallOff && (N - 3) * (N - 3) <= 64;
    const int m3 = N - 3;
    for (int k0 = Team::tid(); k0 < n; k0 += Team::size) {
        int k, j, i;
        if (small) {
            if (k0 >= m3 * m3) break;
            const int mg = (65536 + m3 - 1) / m3;
            const int jj = (k0 * mg) >> 16;
            j = 2 + jj;
            i = 2 + (k0 - jj * m3);
            k = j * N + i;
        } else {
            k = k0;
            j = tail_row(k, Lf.rN);
            i = k - j * N;
            if (i < 2 || j < 2 || i > N - 2 || j > N - 2) continue;
        }
        // (branch-free, see pweight: the four parity cases in one expression)
        x[k] = x[k] + pweight(e, pgeo(j, i, N, Nc, true), Nc);
    }
    Team::sync();
}

// DPP lane moves inside 16-lane rows for the 5x5 coarsest grid (row_shl:n = 0x100 + n,
// row_shr:n = 0x110 + n; lanes without a source read 0)
template <int CTRL> __device__ __forceinline__ double dpp_row(double v) { return dpp64<CTRL>(v); }
template <int CTRL> __device__ __forceinline__ float dpp_row(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// The coarsest solve (JacobiSmoother::smooth with coarse_iter, Smoother.hpp:38-116) of a 5x5
// level held in registers: lane q = 4 (jc - 1) + (ic - 1) owns interior point (jc, ic) for
// ic <= 3 (q & 3 < 3, q < 12: lanes 0-2, 4-6, 8-10); every other lane holds +0 -- the Dirichlet
// boundary -- so the left/right/up/down neighbours are plain DPP moves by 1 and 4 lanes inside
// DPP row 0 (a boundary neighbour is a padding lane, or a lane past the row, which bound_ctrl
// reads as +0: the same +0 the reference adds), with no boundary selects and no LDS round trip
// per sweep.  Same expressions, operand order and fused speculative check as
// tail_smooth_small; the check's sum over the row is the same row scan wave_sum does.
__device__ __forceinline__ int c5_lane(int jc, int ic) { return 4 * (jc - 1) + (ic - 1); }
__device__ __forceinline__ bool c5_act(int lane) { return lane < 12 && (lane & 3) < 3; }

template <class Real>
__device__ __forceinline__ void c5_nbrs(Real v, Real *o)
{
    o[0] = dpp_row<0x111>(v);   // row_shr:1: left (lane q-1)
    o[1] = dpp_row<0x101>(v);   // row_shl:1: right (lane q+1)
    o[2] = dpp_row<0x114>(v);   // row_shr:4: up (lane q-4; lanes 0..3: +0)
    o[3] = dpp_row<0x104>(v);   // row_shl:4: down (lane q+4)
    // all four moves with every lane active (the padding lanes' +0 is read, not assumed)
    __asm__ volatile("" : "+v"(o[0]), "+v"(o[1]), "+v"(o[2]), "+v"(o[3]));
}

template <class Real>
__device__ __forceinline__ Cnt tail_coarse5_regs(Real &x, Real f, const TailLevel<Real> L,
                                                 int num_iter, double eps2)
{
    const int lane = threadIdx.x & 63;
    const bool act = c5_act(lane);
    const Real hh = L.hh, ih = L.ih, hf = hh * f;
    Real xv = x;
    int sweeps = 1, exits = 0;
    {
        Real o[4];
        c5_nbrs(xv, o);
        const Real nx = Real(0.25) * (hf + o[0] + o[1] + o[2] + o[3]);
        xv = act ? nx : Real(0);
    }
    for (int it = 2; it <= num_iter + 1; ++it) {
        Real o[4];
        c5_nbrs(xv, o);
        const Real res = f - ih * (Real(4) * xv - o[0] - o[1] - o[2] - o[3]);
        const double r2 = sq(res);
        double acc = act ? r2 : 0.0;
        const Real nx = Real(0.25) * (hf + o[0] + o[1] + o[2] + o[3]);
        acc += dpp64<0x111>(acc);   // row_shr:1,2,4,8: lane 15 holds the total of row 0
        acc += dpp64<0x112>(acc);
        acc += dpp64<0x114>(acc);
        acc += dpp64<0x118>(acc);
        // wave-uniform: the decision of every lane
        const double s = readlane64(acc, 15);
        if (s < eps2) {   // x_{it-1} is the result: the speculative sweep is dropped
            exits = 1;
            break;
        }
        xv = act ? nx : Real(0);
        ++sweeps;
    }
    x = xv;
    return Cnt{sweeps, exits};
}

// The gamma coarsest solves of one 9x9 visit, each continuing from the previous one's result.
// The iterates x_1, x_2, .. are one Jacobi sequence whatever the call boundaries are (a call
// ends at the first check that fires, the next continues from that iterate), and in a W-cycle
// every call ends at its first check (the oracle's statistics: 1.0 sweeps per call from the
// second cycle on).  So the fast path computes x_1 .. x_gamma back to back — the sweeps are
// the only dependent chain — with their gamma checks beside them, and keeps x_gamma when all
// of them fire (gamma sweeps, gamma exits: exactly the sequential calls' work and counters);
// otherwise the calls run one by one from the untouched x_0.  GAMMA: the W-cycle's alpha = 3
// at compile time (no run-time trip count on the chain), 0 = any.
template <class Real, int GAMMA>
__device__ __forceinline__ Cnt tail_coarse5_gamma(Real &x, Real f, const TailLevel<Real> L,
                                                  int num_iter, double eps2, int gamma)
{
    const int G = GAMMA > 0 ? GAMMA : gamma;
    if (G <= 3 && num_iter >= 1) {
        const int lane = threadIdx.x & 63;
        const bool act = c5_act(lane);
        const Real hh = L.hh, ih = L.ih, hf = hh * f;
        // x_k's neighbours serve both its check r(x_k) and the next sweep J(x_k); the gamma
        // checks are summed per lane and reduced ONCE: every lane's sum bounds each of its
        // terms and the DPP reduction tree is the same for both, so (fl(a + b) is monotone in
        // a and b) the reduced total bounds every reduced check sum — a total below eps2
        // means every check fires; otherwise the exact sequential calls decide
        Real o[4];
        c5_nbrs(x, o);
        const Real x1 = act ? Real(0.25) * (hf + o[0] + o[1] + o[2] + o[3]) : Real(0);
        Real xk = x1, xl = x1;
        double acc = 0.0;
        #pragma unroll
        for (int g = 1; g <= 3; ++g) {
            if (g > G) break;
            c5_nbrs(xk, o);
            const Real res = f - ih * (Real(4) * xk - o[0] - o[1] - o[2] - o[3]);
            const double r2 = sq(res);
            acc += act ? r2 : 0.0;
            xl = xk;
            if (g < G) {
                const Real nx = Real(0.25) * (hf + o[0] + o[1] + o[2] + o[3]);
                xk = act ? nx : Real(0);
            }
        }
        acc += dpp64<0x111>(acc);
        acc += dpp64<0x112>(acc);
        acc += dpp64<0x114>(acc);
        acc += dpp64<0x118>(acc);
        if (readlane64(acc, 15) < eps2) {
            x = xl;
            return Cnt{G, G};
        }
    }
    Cnt c;
    for (int g = 0; g < G; ++g) c += tail_coarse5_regs(x, f, L, num_iter, eps2);
    return c;
}

// `reps` gamma-cycles of a 9x9 level whose coarser level is the 5x5 coarsest one, on wave 0:
// smoothing of the 9x9 level in LDS (tail_smooth_small), its residual and full-weighting
// restriction straight into the coarse lanes' registers, the gamma coarsest solves in
// registers (tail_coarse5_regs), the prolongation from one LDS copy of the correction.
// Replaces, for this (most visited) pair of levels of a W-cycle, the generic loop's
// per-stage LDS grids and index arithmetic.  MultiGrid.hpp:57-136 semantics.
template <class Real>
__device__ __forceinline__ Cnt tail_w9(const TailArgsDev<Real> &d, int l, int reps, Real *E,
                                       Real *F, Real *T)
{
    const TailArgsT<Real> &a = d.a;
    const TailLevel<Real> L9 = d.lv[l], L5 = d.lv[l + 1];   // by value: scalar registers
    Real *x9 = E + L9.off;
    const Real *f9 = F + L9.off;
    Real *e5 = E + L5.off;
    const int lane = threadIdx.x & 63;
    const int jj = lane / 7, ii = lane - 7 * jj;
    const bool in9 = lane < 49;
    const int k9 = in9 ? (1 + jj) * 9 + 1 + ii : 10;
    // coarse lane q (c5_act): (jc, ic) = (1 + q/4, 1 + q%4), fine centre (2jc, 2ic)
    const bool cact = c5_act(lane);
    const int jc = 1 + (lane >> 2), ic = 1 + (lane & 3);
    const int kc = cact ? (2 * jc) * 9 + 2 * ic : 20;
    const double eps2 = d.eps2;
    const int gamma = d.gamma;
    auto fence = [] {
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_wave_barrier();
    };
    const Real hh = L9.hh, ih = L9.ih;
    const Real fk = f9[k9], hf = hh * fk;
    Real x = x9[k9];   // this lane's point; LDS x9 always holds every lane's current value
    const PGeo pg9 = pgeo(1 + jj, 1 + ii, 9, 5, in9);
    // JacobiSmoother::smooth on the 9x9 level with the iterate in registers: sweeps in place
    // (the wave's reads of the old neighbours precede its writes), the check of x_k fused
    // into sweep k+1 and undone from the register copy when it fires (tail_smooth_small)
    // returns true when a check fired: rlast then holds r(result), the residual the
    // restriction needs (the check computed it with the result's neighbours)
    Real rlast = Real(0);
    auto smooth = [&](int num_iter, Cnt &c) __attribute__((always_inline)) -> bool {
        Real nx = Real(0.25) * (hf + x9[k9 - 1] + x9[k9 + 1] + x9[k9 - 9] + x9[k9 + 9]);
        fence();
        if (in9) x9[k9] = nx;
        fence();
        x = nx;
        ++c.sweeps;
        for (int it = 2; it <= num_iter + 1; ++it) {
            const Real l0 = x9[k9 - 1], r0 = x9[k9 + 1], u0 = x9[k9 - 9], d0 = x9[k9 + 9];
            const Real res = fk - ih * (Real(4) * x - l0 - r0 - u0 - d0);
            const double acc = in9 ? sq(res) : 0.0;
            nx = Real(0.25) * (hf + l0 + r0 + u0 + d0);
            fence();
            if (in9) x9[k9] = nx;
            fence();
            const double s = wave_sum(acc);
            if (s < eps2) {   // x_{it-1} is the result
                if (in9) x9[k9] = x;
                fence();
                ++c.exits;
                rlast = res;
                return true;
            }
            x = nx;
            ++c.sweeps;
        }
        return false;
    };
    Cnt cnt;
#ifdef PGMG_TUNING
    // stage clocks of the 9x9 visits (PGMG_TAIL_PROF): prof[8..11] smooth, res+restrict,
    // coarsest solves, prolongation; prof[15] visits
    unsigned long long st[4] = {0, 0, 0, 0}, tc = d.prof ? tail_clock() : 0;
    auto stamp = [&](int i) {
        if (d.prof) {
            const unsigned long long t1 = tail_clock();
            st[i] += t1 - tc;
            tc = t1;
        }
    };
#else
    auto stamp = [](int) {};
#endif
    // the rest of a visit once T holds the residual of the pre-smoothed iterate: restriction,
    // the gamma coarsest solves, prolongation, post-smooth
    auto rest = [&](Cnt &c) __attribute__((always_inline)) {
        // rc = R r (MultiGrid.hpp:187-205); e_coarse = 0 (:81-82)
        Real fc = Real(0), ec = Real(0);
        if (cact)
            fc = Real(0.25) * T[kc] + Real(0.125) * (T[kc + 1] + T[kc - 1] + T[kc + 9] + T[kc - 9]) +
                 Real(0.0625) * (T[kc - 9 - 1] + T[kc - 9 + 1] + T[kc + 9 - 1] + T[kc + 9 + 1]);
        stamp(1);
        c += gamma == 3 ? tail_coarse5_gamma<Real, 3>(ec, fc, L5, a.coarse_iter, eps2, gamma)
                        : tail_coarse5_gamma<Real, 0>(ec, fc, L5, a.coarse_iter, eps2, gamma);
        stamp(2);
        // the correction into LDS (5x5, boundary 0), then x += P e on [2, 7]^2 (:208-226)
        if (lane < 25) e5[lane] = Real(0);
        fence();
        if (cact) e5[jc * 5 + ic] = ec;
        fence();
        {
            const Real w = pweight(e5, pg9, 5);
            if (pg9.cor) {
                x = x + w;
                x9[k9] = x;
            }
        }
        fence();
        stamp(3);
        smooth(a.v2, c);
        stamp(0);
    };
    bool spec = gamma > 1;   // W-cycles (a V-cycle's 9x9 level needs two sweeps early on)
    for (int v = 0; v < reps; ++v) {
        // Fast path: the pre-smooth's first check fires (a 9x9 level of a W-cycle exits after
        // its first sweep in ~99 % of the visits from the second cycle on).  Its decision
        // (the norm's reduction, read-out and compare: a long dependent chain) is taken after
        // the rest of the visit instead of before it, the speculative second sweep is not
        // computed, and when it turns out not to fire the visit is rolled back to its start
        // (x in registers and LDS; the coarse grid and T are rewritten anyway) and run exactly.
        if (spec && a.v1 >= 1) {
            const Real x0 = x;
            Cnt cf;
            const Real nx = Real(0.25) * (hf + x9[k9 - 1] + x9[k9 + 1] + x9[k9 - 9] + x9[k9 + 9]);
            fence();
            if (in9) x9[k9] = nx;
            fence();
            x = nx;
            cf.sweeps = 1;
            const Real l0 = x9[k9 - 1], r0 = x9[k9 + 1], u0 = x9[k9 - 9], d0 = x9[k9 + 9];
            const Real res = fk - ih * (Real(4) * x - l0 - r0 - u0 - d0);
            const double s_pre = wave_sum(in9 ? sq(res) : 0.0);
            cf.exits = 1;
            stamp(0);
            if (in9) T[k9] = res;
            fence();
            rest(cf);
            if (s_pre < eps2) {
                cnt += cf;
                continue;
            }
            x = x0;   // roll back, and decide in order for the rest of this call
            if (in9) x9[k9] = x0;
            fence();
            spec = false;
        }
        const bool have_r = smooth(a.v1, cnt);
        stamp(0);
        // r = f - A x on the interior (DynamicGridUtils.hpp:59-69), into T: the check's
        // residual of the result when a check fired (the same expression on the same values)
        if (have_r) {
            if (in9) T[k9] = rlast;
        } else {
            if (in9) T[k9] = fk - ih * (Real(4) * x - x9[k9 - 1] - x9[k9 + 1] - x9[k9 - 9] - x9[k9 + 9]);
        }
        fence();
        rest(cnt);
    }
#ifdef PGMG_TUNING
    if (d.prof && lane == 0) {
        for (int i = 0; i < 4; ++i) atomicAdd(&d.prof[8 + i], st[i]);
        atomicAdd(&d.prof[15], (unsigned long long)reps);
    }
#endif
    return cnt;
}

// `reps` gamma-cycles of an NN x NN level (NN = 17, 33) whose coarser levels halve down to
// the 5x5 coarsest, on wave 0 (a workgroup barrier per stage costs more than the work of a
// stage at these sizes): Q = ceil((NN-2)^2 / 64) interior points per lane with their
// iterates in registers, flat indices computed once, every stage's LDS reads issued
// together; the next coarser level by tail_wq<NC> (tail_w9 for 9x9).
template <class Real, int NN>
__device__ __forceinline__ Cnt tail_wq(const TailArgsDev<Real> &d, int l, int reps, Real *E,
                                       Real *F, Real *T)
{
    constexpr int M = NN - 2, NI = M * M, Q = (NI + 63) / 64;
    constexpr int NC = (NN - 1) / 2 + 1, MC = NC - 2;
    const TailArgsT<Real> &a = d.a;
    const TailLevel<Real> L = d.lv[l], L9 = d.lv[l + 1];   // by value: scalar registers
    Real *x17 = E + L.off;
    const Real *f17 = F + L.off;
    Real *xc9 = E + L9.off;
    Real *fc9 = F + L9.off;
    const int lane = threadIdx.x & 63;
    const double eps2 = d.eps2;
    const int gamma = d.gamma;
    auto fence = [] {
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_wave_barrier();
    };
    // the right-hand side in registers only while it fits (Q <= 4); otherwise re-read from
    // LDS with the neighbours (h*h*f recomputed: the same IEEE product)
    constexpr bool REGF = Q <= 4;
    int k[Q];
    bool in[Q];
    Real x[Q], fkr[REGF ? Q : 1], hfr[REGF ? Q : 1];
    const Real hh = L.hh, ih = L.ih;
    #pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int p = lane + 64 * q, jj = p / M;
        in[q] = p < NI;
        k[q] = in[q] ? (1 + jj) * NN + 1 + (p - M * jj) : NN + 1;
        if constexpr (REGF) {
            fkr[q] = f17[k[q]];
            hfr[q] = hh * fkr[q];
        }
        x[q] = x17[k[q]];
    }
    auto fk = [&](int q) __attribute__((always_inline)) {
        if constexpr (REGF) return fkr[q];
        else return f17[k[q]];
    };
    auto hf = [&](int q) __attribute__((always_inline)) {
        if constexpr (REGF) return hfr[q];
        else return hh * f17[k[q]];
    };
    // returns true when a check fired: rl[] then holds r(result) (see tail_w9)
    Real rl[Q];
    auto smooth = [&](int num_iter, Cnt &c) __attribute__((always_inline)) -> bool {
        Real nx[Q], rs[Q];
        #pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int kk = k[q];
            nx[q] = Real(0.25) * (hf(q) + x17[kk - 1] + x17[kk + 1] + x17[kk - NN] + x17[kk + NN]);
        }
        fence();
        #pragma unroll
        for (int q = 0; q < Q; ++q) {
            if (in[q]) x17[k[q]] = nx[q];
            x[q] = nx[q];
        }
        fence();
        ++c.sweeps;
        for (int it = 2; it <= num_iter + 1; ++it) {
            double acc = 0.0;
            #pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int kk = k[q];
                const Real l0 = x17[kk - 1], r0 = x17[kk + 1], u0 = x17[kk - NN], d0 = x17[kk + NN];
                const Real res = fk(q) - ih * (Real(4) * x[q] - l0 - r0 - u0 - d0);
                if (in[q]) acc += sq(res);
                rs[q] = res;
                nx[q] = Real(0.25) * (hf(q) + l0 + r0 + u0 + d0);
            }
            fence();
            #pragma unroll
            for (int q = 0; q < Q; ++q)
                if (in[q]) x17[k[q]] = nx[q];
            fence();
            const double s = wave_sum(acc);
            if (s < eps2) {   // x_{it-1} is the result
                #pragma unroll
                for (int q = 0; q < Q; ++q) {
                    if (in[q]) x17[k[q]] = x[q];
                    rl[q] = rs[q];
                }
                fence();
                ++c.exits;
                return true;
            }
            #pragma unroll
            for (int q = 0; q < Q; ++q) x[q] = nx[q];
            ++c.sweeps;
        }
        return false;
    };
    PGeo pg[Q];
    #pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int p = lane + 64 * q, jj = p / M;
        pg[q] = pgeo(1 + jj, 1 + (p - M * jj), NN, NC, in[q]);
    }
    // coarse interior point pc = lane + 64 qc: (1 + pc/MC, 1 + pc%MC), fine centre (2j, 2i)
    constexpr int QC = (MC * MC + 63) / 64;
    int kf[QC], kc9[QC];
    bool inc[QC];
    #pragma unroll
    for (int qc = 0; qc < QC; ++qc) {
        const int pc = lane + 64 * qc, jc = 1 + pc / MC, ic = 1 + pc - MC * (pc / MC);
        inc[qc] = pc < MC * MC;
        kf[qc] = inc[qc] ? (2 * jc) * NN + 2 * ic : 2 * NN + 2;
        kc9[qc] = inc[qc] ? jc * NC + ic : NC + 1;
    }
    Cnt cnt;
#ifdef PGMG_TUNING
    // stage clocks of this level's own stages (PGMG_TAIL_PROF): prof[12..14] smooth,
    // res+restrict, prolongation (the coarser visits excluded)
    unsigned long long st[3] = {0, 0, 0}, tc = d.prof ? tail_clock() : 0;
    auto stamp = [&](int i) {
        if (d.prof) {
            const unsigned long long t1 = tail_clock();
            if (i >= 0) st[i] += t1 - tc;
            tc = t1;
        }
    };
#else
    auto stamp = [](int) {};
#endif
    // rc = R r straight into the coarser level's F and e_coarse = 0 (MultiGrid.hpp:70-82; its
    // boundary is never written, so stays 0), r in T
    auto restrict_T = [&]() __attribute__((always_inline)) {
        #pragma unroll
        for (int qc = 0; qc < QC; ++qc) {
            if (inc[qc]) {
                const int c = kf[qc];
                fc9[kc9[qc]] = Real(0.25) * T[c] + Real(0.125) * (T[c + 1] + T[c - 1] + T[c + NN] + T[c - NN]) +
                               Real(0.0625) * (T[c - NN - 1] + T[c - NN + 1] + T[c + NN - 1] + T[c + NN + 1]);
                xc9[kc9[qc]] = Real(0);
            }
        }
        fence();
    };
    bool spec = gamma > 1;   // W-cycles (see tail_w9)
    for (int v = 0; v < reps; ++v) {
        // Fast path (as tail_w9's, over a shorter span): assume the pre-smooth's first check
        // fires, restrict r(x_1) while its norm is reduced, decide before the coarser visits;
        // when it does not fire, roll x back to x_0 and smooth in order
        bool pre_done = false;
        if (spec && a.v1 >= 1) {
            Real x0[Q], nx[Q];
            #pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int kk = k[q];
                x0[q] = x[q];
                nx[q] = Real(0.25) * (hf(q) + x17[kk - 1] + x17[kk + 1] + x17[kk - NN] + x17[kk + NN]);
            }
            fence();
            #pragma unroll
            for (int q = 0; q < Q; ++q) {
                if (in[q]) x17[k[q]] = nx[q];
                x[q] = nx[q];
            }
            fence();
            double acc = 0.0;
            #pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int kk = k[q];
                const Real l0 = x17[kk - 1], r0 = x17[kk + 1], u0 = x17[kk - NN], d0 = x17[kk + NN];
                const Real res = fk(q) - ih * (Real(4) * x[q] - l0 - r0 - u0 - d0);
                if (in[q]) {
                    acc += sq(res);
                    T[kk] = res;
                }
            }
            const double s_pre = wave_sum(acc);
            fence();
            stamp(0);
            restrict_T();
            if (s_pre < eps2) {
                ++cnt.sweeps;
                ++cnt.exits;
                pre_done = true;
            } else {
                #pragma unroll
                for (int q = 0; q < Q; ++q) {
                    x[q] = x0[q];
                    if (in[q]) x17[k[q]] = x0[q];
                }
                fence();
                spec = false;
            }
        }
        if (!pre_done) {
            const bool have_r = smooth(a.v1, cnt);
            stamp(0);
            // r = f - A x on the interior into T (the check's residual of the result when a
            // check fired)
            if (have_r) {
                #pragma unroll
                for (int q = 0; q < Q; ++q)
                    if (in[q]) T[k[q]] = rl[q];
            } else {
                #pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const int kk = k[q];
                    if (in[q])
                        T[kk] = fk(q) - ih * (Real(4) * x[q] - x17[kk - 1] - x17[kk + 1] - x17[kk - NN] - x17[kk + NN]);
                }
            }
            fence();
            restrict_T();
        }
        stamp(1);
        if constexpr (NC == 9)
            cnt += tail_w9<Real>(d, l + 1, gamma, E, F, T);
        else
            cnt += tail_wq<Real, NC>(d, l + 1, gamma, E, F, T);
        stamp(-1);
        // x += P e on fine points [2, 15]^2 (MultiGrid.hpp:208-226)
        {
            Real w[Q];
            #pragma unroll
            for (int q = 0; q < Q; ++q) w[q] = pweight(xc9, pg[q], NC);
            #pragma unroll
            for (int q = 0; q < Q; ++q) {
                if (pg[q].cor) {
                    x[q] = x[q] + w[q];
                    x17[k[q]] = x[q];
                }
            }
        }
        fence();
        stamp(2);
        smooth(a.v2, cnt);
        stamp(0);
    }
#ifdef PGMG_TUNING
    if (d.prof && lane == 0 && NN == 17)
        for (int q = 0; q < 3; ++q) atomicAdd(&d.prof[12 + q], st[q]);
#endif
    return cnt;
}

// `reps` gamma-cycles (MultiGrid.hpp:57-136) whose top is tail level `top`; levels
// top .. last.  A BlockTeam hands every sub-hierarchy whose top has N <= wave_n to wave 0
// (all gamma visits of it at once) and waits at a barrier.
template <class Team, class Real>
__device__ __forceinline__ Cnt tail_gcycle(const TailArgsDev<Real> &d, int top, int reps, Real *E,
                                           Real *F, Real *T, double *red, int &par)
{
    Cnt cnt;
    constexpr bool kBlock = Team::size == kTailThreads;
    const TailArgsT<Real> &a = d.a;
    // visit counts per level, 4 bits each in one register (a dynamically indexed array
    // would live in scratch memory)
    unsigned visits = 0;
    auto vget = [&](int i) { return (int)((visits >> (4 * i)) & 15u); };
    auto vset = [&](int i, int v) { visits = (visits & ~(15u << (4 * i))) | ((unsigned)v << (4 * i)); };
    int l = top, done = 0;
    bool descending = true;
    const int last = d.nl - 1;
    for (;;) {
        if (descending) {
            const bool w17 = kTailW17 && d.lv[l].N == 17 && l + 2 == last && d.lv[l + 2].N == 5;
            if (kBlock && l != top && w17) {
                // the whole gamma-recursion of this level (and below) on wave 0
                const unsigned long long c0 = d.prof ? tail_clock() : 0;
                if (threadIdx.x < 64) cnt += tail_wq<Real, 17>(d, l, d.gamma, E, F, T);
                __syncthreads();
                if (d.prof && threadIdx.x == 0) d.prof[0] += tail_clock() - c0;
                vset(l, d.gamma - 1);
                descending = false;
                continue;
            }
            if (kBlock && l != top && d.lv[l].N <= d.wave_n) {
                // the whole gamma-recursion of level l on wave 0
                const unsigned long long c0 = d.prof ? tail_clock() : 0;
                if (threadIdx.x < 64) {
                    if (kTailW9 && d.lv[l].N == 9 && l + 1 == last && d.lv[l + 1].N == 5)
                        cnt += tail_w9<Real>(d, l, d.gamma, E, F, T);
                    else
                        cnt += tail_gcycle<WaveTeam, Real>(d, l, d.gamma, E, F, T, red, par);
                }
                __syncthreads();
                if (d.prof && threadIdx.x == 0) d.prof[0] += tail_clock() - c0;
                vset(l, d.gamma - 1);
                descending = false;
                continue;
            }
            if (!kBlock && kTailW9 && l != top && d.lv[l].N == 9 && l + 1 == last &&
                d.lv[l + 1].N == 5) {
                // one visit of the 9x9 level (inside a sub-hierarchy handed to wave 0)
                cnt += tail_w9<Real>(d, l, 1, E, F, T);
                descending = false;
                continue;
            }
            const int pi = kBlock ? 1 : 6, pr = kBlock ? 2 : 7;
            unsigned long long c0 = d.prof ? tail_clock() : 0;
            if (l == last) {
                cnt += tail_smooth<Team>(E + d.lv[l].off, F + d.lv[l].off, d.lv[l], a.coarse_iter,
                                         d.eps2, T, red, par);
                if (d.prof && threadIdx.x == 0) d.prof[pi] += tail_clock() - c0;
                descending = false;
            } else {
                // the block team's register levels leave r(x) in T (no re-read of x)
                const bool rr = tail_rows_level<Team>(d.lv[l].N);
                cnt += tail_smooth<Team>(E + d.lv[l].off, F + d.lv[l].off, d.lv[l], a.v1, d.eps2, T,
                                         red, par, rr ? T : nullptr);
                if (d.prof && threadIdx.x == 0) {
                    const unsigned long long c1 = tail_clock();
                    d.prof[pi] += c1 - c0;
                    c0 = c1;
                }
                if (rr) {
                    Team::sync();
                    tail_restrict_T<Team>(T, d.lv[l], F + d.lv[l + 1].off, E + d.lv[l + 1].off, d.lv[l + 1]);
                } else {
                    tail_res_restrict<Team>(E + d.lv[l].off, F + d.lv[l].off, d.lv[l],
                                            F + d.lv[l + 1].off, E + d.lv[l + 1].off, d.lv[l + 1], T);
                }
                if (d.prof && threadIdx.x == 0) d.prof[pr] += tail_clock() - c0;
                vset(l + 1, 0);
                ++l;
            }
        } else {
            if (l == top) {
                if (++done < reps) {
                    descending = true;   // the caller's next visit of the top level
                    continue;
                }
                break;
            }
            const int p = l - 1;
            vset(l, vget(l) + 1);
            if (vget(l) < d.gamma) {
                descending = true;   // call the cycle on level l again
            } else {
                const int pi = kBlock ? 1 : 6, pr = kBlock ? 3 : 7;
                unsigned long long c0 = d.prof ? tail_clock() : 0;
                tail_prolong<Team>(E + d.lv[p].off, d.lv[p], E + d.lv[l].off, d.lv[l]);
                if (d.prof && threadIdx.x == 0) {
                    const unsigned long long c1 = tail_clock();
                    d.prof[pr] += c1 - c0;
                    c0 = c1;
                }
                cnt += tail_smooth<Team>(E + d.lv[p].off, F + d.lv[p].off, d.lv[p], a.v2, d.eps2, T,
                                         red, par);
                if (d.prof && threadIdx.x == 0) d.prof[pi] += tail_clock() - c0;
                l = p;
            }
        }
    }
    return cnt;
}

// analytic right-hand side of tail level t from host sine tables (DynamicGridUtils.hpp:111-124)
template <class Real>
__device__ __forceinline__ void tail_rhs(const TailArgsDev<Real> &d, int t, Real *F)
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
__device__ __forceinline__ void tail_restrict_values(const Real *x, const TailLevel<Real> &Lf, Real *xc,
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
    const unsigned long long k0 = d.prof ? tail_clock() : 0;
    const TailArgsT<Real> &a = d.a;
    const int S = d.S;
    double *red = lds;                                   // kTailThreads / 64 + 1 partial sums
    Real *E = reinterpret_cast<Real *>(lds + kTailRed);
    Real *F = E + S;
    Real *T = E + 2 * S;

    for (int k = threadIdx.x; k < 2 * S; k += kTailThreads) E[k] = Real(0);
    __syncthreads();
    {
        // the top level from global memory: every load of a thread issued before the first
        // LDS store (a load-store loop waited one global-memory latency per point)
        const int N = d.lv[0].N, n = N * N;
        const long long P = a.P_top;
        const bool ldf = !a.fmg, lde = a.x0_from_global || a.fmg;
        constexpr int KU = (65 * 65 + kTailThreads - 1) / kTailThreads;   // N_top <= 65
        Real fv[KU], ev[KU];
        #pragma unroll
        for (int q = 0; q < KU; ++q) {
            // (clamped: a point past the grid re-reads the last one, never past the array)
            const int k = min((int)threadIdx.x + q * kTailThreads, n - 1);
            const int j = tail_row(k, d.lv[0].rN), i = k - j * N;
            fv[q] = ldf ? a.f_top[j * P + i] : Real(0);
            ev[q] = lde ? a.e_top[j * P + i] : Real(0);
        }
        #pragma unroll
        for (int q = 0; q < KU; ++q) {
            const int k = threadIdx.x + q * kTailThreads;
            if (k < n) {
                if (ldf) F[k] = fv[q];
                if (lde) E[k] = ev[q];
            }
        }
        for (int k = threadIdx.x + KU * kTailThreads; k < n; k += kTailThreads) {
            const int j = k / N;
            const int i = k - j * N;
            if (ldf) F[k] = a.f_top[j * P + i];
            if (lde) E[k] = a.e_top[j * P + i];
        }
    }
    __syncthreads();

    Cnt cnt;   // sweeps and exits of this launch (< 2^31)
    int par = 0;
    const int last = d.nl - 1;
    if (!a.fmg) {
        for (int v = 0; v < max(1, a.visits); ++v)
            cnt += tail_gcycle<BlockTeam>(d, 0, 1, E, F, T, red, par);
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
                tail_prolong<BlockTeam>(Et, d.lv[t], E + d.lv[t + 1].off, d.lv[t + 1]);   // :164
                cnt += tail_gcycle<BlockTeam>(d, t, 1, E, F, T, red, par);  // :167 v_cycle
            } else {
                __syncthreads();
            }
            if (t > 0 || a.fmg_smooth_top)                                   // :153 smooth(3)
                cnt += tail_smooth<BlockTeam>(Et, Ft, d.lv[t], 3, d.eps2, T, red, par);
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
        atomicAdd(&a.stats[0], (unsigned long long)cnt.sweeps);
        atomicAdd(&a.stats[1], (unsigned long long)cnt.exits);
    }
    if (d.prof && threadIdx.x == 0) {
        d.prof[4] += tail_clock() - k0;
        d.prof[5] += 1;
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
    // scratch T: one grid of the top level, and at least tail_smooth_rows' edge-row buffers
    const size_t t = std::max((size_t)N_top * N_top, (size_t)kTailRows * 4 * kTailWaves * 64);
    return kTailRed * sizeof(double) + (2 * S + t) * sizeof(Real);
}

// PGMG_TAIL_PROF=1 (measurement build libpgmg_ab.so only): the per-stage cycle counters
// of k_tail
static unsigned long long *tail_prof_buffer()
{
    static unsigned long long *buf = [] {
        unsigned long long *p = nullptr;
        if (tuning_int("PGMG_TAIL_PROF", 0) == 1 &&
            hipMalloc(&p, 16 * sizeof(unsigned long long)) == hipSuccess)
            (void)hipMemset(p, 0, 16 * sizeof(unsigned long long));
        return p;
    }();
    return buf;
}

template <class Real>
hipError_t launch_tail_gamma(const TailArgsT<Real> &a, int gamma, hipStream_t s)
{
    static bool attr_set = false;
    TailArgsDev<Real> d;
    d.a = a;
    d.gamma = gamma;
    d.eps2 = norm2_threshold(a.eps);
    int N = a.N_top;
    double h = a.h_top;
    int off = 0, nl = 0;
    for (; nl < kTailMaxLevels; ++nl) {
        d.lv[nl].N = N;
        d.lv[nl].off = off;
        d.lv[nl].hh = (Real)(h * h);
        d.lv[nl].ih = (Real)(1.0 / (h * h));
        d.lv[nl].rN = 1.0f / (float)N;
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
    {
        static const int wave_n = tuning_int("PGMG_TAIL_WAVE_N", 9);
        d.wave_n = wave_n;
    }
    d.prof = tail_prof_buffer();
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

}  // namespace pgmg

// Read (and optionally reset) the k_tail cycle counters; -1 when PGMG_TAIL_PROF is unset.
extern "C" int pgmg_tail_prof(unsigned long long *out16, int reset)
{
    unsigned long long *b = pgmg::tail_prof_buffer();
    if (!b || !out16) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpy(out16, b, 16 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return -2;
    if (reset) (void)hipMemset(b, 0, 16 * sizeof(unsigned long long));
    return 0;
}

namespace pgmg {
template hipError_t launch_tail_gamma<float>(const TailArgsT<float> &, int, hipStream_t);
template size_t tail_lds_bytes<double>(int, int);
template size_t tail_lds_bytes<float>(int, int);

}  // namespace pgmg
