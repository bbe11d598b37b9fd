// pgmg_internal.h — device data layout, kernel argument blocks and launchers.
//
// HBM layout of one grid level (see DESIGN.md "Data layout"):
//   element (row j, column i) of an N x N vertex grid lives at o[j*P + i] where
//   o = base + kOff and P = round_up(N, 16) doubles.  kOff = 15 puts column 1 of
//   every row on a 128-byte boundary, so the pair of columns (1+2t, 2+2t) that
//   lane t owns is one aligned 16-byte load and a wave's 64 pairs are exactly
//   eight 128-byte lines.
//
// All kernels keep the reference's left-to-right expression order and are built with
// -ffp-contract=off, so the fp64 instantiations are bit-identical to mg_cpu_exec.  Level
// kernels are templates on the element type T (double, or float for the fp32 variant,
// pgmg_real.h); the argument blocks below are templated alike (XxxArgsT<T>).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "pgmg_real.h"

namespace pgmg {

// Tuning knobs.  The product library (libpgmg.so) reads nothing from the environment: every
// launch geometry and variant is fixed at build time.  The measurement build
// (libpgmg_ab.so, `make ab`, -DPGMG_TUNING) lets A/B scripts override the geometry knobs
// named at the call sites (block counts, band heights, ...), none of which changes a
// result bit.
#ifdef PGMG_TUNING
int tuning_int(const char *name, int dflt);
#else
inline int tuning_int(const char *, int dflt) { return dflt; }
#endif

// The last launch of a finest-pass launcher (launch_pre / post / post_r2 / postpre / sweep) on
// this thread: its kernel's host stub and its algorithmic bytes (the pgmg_fine_pass_bytes
// model applied to what that launch reads and writes).  The timed passes record it per launch
// (timed_end), so bench.py names and charges the kernel that actually ran
// (pgmg_fine_pass_info) instead of deriving both from its own flags.
struct LaunchNote {
    const void *kernel = nullptr;
    double bytes = 0.0;
};
extern thread_local LaunchNote g_last_launch;
template <class... P, class... A>
inline void launchk(void (*k)(P...), dim3 g, dim3 b, hipStream_t s, A &&...args)
{
    k<<<g, b, 0, s>>>(static_cast<P>(args)...);
    g_last_launch.kernel = reinterpret_cast<const void *>(k);
}
// fine points of rows [r0, r1) of an N-point level, times an element size (algorithmic bytes)
inline double row_pts(int r0, int r1, int N) { return r1 > r0 ? (double)(r1 - r0) * (N - 2) : 0.0; }

// The smoother's early exit is sqrt(s) < eps for s = sum of r^2 (Smoother.hpp:77-80).
// sqrt is correctly rounded and monotonic, so for s >= 0 (and NaN) the test equals s < T
// with T = the smallest double whose square root is >= eps: the latency-bound kernels test
// that instead of computing a square root on the dependent chain of every sweep.
inline double norm2_threshold(double eps)
{
    if (!(eps > 0.0)) return 0.0;                       // never fires (eps <= 0 or NaN)
    if (__builtin_isinf(eps)) return __builtin_inf();   // fires for every finite s
    unsigned long long lo = 0, hi = 0x7FF0000000000000ULL;  // sqrt(0) < eps <= sqrt(inf)
    while (hi - lo > 1) {
        const unsigned long long mid = lo + (hi - lo) / 2;
        double m;
        __builtin_memcpy(&m, &mid, 8);
        if (__builtin_sqrt(m) >= eps) hi = mid;
        else lo = mid;
    }
    double t;
    __builtin_memcpy(&t, &hi, 8);
    return t;
}

// one early-exit check recorded by a speculative call: the producing pass's per-block
// partial sums of r^2 (see pgmg_ctx.hip, "speculative calls")
struct CheckRef {
    const double *partials;
    long long np;
    int level;   // host bookkeeping (per-level speculation policy)
    int expect;  // 0: recorded as "does not fire", 1: as "fires", 2: decided in-stream (norm only)
};

constexpr int kOff = 15;          // doubles between allocation base and element (0,0) (fp64)
constexpr int kHalo = 10;         // halo rows allocated above and below a level's rows
constexpr int kPostExt = 4;       // row strips: k_post of a level below the finest also
                                  // computes this many rows of its result past each strip
                                  // edge (bitwise what the neighbour computes), so the
                                  // coarse correction needs no halo exchange
constexpr int kBlock = 256;       // threads per block for streaming kernels (4 waves)
#ifndef PGMG_TAIL_THREADS
#define PGMG_TAIL_THREADS 512    // 512 and 1024 measured equal (W at 4097 82.4 vs 82.9 ms)
#endif
constexpr int kTailThreads = PGMG_TAIL_THREADS;   // the tail workgroup (wave-0 paths fit 128 VGPRs)
constexpr int kTailMaxN = 65;     // largest level the LDS-resident tail holds

// Allocation registry and read/write span checks (DESIGN.md §2 "Read extents").  Every
// level grid (alloc_grid) is registered; the launch wrappers of the fused passes compute,
// from the band geometry the kernel itself uses, the first and last row and column they
// read or write in each array, and check_span verifies that the span lies inside ONE
// registered allocation before the pass is launched (PGMG_ERR_STATE, nothing launched,
// otherwise).  The passes deliberately read rows past their band and columns past their
// tiles (halos, tile margins); this turns a wrong halo or pitch assumption into an error
// code on the host instead of a GPU memory fault.
void register_alloc(const void *base, size_t bytes);
void unregister_alloc(const void *base);
// rows [r0, r1] x columns [c0, c1] (inclusive) of the array with virtual origin o (element
// (0,0)), pitch P elements of es bytes; o == nullptr: nothing to check
int check_span(const void *o, long long P, int es, long long r0, long long r1, long long c0,
               long long c1, const char *what);

inline int pitch_for(int N) { return (N + 15) / 16 * 16; }
inline size_t alloc_elems(int rows, int N) { return (size_t)kOff + (size_t)rows * pitch_for(N) + 64; }

// One sweep x_out = J(x_in) over interior rows [row0,row1) of a W-column grid.
// With partials != nullptr it also accumulates sum r(x_in)^2 over the same points
// per block: the smoother's early-exit norm of the PREVIOUS sweep, fused.
template <class T>
struct SweepArgsT {
    const T *xin;           // origin pointer (element (0,0)); unused when x0 is zero
    const T *f;
    T *xout;
    double *partials;       // one double per block, or nullptr
    const unsigned *skip;   // non-null and *skip != 0: the kernel does nothing
    unsigned *reset;        // non-null: block 0 writes 0 here (start of a smooth call)
    unsigned long long *stats;  // [0] sweeps performed (block 0 adds 1)
    T hh, inv_hh;           // h*h and 1.0/(h*h), rounded once on the host
    int W, P;               // columns, pitch (elements)
    int row0, row1;         // rows to update (local indexing)
    int rows_per_block;
};

// rc = R r(x) on coarse rows [jc0, jc1); the residual is never materialised.
template <class T>
struct ResRestrictArgsT {
    const T *x, *f;
    T *rc;
    T inv_hh;
    int Wf, Pf, Wc, Pc;
    int jc0, jc1;
    int rows_per_block;     // coarse rows per block
};

// fine += P coarse (reference flavour: fine row/col 1 never corrected).
template <class T>
struct ProlongArgsT {
    const T *c;
    T *fine;
    int Wf, Pf, Wc, Pc;
    int row0, row1;         // fine rows to update, inside [2, Nf-2]
    int rows_per_block;
    int assign;             // fine = (+0) + P coarse (prolongation into a zeroed grid)
};

// Early-exit decision for one smoother check plus the undo of the speculative sweep.
template <class T>
struct FixupArgsT {
    const double *partials;
    int np;
    double eps;
    const unsigned *done_prev;  // smoother already exited before this sweep
    unsigned *done_next;        // written: done_prev || (norm < eps)
    const T *src;               // buffer holding x_{k-1}
    T *dst;                     // buffer the speculative sweep k wrote
    unsigned long long *stats;
    int W, P, row0, row1;       // region copied on trigger
    const double *global_sum;   // all-rank sum of the partials (multi-GPU) or nullptr
};

// The whole V-cycle at and below a level with N <= 65, in LDS, one workgroup.
template <class T>
struct TailArgsT {
    const T *f_top;         // rhs of the tail's top level (global origin pointer)
    T *e_top;               // solution of the tail's top level (global origin pointer)
    int P_top;              // pitch of f_top / e_top
    int N_top;
    double h_top;
    int x0_from_global;     // 1: start from e_top's contents; 0: from zero
    // consecutive cycles on the top level with the same right-hand side (the W recursion's
    // alpha visits from its parent, MultiGrid.hpp:126-128), each from the previous one's
    // result, in ONE launch (0 or 1: one cycle)
    int visits;
    int v1, v2, coarse_iter, n_coarse;
    double eps;
    unsigned long long *stats;
    // F-cycle (full multigrid) mode, MultiGrid.hpp:138-183: e_top holds phi on entry;
    // restrict it to the coarsest level, then climb with smooth(3) -> prolong into a
    // zeroed finer grid -> analytic RHS -> V-cycle; result back into e_top.
    int fmg;
    int fmg_smooth_top;          // also run the smooth(3) on the top level (a finer level follows)
    const double *fmg_tab;       // per tail level: sx[N], sy[N] sine tables (host libm)
    int fmg_tab_off[8];          // offset of level t's sx in fmg_tab (sy follows)
    double fmg_factor;           // (pi^2/a^2)(p^2+q^2)
};

using SweepArgs = SweepArgsT<double>;
using ResRestrictArgs = ResRestrictArgsT<double>;
using ProlongArgs = ProlongArgsT<double>;
using FixupArgs = FixupArgsT<double>;
using TailArgs = TailArgsT<double>;

// sweeps on the finest level use a distinct kernel symbol (kFine) so that
// rocprofv3's per-kernel statistics isolate the roofline kernel.
template <class T> void launch_sweep(const SweepArgsT<T> &a, bool x0_zero, bool fine_level, hipStream_t s);
int sweep_blocks(int W, int row0, int row1, int *rows_per_block, int *gx, int *gy);
template <class T> void launch_res_restrict(const ResRestrictArgsT<T> &a, hipStream_t s);
int res_restrict_rows_per_block(int Wc, int nrows);
template <class T> void launch_prolong(const ProlongArgsT<T> &a, hipStream_t s);
template <class T> void launch_fixup(const FixupArgsT<T> &a, hipStream_t s);
template <class T>
void launch_copy_rows(const T *src, T *dst, int W, int P, int row0, int row1, hipStream_t s);
template <class T> hipError_t launch_tail_gamma(const TailArgsT<T> &a, int gamma, hipStream_t s);
template <class T> size_t tail_lds_bytes(int N_top, int n_coarse);
// f = (factor * sx[i]) * sy[j] in double, stored as T
template <class T>
void launch_rhs(T *f, const double *sx, const double *sy, double factor, int W, int P, int row0,
                int row1, hipStream_t s);
// coarse = R fine on interior coarse points (values, not residuals): compute_coarsest_grid;
// coarse rows [jc0, jc1) (clamped to the interior; row strips: the rank's rows)
template <class T>
void launch_restrict_values(const T *fine, int Nf, int Pf, T *coarse, int Nc, int Pc,
                            hipStream_t s, int jc0 = 1, int jc1 = 1 << 30);
// coarse = R R fine (two levels down in one pass, single grid, all interior rows)
template <class T>
void launch_restrict2_values(const T *fine, int Pf, T *coarse, int Nc, int Pc, hipStream_t s);
template <class T> void launch_fill_rows(T *o, int P, int row0, int row1, hipStream_t s);
// zero rows 0, 1, N-1 and columns 0, N-1 of an N x N grid (what a prolongation with
// assign = 1 over rows [2, N-2] leaves unwritten), within rows [r0, r1) (row strips:
// the rank's rows and halo rows)
template <class T>
void launch_zero_frame(T *o, int P, int N, hipStream_t s, int r0 = 0, int r1 = 1 << 30);
// rows 0, N-1 and columns 0, N-1 of a double grid (pitch Ps) into a T grid (pitch Pd)
template <class T>
void launch_copy_frame(const double *src, long long Ps, T *dst, long long Pd, int N, hipStream_t s);
template <class T>
void launch_resnorm_partials(const T *x, const T *f, double *partials, T inv_hh, int W, int P,
                             int row0, int row1, int nblocks, hipStream_t s);
void launch_sum_partials(const double *partials, int np, double *out, hipStream_t s);
// widen / narrow a level's rows between T storage and a double staging array (pitch N)
template <class T>
void launch_to_double(const T *src, int P, double *dst, int N, int row0, int row1, hipStream_t s);
template <class T>
void launch_from_double(const double *src, int N, T *dst, int P, int row0, int row1, hipStream_t s);

// reference-layout (pitch = W, any alignment) op kernels
// one Jacobi sweep; partials != nullptr: per-block sums of r(xin)^2 (g_blocks of them); seed:
// also copy xin's boundary into xout
void launch_g_sweep(const double *xin, const double *f, double *xout, double *partials,
                    const unsigned *skip, unsigned *reset, unsigned long long *stats, double hh,
                    double inv_hh, int H, int W, bool seed, hipStream_t s);
int g_blocks(int H, int W);
constexpr int kOpPartialsCap = 65536;   // partial sums per op scratch set (>= g_blocks)
// in-place sweeps on the caller's x (r05): one sweep / two sweeps per pass, each followed by
// the scatter of its deferred tile-edge outputs; `side` holds g_defer_elems(H, W) doubles
size_t g_defer_elems(int H, int W);
void launch_g_sweep_ip(double *x, const double *f, double *side, unsigned *reset,
                       unsigned long long *stats, double hh, int H, int W, hipStream_t s);
void launch_g_sweep2_ip(double *x, const double *f, double *side, unsigned long long *stats,
                        double hh, int H, int W, hipStream_t s);
void launch_g_fixup(const double *partials, int np, double eps, const unsigned *done_prev,
                    unsigned *done_next, const double *src, double *dst,
                    unsigned long long *stats, int H, int W, hipStream_t s);
void launch_g_residual(double *r, const double *x, const double *f, double inv_hh, int H, int W,
                       hipStream_t s);
void launch_g_restrict(const double *fine, double *coarse, int Nf, int Nc, hipStream_t s);
void launch_g_prolong(const double *coarse, double *fine, int Nc, int Nf, int mode, int ext,
                      hipStream_t s);
void launch_g_sumsq(const double *v, long long n, double *partials, int nblocks, hipStream_t s);
void launch_g_rhs(double *f, const double *sx, const double *sy, double factor, int W, int H,
                  hipStream_t s);

}  // namespace pgmg
