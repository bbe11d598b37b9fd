// pgmg_internal.h — device data layout, kernel argument blocks and launchers.
//
// HBM layout of one grid level (see DESIGN.md "Data layout"):
//   element (row j, column i) of an N x N vertex grid lives at o[j*P + i] where
//   o = base + kOff and P = round_up(N, 16) doubles.  kOff = 15 puts column 1 of
//   every row on a 128-byte boundary, so the pair of columns (1+2t, 2+2t) that
//   lane t owns is one aligned 16-byte load and a wave's 64 pairs are exactly
//   eight 128-byte lines.
//
// All kernels compute in fp64 with -ffp-contract=off and keep the reference's
// left-to-right expression order, so results are bit-identical to mg_cpu_exec.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace pgmg {

constexpr int kOff = 15;          // doubles between allocation base and element (0,0)
constexpr int kHalo = 6;          // halo rows allocated above and below a level's rows
constexpr int kBlock = 256;       // threads per block for streaming kernels (4 waves)
constexpr int kTailThreads = 1024;
constexpr int kTailMaxN = 65;     // largest level the LDS-resident tail holds

inline int pitch_for(int N) { return (N + 15) / 16 * 16; }
inline size_t alloc_elems(int rows, int N) { return (size_t)kOff + (size_t)rows * pitch_for(N) + 64; }

// One sweep x_out = J(x_in) over interior rows [row0,row1) of a W-column grid.
// With partials != nullptr it also accumulates sum r(x_in)^2 over the same points
// per block: the smoother's early-exit norm of the PREVIOUS sweep, fused.
struct SweepArgs {
    const double *xin;      // origin pointer (element (0,0)); unused when x0 is zero
    const double *f;
    double *xout;
    double *partials;       // one double per block, or nullptr
    const unsigned *skip;   // non-null and *skip != 0: the kernel does nothing
    unsigned *reset;        // non-null: block 0 writes 0 here (start of a smooth call)
    unsigned long long *stats;  // [0] sweeps performed (block 0 adds 1)
    double hh, inv_hh;      // h*h and 1.0/(h*h), rounded once on the host
    int W, P;               // columns, pitch (doubles)
    int row0, row1;         // rows to update (local indexing)
    int rows_per_block;
};

// rc = R r(x) on coarse rows [jc0, jc1); the residual is never materialised.
struct ResRestrictArgs {
    const double *x, *f;
    double *rc;
    double inv_hh;
    int Wf, Pf, Wc, Pc;
    int jc0, jc1;
    int rows_per_block;     // coarse rows per block
};

// fine += P coarse (reference flavour: fine row/col 1 never corrected).
struct ProlongArgs {
    const double *c;
    double *fine;
    int Wf, Pf, Wc, Pc;
    int row0, row1;         // fine rows to update, inside [2, Nf-2]
    int rows_per_block;
};

// Early-exit decision for one smoother check plus the undo of the speculative sweep.
struct FixupArgs {
    const double *partials;
    int np;
    double eps;
    const unsigned *done_prev;  // smoother already exited before this sweep
    unsigned *done_next;        // written: done_prev || (norm < eps)
    const double *src;          // buffer holding x_{k-1}
    double *dst;                // buffer the speculative sweep k wrote
    unsigned long long *stats;
    int W, P, row0, row1;       // region copied on trigger
    const double *global_sum;   // all-rank sum of the partials (multi-GPU) or nullptr
};

// The whole V-cycle at and below a level with N <= 65, in LDS, one workgroup.
struct TailArgs {
    const double *f_top;    // rhs of the tail's top level (global origin pointer)
    double *e_top;          // solution of the tail's top level (global origin pointer)
    int P_top;              // pitch of f_top / e_top
    int N_top;
    double h_top;
    int x0_from_global;     // 1: start from e_top's contents; 0: from zero
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

// sweeps on the finest level use a distinct kernel symbol (kFine) so that
// rocprofv3's per-kernel statistics isolate the roofline kernel.
void launch_sweep(const SweepArgs &a, bool x0_zero, bool fine_level, hipStream_t s);
int sweep_blocks(int W, int row0, int row1, int *rows_per_block, int *gx, int *gy);
void launch_res_restrict(const ResRestrictArgs &a, hipStream_t s);
int res_restrict_rows_per_block(int Wc, int nrows);
void launch_prolong(const ProlongArgs &a, hipStream_t s);
void launch_fixup(const FixupArgs &a, hipStream_t s);
void launch_copy_rows(const double *src, double *dst, int W, int P, int row0, int row1,
                      hipStream_t s);
hipError_t launch_tail(const TailArgs &a, hipStream_t s);
hipError_t launch_tail_gamma(const TailArgs &a, int gamma, hipStream_t s);
size_t tail_lds_doubles(int N_top, int n_coarse);
void launch_rhs(double *f, const double *sx, const double *sy, double factor, int W, int P,
                int row0, int row1, hipStream_t s);
// coarse = R fine on interior coarse points (values, not residuals): compute_coarsest_grid
void launch_restrict_values(const double *fine, int Nf, int Pf, double *coarse, int Nc, int Pc,
                            hipStream_t s);
void launch_fill_rows(double *o, int P, int row0, int row1, double v, hipStream_t s);
void launch_resnorm_partials(const double *x, const double *f, double *partials, double inv_hh,
                             int W, int P, int row0, int row1, int nblocks, hipStream_t s);
void launch_sum_partials(const double *partials, int np, double *out, hipStream_t s);

// reference-layout (pitch = W, any alignment) op kernels
void launch_g_sweep(const double *xin, const double *f, double *xout, double *partials,
                    const unsigned *skip, unsigned *reset, unsigned long long *stats, double hh,
                    double inv_hh, int H, int W, int nblocks, hipStream_t s);
int g_blocks(int H, int W);
void launch_g_fixup(const double *partials, int np, double eps, const unsigned *done_prev,
                    unsigned *done_next, const double *src, double *dst,
                    unsigned long long *stats, int H, int W, hipStream_t s);
void launch_g_copy(const double *src, double *dst, long long n, hipStream_t s);
void launch_g_residual(double *r, const double *x, const double *f, double inv_hh, int H, int W,
                       hipStream_t s);
void launch_g_restrict(const double *fine, double *coarse, int Nf, int Nc, hipStream_t s);
void launch_g_prolong(const double *coarse, double *fine, int Nc, int Nf, int mode, hipStream_t s);
void launch_g_sumsq(const double *v, long long n, double *partials, int nblocks, hipStream_t s);
void launch_g_rhs(double *f, const double *sx, const double *sy, double factor, int W, int H,
                  hipStream_t s);

}  // namespace pgmg
