// pgmg_fused.h — argument blocks of the fused smoother passes (pgmg_fused.hip).
// Templates on the grid element type T (double, or float for the fp32 variant);
// partial sums and eps stay double.
#pragma once
#include "pgmg_internal.h"

namespace pgmg {

// pre-smooth (2 sweeps) + residual + full-weighting restriction in one pass
template <class T>
struct PreArgsT {
    const T *x0;                // level solution before smoothing (unused when x0 is zero)
    const T *f;                 // level right-hand side
    T *x2;                      // result of the two sweeps (ping-pong buffer); nullptr: not
                                // stored (x0 = 0: k_post recomputes it from f)
    T *rc;                      // coarse right-hand side R r(x2)
    double *partials;           // per block sum r(x1)^2 (early-exit check)
    unsigned long long *stats;  // [0] sweeps (+2 per launch)
    T hh, ih;
    int N, P, Nc, Pc;
    int jc0, jc1;               // coarse-row segments [jc0, jc1) (fine rows 2jc, 2jc+1)
    int row_lo, row_hi;         // fine rows whose x2 this rank writes
    int rc_lo, rc_hi;           // coarse rows whose rc this rank writes
    int rows_per_block;
    const unsigned *cond;       // non-null: run only when *cond != 0
    unsigned *fired;            // non-null: the fix-up records whether the check fired
    // non-null: f is the analytic RHS, regenerated as (T)(gfx[i] * gsy[j]) (level 0, or
    // the level of the F climb whose V-cycle and smooth(3) run)
    const double *gfx, *gsy;
    int nt;                     // set by launch_pre: bit 0 x2, bit 1 rc stores non-temporal
    // non-null (F-cycle): x0 is not read but is the prolongation of this coarse grid into a
    // zeroed fine grid, x0 = (+0) + P ec on rows/columns [2, N-2], 0 on the frame
    // (MultiGrid.hpp:159-164 followed by the V-cycle's pre-smooth)
    const T *pin_ec;
    // row pitch of x0 in elements (0: P).  Non-zero when x0 is the caller's array in the
    // reference layout (pitch N, pgmg_set_problem_device): the call's first pass reads it in
    // place; its 16-byte column-pair loads are then 8-byte aligned on every other row
    long long Px;
};

// prolongation + post-smooth (2 sweeps) in one pass
template <class T>
struct PostArgsT {
    const T *phi;               // level solution after pre-smoothing
    const T *ec;                // coarse-grid correction
    const T *f;
    T *x2;                      // result (the level's solution buffer)
    double *partials;
    unsigned long long *stats;
    T hh, ih;
    int N, P, Nc, Pc;
    int jc0, jc1;
    int row_lo, row_hi;
    int rows_per_block;
    const unsigned *cond;
    // non-null: phi is not read but recomputed from f as the pre-smoothed iterate of
    // x0 = 0 (x1 = J(0), phi = *pre_fired ? x1 : J(x1)); PreArgs::fired of the same level
    const unsigned *pre_fired;
    int fix_sweeps;             // k_post_fixup: 0/1 -> x1 (the check fired), 2 -> x2
    int sum_lo, sum_hi;         // sum_hi > sum_lo: the early-exit partial sums cover only
                                // these rows (the rank's own) while [row_lo, row_hi) is
                                // written (the strip plus kPostExt rows past each edge)
    // non-null: f is the analytic RHS, regenerated as (T)(gfx[i] * gsy[j]) (level 0, or
    // the level of the F climb whose V-cycle and smooth(3) run)
    const double *gfx, *gsy;
    int nt;                     // set by launch_post: bit 2 x2 stores non-temporal
    // row pitch of x2 in elements (0: P): the call's last pass writes the caller's array
    // (reference layout, pitch N) in place (pgmg_set_problem_device)
    long long Po;
    // k_post_r2 (the finest level's last pass of an F-cycle followed by another, speculative
    // calls): also the two-step full weighting of x2 into level 2 (r2out, pitch Pr2, N = Nr2),
    // the next F-cycle's first restriction step.  With the 116-column tile stride and the
    // 6-column margin the pass forms every level-2 centre column itself: lanes 3..60 own the
    // centres and lane 63 loads its own east coarse column (pgmg_fused.hip "k_post_r2")
    T *r2out;
    long long Pr2;
    int Nr2;
    // added to the sweeps the pass counts (stats[0] += 2 + sw_adj): +2 on the first finest pass
    // of a call that took over a carried pre-smooth (pgmg_ctx.hip "carry"), whose two sweeps
    // were run by the previous call's last pass
    int sw_adj;
};

// post-smooth of cycle k + pre-smooth/residual/restriction of cycle k+1 in one pass
// (the finest level between consecutive cycles of one pgmg_vcycle call)
template <class T>
struct PostPreArgsT {
    const T *phi;               // pre-smoothed solution of cycle k (recompute: its phi)
    const T *ec;                // coarse correction of cycle k
    const T *f;
    T *x4;                      // pre-smoothed solution of cycle k+1 (not the carry pass's)
    T *rc;                      // coarse right-hand side of cycle k+1
    double *partials1;          // sum r(x1)^2 (post-smooth check)
    double *partials2;          // sum r(x3)^2 (pre-smooth check)
    double *partials3;          // non-null (row strips): sum r(x2)^2 (pre check from x1)
    // non-null: f is the analytic RHS, regenerated as (T)(gfx[i] * gsy[j]) (gfx[i] =
    // factor*sx[i]); both tables valid for indices -8 .. (gfx: P + 248, gsy: N + 8)
    const double *gfx, *gsy;
    unsigned long long *stats;
    T hh, ih;
    int N, P, Nc, Pc;
    int jc0, jc1;
    int row_lo, row_hi;
    int rc_lo, rc_hi;
    int rows_per_block;
    int fast;                   // PGMG_FLAG_FAST (one GPU, f regenerated or stored)
    // non-null: the carry pass, the LAST finest pass of a call that also runs the next call's
    // pre-smooth (pgmg_ctx.hip "carry"): x2, the call's result, is stored here instead of x4
    // (x4 = nullptr); its restricted residual goes to rc as usual
    T *x2;
    int sw_adj;                 // stats[0] += 4 + sw_adj (the carry pass: -2; see PostArgsT)
    // nonzero: the recompute form, the first finest pass of a call that took the carry: phi
    // is the previous call's x2 and the pass runs its pre-smooth (the carry pass's, bitwise)
    // before the correction
    int recompute;
    // nonzero: XCD-aware tile order (measurement knob PGMG_PP_XCD): the workgroups the hardware
    // places on one XCD (linear id = x mod 8) take a contiguous run of tiles
    int xcd;
};

struct FixArgsF {
    const double *partials;
    int np;
    double eps;
    const double *global_sum;   // all-rank sum (multi-GPU) or nullptr: sum the partials
    unsigned long long *stats;
    const unsigned *cond;       // non-null: run only when *cond != 0
    int force;                  // recompute without deciding (rare path of k_postpre)
};


using PreArgs = PreArgsT<double>;
using PostArgs = PostArgsT<double>;
using PostPreArgs = PostPreArgsT<double>;

int fused_blocks(int N, int jc0, int jc1);
int post_r2_blocks(int N, int jc0, int jc1);   // k_post_r2's workgroups (check partials)
// the fused-pass launchers return PGMG_ERR_STATE (and launch nothing) when a span the pass
// would read or write lies outside its array's allocation (check_span)
template <class T> int launch_pre(const PreArgsT<T> &a, bool x0_zero, bool fine, hipStream_t s);
template <class T> int launch_post(const PostArgsT<T> &a, bool fine, hipStream_t s);
// the finest level's k_post with the two-step restriction of its result into a.r2out (every
// level-2 centre column formed by the pass's own wave tiles): one GPU, the analytic f
// regenerated or streamed, phi read (not RECOMP)
template <class T> int launch_post_r2(const PostArgsT<T> &a, hipStream_t s);
// coarse levels (x0 = 0, RECOMP) whose checks are predicted to fire: the one-sweep passes
// with the checks' partials (k_pre1 / k_post1)
template <class T> int launch_pre1(const PreArgsT<T> &a, bool x0_zero, hipStream_t s);
template <class T> int launch_post1(const PostArgsT<T> &a, hipStream_t s);
template <class T>
void launch_pre_fixup(const FixArgsF &a, const PreArgsT<T> &p, bool x0_zero, hipStream_t s);
template <class T> void launch_post_fixup(const FixArgsF &a, const PostArgsT<T> &p, hipStream_t s);
// the same rare paths as fused one-sweep passes (in-stream checks of enqueue_fused_level)
template <class T>
int launch_pre_rare(const FixArgsF &f, const PreArgsT<T> &a, bool x0_zero, hipStream_t s);
template <class T> int launch_post_rare(const FixArgsF &f, const PostArgsT<T> &a, hipStream_t s);
// k_postpre's workgroups (check partials); rc: the recompute form's (112-column tiles)
int postpre_blocks(int N, int jc0, int jc1, bool rc = false);
template <class T> int launch_postpre(const PostPreArgsT<T> &a, hipStream_t s);
// fused smooth(3): x4 of a.phi into a.x4 with the three checks' partial sums
// (partials1 r(x1), partials3 r(x2), partials2 r(x3)); then the decision + rare path
template <class T> int launch_smooth4(const PostPreArgsT<T> &a, hipStream_t s);
template <class T>
void launch_smooth4_finish(const PostPreArgsT<T> &a, int np, const double *global3, double eps,
                           unsigned *flags, unsigned long long *stats, hipStream_t s);
// flags[0] = post check fired; flags[1] = pre check fired (and post did not).
// global != nullptr: all-rank sums {post, pre} (row strips) instead of the partials.
void launch_postpre_decide(const double *partials1, const double *partials2,
                           unsigned long long *stats, int np, const double *global, double eps,
                           unsigned *flags, hipStream_t s);
// out[i] = 1 when check i could fire: sqrt(sum of its partials) < eps * (1 + 1e-12), the
// sum taken in the fix-ups' order (one workgroup per check); norm[i] = that sqrt
void launch_verify_checks(const CheckRef *checks, int n, double eps, unsigned *out, double *norm,
                          hipStream_t s);

// the validation's reply, straight into pinned host memory (no copies): any = OR over the
// first n_any verdicts, and the n norms and verdicts themselves; then *h_seq = seq (system
// scope, after the rest: the host polls it)
void launch_spec_reply(const unsigned *flags, const double *norm, int n, int n_any, unsigned *h_any,
                       double *h_norm, unsigned *h_flags, unsigned *h_seq, unsigned seq, hipStream_t s);
// a speculative segment's opening: stats_bk = stats (4 words), flags[0, nflags) = 0
void launch_spec_open(const unsigned long long *stats, unsigned long long *stats_bk, unsigned *flags,
                      int nflags, hipStream_t s);

}  // namespace pgmg
