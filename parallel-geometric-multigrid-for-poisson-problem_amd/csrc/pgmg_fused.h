// pgmg_fused.h — argument blocks of the fused smoother passes (pgmg_fused.hip).
#pragma once
#include "pgmg_internal.h"

namespace pgmg {

// pre-smooth (2 sweeps) + residual + full-weighting restriction in one pass
struct PreArgs {
    const double *x0;           // level solution before smoothing (unused when x0 is zero)
    const double *f;            // level right-hand side
    double *x2;                 // result of the two sweeps (ping-pong buffer); nullptr: not
                                // stored (x0 = 0: k_post recomputes it from f)
    double *rc;                 // coarse right-hand side R r(x2)
    double *partials;           // per block sum r(x1)^2 (early-exit check)
    unsigned long long *stats;  // [0] sweeps (+2 per launch)
    double hh, ih;
    int N, P, Nc, Pc;
    int jc0, jc1;               // coarse-row segments [jc0, jc1) (fine rows 2jc, 2jc+1)
    int row_lo, row_hi;         // fine rows whose x2 this rank writes
    int rc_lo, rc_hi;           // coarse rows whose rc this rank writes
    int rows_per_block;
    const unsigned *cond;       // non-null: run only when *cond != 0
    unsigned *fired;            // non-null: the fix-up records whether the check fired
};

// prolongation + post-smooth (2 sweeps) in one pass
struct PostArgs {
    const double *phi;          // level solution after pre-smoothing
    const double *ec;           // coarse-grid correction
    const double *f;
    double *x2;                 // result (the level's solution buffer)
    double *partials;
    unsigned long long *stats;
    double hh, ih;
    int N, P, Nc, Pc;
    int jc0, jc1;
    int row_lo, row_hi;
    int rows_per_block;
    const unsigned *cond;
    // non-null: phi is not read but recomputed from f as the pre-smoothed iterate of
    // x0 = 0 (x1 = J(0), phi = *pre_fired ? x1 : J(x1)); PreArgs::fired of the same level
    const unsigned *pre_fired;
};

// post-smooth of cycle k + pre-smooth/residual/restriction of cycle k+1 in one pass
// (the finest level between consecutive cycles of one pgmg_vcycle call)
struct PostPreArgs {
    const double *phi;          // pre-smoothed solution of cycle k
    const double *ec;           // coarse correction of cycle k
    const double *f;
    double *x4;                 // pre-smoothed solution of cycle k+1
    double *rc;                 // coarse right-hand side of cycle k+1
    double *partials1;          // sum r(x1)^2 (post-smooth check)
    double *partials2;          // sum r(x3)^2 (pre-smooth check)
    unsigned long long *stats;
    double hh, ih;
    int N, P, Nc, Pc;
    int jc0, jc1;
    int row_lo, row_hi;
    int rc_lo, rc_hi;
    int rows_per_block;
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

int fused_blocks(int N, int jc0, int jc1);
void launch_pre(const PreArgs &a, bool x0_zero, bool fine, hipStream_t s);
void launch_post(const PostArgs &a, bool fine, hipStream_t s);
void launch_pre_fixup(const FixArgsF &a, const PreArgs &p, bool x0_zero, hipStream_t s);
void launch_post_fixup(const FixArgsF &a, const PostArgs &p, hipStream_t s);
int postpre_blocks(int N, int jc0, int jc1);
void launch_postpre(const PostPreArgs &a, hipStream_t s);
// flags[0] = post check fired; flags[1] = pre check fired (and post did not)
void launch_postpre_decide(const PostPreArgs &a, int np, double eps, unsigned *flags,
                           hipStream_t s);

}  // namespace pgmg
