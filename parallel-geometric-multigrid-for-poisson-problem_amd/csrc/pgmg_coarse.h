// pgmg_coarse.h — the small coarse levels' passes as 2D LDS tiles (pgmg_coarse.hip).
#pragma once
#include "pgmg_internal.h"

namespace pgmg {

// a level entered with x0 = 0 (RECOMP), f stored (not regenerated); the whole grid or a row
// strip's rows (global row numbers, as every level kernel)
template <class T>
struct CoarseArgsT {
    const T *f;                  // level right-hand side (pitch P)
    const T *ec;                 // k_post: coarse correction (pitch Pc)
    T *rc;                       // k_pre: coarse right-hand side R r(x2) (pitch Pc)
    T *x2;                       // k_post: the level's solution (pitch P)
    double *partials;            // per tile: sum of the check's r(x1)^2
    unsigned long long *stats;   // [0] += 2 per pass
    unsigned *fired;             // k_pre: cleared (the pre check's outcome, for k_post)
    const unsigned *pre_fired;   // k_post: the pre check fired -> the iterate is x1, not x2
    T hh, ih;
    int N, P, Nc, Pc;
    // tiles over the coarse rows [jt0, jt1); each tile owns the fine rows [2 jca, 2 jcb) of its
    // coarse rows [jca, jcb), the first from own_lo, the last up to own_hi: k_pre's check terms
    // (own = the rank's interior rows), k_post's written rows (own = its output rows); k_post
    // sums its check over [sum_lo, sum_hi) only (a strip's own rows)
    int jt0, jt1, own_lo, own_hi, sum_lo, sum_hi;
    // mode 2 (the in-stream rare path): the check to decide -- the mode-0 pass's partials, or
    // the all-rank sum of a distributed level's (global_sum != nullptr)
    const double *dec_partials;
    int dec_np;
    double eps;
    const double *global_sum;
};

// the tile passes apply to this level size (small, latency-bound levels; dist: a level split
// into row strips, whose thin strips are latency-bound up to larger N)
bool coarse_tile_ok(int N, bool dist = false);
// per-tile partial sums one tile pass over the whole grid writes (0 when !coarse_tile_ok): an
// upper bound of a strip's
int coarse_tile_blocks(int N);
// the same for a pass over the coarse rows [jt0, jt1)
int coarse_tile_blocks_rows(int N, int jt0, int jt1);
// mode 0: the pass (two sweeps + the check's partials); 1: the check predicted to fire (one
// sweep, partials, the exit booked); 2: the in-stream rare path (decide the mode-0 pass's
// check; if it fired, the one-sweep pass)
template <class T> void launch_pre_tile(const CoarseArgsT<T> &a, int mode, hipStream_t s);
template <class T> void launch_post_tile(const CoarseArgsT<T> &a, int mode, hipStream_t s);

}  // namespace pgmg
