// pgmg_coarse.h — the small coarse levels' passes as 2D LDS tiles (pgmg_coarse.hip).
#pragma once
#include "pgmg_internal.h"

namespace pgmg {

// a level entered with x0 = 0 (RECOMP), whole grid on this rank, f stored (not regenerated)
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
    // mode 2 (the in-stream rare path): the check to decide -- the mode-0 pass's partials
    const double *dec_partials;
    int dec_np;
    double eps;
};

// the tile passes apply to this level size (small, latency-bound levels)
bool coarse_tile_ok(int N);
// per-tile partial sums one tile pass writes (0 when !coarse_tile_ok)
int coarse_tile_blocks(int N);
// mode 0: the pass (two sweeps + the check's partials); 1: the check predicted to fire (one
// sweep, partials, the exit booked); 2: the in-stream rare path (decide the mode-0 pass's
// check; if it fired, the one-sweep pass)
template <class T> void launch_pre_tile(const CoarseArgsT<T> &a, int mode, hipStream_t s);
template <class T> void launch_post_tile(const CoarseArgsT<T> &a, int mode, hipStream_t s);

}  // namespace pgmg
