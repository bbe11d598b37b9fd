// pgmg_ctx.h — the context object behind the C ABI (shared by the orchestration
// in pgmg_ctx.hip and the row-strip communication layer in pgmg_comm.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/pgmg.h"
#include "pgmg_internal.h"

namespace pgmg {

constexpr int kMaxSweeps = 64;  // early-exit flag slots per smooth call

int set_err(int code, const std::string &msg);

#define PGMG_HIPC(expr)                                                                           \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return ::pgmg::set_err(PGMG_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Grid {
    void *base = nullptr;    // allocation
    void *o = nullptr;       // virtual origin: element (global row j, col i) at o[j*P + i]
    size_t bytes = 0;        // allocation size
};

// typed view of a grid's origin (T = the context's element type)
template <class T> inline T *G(const Grid &g) { return static_cast<T *>(g.o); }
// element (row, 0) of a grid with element size es and pitch P, as bytes
inline char *row_ptr(const Grid &g, long long row, int P, int es)
{
    return static_cast<char *>(g.o) + row * (long long)P * es;
}

struct Level {
    int N = 0, P = 0;        // points per side, row pitch (elements)
    int es = 8;              // element bytes: 8 (fp64) or 4 (fp32)
    double h = 0, hh = 0, ih = 0;
    int lo = 0, hi = 0;      // owned global rows [lo, hi) (row 0 / N-1 belong to the ends)
    int u0 = 0, u1 = 0;      // interior rows this rank updates: [max(lo,1), min(hi,N-1))
    Grid A, B, F;            // solution (phi or e), ping-pong, right-hand side (f or rc)
    bool on_this_rank = true;
    bool gathered = false;   // the level is not split: every rank holds and computes all of it
};

class Comm;

// one array's halo exchange inside a grouped exchange (Comm::halos)
struct HaloReq {
    const Grid *g;
    const Level *L;
    int depth;
};

}  // namespace pgmg

struct pgmg_ctx {
    pgmg_config cfg{};
    bool fp32 = false;            // PGMG_PRECISION_FP32: every level grid stores float
    bool shuffle = false;         // large grids from shuffled physical chunks (one GPU)
    hipStream_t s = nullptr;
    std::vector<pgmg::Level> lv;  // 0 .. nb-1 bulk levels, nb = the tail's top level
    int nb = 0;
    double *partials = nullptr;
    int partials_cap = 0;
    unsigned *flags = nullptr;
    unsigned long long *stats = nullptr;
    double *scalar = nullptr;
    hipGraphExec_t gexec = nullptr;
    bool fsmooth_swapped = false; // an F-cycle swapped L.A / L.B of a level (fused smooth(3))
    bool have_problem = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // device-bound calls: recorded on the null stream at entry, so c->s (non-blocking) starts
    // after the caller's outstanding default-stream work (order_after_caller)
    hipEvent_t ev_caller = nullptr;
    struct EventPool {
        std::vector<hipEvent_t> ev;
        int used = 0;
    };
    // finest-level kernel timing (PGMG_FLAG_TIME_FINE): 0 plain sweep, 1 k_pre, 2 k_post
    EventPool tpool[6];           // 3: k_postpre, 4: the carry pass, 5: the recompute form
    // per timed pass: the kernels and algorithmic bytes of the launches timed since the last
    // pgmg_fine_pass_time (LaunchNote), and what that call averaged (pgmg_fine_pass_info)
    double tbytes[6] = {};
    const void *tkern[6] = {};
    double info_bytes[6] = {};
    const void *info_kern[6] = {};
    bool fused = false;           // v1 = v2 = 1: two fused passes per level
    bool cross = false;           // finest level fuses post(k) with pre(k+1) across cycles
    bool recompute = true;        // levels entered with x0 = 0 recompute x2 in k_post
    pgmg::Grid S;                 // finest-level scratch for k_postpre's rare paths
    double *partials2 = nullptr;  // second partials buffer (k_postpre's pre check)
    double *partials3 = nullptr;  // third (row strips: k_postpre's pre check from x1)
    // analytic RHS (set_problem with f = NULL): level-0 passes may regenerate f in-kernel
    // as gfx[i] * gsy[j] instead of streaming it (bitwise the stored values)
    double *rhs_tab = nullptr;
    const double *gfx = nullptr, *gsy = nullptr;   // valid for indices -8 ..
    bool gen_rhs = false;
    // the tables matching the CURRENT level-0 F (gfx/gsy, or the F-cycle's own during
    // pgmg_fcycle), nullptr when level-0 f must be streamed
    const double *rgfx = nullptr, *rgsy = nullptr;
    double *fmg_gtab = nullptr;   // fx/sy tables of the F-cycle's level-0 RHS
    // speculative calls (pgmg_ctx.hip "speculative calls"): the early-exit checks of a
    // call are recorded instead of decided in-stream, validated once after the call
    bool spec = false;            // enabled for this context (fused cycle, no EXACT flag)
    bool spec_off = false;        // switched off: a finest-level check fires
    std::vector<char> lvl_exact;  // per bulk level: its checks fire (soon): decide in-stream
    std::vector<char> lvl_fire;   // per bulk level: its checks keep firing: predicted to fire
    std::vector<char> lvl_fire_block;   // a "fires" prediction failed: never again (this problem)
    std::vector<int> lvl_kx;      // per bulk level: its first cycles of the segment recorded
                                  // "does not fire" (then in-stream); lvl_vis counts its visits
    std::vector<int> lvl_vis;
    std::vector<double> lvl_fire_try;   // norm at the last segment split made for the level to
                                        // become "fires" (0: none; no second split before it halves)
    std::vector<std::vector<double>> lvl_hist;   // per bulk level: its last check norms
    double *chk_norm = nullptr;   // per-check norms of the last validation
    unsigned *mark_dev = nullptr; // row strips: per-level marks agreed by allreduce
    std::vector<double> hnorm;
    std::vector<unsigned> hflag;
    bool lean = false;            // the cycles being enqueued record their checks
    int spec_gamma = 1;           // gamma of the speculative call being enqueued
    // W-cycle plan (pgmg_ctx.hip "W-cycle plans"): per visit of a bulk level in the cycle, the
    // largest and smallest check norm of that visit in the last validated cycle
    std::vector<double> wmax, wmin, wrho;   // wrho: the visit's decay over the last two cycles
    int wplan_gamma = 0;          // gamma of the plan (0: none)
    int wplan_seg = 0;            // cycles of the segment the plan was taken from
    bool wplan_off = false;       // a plan's prediction failed: none for this problem
    int wvisit = 0, wseg = 0;     // visits enqueued in this segment; its cycles
    int cur_visit = -1;           // the visit whose checks chk_log records (-1: none)
    long long wcount[3] = {0, 0, 0};   // the last W call's visits per mode
    std::vector<int> chk_visit;   // per recorded check: its visit (-1: level 0)
    double *plog = nullptr;       // partials of every recorded check of the current call
    long long plog_cap = 0, plog_used = 0;
    std::vector<pgmg::CheckRef> chks;
    unsigned *uflags = nullptr;   // per-check verdicts (+ one spare word: any)
    char *pin = nullptr;          // pinned coherent host staging of the validation: chk_cap
                                  // CheckRefs (read by k_verify_checks), norms, verdicts + any
                                  // (written by k_spec_reply)
    long long chk_cap = 0;
    unsigned pin_seq = 0;         // the last validation reply's sequence word
    pgmg::Grid bk;                // level-0 solution at the start of the call (rollback)
    // speculative F-cycles (pgmg_ctx.hip "speculative F-cycles"): every bulk check of the
    // climb recorded "does not fire"; a rollback restarts the call's first climb from the
    // tail top's restricted grid, saved here (the only input of the climb)
    bool fspec = false;           // the F-cycles being enqueued are speculative
    bool fspec_off = false;       // a speculative F call was rolled back: in-stream (problem)
    pgmg::Grid ftop;
    // speculative F-cycle followed by another in the call: its finest k_post also forms level
    // 2's restriction (k_post_r2; fr2_want while it is enqueued, fr2_made once it was)
    bool fr2_want = false, fr2_made = false;
    unsigned long long *stats_bk = nullptr;
    long long rollbacks = 0;
    unsigned *ppflags = nullptr;  // k_postpre_decide flags
    pgmg::Comm *comm = nullptr;   // non-null when world > 1
    // F-cycle (pgmg_fcycle): analytic level-0 RHS of the FMG h chain, and the sine
    // tables of every level (built on the first call)
    pgmg::Grid Ffmg;
    // F-cycle climb: regenerated-RHS tables (factor*sx, sy) of every bulk level of the FMG
    // chain (level l at fmg_gtab + fmg_goff[l]); the level whose V-cycle and smooth(3) are
    // being enqueued regenerates its analytic f in-kernel (gen_level, lgfx, lgsy)
    std::vector<size_t> fmg_goff;
    int gen_level = 0;
    const double *lgfx = nullptr, *lgsy = nullptr;
    int fmg_f_swapped = -1;   // bulk level whose L.F is traded with Ffmg_l (climb), or -1
    std::vector<pgmg::Grid> Ffmg_l;   // the analytic RHS of bulk levels 1.. of the FMG climb
    bool fmg_rhs_ready = false;   // Ffmg holds the level-0 analytic RHS of the FMG h chain
    double *fmg_tab = nullptr;
    std::vector<int> fmg_off;     // per level 0..nb then tail levels below nb: sx offset
    // pgmg_set_problem_device: the caller's arrays in the reference layout (pitch N, double),
    // the problem of every following cycle call (phi updated in place)
    double *ext_phi = nullptr;
    const double *ext_f = nullptr;   // nullptr: the analytic RHS (regenerated in-kernel)
    bool ext_inplace = false;        // the finest passes read / write ext_phi in place
    // while a call is enqueued: the first k_pre reads x_in, the last k_post writes x_out
    // (pitch ext_P) instead of the level-0 grids; defer_post stops before that last k_post
    // (a speculative call validates its checks first: x_out is also x_in), pend_pr is the
    // pre-smoothed iterate it will read
    const void *x_in = nullptr;
    void *x_out = nullptr;
    long long ext_P = 0;
    bool defer_post = false;
    void *pend_pr = nullptr;
    // the carry (pgmg_ctx.hip "carry"): a speculative V call on the context's own grids ends
    // with the carry pass, which stores its result and the next cycle's restriction into
    // lv[1].F; the next V call starts from them (its first finest pass recomputes the
    // pre-smooth) when no entry touched the problem in between
    bool carry = false;           // lv[1].F holds the validated restriction of lv[0].A's pre-smooth
    bool carry_use = false;       // the segment being enqueued starts from the carry
    bool carry_make = false;      // the segment being enqueued ends with the carry pass
    bool carry_made = false;      // ... and it did
    bool carry_took = false;      // the last segment enqueued started from the carry
    int carry_chk = -1;           // index in chks of the carried pre-smooth's check
    long long carry_n[3] = {0, 0, 0};   // calls that took a carry, carries made, dropped
};

namespace pgmg {

// stagger: the origin shifted by this many bytes (a multiple of 128) past the usual one;
// shuffle: a grid of 256 MB or more is built from shuffled physical chunks (pgmg_ctx.hip)
int alloc_grid(Grid &g, const Level &L, size_t stagger = 0, bool shuffle = false);
void free_grid(Grid &g);
// dispatch on the context's element type
int enqueue_cycle(pgmg_ctx *c, int l, int gamma, bool x0_zero);
int enqueue_tail(pgmg_ctx *c, int gamma, bool x0_from_global);
// copy rows [0, N) of a level-0-shaped grid (origin o, pitch P, the context's element
// type) to a dense host array of doubles (synchronous)
int download_grid(pgmg_ctx *c, const void *o, int P, int N, double *host);

// Row-strip domain decomposition (one process per GPU, RCCL), pgmg_comm.hip.
// Levels 0 .. gathered_level()-1 are split into row strips with halo exchange;
// the first gathered level and everything below it are collapsed to one (replicated) grid.
class Comm {
  public:
    virtual ~Comm() {}
    // ownership (lo/hi/u0/u1, on_this_rank, gathered) for every level, before allocation
    virtual int plan(pgmg_ctx *c) = 0;
    // after allocation
    virtual int setup(pgmg_ctx *c) = 0;
    virtual int gathered_level() const = 0;
    virtual int rank() const = 0;
    // exchange `depth` halo rows of strip-distributed arrays, all in one group
    virtual int halos(const HaloReq *reqs, int n, hipStream_t s) = 0;
    int halo(const Grid &g, const Level &L, int depth, hipStream_t s)
    {
        const HaloReq r{&g, &L, depth};
        return halos(&r, 1, s);
    }
    // The same exchange started early: as soon as stream s reaches this point (the rows to
    // send are final), on a side stream of the comm, overlapping whatever s does next;
    // halo_end(s) makes s wait for it.  Used for the finest level's halos, which are final
    // a whole coarse hierarchy before they are read.  Default: exchange in place on s.
    virtual int halo_begin(const Grid &g, const Level &L, int depth, hipStream_t s)
    {
        return halo(g, L, depth, s);
    }
    virtual int halo_end(hipStream_t) { return 0; }
    // in-place sum of n device doubles over all ranks
    virtual int allreduce_sum(double *d, int n, hipStream_t s) = 0;
    // in-place element-wise minimum of n device unsigned ints over all ranks
    virtual int allreduce_min_u32(unsigned *d, int n, hipStream_t s) = 0;
    // the parent produced rc of gathered level l: gather it on every rank, run `repeats`
    // cycles on every rank's full copy (identical results; no scatter needed)
    virtual int run_gathered(pgmg_ctx *c, int l, int gamma, int repeats) = 0;
    // grid g of gathered level l: every rank's rows (the ones its parent strip restricts
    // into) to every other rank, so every rank holds the full grid (one grouped exchange)
    virtual int allgather_rows(pgmg_ctx *c, int l, const Grid &g) = 0;
    // the strips of phi to every rank (root < 0) or to rank `root` only (others: phi_host
    // may be null)
    virtual int gather_solution(pgmg_ctx *c, double *phi_host, int root) = 0;
    // hipStreamSynchronize that cannot hang on a dead or stuck peer: RCCL's asynchronous
    // error state is polled while waiting, and after cfg.comm_timeout_s the communicator is
    // aborted; PGMG_ERR_COMM then
    virtual int wait(hipStream_t s) = 0;
    // collective groups (grouped exchanges and allreduces) enqueued since the last call and,
    // with PGMG_FLAG_TIME_COMM, the stream time spent inside them (events around each group:
    // the transfer plus any wait for a peer), else ms = -1; synchronous, resets both
    virtual int comm_stats(hipStream_t s, long long *groups, double *ms) = 0;
    // ranks of the communicator (RCCL: ncclCommCount), the world for the other transports
    virtual int comm_ranks(int *n) = 0;
    static Comm *create(pgmg_ctx *c, int *rc);
};

// true when level l is split across ranks (halos, global norms)
inline bool is_dist(const pgmg_ctx *c, int l);

}  // namespace pgmg

inline bool pgmg::is_dist(const pgmg_ctx *c, int l)
{
    return c->comm != nullptr && l < c->comm->gathered_level();
}
