/*
 * pgmg.h — C ABI of the MI355X geometric-multigrid library (libpgmg.so).
 *
 * The drop-in boundary for the reference's GPU path.  Every entry point is
 * extern "C" with plain pointers, sizes and int return codes (0 = success,
 * negative = error; pgmg_last_error() gives the message).  No C++ exceptions
 * and no HIP/torch types cross it.  Host code that binds it: the C++ mirror of
 * the reference interface (host/Parallel_*.hpp, host/ParallelTestRunner.hpp,
 * host/gpu_exec.cpp) and the Python ctypes plumbing used by tests and bench.py.
 *
 * What each entry replaces in the reference (/root/reference/...):
 *
 *   cycle level (context API)
 *     pgmg_create / pgmg_set_problem / pgmg_vcycle / pgmg_get_solution
 *         ParallelMultiGridSolver::v_cycle(double*, double*, int, double)
 *             3_part_parallel/Parallel_Mg.cu:21-60, driven by
 *         ParallelTestRunner::run_v_cycle()  3_part_parallel/ParallelTestRunner.cu:152-186
 *         (numerics: MultigridSolver::v_cycle, 2_part_MG/MultiGrid.hpp:57-94)
 *     pgmg_wcycle
 *         ParallelMultiGridSolver::w_cycle  3_part_parallel/Parallel_Mg.cu:62-102
 *         (numerics: MultigridSolver::w_cycle, 2_part_MG/MultiGrid.hpp:96-136)
 *     pgmg_fcycle
 *         MultigridTestRunner::run_cycle("F-cycle") 2_part_MG/MultiGridTestRunner.hpp:192-205
 *         + MultigridSolver::f_cycle / compute_coarsest_grid, MultiGrid.hpp:28-55,138-183
 *
 *   op level (caller-owned device arrays in the reference's row-major layout,
 *   element (y, x) at p[y*W + x]; the optional `stream` is a hipStream_t)
 *     pgmg_jacobi    Parallel::ComputeJacobi       3_part_parallel/Parallel_Method.cu:144-160
 *                    (in place on d_x like the reference's, each sweep exactly the
 *                    out-of-place sweep; numerics of JacobiSmoother::smooth,
 *                    Smoother.hpp:38-116: v+1 sweeps with the residual-norm early exit)
 *     pgmg_residual  Parallel::ComputeResidual     Parallel_Method.cu:162-173
 *                    (DynamicGridUtils::compute_residual, DynamicGridUtils.hpp:59-69)
 *     pgmg_restrict  Parallel::ComputeRestriction  Parallel_Method.cu:175-186
 *                    (MultigridSolver::restrict_full_weighting, MultiGrid.hpp:187-205)
 *     pgmg_prolong   Parallel::ComputeProlungator  Parallel_Method.cu:188-199
 *                    (mode 0: MultigridSolver::prolongation, MultiGrid.hpp:208-226;
 *                     mode 1: the symmetric prolungator_kernel, Parallel_Method.cu:79-138)
 *     pgmg_norm      DynamicGridUtils::norm        DynamicGridUtils.hpp:21-27
 *     pgmg_rhs       DynamicGridUtils::compute_rhs DynamicGridUtils.hpp:111-124
 *
 * Threading: a context is driven by one host thread; not thread-safe.
 */
#ifndef PGMG_H
#define PGMG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGMG_OK 0
#define PGMG_ERR_ARG (-1)     /* bad argument (N not 2^k+1, null pointer, ...) */
#define PGMG_ERR_HIP (-2)     /* HIP runtime error                              */
#define PGMG_ERR_NOMEM (-3)   /* device allocation failed                       */
#define PGMG_ERR_COMM (-4)    /* RCCL error                                     */
#define PGMG_ERR_STATE (-5)   /* call out of order (e.g. vcycle before set_problem) */

/* prolongation flavours */
#define PGMG_PROLONG_REFERENCE 0 /* mg_cpu_exec: fine row/col 1 uncorrected */
#define PGMG_PROLONG_SYMMETRIC 1 /* gpu_exec's prolungator_kernel; fine boundary set 0  */

/* element type of every level grid (pgmg_config.precision) */
#define PGMG_PRECISION_FP64 0    /* bit-identical to mg_cpu_exec (the default)            */
#define PGMG_PRECISION_FP32 1    /* fp32 storage and arithmetic, half the HBM bytes; norms
                                    accumulated in fp64; parity stated as a tolerance
                                    against fp64 (the reference is fp64-only).
                                    Host arrays at the ABI stay double.                     */

/* config flags */
#define PGMG_FLAG_NO_GRAPH 1u    /* launch eagerly instead of replaying a hipGraph */
#define PGMG_FLAG_TIME_FINE 2u   /* eager launches + hipEvents around every finest-level
                                    pass (see pgmg_fine_pass_time)                  */
#define PGMG_FLAG_UNFUSED 4u     /* one kernel per smoother sweep even when v1 = v2 = 1
                                    (the general path; same results)                */
#define PGMG_FLAG_NO_CROSS 16u   /* do not fuse the finest level's post-smooth with the
                                    next cycle's pre-smooth (same results)           */
#define PGMG_FLAG_STORED_RHS 32u /* always stream f from HBM; by default, when f is the
                                    analytic RHS (set_problem f = NULL), the finest-level
                                    cross-cycle pass regenerates it in-kernel from two
                                    sine tables (bitwise the same values, 8 B/pt less) */
#define PGMG_FLAG_EXACT_DIST 64u /* decide every smoother early-exit check in-stream (a
                                    fix-up launch per check; on row strips an allreduce
                                    each) instead of speculatively (validated once per
                                    call, rollback on doubt; same results)            */
#define PGMG_FLAG_SOLO 128u     /* measurement only: world > 1 with a null transport — this
                                    rank's share of the strip work on one GPU, no messages
                                    (halos/gathered rows stale, allreduces local); results
                                    are meaningless, timings are one rank's compute     */
#define PGMG_FLAG_LOOPBACK 8u    /* world > 1 with ranks as threads of one process on
                                    one GPU: nccl_unique_id is a pgmg_loopback hub
                                    (test transport for the strip decomposition)    */
/* Alternative execution plans with the same results (each is bitwise-tested against the
 * default and the oracle; they exist to test the default's building blocks apart): */
#define PGMG_FLAG_NO_RECOMPUTE 256u /* coarse levels store their pre-smoothed iterate
                                       instead of recomputing it from f in k_post     */
#define PGMG_FLAG_NO_PIN 512u       /* F-cycle: a separate prolongation pass into the
                                       zeroed finer grid instead of k_pre computing it
                                       on the fly                                      */
#define PGMG_FLAG_NO_R2 1024u       /* F-cycle: one full-weighting level per restriction
                                       pass instead of two                             */
#define PGMG_FLAG_FAST 4096u    /* FAST mode: the finest
                                   level's cross-cycle pass shares each iterate's neighbour
                                   sum between its Jacobi sweep and its residual and forms
                                   the residuals with FMA — not the reference's expression
                                   order, so phi agrees with the EXACT default within
                                   1e-12 relative (after <= 10 cycles) instead of bitwise.
                                   One GPU (row strips ignore it); everything else exact */
#define PGMG_FLAG_NO_SPEC_FIRE 32768u /* speculative calls without segment planning,
                                       per-cycle speculation windows and levels predicted
                                       to fire (the r02 policy: a level that will fire
                                       decides in-stream from the call's start), and
                                       W-cycles without plans (every bulk check
                                       in-stream).  Results are identical either way.
                                       (8192u until r03.)                              */
/* Retired bits, rejected by pgmg_create with PGMG_ERR_ARG so that a caller built against an
   older header fails loudly instead of silently getting another option:
   8192u  -- PGMG_FLAG_L1POST until r02 (level 1's post-smooth inside the finest pass; removed
             in r03), then PGMG_FLAG_NO_SPEC_FIRE in r03;
   16384u -- the 129x129 level inside the tail's launch (built in r03, bitwise, measured
             slower: one CU's fp64 VALU needs ~1.2 us per pass over 129^2 points; removed) */
#define PGMG_FLAGS_RETIRED (8192u | 16384u)
#define PGMG_FLAG_NO_CTILE 65536u /* the small coarse levels (N <= 513, entered with x0 = 0)
                                     run the row-marching fused passes instead of the 2D LDS
                                     tile passes (r04).  Results are identical either way */
#define PGMG_FLAG_NO_CARRY 131072u /* do not carry the next call's pre-smooth across
                                      pgmg_vcycle calls (the carry: below pgmg_vcycle).  Results
                                      and statistics are identical either way */
#define PGMG_FLAG_TIME_COMM 262144u /* world > 1: hipEvents around every collective group
                                       (grouped halo exchange, all-to-all, allreduce) on the
                                       context's stream, read by pgmg_comm_stats */
#define PGMG_FLAG_NO_SHUFFLE 524288u /* one GPU: allocate the grids of 256 MB and more with
                                        plain hipMalloc instead of from 2 MB physical chunks
                                        mapped in a shuffled order (the finest
                                        pass runs ~3-4 % faster in a process's first context) */
#define PGMG_FLAG_NO_SPIN 1048576u /* one GPU: a speculative call waits for its validation with a
                                      blocking stream wait instead of polling the reply word in
                                      pinned memory (pgmg_ctx.hip reply_wait) */
#define PGMG_FLAG_HOST_TRANSPORT 2048u /* world > 1 without RCCL: nccl_unique_id points to
                                       a pgmg_host_transport; every message and reduction
                                       is staged through host memory and handed to the
                                       caller's functions (MPI, torch.distributed/gloo,
                                       ...; several ranks may share one GPU)           */

/* The caller's transport for PGMG_FLAG_HOST_TRANSPORT.  Every function is called by all
 * ranks in the same order (collective, blocking) and returns 0 on success; any other value
 * fails the library call with PGMG_ERR_COMM.
 *   exchange: one group of point-to-point messages: send send_bytes[i] bytes of host
 *     buffer send_buf[i] to rank send_peer[i], receive recv_bytes[i] bytes from
 *     recv_peer[i] into recv_buf[i]; messages between two ranks match in posting order
 *     (the semantics of the RCCL path's grouped ncclSend/ncclRecv).
 *   allreduce_sum_f64: v[i] = sum over ranks, in place; the sum taken in rank order
 *     (0.0 + v_0 + v_1 + ...) keeps every rank's decisions identical and equal to the
 *     in-process loopback transport's.
 *   allreduce_min_u32: v[i] = min over ranks, in place. */
typedef struct pgmg_host_transport {
    void *user;
    int (*exchange)(void *user, int nsend, const int *send_peer, const void *const *send_buf,
                    const unsigned long long *send_bytes, int nrecv, const int *recv_peer,
                    void *const *recv_buf, const unsigned long long *recv_bytes);
    int (*allreduce_sum_f64)(void *user, double *v, int n);
    int (*allreduce_min_u32)(void *user, unsigned *v, int n);
} pgmg_host_transport;

typedef struct pgmg_config {
    int N;             /* points per side incl. boundary; 2^k + 1, k >= 2        */
    int v1, v2;        /* pre/post smoother num_iter (v+1 sweeps), default 1, 1  */
    int coarse_iter;   /* num_iter on the coarsest grid, default 10 (11 sweeps)  */
    int n_coarse;      /* recursion floor N_coarse, default 5                    */
    int alpha;         /* W-cycle recursion count, default 3                     */
    double eps;        /* smoother early-exit tolerance, default 1e-7; <0: never */
    double a, p, q;    /* domain edge and RHS wave numbers, default 1, 1, 1      */
    int tail_n;        /* levels with N <= tail_n run in one workgroup (<= 65)   */
    int device;        /* HIP device ordinal, default 0                          */
    unsigned flags;    /* PGMG_FLAG_*                                            */
    /* row-strip domain decomposition over `world` ranks (one process per GPU). */
    int rank, world;   /* default 0, 1                                           */
    const void *nccl_unique_id;  /* 128-byte ncclUniqueId when world > 1      */
    int gather_n;      /* levels with N <= gather_n collapse to one grid, replicated
                          on every rank (world > 1)                               */
    int precision;     /* PGMG_PRECISION_FP64 (default) or PGMG_PRECISION_FP32    */
    int cross_min_n;   /* the finest level's post-smooth of cycle k and pre-smooth of
                          cycle k+1 are one pass from this N up (default 2049; small
                          values let tests exercise it on small grids)            */
    int spec_segment;  /* speculative calls: at most this many cycles per validated
                          segment (0 = sized by the log buffer; tests set it small) */
    double comm_timeout_s; /* row strips over RCCL: a stream wait that sees no progress
                          for this long aborts the communicator and returns
                          PGMG_ERR_COMM (default 600); RCCL's asynchronous error
                          state is polled while waiting                            */
    double h0;         /* finest-level mesh width; 0 (default): a / (N - 1).  The
                          reference's cycle entry points take h from the caller
                          (MultiGrid.hpp:57, Parallel_Mg.cu:21); coarse levels double
                          it (MultiGrid.hpp:83)                                    */
} pgmg_config;

typedef struct pgmg_ctx pgmg_ctx;

/* Fill `cfg` with the reference defaults for grid size N. */
int pgmg_config_default(pgmg_config *cfg, int N);

int pgmg_create(pgmg_ctx **ctx, const pgmg_config *cfg);
int pgmg_destroy(pgmg_ctx *ctx);

/* Upload phi0 (N*N, NULL -> zeros) and f (N*N, NULL -> the analytic RHS of
 * DynamicGridUtils::compute_rhs, generated on the device bit-identically from
 * host libm sine tables).  Host arrays in the reference layout (pitch N).  With
 * world > 1 every rank passes the full arrays (or NULLs) and keeps its strip. */
int pgmg_set_problem(pgmg_ctx *ctx, const double *phi0, const double *f);

/* Device-resident problem: the reference's memory contract.  ParallelMultiGridSolver::
 * v_cycle(phi, f, N, h) (3_part_parallel/Parallel_Mg.cu:21-60) updates in place arrays the
 * caller allocated in device-accessible memory (cudaMallocManaged,
 * ParallelTestRunner.cu:162-163).  After this call every pgmg_vcycle / wcycle / fcycle works
 * on the caller's DEVICE arrays in the reference layout (N*N doubles, pitch N): phi is read
 * and updated in place, synchronously (the call returns when phi holds the result), with no
 * host transfer.  f = NULL: the analytic RHS of compute_rhs (regenerated in-kernel, never
 * read); otherwise the caller's f, copied on the device into the context at every call (the
 * caller may change it between calls).  With phi from pgmg_alloc_grid on a cross-fused fp64
 * context (N >= cross_min_n) the finest-level passes read and write phi where it lies (the
 * same HBM bytes as a call on the context's own grids); any other device pointer is staged
 * with device-to-device copies before and after each call.  One GPU (world 1).  Resets the
 * statistics like pgmg_set_problem; pgmg_set_problem unbinds.  pgmg_get_solution /
 * pgmg_solution_hash / pgmg_residual_norm read the bound phi. */
int pgmg_set_problem_device(pgmg_ctx *ctx, double *phi, const double *f);
/* bound = a device problem is bound; inplace = its calls read / write phi in place */
int pgmg_problem_device_info(pgmg_ctx *ctx, int *bound, int *inplace);
/* An N*N device grid in the reference layout (pitch N, zeroed) with guard rows before and
 * after it, so the finest passes may read past its edges: what the in-place path of
 * pgmg_set_problem_device needs (the mirror's stand-in for cudaMallocManaged). */
int pgmg_alloc_grid(double **ptr, int N);
int pgmg_free_grid(double *ptr);
/* *serial = a number unique to this pgmg_alloc_grid allocation (never reused), 0 when ptr is
 * not a live pgmg_alloc_grid grid: lets a caller that caches a binding by pointer (the mirror's
 * ParallelMultiGridSolver) notice a grid freed and re-allocated at the same address. */
int pgmg_grid_serial(const double *ptr, unsigned long long *serial);
/* *is_device = 1 when p is device (or managed) memory of the HIP runtime. */
int pgmg_pointer_is_device(const void *p, int *is_device);

/* Enqueue `ncycles` cycles on the context's stream (asynchronous; a speculative call,
 * see pgmg_dist_info, returns after the device has finished it).
 * pgmg_fcycle: one F-cycle = restrict phi to n_coarse, then per level up smooth(3),
 * prolongation into a zeroed finer grid, analytic RHS of that grid (h chain starting at
 * 1/(n_coarse-1)), one V-cycle; the f given to pgmg_set_problem is left untouched
 * (MultiGridTestRunner.hpp:192-205).  On row strips as well (world > 1).  On one GPU an
 * F-cycle call is speculative too (its bulk checks recorded "does not fire" and validated once
 * after the call; a rollback reruns the call in-stream from the saved restricted grid and the
 * problem's later F calls decide in-stream); PGMG_FLAG_EXACT_DIST turns that off. */
/* The carry (r06; one GPU, cross-fused contexts, problems set with pgmg_set_problem): a
 * speculative V call ends with a finest-level pass that also runs the NEXT cycle's pre-smooth,
 * residual and restriction (MultiGrid.hpp:57-94's first half), keeps the restriction in a
 * context-owned buffer and checks it; the next pgmg_vcycle on the same problem starts from it
 * instead of running its own first pass (its first finest pass recomputes the pre-smooth from
 * phi in registers: no pass and no byte is added).  Entries that only read the problem (pgmg_get_solution, pgmg_solution_hash,
 * pgmg_residual_norm, pgmg_stats*, pgmg_sync ...) keep the carry; every entry that changes phi,
 * f, eps, the flags or the cycle kind (pgmg_set_problem*, pgmg_set_eps, pgmg_wcycle,
 * pgmg_fcycle, pgmg_bench_sweep, pgmg_phi_device -- its pointer allows writes -- ) drops it.
 * A carried pre-smooth whose early-exit check could fire is dropped, not rolled back.  Results
 * and statistics (its two sweeps count in the call that uses them) equal the uncarried ones,
 * bit for bit.  PGMG_FLAG_NO_CARRY turns it off; pgmg_carry_info counts it. */
int pgmg_vcycle(pgmg_ctx *ctx, int ncycles);
int pgmg_wcycle(pgmg_ctx *ctx, int ncycles);
int pgmg_fcycle(pgmg_ctx *ctx, int ncycles);
int pgmg_sync(pgmg_ctx *ctx);

/* Download phi (N*N, reference layout).  world > 1: every rank receives the
 * full grid (strips are gathered to all ranks). */
int pgmg_get_solution(pgmg_ctx *ctx, double *phi_host);
/* The same with the strips gathered to rank `root` only (collective: every rank calls it;
 * ranks other than root may pass phi_host = NULL).  root < 0: every rank, as above. */
int pgmg_gather_solution(pgmg_ctx *ctx, int root, double *phi_host);

/* FNV-64-style hash of phi's IEEE words in the reference layout (h = 1469598103934665603,
 * h = (h ^ word) * 1099511628211 per element, row-major N*N): the checksum of the golden
 * fixtures (tests/golden/cycles.json).  Collective on row strips; the value lands on rank
 * `root` (root < 0: every rank), the others get 0. */
int pgmg_solution_hash(pgmg_ctx *ctx, int root, unsigned long long *hash);

/* sqrt(sum over interior of r^2) for the current phi (synchronous). */
int pgmg_residual_norm(pgmg_ctx *ctx, double *out);

/* Cumulative smoother sweeps and early exits since set_problem
 * (comparable with the oracle's counters). */
int pgmg_stats(pgmg_ctx *ctx, long long *sweeps, long long *early_exits);

/* [0] sweeps, [1] early exits, [2] k_postpre post-check rare paths taken (-1 when
 * cross-cycle fusion is off), [3] k_postpre pre-check rare paths taken. */
int pgmg_stats_detail(pgmg_ctx *ctx, long long *out4);

/* Device time of the last pgmg_vcycle/wcycle call in ms (hipEvents on the
 * context stream; synchronous). */
int pgmg_last_elapsed_ms(pgmg_ctx *ctx, double *ms);

/* Number of bulk (multi-kernel) levels and the tail's top N. */
int pgmg_levels(pgmg_ctx *ctx, int *bulk_levels, int *tail_top_n);

/* Algorithmic HBM bytes one V-cycle moves (per rank), summed per kernel. */
int pgmg_vcycle_bytes(pgmg_ctx *ctx, double *bytes);

/* Raw device pointer and pitch (in elements) of phi's element (0,0) on this
 * rank, for callers that want to read it in place.  The elements are double, or
 * float when the context was created with PGMG_PRECISION_FP32 (pgmg_precision). */
int pgmg_phi_device(pgmg_ctx *ctx, double **ptr, int *pitch, int *row0, int *rows);

/* Is rows [row0, row1] x columns [col0, col1] (inclusive, elements of elem_bytes, row pitch
 * `pitch` elements, relative to element (0,0) at `origin`) inside ONE device allocation of
 * this library (a level grid)?  PGMG_OK if so, PGMG_ERR_STATE otherwise.  The fused passes
 * run this check on every array before each launch (they read halo rows past their bands
 * and margin columns past their tiles); callers reading a grid in place through
 * pgmg_phi_device can use it too. */
int pgmg_check_span(const void *origin, long long pitch, int elem_bytes, long long row0,
                    long long row1, long long col0, long long col1);

/* Algorithmic HBM bytes of one launch of finest-level pass `pass` (numbering of
 * pgmg_fine_pass_time) on this rank: every input read once, every output written once
 * (24 B per fine point for x, f -> x; +8 B per coarse point per coarse array; 16 B when
 * k_postpre regenerates the analytic f in-kernel), times elem_bytes / 8. */
int pgmg_fine_pass_bytes(pgmg_ctx *ctx, int pass, double *bytes);

/* Whether V/W-cycle calls decide the smoother early-exit checks speculatively (1: the
 * checks are recorded, validated once after the call, and the call is rolled back and
 * rerun with in-stream decisions when one could fire; cross-fused or row-strip contexts
 * without PGMG_FLAG_EXACT_DIST) or in-stream (0), and how many calls (V, W or F) were rolled
 * back.  After a rollback the context decides in-stream until the next pgmg_set_problem. */
int pgmg_dist_info(pgmg_ctx *ctx, int *speculative, long long *rollbacks);

/* Which bulk levels decide their early-exit checks in-stream in the next speculative call:
 * bit l (l >= 1) = level l's checks fired or are predicted to fire soon; bit 0 = no
 * speculation at all (disabled, or a finest-level check fires). */
int pgmg_spec_levels(pgmg_ctx *ctx, unsigned long long *in_stream);
/* Of those, the levels whose checks are predicted to FIRE in the next speculative call (one
 * GPU; converged levels: each visit runs the one-sweep passes the in-stream rare paths would
 * run, and the validation confirms every such check fired, else the call is rolled back). */
int pgmg_spec_fire_levels(pgmg_ctx *ctx, unsigned long long *fire);
/* W-cycle plans (one GPU): how the last speculative W call enqueued the visits of its bulk
 * levels -- counts[0] recorded "does not fire", counts[1] predicted to fire, counts[2] decided
 * in-stream -- each visit planned from the same visit of the previous cycle.  Zeros after a
 * V call. */
int pgmg_spec_visit_modes(pgmg_ctx *ctx, long long counts[3]);

/* Row strips (world > 1): the collective groups enqueued since the last call and, with
 * PGMG_FLAG_TIME_COMM, the stream time spent inside them in ms (-1 without the flag; the
 * transfer plus any wait for a peer, i.e. the part of a rank's cycle not spent computing);
 * synchronous, resets both.  One GPU: 0 and 0. */
int pgmg_comm_stats(pgmg_ctx *ctx, long long *groups, double *ms);
/* The communicator's rank count (RCCL: ncclCommCount; the world for the loopback / host /
 * null transports; 1 without strips). */
int pgmg_comm_ranks(pgmg_ctx *ctx, int *ranks);

/* The carry (above pgmg_vcycle): out[0] calls that started from a carried pre-smooth, out[1]
 * carries made, out[2] carries dropped because their check could fire. */
int pgmg_carry_info(pgmg_ctx *ctx, long long out[3]);

/* A new early-exit threshold (JacobiSmoother's eps, Smoother.hpp:38) for the following calls:
 * drops the carry and the speculation history (the statistics continue). */
int pgmg_set_eps(pgmg_ctx *ctx, double eps);

/* The context's PGMG_PRECISION_* and its grid element size in bytes (8 or 4). */
int pgmg_precision(pgmg_ctx *ctx, int *precision, int *elem_bytes);

/* Count and mean device duration (ms) of the finest-level kernels launched since
 * the last call (needs PGMG_FLAG_TIME_FINE; synchronous).  pass 0: plain Jacobi
 * sweep (unfused path), 1: fused pre-smooth+residual+restriction (k_pre),
 * 2: fused prolongation+post-smooth (k_post), 3: cross-cycle k_postpre, 4: the carry pass
 * (k_postpre that stores the call's result instead of the next pre-smooth), 5: the recompute
 * form (the first k_postpre of a call that took the carry). */
int pgmg_fine_pass_time(pgmg_ctx *ctx, int pass, int *count, double *mean_ms);
/* What the launches the last pgmg_fine_pass_time(pass) averaged were: the kernel symbol of the
 * last of them (demangled, e.g. "pgmg::k_postpre_lds<double, false, true, 2>"; "" when none was
 * timed) and the mean of their algorithmic bytes (the pgmg_fine_pass_bytes model applied to
 * what each launch actually read and wrote: an F-cycle's k_pre reads no x0, ...). */
int pgmg_fine_pass_info(pgmg_ctx *ctx, int pass, char *symbol, int len, double *bytes_per_launch);
int pgmg_fine_sweep_time(pgmg_ctx *ctx, int *count, double *mean_ms);  /* pass 0 */

/* 1 when the context runs the fused two-pass-per-level cycle (v1 = v2 = 1). */
int pgmg_fused(pgmg_ctx *ctx, int *fused);

/* Time `reps` back-to-back fine-grid Jacobi sweeps (the roofline kernel) on the
 * context's level-0 buffers with hipEvents; returns the mean per sweep in ms.
 * Leaves phi changed (call set_problem again before parity checks). */
int pgmg_bench_sweep(pgmg_ctx *ctx, int reps, double *ms_per_sweep);

/* ---- op level (device pointers, reference layout, pitch = W) ------------- */
/* v+1 sweeps on d_x IN PLACE (Parallel::ComputeJacobi, Parallel_Method.cu:144-160; each
 * sweep is exactly the out-of-place Jacobi sweep: tile-edge outputs another workgroup reads
 * are deferred and scattered after each pass).  eps < 0 disables the early exit.  d_tmp: W*H
 * scratch or NULL (allocated internally), used only by checked calls (eps >= 0) with v >= 1.
 * *sweeps_done (may be NULL) receives the sweep count (synchronous when non-NULL; NULL keeps
 * the call asynchronous on `stream`). */
int pgmg_jacobi(double *d_x, double *d_tmp, const double *d_f, int H, int W, double h, int v,
                double eps, int *sweeps_done, void *stream);
int pgmg_residual(double *d_r, const double *d_x, const double *d_f, int H, int W, double h,
                  void *stream);
int pgmg_restrict(const double *d_fine, double *d_coarse, int Nf, int Nc, void *stream);
int pgmg_prolong(const double *d_coarse, double *d_fine, int Nc, int Nf, int mode, void *stream);
/* The same with the reference's thread grid (Parallel::ComputeProlungator,
 * Parallel_Method.cu:188-199): only fine rows and columns below max(1, Nf / num_thread) *
 * num_thread are touched -- for Nf = 2^k + 1 > num_thread the last fine row and column keep
 * their values, as in the reference.  num_thread = 0: the whole grid (pgmg_prolong). */
int pgmg_prolong_grid(const double *d_coarse, double *d_fine, int Nc, int Nf, int mode,
                      int num_thread, void *stream);
int pgmg_norm(const double *d_v, long long n, double *result, void *stream);
int pgmg_rhs(double *d_f, int W, int H, double h, double a, double p, double q, void *stream);
/* The op-level entries keep one scratch set (partial sums, flags, ping-pong buffer) per
 * stream they were called on; this waits for `stream` and frees its set (a later op on the
 * same stream allocates a fresh one).  Call it before destroying a stream the ops used. */
int pgmg_ops_release(void *stream);

/* ---- device memory helpers (for host code built without HIP headers) ----- */
int pgmg_device_alloc(void **ptr, size_t bytes);
int pgmg_device_free(void *ptr);
int pgmg_memcpy_h2d(void *dst, const void *src, size_t bytes);
int pgmg_memcpy_d2h(void *dst, const void *src, size_t bytes);
int pgmg_device_sync(void);
int pgmg_device_count(int *n);

/* RCCL bootstrap: fill a 128-byte buffer with a fresh ncclUniqueId (rank 0). */
int pgmg_comm_unique_id(void *out128);

/* Self-test of the RCCL transport on one GPU (a world-1 communicator): the strip path's
 * grouped send/recv, allreduce(sum, double) and allreduce(min, u32) on a stream; 0 = ok. */
int pgmg_rccl_selftest(const void *uid128, int device);
/* Latency floor of the strips' collectives on THIS device: a world-1 RCCL communicator
 * (unique id uid128) times, over `reps` repetitions after 3 warm ones with hipEvents on one
 * stream, us[0] one grouped send + recv of 2 rows of 16385 doubles to itself (the finest
 * level's halo at N = 16385), us[1] an allreduce(sum) of 3 doubles (k_postpre's decision),
 * us[2] an allreduce(min) of 9 u32 (the speculation marks); mean microseconds per call.  A
 * lower bound of the per-group cost between ranks (no xGMI hop, no peer to wait for). */
int pgmg_rccl_latency(const void *uid128, int device, int reps, double *us3);

/* Measurement (libpgmg_ab.so, built with -DPGMG_TUNING; the product library always
 * returns -1): with PGMG_TAIL_PROF=1 in the environment, the LDS tail accumulates shader-
 * clock cycles per stage kind ([0] wave-team hand-offs, [1] block smooth, [2] block
 * res+restrict, [3] block prolong, [4] whole kernel, [5] launches, [6] wave smooth, [7] wave
 * res+restrict+prolong); read (and reset) them.  -1 when the variable is unset. */
int pgmg_tail_prof(unsigned long long *out16, int reset);

/* In-process rank hub for PGMG_FLAG_LOOPBACK (tests of the strip decomposition). */
int pgmg_loopback_create(int world, void **hub);
int pgmg_loopback_destroy(void *hub);
/* Test hook: the at_group-th transport group (halo exchange, gather) rank `rank` starts
 * from now on fails with PGMG_ERR_COMM (0 = never). */
int pgmg_loopback_fail(void *hub, int rank, long long at_group);

/* Host-only strip plan: the finest-level rows [lo, hi) rank `rank` owns and the
 * number of strip-distributed levels (0: too small to split, replicas). */
int pgmg_plan_strips(int N, int world, int rank, int tail_n, int gather_n, int *lo, int *hi,
                     int *dist_levels);

const char *pgmg_last_error(void);
const char *pgmg_version(void);
/* First 16 hex digits of the sha256 of the sources this library was built from (the csrc .hip
 * and .h files, include/pgmg.h, concatenated in path order; Makefile "srchash"). */
const char *pgmg_source_hash(void);

#ifdef __cplusplus
}
#endif
#endif /* PGMG_H */
