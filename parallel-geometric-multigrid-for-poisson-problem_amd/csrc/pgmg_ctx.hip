// pgmg_ctx.hip — context, level pyramid, cycle orchestration and the C ABI.
//
// Replaces the reference's ParallelMultiGridSolver (3_part_parallel/Parallel_Mg.cu)
// and the allocation/timing plumbing of ParallelTestRunner::run_v_cycle
// (3_part_parallel/ParallelTestRunner.cu:152-186), MI355X-first:
//   * the whole level pyramid is allocated once in HBM (no per-level, per-cycle
//     cudaMallocManaged, no unified-memory migration, no host sync per kernel);
//   * each bulk level (N > tail_n) is 2 pre sweeps + fused residual/restriction
//     + prolongation + 2 post sweeps on ping-pong buffers; the smoother's
//     per-sweep early exit (Smoother.hpp:75-88) is evaluated on the device by
//     speculating the next sweep and undoing it when the check fires;
//   * the coarse end (N <= tail_n) is one LDS-resident workgroup (pgmg_tail.hip);
//   * a V-cycle is captured once into a hipGraph and replayed.
//
// Row strips: every per-level array is addressed through a "virtual origin"
// pointer o with element (global row j, column i) at o[j*P + i]; a rank only
// allocates its owned rows plus two halo rows each side, so all kernels work in
// global row numbers and the fine/coarse row parity (j = 2 jc) is preserved.
#include <hip/hip_runtime.h>

#include <cxxabi.h>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <numeric>
#include <string>
#include <utility>
#include <vector>

#include "pgmg_ctx.h"
#include "pgmg_coarse.h"
#include "pgmg_fused.h"

using namespace pgmg;

// Wait for the context's stream.  On row strips through the transport's wait, which polls
// RCCL's asynchronous error state and gives up after cfg.comm_timeout_s instead of hanging
// on a dead or stuck peer.
static int stream_wait(pgmg_ctx *c)
{
    if (c->comm) return c->comm->wait(c->s);
    PGMG_HIPC(hipStreamSynchronize(c->s));
    return PGMG_OK;
}
#define PGMG_TRY(expr)            \
    do {                          \
        const int e_ = (expr);    \
        if (e_) return e_;        \
    } while (0)

static thread_local std::string g_err;

int pgmg::set_err(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

#define HIPC(expr) PGMG_HIPC(expr)

// ---------------------------------------------------------------------------
// allocation
// ---------------------------------------------------------------------------
namespace {
std::mutex g_alloc_mu;
std::map<uintptr_t, size_t> g_allocs;   // base -> bytes of every registered allocation
}  // namespace

void pgmg::register_alloc(const void *base, size_t bytes)
{
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    g_allocs[(uintptr_t)base] = bytes;
}

void pgmg::unregister_alloc(const void *base)
{
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    g_allocs.erase((uintptr_t)base);
}

// is [lo, hi) inside ONE registered allocation?
static bool registered_span(intptr_t lo, intptr_t hi)
{
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    auto it = g_allocs.upper_bound((uintptr_t)lo);
    if (it == g_allocs.begin()) return false;
    --it;
    const intptr_t b = (intptr_t)it->first, e = b + (intptr_t)it->second;
    return lo >= b && hi <= e;
}

namespace {
std::mutex g_user_mu;
struct UserGrid {
    void *alloc;
    unsigned long long serial;   // distinct for every pgmg_alloc_grid call (pgmg_grid_serial)
};
std::map<uintptr_t, UserGrid> g_user_grids;   // pgmg_alloc_grid: element (0,0) -> allocation
unsigned long long g_user_serial = 0;
}  // namespace

static bool is_device_ptr(const void *p)
{
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();   // unregistered host memory: not an error to keep
        return false;
    }
    return at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
}

int pgmg::check_span(const void *o, long long P, int es, long long r0, long long r1,
                     long long c0, long long c1, const char *what)
{
    if (o == nullptr || r1 < r0 || c1 < c0) return PGMG_OK;
    const intptr_t org = (intptr_t)o;
    const intptr_t lo = org + (intptr_t)((r0 * P + c0) * es);
    const intptr_t hi = org + (intptr_t)((r1 * P + c1 + 1) * es);   // one past the last byte
    if (registered_span(lo, hi)) return PGMG_OK;
    char buf[256];
    std::snprintf(buf, sizeof(buf),
                  "%s: rows %lld..%lld, columns %lld..%lld (pitch %lld) outside the array's "
                  "allocation",
                  what, r0, r1, c0, c1, P);
    return set_err(PGMG_ERR_STATE, buf);
}

// ---------------------------------------------------------------------------
// Shuffled physical placement (large grids).  The finest pass streams two 2 GB grids at once
// (reads one, writes the other a few rows behind); how fast depends on where their PHYSICAL
// pages lie relative to each other (profiles/r06/probes/: the same kernel on the same data runs
// 1.02 or 1.09 ms depending on the context's allocation, 1.14-1.29 ms with physically
// contiguous grids).  A grid of this kind is instead built from physical chunks mapped into one
// virtual range in a fixed pseudo-random order (HIP virtual memory API): whatever the
// allocator hands out, consecutive chunks of a grid do not sit at a fixed physical distance from
// the chunks of the other grids the pass streams at the same time.
// ---------------------------------------------------------------------------
namespace {
struct VmmAlloc {
    size_t bytes = 0, chunk = 0;
    std::vector<hipMemGenericAllocationHandle_t> h;
};
std::mutex g_vmm_mu;
std::map<uintptr_t, VmmAlloc> g_vmm;   // reserved base -> its chunks
}  // namespace

// does p lie in a shuffled (virtual-memory-mapped) grid?  The runtime's 2D copies and memsets
// refuse those ranges, so every grid transfer checks and takes a kernel or a 1D copy instead
static bool is_vmm(const void *p)
{
    std::lock_guard<std::mutex> lk(g_vmm_mu);
    auto it = g_vmm.upper_bound((uintptr_t)p);
    if (it == g_vmm.begin()) return false;
    --it;
    return (uintptr_t)p < it->first + it->second.bytes;
}

static hipError_t vmm_free(void *base)
{
    VmmAlloc a;
    {
        std::lock_guard<std::mutex> lk(g_vmm_mu);
        auto it = g_vmm.find((uintptr_t)base);
        if (it == g_vmm.end()) return hipErrorInvalidValue;
        a = std::move(it->second);
        g_vmm.erase(it);
    }
    hipError_t e = hipSuccess;
    for (size_t i = 0; i < a.h.size(); ++i) {
        if (a.h[i] == 0) continue;
        const hipError_t u = hipMemUnmap(static_cast<char *>(base) + i * a.chunk, a.chunk);
        const hipError_t r = hipMemRelease(a.h[i]);
        if (e == hipSuccess) e = u != hipSuccess ? u : r;
    }
    const hipError_t f = hipMemAddressFree(base, a.bytes);
    return e != hipSuccess ? e : f;
}

// `bytes` of device memory on the current device from chunks of `chunk_mb` MB (rounded to the
// allocation granularity) mapped in a fixed shuffled order; *out = nullptr on failure
static hipError_t vmm_alloc(void **out, size_t bytes, size_t chunk_mb)
{
    *out = nullptr;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    size_t gran = 0;
    if ((e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum)) != hipSuccess)
        return e;
    size_t chunk = std::max(gran, (chunk_mb << 20) / gran * gran);
    const size_t n = (bytes + chunk - 1) / chunk, total = n * chunk;
    void *base = nullptr;
    if ((e = hipMemAddressReserve(&base, total, 0, nullptr, 0)) != hipSuccess) return e;
    VmmAlloc a;
    a.bytes = total;
    a.chunk = chunk;
    a.h.assign(n, 0);
    {
        std::lock_guard<std::mutex> lk(g_vmm_mu);
        g_vmm[(uintptr_t)base] = a;
    }
    // the k-th physical chunk created goes to virtual slot (k * stride + shift) % n: a
    // multiplicative permutation (stride coprime to n) scattering consecutive chunks, different
    // for every grid (the relative placement of two grids' chunks at the same virtual offset --
    // what two streams of one pass touch together -- then varies from chunk to chunk)
    static std::atomic<unsigned> serial{0};
    const unsigned g = serial.fetch_add(1);
    const double phi = 0.6180339887 + 0.0731 * (double)(g % 7);
    size_t stride = ((size_t)(phi * (double)n) % n) | 1;
    while (std::gcd(stride, n) != 1) stride += 2;
    const size_t shift = ((size_t)g * 40503u) % n;
    for (size_t k = 0; k < n && e == hipSuccess; ++k) {
        const size_t slot = (k * stride + shift) % n;
        hipMemGenericAllocationHandle_t h = 0;
        if ((e = hipMemCreate(&h, chunk, &prop, 0)) != hipSuccess) break;
        {
            std::lock_guard<std::mutex> lk(g_vmm_mu);
            g_vmm[(uintptr_t)base].h[slot] = h;
        }
        e = hipMemMap(static_cast<char *>(base) + slot * chunk, chunk, 0, h, 0);
    }
    if (e == hipSuccess) {
        hipMemAccessDesc acc{};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        e = hipMemSetAccess(base, total, &acc, 1);
    }
    if (e != hipSuccess) {
        (void)vmm_free(base);
        return e;
    }
    *out = base;
    return hipSuccess;
}

int pgmg::alloc_grid(Grid &g, const Level &L, size_t stagger, bool shuffle)
{
    // owned rows + kHalo halo rows each side (the fused passes read 4 rows past a
    // segment); the slack covers the last wave tile reading past the row end
    const int rows = (L.hi - L.lo) + 2 * kHalo;
    // column 1 of every row on a 128-byte boundary: 128/es - 1 elements before (0,0)
    const size_t off = (size_t)(128 / L.es - 1) + (stagger / 128) * (128 / L.es);
    const size_t n = off + (size_t)rows * L.P + 512;
    void *p = nullptr;
    // (measurement build: PGMG_CONTIG=1 asks for physically contiguous memory for grids of
    // 64 MB and more: a placement probe)
    // (measurement build: PGMG_CONTIG=1 physically contiguous grids, PGMG_SHUFFLE_MB the chunk
    // size of the shuffled ones, 0 = no shuffling)
    const bool contig = tuning_int("PGMG_CONTIG", 0) != 0 && n * L.es >= (64u << 20);
    const int shuffle_mb = tuning_int("PGMG_SHUFFLE_MB", 2);
    const bool shuffled = shuffle && shuffle_mb > 0 && n * L.es >= (256u << 20);
    hipError_t ae = hipErrorUnknown;
    if (shuffled) ae = vmm_alloc(&p, n * L.es, (size_t)shuffle_mb);
    if (shuffled && ae != hipSuccess) (void)hipGetLastError();   // no VMM here: plain memory
    if (ae == hipSuccess) {
    } else if (contig) ae = hipExtMallocWithFlags(&p, n * L.es, hipDeviceMallocContiguous);
    else ae = hipMalloc(&p, n * L.es);
    if (ae != hipSuccess)
        return set_err(PGMG_ERR_NOMEM, "hipMalloc failed for a level of N=" + std::to_string(L.N) + ": " +
                                           hipGetErrorString(ae));
    HIPC(hipMemset(p, 0, n * L.es));
    g.base = p;
    g.bytes = n * L.es;
    register_alloc(p, g.bytes);
    g.o = static_cast<char *>(p) + (off + (ptrdiff_t)(kHalo - L.lo) * L.P) * L.es;
    return PGMG_OK;
}

void pgmg::free_grid(Grid &g)
{
    if (g.base) {
        unregister_alloc(g.base);
        if (vmm_free(g.base) != hipSuccess) (void)hipFree(g.base);   // (not a shuffled grid)
    }
    g.base = g.o = nullptr;
    g.bytes = 0;
}

// Speculative call: a fresh slice of the partials log for one early-exit check, recorded
// for the validation after the call (nullptr when the cycles being enqueued decide every
// check in-stream).  The log is sized beforehand (spec_need); running past it would be a
// bug: the check then writes the shared partials and the call is treated as failed
// validation (rolled back), never read out of bounds.
// How a speculative call enqueues level l's checks: 0 recorded as "does not fire" (no
// fix-up), 1 recorded as "fires" (the one-sweep passes, no fix-up), 2 decided in-stream (the
// fix-ups; outside speculative calls every check).
// W-cycles (gamma > 1): a bulk level's visits are planned one by one (w_visit_mode)
static int chk_mode(const pgmg_ctx *c, int level)
{
    if (c->lean && c->fspec) return 0;   // speculative F-cycles: every bulk check
    if (!c->lean || (c->spec_gamma > 1 && level > 0) || c->lvl_exact[level]) return 2;
    return c->lvl_fire[level] ? 1 : 0;
}

// W-cycle plans (one GPU).  A W-cycle visits level l 3^l times and every visit's checks are a
// different story: a visit right after its parent's restriction starts from a large residual,
// the later ones from a nearly solved one -- per level, some visits fire and some do not in
// every cycle, so the per-level policy of the V-cycles leaves every bulk check in-stream (a
// pass and a rare-path launch each, ~5 % of a W-cycle at 4097).  The visits of a cycle come
// in the same order every cycle and their norms fall from cycle to cycle (by ~0.15 at 4097 in
// the steady phase, by orders of magnitude in the first cycles), so visit v of the next cycle
// is planned from visit v of the last validated one: predicted to fire (k_pre1 / k_post1) when
// both of its checks were below eps / 4, recorded "does not fire" when both stay above eps
// with the decay the visit showed since the previous plan, per cycle of the new segment, and a
// further 100-fold margin; in-stream otherwise.  A failed prediction rolls the segment back and ends the plans for the
// problem.
static int w_visit_mode(pgmg_ctx *c, int l)
{
    if (!c->lean || c->spec_gamma <= 1 || l == 0) return -1;
    const int v = c->wvisit++;
    c->cur_visit = v;
    const int vc = (int)c->wmax.size();
    int m = 2;
    if (!c->wplan_off && c->wplan_gamma == c->spec_gamma && vc > 0) {
        const int pos = v % vc;
        const double eps = c->cfg.eps;
        if (c->wmax[pos] >= 0.0 && c->wmax[pos] < 0.25 * eps) m = 1;
        else if (c->wrho[pos] > 0.0 &&
                 c->wmin[pos] * std::pow(c->wrho[pos], (double)c->wseg) * 0.01 >= eps)
            m = 0;
    }
    ++c->wcount[m];
    return m;
}

// A log slice for one check of mode `mode` (nullptr outside speculative calls; an in-stream
// check is logged -- its norm only, for the per-level policy -- on one GPU)
static double *chk_log(pgmg_ctx *c, int np, int level, int mode)
{
    if (!c->lean || (mode == 2 && c->comm != nullptr)) return nullptr;
    c->chk_visit.push_back(level > 0 ? c->cur_visit : -1);
    if (c->plog_used + np > c->plog_cap) {
        c->chks.push_back({nullptr, -1, level, mode});
        return c->partials;
    }
    double *p = c->plog + c->plog_used;
    c->plog_used += np;
    c->chks.push_back({p, np, level, mode});
    return p;
}

// the slice of a check recorded as "does not fire" (nullptr: decide it in-stream)
static double *chk_partials(pgmg_ctx *c, int np, int level)
{
    return chk_mode(c, level) == 0 ? chk_log(c, np, level, 0) : nullptr;
}

// ---------------------------------------------------------------------------
// kernel sequences
// ---------------------------------------------------------------------------
static unsigned *smooth_flags(pgmg_ctx *c, int l, int which)
{
    return c->flags + ((size_t)l * 2 + which) * kMaxSweeps;
}

static int timed_begin(pgmg_ctx *c, int slot);
static int timed_end(pgmg_ctx *c, int slot, int idx);
// k_post row range of a fused level: the strip, or on distributed levels below the finest
// the strip plus kPostExt rows past each edge (see enqueue_fused_level)
struct PostRows {
    int jc0, jc1, row_lo, row_hi;
};
static PostRows post_rows(const pgmg_ctx *c, int l)
{
    const Level &L = c->lv[l];
    PostRows r{L.lo / 2, (L.hi < L.N ? L.hi : L.N - 1) / 2, L.u0, L.u1};
    if (l > 0 && is_dist(c, l)) {
        const int r0 = std::max(L.lo - kPostExt, 0), r1 = std::min(L.hi + kPostExt, L.N - 1);
        r = {r0 / 2, r1 / 2, std::max(r0, 1), r1};
    }
    return r;
}

// partial sums a tile pass of bulk level l writes on this rank (0: no tile pass there);
// pre: the rank's coarse rows, post: its k_post rows (post_rows)
static int tile_np(const pgmg_ctx *c, int l, bool post)
{
    if (l < 1 || l >= c->nb) return 0;
    const Level &L = c->lv[l];
    if (!coarse_tile_ok(L.N, is_dist(c, l))) return 0;
    const int Nc = c->lv[l + 1].N;
    int jc0 = L.lo / 2, jc1 = (L.hi < L.N ? L.hi : L.N - 1) / 2;
    if (post) {
        const PostRows pr = post_rows(c, l);
        jc0 = pr.jc0;
        jc1 = pr.jc1;
    }
    return coarse_tile_blocks_rows(L.N, std::max(jc0, 1), std::min(jc1, Nc - 1));
}

template <class T> static int enqueue_children(pgmg_ctx *c, int l, int gamma);
template <class T> static int enqueue_cycle_t(pgmg_ctx *c, int l, int gamma, bool x0_zero);

// one JacobiSmoother::smooth(x = L.A, f = L.F, num_iter = v) on a bulk level
template <class T>
static int enqueue_smooth(pgmg_ctx *c, int l, int which, int v, bool x0_zero)
{
    Level &L = c->lv[l];
    const int S = v + 1;
    unsigned *D = smooth_flags(c, l, which);
    const bool fine = (l == 0);
    for (int k = 1; k <= S; ++k) {
        T *in = G<T>((k & 1) ? L.A : L.B);
        T *out = G<T>((k & 1) ? L.B : L.A);
        if (is_dist(c, l) && !(k == 1 && x0_zero)) {
            int e = c->comm->halo((k & 1) ? L.A : L.B, L, 1, c->s);
            if (e) return e;
        }
        SweepArgsT<T> a{};
        a.xin = (k == 1 && x0_zero) ? nullptr : in;
        a.f = G<T>(L.F);
        a.xout = out;
        a.partials = (k >= 2) ? c->partials : nullptr;
        a.skip = (k >= 2) ? &D[k - 1] : nullptr;
        a.reset = (k == 1) ? &D[1] : nullptr;
        a.stats = c->stats;
        a.hh = (T)L.hh;
        a.inv_hh = (T)L.ih;
        a.W = L.N;
        a.P = L.P;
        a.row0 = L.u0;
        a.row1 = L.u1;
        const int ev = (fine && a.partials == nullptr && !(k == 1 && x0_zero)) ? timed_begin(c, 0) : -1;
        launch_sweep(a, k == 1 && x0_zero, l == 0, c->s);
        int te = timed_end(c, 0, ev);
        if (te) return te;
        if (k >= 2) {
            int rpb, gx, gy;
            const int np = sweep_blocks(L.N, L.u0, L.u1, &rpb, &gx, &gy);
            FixupArgsT<T> f{};
            f.partials = c->partials;
            f.np = np;
            f.eps = c->cfg.eps;
            f.done_prev = &D[k - 1];
            f.done_next = &D[k];
            f.src = in;
            f.dst = out;
            f.stats = c->stats;
            f.W = L.N;
            f.P = L.P;
            f.row0 = L.u0;
            f.row1 = L.u1;
            f.global_sum = nullptr;
            if (is_dist(c, l)) {
                launch_sum_partials(c->partials, np, c->scalar, c->s);
                int e = c->comm->allreduce_sum(c->scalar, 1, c->s);
                if (e) return e;
                f.global_sum = c->scalar;
            }
            launch_fixup(f, c->s);
        }
    }
    if (S & 1) launch_copy_rows(G<T>(L.B), G<T>(L.A), L.N, L.P, L.u0, L.u1, c->s);
    return PGMG_OK;
}

template <class T>
static int enqueue_tail_t(pgmg_ctx *c, int gamma, bool x0_from_global, int visits = 1)
{
    Level &Lt = c->lv[c->nb];
    TailArgsT<T> t{};
    t.visits = visits;
    t.f_top = G<T>(Lt.F);
    t.e_top = G<T>(Lt.A);
    t.P_top = Lt.P;
    t.N_top = Lt.N;
    t.h_top = Lt.h;
    t.x0_from_global = x0_from_global ? 1 : 0;
    t.v1 = c->cfg.v1;
    t.v2 = c->cfg.v2;
    t.coarse_iter = c->cfg.coarse_iter;
    t.n_coarse = c->cfg.n_coarse;
    t.eps = c->cfg.eps;
    t.stats = c->stats;
    HIPC(launch_tail_gamma(t, gamma, c->s));
    return PGMG_OK;
}

int pgmg::enqueue_tail(pgmg_ctx *c, int gamma, bool x0_from_global)
{
    return c->fp32 ? enqueue_tail_t<float>(c, gamma, x0_from_global)
                   : enqueue_tail_t<double>(c, gamma, x0_from_global);
}

static int timed_begin(pgmg_ctx *c, int slot)
{
    auto &pool = c->tpool[slot];
    if (!(c->cfg.flags & PGMG_FLAG_TIME_FINE) || pool.used + 2 > (int)pool.ev.size()) return -1;
    HIPC(hipEventRecord(pool.ev[pool.used], c->s));
    return pool.used;
}

static int timed_end(pgmg_ctx *c, int slot, int idx)
{
    if (idx < 0) return PGMG_OK;
    auto &pool = c->tpool[slot];
    HIPC(hipEventRecord(pool.ev[idx + 1], c->s));
    pool.used = idx + 2;
    c->tbytes[slot] += g_last_launch.bytes;   // the launch just timed (LaunchNote)
    c->tkern[slot] = g_last_launch.kernel;
    return PGMG_OK;
}

// children of level l: gamma cycles on level l+1 (on rank 0 alone if it is gathered)
template <class T>
static int enqueue_children(pgmg_ctx *c, int l, int gamma)
{
    if (c->comm && l + 1 == c->comm->gathered_level())
        return c->comm->run_gathered(c, l + 1, gamma, gamma);
    // the tail level: the gamma visits (same right-hand side, each from the previous one's
    // result; the first from zero) in one launch -- at N = 32769 a W-cycle launches the tail
    // 3^9 times, one launch per visit cost ~8 % of its time in launch overhead
    if (l + 1 == c->nb && gamma > 1 && tuning_int("PGMG_TAIL_VISITS", 1) != 0)
        return enqueue_tail_t<T>(c, gamma, false, gamma);
    for (int i = 0; i < gamma; ++i) {
        int e = enqueue_cycle_t<T>(c, l + 1, gamma, i == 0);
        if (e) return e;
    }
    return PGMG_OK;
}

// global early-exit sum for a distributed level: local partial sum, then all ranks
static int global_sum(pgmg_ctx *c, int np, const double **out)
{
    launch_sum_partials(c->partials, np, c->scalar, c->s);
    int e = c->comm->allreduce_sum(c->scalar, 1, c->s);
    *out = c->scalar;
    return e;
}

// fused level (v1 = v2 = 1): k_pre (+fixup), children, k_post (+fixup)
// pin (F-cycle climb, x0_zero false): the level's x0 is the prolongation of level l+1's
// grid into a zeroed grid; k_pre computes it on the fly instead of reading L.A
template <class T>
static int enqueue_fused_level(pgmg_ctx *c, int l, int gamma, bool x0_zero, bool pin = false)
{
    Level &L = c->lv[l];
    Level &C = c->lv[l + 1];
    const bool dist = is_dist(c, l);
    // entered with x0 = 0: the pre-smoothed iterate is a function of f alone, so k_pre
    // does not store it and k_post recomputes it (x1 = J(0) is pointwise)
    const bool recomp = x0_zero && l > 0 && c->recompute;
    unsigned *fired = smooth_flags(c, l, 0) + (kMaxSweeps - 1);
    int e;
    // row strips, levels below the finest: k_post also computes kPostExt rows past each
    // strip edge (from deeper halos of f and phi, exchanged with the pre-smooth's anyway),
    // so the parent's prolongation reads this level's correction without an exchange
    const bool ext = dist && l > 0;
    if (dist) {
        if (!x0_zero && !pin && (e = c->comm->halo(L.A, L, 4, c->s))) return e;
        // f: 4 rows for k_pre, 3 + kPostExt for the extended k_post (RECOMP reads f 3 rows
        // past its first output row)
        if (l > 0 && (e = c->comm->halo(L.F, L, 3 + kPostExt, c->s))) return e;
    }
    PreArgsT<T> pa{};
    pa.x0 = G<T>(L.A);
    pa.f = G<T>(L.F);
    pa.x2 = recomp ? nullptr : G<T>(L.B);
    pa.fired = recomp ? fired : nullptr;
    pa.rc = G<T>(C.F);
    pa.partials = c->partials;
    pa.stats = c->stats;
    pa.hh = (T)L.hh;
    pa.ih = (T)L.ih;
    pa.N = L.N;
    pa.P = L.P;
    pa.Nc = C.N;
    pa.Pc = C.P;
    pa.jc0 = L.lo / 2;
    pa.jc1 = (L.hi < L.N ? L.hi : L.N - 1) / 2;
    pa.row_lo = L.u0;
    pa.row_hi = L.u1;
    // coarse rows this rank restricts into (its strip's rows; the fix-up honours them too)
    pa.rc_lo = pa.jc0 > 1 ? pa.jc0 : 1;
    pa.rc_hi = pa.jc1 < C.N - 1 ? pa.jc1 : C.N - 1;
    // level 0 with an analytic RHS, or the F climb's current level: regenerate f in-kernel
    pa.gfx = l == 0 ? c->rgfx : (l == c->gen_level ? c->lgfx : nullptr);
    pa.gsy = l == 0 ? c->rgsy : (l == c->gen_level ? c->lgsy : nullptr);
    pa.pin_ec = pin ? G<T>(C.A) : nullptr;
    FixArgsF fa{};
    fa.partials = c->partials;
    fa.np = fused_blocks(L.N, pa.jc0, pa.jc1);
    fa.eps = c->cfg.eps;
    fa.stats = c->stats;
    const bool fine = (l == 0);
    // speculative call: record the check (mode 0: no fix-up; 1: predicted to fire, the
    // one-sweep passes; 2: in-stream, logged for its norm)
    int mode = chk_mode(c, l);
    // V-cycles: a speculating level records "does not fire" up to its predicted crossing of
    // 100 eps (spec_mark_levels), in-stream after it
    if (mode == 0 && l > 0 && c->spec_gamma == 1 && !c->fspec && c->lvl_vis[l]++ >= c->lvl_kx[l])
        mode = 2;
    const int wm = w_visit_mode(c, l);
    const int visit = c->cur_visit;   // (the children's visits move it)
    if (wm >= 0) mode = wm;
    if (mode == 1 && (dist || pin || (x0_zero && !recomp))) mode = 2;
    // the small coarse levels (pgmg_coarse.hip): both passes, their predicted-to-fire
    // one-sweep forms and their in-stream rare paths as 2D LDS tiles; the checks' partial
    // count is the tile count
    // (row strips too: the tiles cover the rank's coarse rows, its interior rows own the check)
    const bool tile = recomp && !pin && pa.gfx == nullptr &&
                      !(c->cfg.flags & PGMG_FLAG_NO_CTILE) && coarse_tile_ok(L.N, dist) &&
                      pa.rc_hi > pa.rc_lo;
    CoarseArgsT<T> ca{};
    if (tile) {
        ca.jt0 = pa.rc_lo;
        ca.jt1 = pa.rc_hi;
        ca.own_lo = L.u0;
        ca.own_hi = L.u1;
        fa.np = coarse_tile_blocks_rows(L.N, ca.jt0, ca.jt1);
        ca.f = pa.f;
        ca.ec = G<T>(C.A);
        ca.rc = pa.rc;
        ca.x2 = G<T>(L.A);
        ca.stats = c->stats;
        ca.fired = fired;
        ca.pre_fired = fired;
        ca.hh = pa.hh;
        ca.ih = pa.ih;
        ca.N = L.N;
        ca.P = L.P;
        ca.Nc = C.N;
        ca.Pc = C.P;
    }
    double *lp = chk_log(c, fa.np, l, mode);
    if (lp) pa.partials = lp;
    int ev = fine ? timed_begin(c, 1) : -1;
    if (tile) {
        ca.partials = pa.partials;
        launch_pre_tile(ca, mode == 1 ? 1 : 0, c->s);
        HIPC(hipGetLastError());
    } else if ((e = mode == 1 ? launch_pre1(pa, x0_zero, c->s) : launch_pre(pa, x0_zero, fine, c->s))) {
        return e;
    }
    if ((e = timed_end(c, 1, ev))) return e;
    if (mode == 2) {
        if (lp) fa.partials = lp;
        if (tile) {
            ca.global_sum = nullptr;
            if (dist && (e = global_sum(c, fa.np, &ca.global_sum))) return e;
            ca.dec_partials = fa.partials;
            ca.dec_np = fa.np;
            ca.eps = fa.eps;
            launch_pre_tile(ca, 2, c->s);
            HIPC(hipGetLastError());
        } else {
            if (dist && (e = global_sum(c, fa.np, &fa.global_sum))) return e;
            if ((e = launch_pre_rare(fa, pa, x0_zero, c->s))) return e;
        }
        fa.partials = c->partials;
    }
    if ((e = enqueue_children<T>(c, l, gamma))) return e;
    // the correction of level l+1 is not exchanged: a distributed child's k_post computed
    // it kPostExt rows past its strip (a gathered child's is replicated)
    if (dist && !recomp && (e = c->comm->halo(L.B, L, ext ? 2 + kPostExt : 2, c->s))) return e;
    PostArgsT<T> po{};
    po.phi = G<T>(L.B);
    po.pre_fired = recomp ? fired : nullptr;
    po.ec = G<T>(C.A);
    po.f = G<T>(L.F);
    po.x2 = G<T>(L.A);
    po.partials = c->partials;
    po.stats = c->stats;
    po.hh = (T)L.hh;
    po.ih = (T)L.ih;
    po.N = L.N;
    po.P = L.P;
    po.Nc = C.N;
    po.Pc = C.P;
    po.jc0 = pa.jc0;
    po.jc1 = pa.jc1;
    po.row_lo = L.u0;
    po.row_hi = L.u1;
    if (ext) {   // rows [lo - kPostExt, hi + kPostExt) written, the strip's rows summed
        const PostRows pr = post_rows(c, l);
        po.jc0 = pr.jc0;
        po.jc1 = pr.jc1;
        po.row_lo = pr.row_lo;
        po.row_hi = pr.row_hi;
        po.sum_lo = L.u0;
        po.sum_hi = L.u1;
        fa.np = fused_blocks(L.N, po.jc0, po.jc1);
    }
    po.gfx = pa.gfx;
    po.gsy = pa.gsy;
    if (tile) {   // k_post's rows: the strip plus kPostExt rows (dist), its own rows summed
        ca.jt0 = std::max(po.jc0, 1);
        ca.jt1 = std::min(po.jc1, C.N - 1);
        ca.own_lo = po.row_lo;
        ca.own_hi = po.row_hi;
        ca.sum_lo = po.sum_hi > po.sum_lo ? po.sum_lo : po.row_lo;
        ca.sum_hi = po.sum_hi > po.sum_lo ? po.sum_hi : po.row_hi;
        fa.np = coarse_tile_blocks_rows(L.N, ca.jt0, ca.jt1);
    }
    c->cur_visit = visit;
    // speculative F-cycle followed by another: the finest k_post also restricts its result to
    // level 2 (the next F-cycle's first restriction step; only when its check is recorded
    // "does not fire", so x2 is the result); its 116-column tiles write more partials
    const bool r2 = fine && mode == 0 && c->fr2_want && !dist && !recomp && po.Po == 0 &&
                    c->nb >= 2 && !is_dist(c, 1) && tuning_int("PGMG_F_R2", 1) != 0;
    if (r2) fa.np = post_r2_blocks(L.N, po.jc0, po.jc1);
    lp = chk_log(c, fa.np, l, mode);
    if (lp) po.partials = lp;
    ev = fine ? timed_begin(c, 2) : -1;
    if (r2) {
        po.r2out = G<T>(c->lv[2].A);
        po.Pr2 = c->lv[2].P;
        po.Nr2 = c->lv[2].N;
        if ((e = launch_post_r2(po, c->s))) return e;
        c->fr2_made = true;
    } else if (tile) {
        ca.partials = po.partials;
        launch_post_tile(ca, mode == 1 ? 1 : 0, c->s);
        HIPC(hipGetLastError());
    } else if ((e = mode == 1 ? launch_post1(po, c->s) : launch_post(po, fine, c->s))) {
        return e;
    }
    if ((e = timed_end(c, 2, ev))) return e;
    if (mode == 2) {
        if (lp) fa.partials = lp;
        if (tile) {
            ca.global_sum = nullptr;
            if (dist && (e = global_sum(c, fa.np, &ca.global_sum))) return e;
            ca.dec_partials = fa.partials;
            ca.dec_np = fa.np;
            ca.eps = fa.eps;
            launch_post_tile(ca, 2, c->s);
            HIPC(hipGetLastError());
        } else {
            fa.global_sum = nullptr;
            if (dist && (e = global_sum(c, fa.np, &fa.global_sum))) return e;
            if ((e = launch_post_rare(fa, po, c->s))) return e;
        }
    }
    return PGMG_OK;
}

// ---------------------------------------------------------------------------
// Cross-cycle fusion of the finest level (v1 = v2 = 1): for n consecutive cycles
// the finest level runs k_pre, (children, k_postpre) x (n-1), children, k_post.
// k_postpre reads the pre-smoothed solution of cycle k from one level-0 buffer and
// writes that of cycle k+1 into the other, so the buffers alternate; at the end the
// solution is moved back under L.A by swapping the host pointers (B always mirrors
// A's boundary, so either may play either role).
//
// Row strips (level 0 distributed): every pass covers the rank's rows; before
// k_postpre one grouped exchange brings 6 halo rows of phi and 4 of the coarse
// correction; k_postpre also sums r(x2)^2 (the pre check of rare path 1, which
// restarts the pre-smooth from x1: J(x1) = x2), so ONE allreduce of three sums
// decides every rare path on every rank.  The rare paths rebuild their scratch
// iterate S on the rows the following k_pre reads (4 past the strip) from the
// exchanged halos instead of exchanging S.
// ---------------------------------------------------------------------------
struct StripRows {
    int jc0, jc1;         // coarse-row segments [jc0, jc1)
    int row_lo, row_hi;   // fine rows this rank writes
    int rc_lo, rc_hi;     // coarse rows this rank restricts into
    int x_lo, x_hi;       // rows of the rare-path scratch S (row_lo - 4 .. row_hi + 4)
};

static StripRows strip_rows(const Level &L, const Level &C)
{
    StripRows r;
    r.jc0 = L.lo / 2;
    r.jc1 = (L.hi < L.N ? L.hi : L.N - 1) / 2;
    r.row_lo = L.u0;
    r.row_hi = L.u1;
    r.rc_lo = r.jc0 > 1 ? r.jc0 : 1;
    r.rc_hi = r.jc1 < C.N - 1 ? r.jc1 : C.N - 1;
    r.x_lo = L.u0 - 4 > 1 ? L.u0 - 4 : 1;
    r.x_hi = L.u1 + 4 < L.N - 1 ? L.u1 + 4 : L.N - 1;
    return r;
}

template <class T>
static PreArgsT<T> make_pre(pgmg_ctx *c, const T *x0, T *x2)
{
    Level &L = c->lv[0], &C = c->lv[1];
    const StripRows sr = strip_rows(L, C);
    PreArgsT<T> pa{};
    pa.x0 = x0;
    pa.f = G<T>(L.F);
    pa.x2 = x2;
    pa.rc = G<T>(C.F);
    pa.partials = c->partials;
    pa.stats = c->stats;
    pa.hh = (T)L.hh;
    pa.ih = (T)L.ih;
    pa.N = L.N;
    pa.P = L.P;
    pa.Nc = C.N;
    pa.Pc = C.P;
    pa.jc0 = sr.jc0;
    pa.jc1 = sr.jc1;
    pa.row_lo = sr.row_lo;
    pa.row_hi = sr.row_hi;
    pa.rc_lo = sr.rc_lo;
    pa.rc_hi = sr.rc_hi;
    pa.gfx = c->rgfx;
    pa.gsy = c->rgsy;
    return pa;
}

template <class T>
static PostArgsT<T> make_post(pgmg_ctx *c, const T *phi, T *x2)
{
    Level &L = c->lv[0], &C = c->lv[1];
    const StripRows sr = strip_rows(L, C);
    PostArgsT<T> po{};
    po.phi = phi;
    po.ec = G<T>(C.A);
    po.f = G<T>(L.F);
    po.x2 = x2;
    po.partials = c->partials;
    po.stats = c->stats;
    po.hh = (T)L.hh;
    po.ih = (T)L.ih;
    po.N = L.N;
    po.P = L.P;
    po.Nc = C.N;
    po.Pc = C.P;
    po.jc0 = sr.jc0;
    po.jc1 = sr.jc1;
    po.row_lo = sr.row_lo;
    po.row_hi = sr.row_hi;
    po.gfx = c->rgfx;
    po.gsy = c->rgsy;
    return po;
}

// ---------------------------------------------------------------------------
// The carry (r06).  A call's cycles are cross-fused (k_pre, k_postpre ..., k_post), but a
// caller that runs one cycle per call, or checks the residual between calls (the reference
// harness, ParallelTestRunner.cu:172-173), pays the opening k_pre and the closing k_post of
// every call: two passes over the finest grid where a multi-cycle call runs one k_postpre.
// So a speculative V call on the context's own grids (one GPU) ends with the CARRY PASS: the
// last cycle's k_postpre, which stores x2 -- the call's result -- where a k_postpre stores the
// next cycle's pre-smoothed iterate x4, and the next cycle's restricted residual into lv[1].F
// as usual (so it moves the bytes of a k_postpre).  The pre-smooth's early-exit check is
// logged beside the call's own checks and validated with them; it never rolls the call back: a
// carry whose check could fire is dropped (carry_n[2]) and the next call runs its own k_pre.
// The next pgmg_vcycle on the same problem starts from the carry: no k_pre, straight into the
// coarse levels (MultiGrid.hpp:57-94 from line 69 on); its first finest pass is the RECOMPUTE
// FORM of k_postpre, which reads the previous call's x2 (lv[0].A), runs the carried
// pre-smooth again in registers -- the carry pass's own expressions on the same values, so
// bitwise the x4 it did not store -- and goes on as a k_postpre; it counts the carried
// pre-smooth's two sweeps (sw_adj).  A one-cycle call that took the carry and makes the next
// runs one finest pass, both forms at once.  Every entry that changes phi, f, eps, the flags or
// the cycle kind drops the carry (run_cycles takes it or drops it at every call); caller-owned
// arrays (pgmg_set_problem_device) never carry: the caller may change them between calls.  A
// rollback of the call that took a carry reruns from lv[0].A, which no pass of the call writes,
// with its own k_pre.  Cost: none in bytes (the carry pass and the recompute form each move a
// k_postpre's); two more Jacobi stages per point in the recompute form.
// ---------------------------------------------------------------------------
template <class T>
static int enqueue_cross_cycles(pgmg_ctx *c, int n, int gamma)
{
    Level &L = c->lv[0], &C = c->lv[1];
    const bool dist = is_dist(c, 0);
    const StripRows sr = strip_rows(L, C);
    Grid gA = L.A, gB = L.B, gS = c->S;
    T *A = G<T>(gA), *B = G<T>(gB);
    T *S = G<T>(gS);
    // speculative call: no rare path can run, so the scratch S is free and the level-0
    // buffers rotate through B and S; A (the call's input) is never written and a rollback
    // restarts from it
    const bool lean = c->lean;
    auto grid_of = [&](const T *p) -> const Grid * { return p == A ? &gA : p == B ? &gB : &gS; };
    // (an external input is followed by B: the first k_pre writes B, then B <-> S (lean) or
    // B <-> A, both free of the input; a carried input -- A itself -- is followed by B as well)
    auto next_of = [&](const T *p) -> T * { return lean ? (p == B ? S : B) : (p == B ? A : B); };
    // the caller's array (pgmg_set_problem_device) as the call's input / output
    const T *in = c->x_in != nullptr ? static_cast<const T *>(c->x_in) : A;
    T *const xout = static_cast<T *>(c->x_out);
    const int np = fused_blocks(L.N, sr.jc0, sr.jc1);
    const int npp = postpre_blocks(L.N, sr.jc0, sr.jc1);
    const int npp_rc = postpre_blocks(L.N, sr.jc0, sr.jc1, true);   // the recompute form's
    // the carry: made (the call ends with the carry pass) / taken (it starts from lv[0].A's
    // pre-smooth and lv[1].F, its first finest pass the recompute form -- a k_postpre, so a
    // call of one cycle takes it only when it also makes the next); both only on speculative
    // calls on the context's own grids, one GPU
    const bool make = c->carry_make && lean && !dist && xout == nullptr && !c->defer_post;
    const bool take = c->carry_use && lean && !dist && c->x_in == nullptr && (n > 1 || make);
    if (tuning_int("PGMG_ROLE_TRACE", 0))   // measurement build: which grids play which role
        fprintf(stderr, "roles A %p B %p S %p n %d take %d make %d\n", gA.base, gB.base, gS.base, n,
                (int)take, (int)make);
    c->carry_use = false;
    c->carry_made = false;
    c->carry_took = take;
    int sw_adj = take ? 2 : 0;   // the carried pre-smooth's two sweeps: counted by the next pass
    FixArgsF fa{};
    fa.partials = c->partials;
    fa.np = np;
    fa.eps = c->cfg.eps;
    fa.stats = c->stats;
    int e, ev;
    T *pr;   // pre-smoothed solution of the current cycle (a taken carry: the solution A)
    bool recompute = take;   // the next finest pass recomputes pr's pre-smooth
    if (take) {
        pr = A;
    } else {
        // cycle 1: pre-smooth (+ residual, restriction) A -> B
        if (dist && (e = c->comm->halo(gA, L, 4, c->s))) return e;
        PreArgsT<T> pa = make_pre<T>(c, in, B);
        if (c->x_in != nullptr) pa.Px = c->ext_P;
        double *lp = chk_partials(c, np, 0);
        if (lp) pa.partials = lp;
        ev = timed_begin(c, 1);
        if ((e = launch_pre(pa, false, true, c->s))) return e;
        if ((e = timed_end(c, 1, ev))) return e;
        if (!lp) {
            if (dist && (e = global_sum(c, np, &fa.global_sum))) return e;
            launch_pre_fixup(fa, pa, false, c->s);
            fa.global_sum = nullptr;
        }
        pr = B;
    }
    // its halo rows (6 for k_postpre, 2 for the last k_post) are final now and read only
    // after the whole coarse hierarchy: the exchange runs on the comm's side stream
    // meanwhile (the coarse correction's halo rows are computed locally, kPostExt)
    if (dist && (e = c->comm->halo_begin(*grid_of(pr), L, 6, c->s))) return e;
    if ((e = enqueue_children<T>(c, 0, gamma))) return e;
    auto postpre_args = [&](T *phi, T *x4) {
        PostPreArgsT<T> q{};
        q.phi = phi;
        q.ec = G<T>(C.A);
        q.f = G<T>(L.F);
        q.x4 = x4;
        q.rc = G<T>(C.F);
        q.gfx = c->rgfx;
        q.gsy = c->rgsy;
        q.stats = c->stats;
        q.hh = (T)L.hh;
        q.ih = (T)L.ih;
        q.N = L.N;
        q.P = L.P;
        q.Nc = C.N;
        q.Pc = C.P;
        q.jc0 = sr.jc0;
        q.jc1 = sr.jc1;
        q.row_lo = sr.row_lo;
        q.row_hi = sr.row_hi;
        q.rc_lo = sr.rc_lo;
        q.rc_hi = sr.rc_hi;
        q.fast = (c->cfg.flags & PGMG_FLAG_FAST) != 0 && !dist;
        q.sw_adj = sw_adj;
        sw_adj = 0;
        q.recompute = recompute ? 1 : 0;
        recompute = false;
        return q;
    };
    for (int k = 1; k < n; ++k) {
        T *nx = next_of(pr);
        if (dist && (e = c->comm->halo_end(c->s))) return e;
        const int nq = recompute ? npp_rc : npp;
        PostPreArgsT<T> q = postpre_args(pr, nx);
        q.partials1 = lean ? chk_partials(c, nq, 0) : c->partials;
        q.partials2 = lean ? chk_partials(c, nq, 0) : c->partials2;
        q.partials3 = (dist && !lean) ? c->partials3 : nullptr;   // lean: no rare path runs
        const int slot = q.recompute ? 5 : 3;   // (the recompute form: its own timed slot)
        ev = timed_begin(c, slot);
        if ((e = launch_postpre(q, c->s))) return e;
        if ((e = timed_end(c, slot, ev))) return e;
        const double *g3 = nullptr;   // all-rank {post, pre, pre-from-x1} sums
        if (lean) {
            pr = nx;
            if (dist && (e = c->comm->halo_begin(*grid_of(pr), L, 6, c->s))) return e;
            if ((e = enqueue_children<T>(c, 0, gamma))) return e;
            continue;
        }
        if (dist) {
            launch_sum_partials(q.partials1, npp, c->scalar, c->s);
            launch_sum_partials(q.partials2, npp, c->scalar + 1, c->s);
            launch_sum_partials(q.partials3, npp, c->scalar + 2, c->s);
            if ((e = c->comm->allreduce_sum(c->scalar, 3, c->s))) return e;
            g3 = c->scalar;
        }
        launch_postpre_decide(q.partials1, q.partials2, q.stats, npp, g3, c->cfg.eps, c->ppflags,
                              c->s);
        // rare path 1 (post check fired): S = x1 of the post-smooth, then a full
        // pre-smooth from S (conditional k_pre + its own fix-up)
        PostArgsT<T> po = make_post<T>(c, pr, S);
        po.row_lo = sr.x_lo;
        po.row_hi = sr.x_hi;
        FixArgsF f1 = fa;
        f1.cond = &c->ppflags[0];
        f1.force = 1;
        f1.stats = nullptr;
        launch_post_fixup(f1, po, c->s);
        PreArgsT<T> p1 = make_pre<T>(c, S, nx);
        p1.cond = &c->ppflags[0];
        if ((e = launch_pre(p1, false, false, c->s))) return e;
        FixArgsF f1b = fa;
        f1b.cond = &c->ppflags[0];
        f1b.global_sum = dist ? c->scalar + 2 : nullptr;
        launch_pre_fixup(f1b, p1, false, c->s);
        // rare path 2 (only the pre check fired): S = x2 of the post-smooth, then the
        // pre-smooth result is J(S) and rc = R r(J(S))
        PostArgsT<T> p2 = make_post<T>(c, pr, S);
        if (dist) {   // x2 on the strip and 4 rows past it, from the exchanged halos
            p2.row_lo = sr.x_lo;
            p2.row_hi = sr.x_hi;
            p2.fix_sweeps = 2;
            FixArgsF f2a = fa;
            f2a.cond = &c->ppflags[1];
            f2a.force = 1;
            f2a.stats = nullptr;
            launch_post_fixup(f2a, p2, c->s);
        } else {
            p2.cond = &c->ppflags[1];
            p2.stats = nullptr;
            if ((e = launch_post(p2, false, c->s))) return e;
        }
        PreArgsT<T> p3 = make_pre<T>(c, S, nx);
        FixArgsF f2 = fa;
        f2.cond = &c->ppflags[1];
        f2.force = 1;
        f2.stats = nullptr;
        launch_pre_fixup(f2, p3, false, c->s);
        pr = nx;   // final after the rare paths
        if (dist && (e = c->comm->halo_begin(*grid_of(pr), L, 6, c->s))) return e;
        if ((e = enqueue_children<T>(c, 0, gamma))) return e;
    }
    // last cycle: post-smooth
    if (c->defer_post) {   // enqueued by run_cycles_spec after the validation
        c->pend_pr = pr;
        return PGMG_OK;
    }
    // the solution's buffer becomes L.A (every level-0 grid mirrors the boundary, so any may
    // play any role); an external output holds the solution instead (the level-0 grids keep
    // their roles)
    auto set_roles = [&](const T *sol) {
        const Grid *all[3] = {&gA, &gB, &gS};
        std::vector<Grid> rest;
        for (const Grid *g : all)
            if (g != grid_of(sol)) rest.push_back(*g);
        L.A = *grid_of(sol);
        L.B = rest[0];
        c->S = rest[1];
    };
    if (make) {
        // the carry pass: x2 (the result) into a grid that is neither the input A nor pr (pr is
        // A itself when this one pass also takes the carry); its post check is this call's, its
        // pre check the carry's
        T *const out = (pr == B) ? S : B;
        const int nq = recompute ? npp_rc : npp;
        PostPreArgsT<T> q = postpre_args(pr, nullptr);
        q.x2 = out;
        q.sw_adj -= 2;   // the pre-smooth's sweeps count in the call that uses them
        q.partials1 = chk_partials(c, nq, 0);
        q.partials2 = chk_log(c, nq, 0, 0);
        c->carry_chk = (int)c->chks.size() - 1;
        if (q.partials1 == nullptr || q.partials2 == nullptr) return set_err(PGMG_ERR_STATE, "carry pass: check log");
        ev = timed_begin(c, 4);
        if ((e = launch_postpre(q, c->s))) return e;
        if ((e = timed_end(c, 4, ev))) return e;
        set_roles(out);
        c->carry_made = true;
        return PGMG_OK;
    }
    if (recompute) return set_err(PGMG_ERR_STATE, "a taken carry without a k_postpre");
    T *out = xout != nullptr ? xout : next_of(pr);
    if (dist && (e = c->comm->halo_end(c->s))) return e;
    PostArgsT<T> po = make_post<T>(c, pr, out);
    if (xout != nullptr) po.Po = c->ext_P;
    po.sw_adj = sw_adj;
    double *lp = chk_partials(c, np, 0);
    if (lp) po.partials = lp;
    ev = timed_begin(c, 2);
    if ((e = launch_post(po, true, c->s))) return e;
    if ((e = timed_end(c, 2, ev))) return e;
    if (!lp) {
        if (dist && (e = global_sum(c, np, &fa.global_sum))) return e;
        launch_post_fixup(fa, po, c->s);
    }
    if (xout != nullptr) {
    } else if (lean) {
        set_roles(out);
    } else if (out != A) {
        std::swap(L.A, L.B);
    }
    return PGMG_OK;
}

// MultigridSolver::v_cycle / w_cycle (MultiGrid.hpp:57-136) on level l
template <class T>
static int enqueue_cycle_t(pgmg_ctx *c, int l, int gamma, bool x0_zero)
{
    if (l == c->nb) return enqueue_tail_t<T>(c, gamma, !x0_zero);
    if (c->fused) return enqueue_fused_level<T>(c, l, gamma, x0_zero);
    Level &L = c->lv[l];
    Level &C = c->lv[l + 1];
    const bool dist = is_dist(c, l);
    int e;
    if (dist && l > 0 && (e = c->comm->halo(L.F, L, 1, c->s))) return e;
    e = enqueue_smooth<T>(c, l, 0, c->cfg.v1, x0_zero);
    if (e) return e;
    if (dist && (e = c->comm->halo(L.A, L, 2, c->s))) return e;
    ResRestrictArgsT<T> r{};
    r.x = G<T>(L.A);
    r.f = G<T>(L.F);
    r.rc = G<T>(C.F);
    r.inv_hh = (T)L.ih;
    r.Wf = L.N;
    r.Pf = L.P;
    r.Wc = C.N;
    r.Pc = C.P;
    // coarse rows jc whose centre fine row 2jc this rank owns
    r.jc0 = L.lo / 2 > 1 ? L.lo / 2 : 1;
    r.jc1 = (L.hi + 1) / 2 < C.N - 1 ? (L.hi + 1) / 2 : C.N - 1;
    launch_res_restrict(r, c->s);
    if ((e = enqueue_children<T>(c, l, gamma))) return e;
    if (dist && is_dist(c, l + 1) && (e = c->comm->halo(C.A, C, 2, c->s))) return e;
    ProlongArgsT<T> p{};
    p.c = G<T>(C.A);
    p.fine = G<T>(L.A);
    p.Wf = L.N;
    p.Pf = L.P;
    p.Wc = C.N;
    p.Pc = C.P;
    p.row0 = L.u0 > 2 ? L.u0 : 2;
    p.row1 = L.u1 < L.N - 1 ? L.u1 : L.N - 1;
    if (p.row1 > p.row0) launch_prolong(p, c->s);
    return enqueue_smooth<T>(c, l, 1, c->cfg.v2, false);
}

int pgmg::enqueue_cycle(pgmg_ctx *c, int l, int gamma, bool x0_zero)
{
    return c->fp32 ? enqueue_cycle_t<float>(c, l, gamma, x0_zero)
                   : enqueue_cycle_t<double>(c, l, gamma, x0_zero);
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char *pgmg_last_error(void) { return g_err.c_str(); }
const char *pgmg_version(void) { return "pgmg 0.2 (gfx950, fp64 | fp32, row-strip RCCL)"; }

int pgmg_config_default(pgmg_config *cfg, int N)
{
    if (!cfg) return set_err(PGMG_ERR_ARG, "null cfg");
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->N = N;
    cfg->v1 = 1;           // MultiGrid.hpp:15
    cfg->v2 = 1;           // MultiGrid.hpp:16
    cfg->coarse_iter = 10; // MultiGrid.hpp:61
    cfg->n_coarse = 5;     // MultiGrid.hpp:19
    cfg->alpha = 3;        // 2_part_MG/main.cpp:15
    cfg->eps = 1e-7;       // 2_part_MG/main.cpp:12
    cfg->a = 1.0;          // globals.cpp:2-4
    cfg->p = 1.0;
    cfg->q = 1.0;
    cfg->tail_n = kTailMaxN;
    cfg->device = 0;
    cfg->flags = 0;
    cfg->rank = 0;
    cfg->world = 1;
    cfg->nccl_unique_id = nullptr;
    cfg->gather_n = 1025;
    cfg->precision = PGMG_PRECISION_FP64;
    cfg->cross_min_n = 2049;
    cfg->spec_segment = 0;
    cfg->comm_timeout_s = 600.0;
    cfg->h0 = 0.0;
    return PGMG_OK;
}

static bool is_pow2p1(int N)
{
    if (N < 3) return false;
    const int g = N - 1;
    return (g & (g - 1)) == 0;
}

int pgmg_destroy(pgmg_ctx *c)
{
    if (!c) return PGMG_OK;
    if (c->s) (void)hipStreamSynchronize(c->s);
    if (c->gexec) (void)hipGraphExecDestroy(c->gexec);
    for (auto &L : c->lv) {
        free_grid(L.A);
        free_grid(L.B);
        free_grid(L.F);
    }
    if (c->partials) (void)hipFree(c->partials);
    if (c->partials2) (void)hipFree(c->partials2);
    if (c->partials3) (void)hipFree(c->partials3);
    if (c->rhs_tab) (void)hipFree(c->rhs_tab);
    if (c->fmg_gtab) (void)hipFree(c->fmg_gtab);
    if (c->uflags) (void)hipFree(c->uflags);
    if (c->pin) (void)hipHostFree(c->pin);
    if (c->plog) (void)hipFree(c->plog);
    if (c->chk_norm) (void)hipFree(c->chk_norm);
    if (c->mark_dev) (void)hipFree(c->mark_dev);
    if (c->stats_bk) (void)hipFree(c->stats_bk);
    free_grid(c->bk);
    free_grid(c->ftop);
    if (c->ppflags) (void)hipFree(c->ppflags);
    free_grid(c->S);
    free_grid(c->Ffmg);
    for (auto &g : c->Ffmg_l) free_grid(g);
    if (c->fmg_tab) (void)hipFree(c->fmg_tab);
    if (c->flags) (void)hipFree(c->flags);
    if (c->stats) (void)hipFree(c->stats);
    if (c->scalar) (void)hipFree(c->scalar);
    for (auto &pool : c->tpool)
        for (auto e : pool.ev) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev_caller) (void)hipEventDestroy(c->ev_caller);
    delete c->comm;
    if (c->s) (void)hipStreamDestroy(c->s);
    delete c;
    return PGMG_OK;
}

int pgmg_create(pgmg_ctx **out, const pgmg_config *cfg)
{
    if (!out || !cfg) return set_err(PGMG_ERR_ARG, "null argument");
    *out = nullptr;
    if (!is_pow2p1(cfg->N) || cfg->N < 5)
        return set_err(PGMG_ERR_ARG, "N must be 2^k + 1 with N >= 5 (2_part_MG/main.cpp:6)");
    if (cfg->v1 < 0 || cfg->v2 < 0 || cfg->v1 + 1 >= kMaxSweeps || cfg->v2 + 1 >= kMaxSweeps ||
        cfg->coarse_iter < 0 || cfg->n_coarse < 3 || cfg->alpha < 1)
        return set_err(PGMG_ERR_ARG, "bad smoother/cycle parameters");
    if (cfg->world < 1 || cfg->rank < 0 || cfg->rank >= cfg->world)
        return set_err(PGMG_ERR_ARG, "bad rank/world");
    if (cfg->precision != PGMG_PRECISION_FP64 && cfg->precision != PGMG_PRECISION_FP32)
        return set_err(PGMG_ERR_ARG, "precision must be PGMG_PRECISION_FP64 or _FP32");
    if (!(cfg->h0 >= 0.0) || !std::isfinite(cfg->h0))
        return set_err(PGMG_ERR_ARG, "h0 must be finite and >= 0 (0: a / (N - 1))");
    if (cfg->flags & PGMG_FLAGS_RETIRED)
        return set_err(PGMG_ERR_ARG, "retired PGMG_FLAG_* bit (8192 / 16384; include/pgmg.h): "
                                     "PGMG_FLAG_NO_SPEC_FIRE is 32768 since r04");
    int ndev = 0;
    HIPC(hipGetDeviceCount(&ndev));
    if (cfg->device < 0 || cfg->device >= ndev) return set_err(PGMG_ERR_ARG, "bad device ordinal");
    HIPC(hipSetDevice(cfg->device));

    pgmg_ctx *c = new pgmg_ctx();
    c->cfg = *cfg;
    c->fp32 = cfg->precision == PGMG_PRECISION_FP32;
    // one GPU: the big grids from shuffled physical chunks (vmm_alloc); row strips keep plain
    // device memory (what RCCL's transfers were validated on)
    c->shuffle = cfg->world <= 1 && !(cfg->flags & PGMG_FLAG_NO_SHUFFLE);
    int tail_n = cfg->tail_n;
    if (tail_n > kTailMaxN) tail_n = kTailMaxN;
    if (tail_n < cfg->n_coarse) tail_n = cfg->n_coarse;
    c->cfg.tail_n = tail_n;

    // level sizes: bulk while N > tail_n, then the tail's top level
    int N = cfg->N;
    // MultiGridTestRunner.hpp:131, or the caller's h (MultiGrid.hpp:57's argument)
    double h = cfg->h0 > 0.0 ? cfg->h0 : cfg->a / (N - 1);
    for (;;) {
        Level L;
        L.N = N;
        L.es = c->fp32 ? 4 : 8;
        L.P = c->fp32 ? pitch_elems<float>(N) : pitch_elems<double>(N);
        L.h = h;
        L.hh = h * h;
        L.ih = 1.0 / (h * h);
        L.lo = 0;
        L.hi = N;
        L.u0 = 1;
        L.u1 = N - 1;
        c->lv.push_back(L);
        if (N <= tail_n || N <= cfg->n_coarse) break;
        N = (N - 1) / 2 + 1;
        h = 2 * h;  // MultiGrid.hpp:83
    }
    c->nb = (int)c->lv.size() - 1;

    int rc = PGMG_OK;
    if (cfg->world > 1) {
        c->comm = Comm::create(c, &rc);
        if (!c->comm) {
            pgmg_destroy(c);
            return rc;
        }
        rc = c->comm->plan(c);
        if (rc == 1) {  // grid too small to split: every rank runs an independent replica
            delete c->comm;
            c->comm = nullptr;
            rc = PGMG_OK;
        }
    }

    // (measurement build: PGMG_DUMMY_MB a dummy buffer of that size before every level grid:
    // placement probes)
    Grid dummy;
    if (tuning_int("PGMG_DUMMY_MB", 0) > 0) {
        Level Ld = c->lv[0];
        Ld.hi = Ld.lo + (int)(((size_t)tuning_int("PGMG_DUMMY_MB", 0) << 20) / ((size_t)Ld.P * Ld.es));
        rc = alloc_grid(dummy, Ld);
    }
    for (int l = 0; l < (int)c->lv.size() && rc == PGMG_OK; ++l) {
        Level &L = c->lv[l];
        if (!L.on_this_rank) continue;
        // (measurement build: PGMG_GRID_STAGGER bytes times a per-grid index of level 0)
        const size_t st = l == 0 ? (size_t)tuning_int("PGMG_GRID_STAGGER", 0) : 0;
        rc = alloc_grid(L.A, L, 0 * st, c->shuffle);
        if (rc == PGMG_OK) rc = alloc_grid(L.F, L, 1 * st, c->shuffle);
        if (rc == PGMG_OK && l < c->nb) rc = alloc_grid(L.B, L, 2 * st, c->shuffle);
    }
    c->fused = cfg->v1 == 1 && cfg->v2 == 1 && !(cfg->flags & PGMG_FLAG_UNFUSED);
    c->recompute = !(cfg->flags & PGMG_FLAG_NO_RECOMPUTE);
    {
        const int cross_min = cfg->cross_min_n > 0 ? cfg->cross_min_n : 2049;
        c->cross = c->fused && c->nb >= 1 && c->lv[0].N >= cross_min &&
                   !(cfg->flags & PGMG_FLAG_NO_CROSS);
    }
    int maxblocks = 256;
    for (int l = 0; l < c->nb; ++l) {
        int rpb, gx, gy;
        const Level &L = c->lv[l];
        int nbk = sweep_blocks(L.N, L.u0, L.u1, &rpb, &gx, &gy);
        if (nbk > maxblocks) maxblocks = nbk;
        nbk = fused_blocks(L.N, L.lo / 2, (L.hi < L.N ? L.hi : L.N - 1) / 2);
        if (nbk > maxblocks) maxblocks = nbk;
        const PostRows pr = post_rows(c, l);
        nbk = fused_blocks(L.N, pr.jc0, pr.jc1);
        if (nbk > maxblocks) maxblocks = nbk;
        nbk = postpre_blocks(L.N, L.lo / 2, (L.hi < L.N ? L.hi : L.N - 1) / 2);
        if (nbk > maxblocks) maxblocks = nbk;
        nbk = postpre_blocks(L.N, L.lo / 2, (L.hi < L.N ? L.hi : L.N - 1) / 2, true);
        if (nbk > maxblocks) maxblocks = nbk;
        nbk = std::max(tile_np(c, l, false), tile_np(c, l, true));
        if (nbk > maxblocks) maxblocks = nbk;
        // k_post_r2 (the finest k_post of consecutive F-cycles, 116-column stride): its
        // partials may land in c->partials when the check log is full
        if (l == 0) {
            nbk = post_r2_blocks(L.N, L.lo / 2, (L.hi < L.N ? L.hi : L.N - 1) / 2);
            if (nbk > maxblocks) maxblocks = nbk;
        }
    }
    const size_t st0 = (size_t)tuning_int("PGMG_GRID_STAGGER", 0);
    if (rc == PGMG_OK && c->cross) rc = alloc_grid(c->S, c->lv[0], 3 * st0, c->shuffle);
    (void)dummy;   // (the probe's dummy buffer stays allocated: the context leaks it)
    // partial sums of k_postpre's second and third checks (cross-cycle fusion, and the
    // F-cycle's fused smooth(3)), its decision flags
    if (rc == PGMG_OK && (hipMalloc((void **)&c->partials2, sizeof(double) * maxblocks) != hipSuccess ||
                          hipMalloc((void **)&c->partials3, sizeof(double) * maxblocks) != hipSuccess ||
                          hipMalloc((void **)&c->ppflags, 4 * sizeof(unsigned)) != hipSuccess))
        rc = set_err(PGMG_ERR_NOMEM, "cross-cycle buffers");
    c->partials_cap = maxblocks;
    if (rc == PGMG_OK && hipMalloc((void **)&c->partials, sizeof(double) * maxblocks) != hipSuccess)
        rc = set_err(PGMG_ERR_NOMEM, "partials");
    const size_t nflags = (size_t)(c->lv.size() + 1) * 2 * kMaxSweeps;
    if (rc == PGMG_OK && hipMalloc((void **)&c->flags, sizeof(unsigned) * nflags) != hipSuccess)
        rc = set_err(PGMG_ERR_NOMEM, "flags");
    if (rc == PGMG_OK && hipMalloc((void **)&c->stats, 4 * sizeof(unsigned long long)) != hipSuccess)
        rc = set_err(PGMG_ERR_NOMEM, "stats");
    if (rc == PGMG_OK && hipMalloc((void **)&c->scalar, 8 * sizeof(double)) != hipSuccess)
        rc = set_err(PGMG_ERR_NOMEM, "scalar");
    if (rc == PGMG_OK) {
        if (hipMemset(c->flags, 0, sizeof(unsigned) * nflags) != hipSuccess ||
            hipMemset(c->stats, 0, 4 * sizeof(unsigned long long)) != hipSuccess ||
            hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_caller, hipEventDisableTiming) != hipSuccess)
            rc = set_err(PGMG_ERR_HIP, "stream/event setup failed");
    }
    if (rc == PGMG_OK && (cfg->flags & PGMG_FLAG_TIME_FINE)) {
        for (auto &pool : c->tpool) {
            pool.ev.resize(512);
            for (auto &e : pool.ev)
                if (hipEventCreate(&e) != hipSuccess) rc = set_err(PGMG_ERR_HIP, "event pool");
        }
    }
    if (rc == PGMG_OK && c->comm) rc = c->comm->setup(c);
    c->spec = c->fused && (c->cross || c->comm != nullptr) && !(cfg->flags & PGMG_FLAG_EXACT_DIST);
    if (rc != PGMG_OK) {
        pgmg_destroy(c);
        return rc;
    }
    *out = c;
    return PGMG_OK;
}

// host sine tables -> bit-identical compute_rhs on the device
static void sine_tables(const pgmg_config &cfg, int N, double h, std::vector<double> &sx,
                        std::vector<double> &sy, double &factor)
{
    factor = (M_PI * M_PI / (cfg.a * cfg.a)) * (cfg.p * cfg.p + cfg.q * cfg.q);
    sx.resize(N);
    sy.resize(N);
    for (int i = 0; i < N; ++i) {
        const double x = i * h;
        sx[i] = std::sin(cfg.p * M_PI * x / cfg.a);
        sy[i] = std::sin(cfg.q * M_PI * x / cfg.a);
    }
}

}  // extern "C"

// rows [r0, r1) of a dense host array (pitch N) -> grid g (the context's element type)
static int upload_rows(pgmg_ctx *c, const Level &L, const Grid &g, const double *host, int r0,
                       int r1)
{
    const int N = L.N;
    const size_t rows = (size_t)(r1 - r0);
    if (!c->fp32 && !is_vmm(g.base)) {
        HIPC(hipMemcpy2D(row_ptr(g, r0, L.P, 8), L.P * sizeof(double), host + (size_t)r0 * N,
                         N * sizeof(double), N * sizeof(double), rows, hipMemcpyHostToDevice));
        return PGMG_OK;
    }
    // fp32 (or a shuffled grid): stage the doubles on the device, narrow / place them there
    double *d = nullptr;
    HIPC(hipMalloc((void **)&d, rows * N * sizeof(double)));
    HIPC(hipMemcpy(d, host + (size_t)r0 * N, rows * N * sizeof(double), hipMemcpyHostToDevice));
    if (c->fp32) launch_from_double(d - (size_t)r0 * N, N, G<float>(g), L.P, r0, r1, c->s);
    else launch_from_double(d - (size_t)r0 * N, N, G<double>(g), L.P, r0, r1, c->s);
    HIPC(hipGetLastError());
    PGMG_TRY(stream_wait(c));
    HIPC(hipFree(d));
    return PGMG_OK;
}

int pgmg::download_grid(pgmg_ctx *c, const void *o, int P, int N, double *host)
{
    if (!c->fp32 && is_vmm(o)) {   // a shuffled grid: widen/copy on the device, then 1D
        double *d = nullptr;
        HIPC(hipMalloc((void **)&d, (size_t)N * N * sizeof(double)));
        launch_to_double(static_cast<const double *>(o), P, d, N, 0, N, c->s);
        HIPC(hipGetLastError());
        HIPC(hipMemcpyAsync(host, d, (size_t)N * N * sizeof(double), hipMemcpyDeviceToHost, c->s));
        PGMG_TRY(stream_wait(c));
        HIPC(hipFree(d));
        return PGMG_OK;
    }
    if (!c->fp32) {
        HIPC(hipMemcpy2DAsync(host, N * sizeof(double), o, P * sizeof(double), N * sizeof(double),
                              N, hipMemcpyDeviceToHost, c->s));
        PGMG_TRY(stream_wait(c));
        return PGMG_OK;
    }
    double *d = nullptr;
    HIPC(hipMalloc((void **)&d, (size_t)N * N * sizeof(double)));
    launch_to_double(static_cast<const float *>(o), P, d, N, 0, N, c->s);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(host, d, (size_t)N * N * sizeof(double), hipMemcpyDeviceToHost, c->s));
    PGMG_TRY(stream_wait(c));
    HIPC(hipFree(d));
    return PGMG_OK;
}

// statistics and speculation history of a new problem
static int problem_reset(pgmg_ctx *c)
{
    HIPC(hipMemset(c->stats, 0, 4 * sizeof(unsigned long long)));
    HIPC(hipDeviceSynchronize());
    c->have_problem = true;
    c->carry = false;
    c->spec_off = false;   // a new problem: speculate again, every level
    c->fspec_off = false;
    c->lvl_exact.assign(c->nb + 1, 0);
    c->lvl_fire.assign(c->nb + 1, 0);
    c->lvl_fire_block.assign(c->nb + 1, 0);
    c->lvl_fire_try.assign(c->nb + 1, 0.0);
    c->lvl_kx.assign(c->nb + 1, 0);
    c->lvl_vis.assign(c->nb + 1, 0);
    c->wmax.clear();
    c->wmin.clear();
    c->wrho.clear();
    c->wplan_gamma = 0;
    c->wplan_off = false;
    c->lvl_hist.assign(c->nb + 1, std::vector<double>());
    return PGMG_OK;
}

// level-0 right-hand side rows [r0, r1): the host array f, or (f = NULL) the analytic RHS of
// compute_rhs, stored and, unless PGMG_FLAG_STORED_RHS, regenerated by the level-0 passes
static int setup_rhs(pgmg_ctx *c, const double *f, int r0, int r1)
{
    Level &L = c->lv[0];
    const int N = L.N;
    int e;
    c->gen_rhs = false;
    c->rgfx = c->rgsy = nullptr;
    if (f) {
        if ((e = upload_rows(c, L, L.F, f, r0, r1))) return e;
    } else {
        std::vector<double> sx, sy;
        double factor;
        sine_tables(c->cfg, N, L.h, sx, sy, factor);
        double *d = nullptr;
        HIPC(hipMalloc((void **)&d, 2 * N * sizeof(double)));
        HIPC(hipMemcpy(d, sx.data(), N * sizeof(double), hipMemcpyHostToDevice));
        HIPC(hipMemcpy(d + N, sy.data(), N * sizeof(double), hipMemcpyHostToDevice));
        if (c->fp32) launch_rhs(G<float>(L.F), d, d + N, factor, N, L.P, r0, r1, c->s);
        else launch_rhs(G<double>(L.F), d, d + N, factor, N, L.P, r0, r1, c->s);
        HIPC(hipGetLastError());
        PGMG_TRY(stream_wait(c));
        HIPC(hipFree(d));
        // tables for regenerating f inside the level-0 passes: fx[i] = factor * sx[i]
        // (the first product of k_rhs's factor * sx[i] * sy[j]) and sy[j], zero-padded
        // past the grid (columns / rows -8 .. N + 1024 / N + 16, like the stored f's
        // zero padding)
        if (!(c->cfg.flags & PGMG_FLAG_STORED_RHS)) {
            const int nx = 8 + N + 1024, ny = 8 + N + 16;
            std::vector<double> tab((size_t)nx + ny, 0.0);
            for (int i = 0; i < N; ++i) tab[8 + i] = factor * sx[i];
            for (int j = 0; j < N; ++j) tab[(size_t)nx + 8 + j] = sy[j];
            if (!c->rhs_tab) HIPC(hipMalloc((void **)&c->rhs_tab, tab.size() * sizeof(double)));
            HIPC(hipMemcpy(c->rhs_tab, tab.data(), tab.size() * sizeof(double),
                           hipMemcpyHostToDevice));
            c->gfx = c->rhs_tab + 8;
            c->gsy = c->rhs_tab + nx + 8;
            c->gen_rhs = true;
            c->rgfx = c->gfx;
            c->rgsy = c->gsy;
        }
    }
    return PGMG_OK;
}

extern "C" {

int pgmg_set_problem(pgmg_ctx *c, const double *phi0, const double *f)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    Level &L = c->lv[0];
    const int N = L.N;
    if (!L.on_this_rank) return set_err(PGMG_ERR_STATE, "level 0 not on this rank");
    // owned rows + the halo rows the fused passes read (every rank has the full host arrays)
    const int r0 = L.lo - kHalo > 0 ? L.lo - kHalo : 0;
    const int r1 = L.hi + kHalo < N ? L.hi + kHalo : N;
    const size_t rows = (size_t)(r1 - r0);
    const size_t pitch = (size_t)L.P * L.es, width = (size_t)N * L.es;
    int e;
    PGMG_TRY(stream_wait(c));
    c->ext_phi = nullptr;   // host arrays: the problem lives in the context again
    c->ext_f = nullptr;
    // phi (and its boundary copy in the ping-pong buffer B)
    // (the rows r0 .. r1 of a level-0 grid are one contiguous range, padding included: zeroed
    // and copied whole with 1D operations, which shuffled grids accept)
    (void)width;
    if (phi0) {
        if ((e = upload_rows(c, L, L.A, phi0, r0, r1))) return e;
    } else {
        HIPC(hipMemset(row_ptr(L.A, r0, L.P, L.es), 0, pitch * rows));
    }
    auto mirror = [&](const Grid &g) -> int {
        HIPC(hipMemcpy(row_ptr(g, r0, L.P, L.es), row_ptr(L.A, r0, L.P, L.es), pitch * rows,
                       hipMemcpyDeviceToDevice));
        return PGMG_OK;
    };
    if (c->nb > 0) PGMG_TRY(mirror(L.B));
    // the cross-cycle rare-path scratch S mirrors phi's boundary too (its passes never
    // write boundary rows/columns, the k_pre that reads it passes them through)
    if (c->S.base) PGMG_TRY(mirror(c->S));
    if ((e = setup_rhs(c, f, r0, r1))) return e;
    return problem_reset(c);
}

int pgmg_set_problem_device(pgmg_ctx *c, double *phi, const double *f)
{
    if (!c || !phi) return set_err(PGMG_ERR_ARG, "null argument");
    if (c->comm) return set_err(PGMG_ERR_STATE, "pgmg_set_problem_device: one GPU only (world 1)");
    if (!is_device_ptr(phi) || (f && !is_device_ptr(f)))
        return set_err(PGMG_ERR_ARG, "pgmg_set_problem_device: phi and f must be device memory");
    Level &L = c->lv[0];
    const int N = L.N;
    PGMG_TRY(stream_wait(c));
    int e;
    if (!f) {
        if ((e = setup_rhs(c, nullptr, 0, N))) return e;
    } else {
        c->gen_rhs = false;
        c->rgfx = c->rgsy = nullptr;
    }
    // in place: a cross-fused fp64 context and phi inside an allocation that covers the rows
    // and columns the finest passes read past the grid (pgmg_alloc_grid's guard)
    const intptr_t o = (intptr_t)phi;
    const long long lo = -(long long)kHalo * N - 8, hi = (long long)(N + kHalo) * N + 8;
    c->ext_inplace = c->cross && !c->fp32 &&
                     registered_span(o + (intptr_t)(lo * 8), o + (intptr_t)(hi * 8));
    c->ext_phi = phi;
    c->ext_f = f;
    return problem_reset(c);
}

int pgmg_problem_device_info(pgmg_ctx *c, int *bound, int *inplace)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    if (bound) *bound = c->ext_phi != nullptr ? 1 : 0;
    if (inplace) *inplace = c->ext_phi != nullptr && c->ext_inplace ? 1 : 0;
    return PGMG_OK;
}

int pgmg_alloc_grid(double **out, int N)
{
    if (!out || N < 3) return set_err(PGMG_ERR_ARG, "pgmg_alloc_grid: null pointer or N < 3");
    *out = nullptr;
    // (kHalo + 2) rows + 1024 elements before element (0,0) and after element (N-1, N-1);
    // column 1 of row 0 on a 128-byte boundary
    const size_t guard = (size_t)(kHalo + 2) * N + 1024 + 15;
    const size_t n = 2 * guard + (size_t)N * N;
    void *p = nullptr;
    if (hipMalloc(&p, n * sizeof(double)) != hipSuccess)
        return set_err(PGMG_ERR_NOMEM, "pgmg_alloc_grid: hipMalloc failed");
    HIPC(hipMemset(p, 0, n * sizeof(double)));
    register_alloc(p, n * sizeof(double));
    double *o = static_cast<double *>(p) + guard;
    {
        std::lock_guard<std::mutex> lk(g_user_mu);
        g_user_grids[(uintptr_t)o] = UserGrid{p, ++g_user_serial};
    }
    *out = o;
    return PGMG_OK;
}

int pgmg_free_grid(double *o)
{
    if (!o) return PGMG_OK;
    void *p = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_user_mu);
        auto it = g_user_grids.find((uintptr_t)o);
        if (it == g_user_grids.end()) return set_err(PGMG_ERR_ARG, "pgmg_free_grid: not from pgmg_alloc_grid");
        p = it->second.alloc;
        g_user_grids.erase(it);
    }
    unregister_alloc(p);
    HIPC(hipFree(p));
    return PGMG_OK;
}

int pgmg_grid_serial(const double *o, unsigned long long *serial)
{
    if (!serial) return set_err(PGMG_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> lk(g_user_mu);
    auto it = g_user_grids.find((uintptr_t)o);
    *serial = it == g_user_grids.end() ? 0ull : it->second.serial;
    return PGMG_OK;
}

int pgmg_pointer_is_device(const void *p, int *is_device)
{
    if (!is_device) return set_err(PGMG_ERR_ARG, "null argument");
    *is_device = (p != nullptr && is_device_ptr(p)) ? 1 : 0;
    return PGMG_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Device-resident problems (pgmg_set_problem_device): the reference's contract.
// ParallelMultiGridSolver::v_cycle(phi, f, N, h) (Parallel_Mg.cu:21-60) works on arrays the
// caller allocated in device-accessible memory (cudaMallocManaged, ParallelTestRunner.cu:
// 162-163) and updates phi in place; nothing crosses PCIe per call.  Here phi and f are
// device arrays in the reference layout (pitch N, double).
//   * in place (cross-fused fp64 contexts, phi from pgmg_alloc_grid): the call's first
//     finest-level pass (k_pre) reads phi where it lies and its last (k_post) writes the
//     result there (PreArgs::Px, PostArgs::Po = N); the level-0 grids only carry the
//     iterates in between, so a call moves the same bytes as on the context's own grids.
//     The passes read rows and columns past the grid (halos, tile margins): the guard rows
//     of pgmg_alloc_grid keep those reads inside the allocation (span-checked per launch).
//   * staged (any other device pointer, fp32, or contexts without cross-cycle fusion):
//     phi is copied device-to-device into the level-0 grid before the call and back after.
// f = NULL is the analytic RHS of compute_rhs, regenerated in-kernel (never read); a
// caller's f is copied into the level-0 RHS grid at every call (the caller may change it).
// ---------------------------------------------------------------------------
// the boundary of the caller's phi into every level-0 grid the passes pass it through
template <class T>
static void ext_frames(pgmg_ctx *c)
{
    Level &L = c->lv[0];
    const Grid *gs[3] = {&L.A, &L.B, &c->S};
    for (const Grid *g : gs)
        if (g->base) launch_copy_frame<T>(c->ext_phi, L.N, G<T>(*g), L.P, L.N, c->s);
}

// The reference's v_cycle is synchronous on the default stream; the context's stream is
// non-blocking, so a device-bound call first orders it after whatever the caller queued on
// the null stream (an async copy into phi, a kernel writing f).  Work on the caller's own
// non-blocking streams is the caller's to synchronise (include/pgmg.h).  The wait is skipped
// when the null stream is already idle (the usual case: the previous call synchronised).
// The null stream is the CALLING thread's current device's, so the record runs with the
// context's device made current (and the caller's restored): one thread may drive contexts on
// several devices.
static int order_after_caller(pgmg_ctx *c)
{
    int prev = -1;
    HIPC(hipGetDevice(&prev));
    const bool swap = prev != c->cfg.device;
    if (swap) HIPC(hipSetDevice(c->cfg.device));
    hipError_t e = hipEventRecord(c->ev_caller, nullptr);
    hipError_t q = e == hipSuccess ? hipEventQuery(c->ev_caller) : e;
    if (q == hipErrorNotReady) q = hipStreamWaitEvent(c->s, c->ev_caller, 0);
    if (swap) {
        const hipError_t r = hipSetDevice(prev);
        if (q == hipSuccess) q = r;
    }
    if (q != hipSuccess) return set_err(PGMG_ERR_HIP, hipGetErrorString(q));
    return PGMG_OK;
}

// before a call: the caller's f into the level-0 RHS grid (unless analytic) and phi's frame
// (in place) or all of phi (staged) into the level-0 grids
static int ext_stage_in(pgmg_ctx *c, bool inplace)
{
    PGMG_TRY(order_after_caller(c));
    Level &L = c->lv[0];
    const int N = L.N;
    if (c->ext_f) {
        if (c->fp32) launch_from_double(c->ext_f, N, G<float>(L.F), L.P, 0, N, c->s);
        else if (is_vmm(L.F.base)) launch_from_double(c->ext_f, N, G<double>(L.F), L.P, 0, N, c->s);
        else HIPC(hipMemcpy2DAsync(L.F.o, L.P * sizeof(double), c->ext_f, N * sizeof(double),
                                   N * sizeof(double), N, hipMemcpyDeviceToDevice, c->s));
    }
    if (!inplace) {
        if (c->fp32) launch_from_double(c->ext_phi, N, G<float>(L.A), L.P, 0, N, c->s);
        else if (is_vmm(L.A.base)) launch_from_double(c->ext_phi, N, G<double>(L.A), L.P, 0, N, c->s);
        else HIPC(hipMemcpy2DAsync(L.A.o, L.P * sizeof(double), c->ext_phi, N * sizeof(double),
                                   N * sizeof(double), N, hipMemcpyDeviceToDevice, c->s));
    }
    if (c->fp32) ext_frames<float>(c);
    else ext_frames<double>(c);
    HIPC(hipGetLastError());
    return PGMG_OK;
}

static int ext_stage_out(pgmg_ctx *c)
{
    Level &L = c->lv[0];
    const int N = L.N;
    if (c->fp32) launch_to_double(G<float>(L.A), L.P, c->ext_phi, N, 0, N, c->s);
    else if (is_vmm(L.A.base)) launch_to_double(G<double>(L.A), L.P, c->ext_phi, N, 0, N, c->s);
    else HIPC(hipMemcpy2DAsync(c->ext_phi, N * sizeof(double), L.A.o, L.P * sizeof(double),
                               N * sizeof(double), N, hipMemcpyDeviceToDevice, c->s));
    HIPC(hipGetLastError());
    return PGMG_OK;
}

// the last k_post of an in-place call whose speculative checks were validated first (its
// input survives until then): from the pre-smoothed iterate into the caller's phi, its own
// early-exit check decided in-stream
template <class T>
static int enqueue_last_post(pgmg_ctx *c)
{
    Level &L = c->lv[0];
    const StripRows sr = strip_rows(L, c->lv[1]);
    PostArgsT<T> po = make_post<T>(c, static_cast<const T *>(c->pend_pr), static_cast<T *>(c->x_out));
    po.Po = c->ext_P;
    const int ev = timed_begin(c, 2);
    PGMG_TRY(launch_post(po, true, c->s));
    PGMG_TRY(timed_end(c, 2, ev));
    FixArgsF fa{};
    fa.partials = c->partials;
    fa.np = fused_blocks(L.N, sr.jc0, sr.jc1);
    fa.eps = c->cfg.eps;
    fa.stats = c->stats;
    launch_post_fixup(fa, po, c->s);
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(c->ev1, c->s));
    c->pend_pr = nullptr;
    return PGMG_OK;
}

extern "C" {

static int run_cycles_plain(pgmg_ctx *c, int ncycles, int gamma, bool rec0 = true)
{
    if (rec0) HIPC(hipEventRecord(c->ev0, c->s));
    const bool use_graph = gamma == 1 && !(c->cfg.flags & PGMG_FLAG_NO_GRAPH) &&
                           !(c->cfg.flags & PGMG_FLAG_TIME_FINE) && c->comm == nullptr &&
                           !c->cross;
    if (use_graph && !c->gexec) {
        // first cycle eagerly (sets kernel attributes), the rest from a captured graph
        int e = enqueue_cycle(c, 0, 1, false);
        if (e) return e;
        HIPC(hipGetLastError());
        --ncycles;
        hipGraph_t g = nullptr;
        HIPC(hipStreamBeginCapture(c->s, hipStreamCaptureModeThreadLocal));
        e = enqueue_cycle(c, 0, 1, false);
        hipError_t ce = hipStreamEndCapture(c->s, &g);
        if (e) return e;
        if (ce != hipSuccess) return set_err(PGMG_ERR_HIP, std::string("capture: ") + hipGetErrorString(ce));
        HIPC(hipGraphInstantiate(&c->gexec, g, nullptr, nullptr, 0));
        HIPC(hipGraphDestroy(g));
    }
    if (c->cross && !use_graph) {
        int e = c->fp32 ? enqueue_cross_cycles<float>(c, ncycles, gamma)
                        : enqueue_cross_cycles<double>(c, ncycles, gamma);
        if (e) return e;
        HIPC(hipGetLastError());
        HIPC(hipEventRecord(c->ev1, c->s));
        return PGMG_OK;
    }
    for (int k = 0; k < ncycles; ++k) {
        if (use_graph) {
            HIPC(hipGraphLaunch(c->gexec, c->s));
        } else {
            int e = enqueue_cycle(c, 0, gamma, false);
            if (e) return e;
        }
    }
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(c->ev1, c->s));
    return PGMG_OK;
}

// ---------------------------------------------------------------------------
// Speculative calls.  Every smoother's early-exit check (MultiGrid.hpp via Smoother.hpp:
// 75-88, ||r(x1)|| < eps after the first of the two sweeps) needs a grid-wide sum, so the
// exact path follows each fused pass with a fix-up launch that reduces the pass's per-
// block partials, decides, and recomputes the reference result when the check fired
// (plus, at level 0 between cycles, a decision kernel and four conditional rare-path
// launches): ~22 launches per V-cycle of a few microseconds each that almost never do
// work.  A speculative call instead enqueues all its cycles with every check decided
// "does not fire": each pass writes its partials into a fresh slice of a per-call log and
// no fix-up is launched.  After the call one kernel re-reduces every recorded check
// exactly as the fix-ups would and flags those that could fire; on row strips a rank's
// partial is a lower bound of the all-rank sum (a sum of non-negative doubles never
// rounds below one of its terms, sqrt is monotonic), so one allreduce(min) of the flags
// finds the checks no rank could rule out.  If any check could fire, the call is rolled
// back (the level-0 solution -- untouched: the cross-fused cycles rotate through the
// scratch buffer S instead of writing A -- buffer roles and statistics restored) and run
// again with in-stream decisions, and the context stops speculating (a fired check means
// the solver is near convergence, where checks keep firing).  Results and statistics
// are therefore always the exact path's.  The call ends with one host synchronisation.
// ---------------------------------------------------------------------------

// log doubles and checks of one visit of level l >= 1 (the tail decides in-kernel)
static void spec_need_level(pgmg_ctx *c, int l, int gamma, long long *dbl, long long *nchk)
{
    *dbl = 0;
    *nchk = 0;
    if (l >= c->nb) return;
    const Level &L = c->lv[l];
    // the small levels' tile passes (pgmg_coarse.hip) may write more partials than the
    // row-marching passes: reserve for the larger
    const int np = std::max(fused_blocks(L.N, L.lo / 2, (L.hi < L.N ? L.hi : L.N - 1) / 2),
                            tile_np(c, l, false));
    const PostRows pr = post_rows(c, l);
    const int npo = std::max(fused_blocks(L.N, pr.jc0, pr.jc1), tile_np(c, l, true));
    long long d, k;
    spec_need_level(c, l + 1, gamma, &d, &k);
    *dbl = (long long)np + npo + gamma * d;
    *nchk = 2 + gamma * k;
}

// the pinned validation staging (pgmg_ctx::pin) for cap checks: CheckRefs, norms, verdicts + any
static size_t pin_norm_off(long long cap) { return ((size_t)cap * sizeof(CheckRef) + 15) / 16 * 16; }
static size_t pin_flag_off(long long cap) { return pin_norm_off(cap) + (size_t)cap * sizeof(double); }
static size_t pin_seq_off(long long cap) { return pin_flag_off(cap) + ((size_t)cap + 1) * sizeof(unsigned); }
static size_t pin_bytes(long long cap) { return pin_seq_off(cap) + 64; }

// The validation's wait: poll the reply's sequence word in pinned memory (the call's
// critical path: a blocking stream wait wakes the host late -- tens of us on a busy host --
// and the next call's kernels queue behind that), asking the runtime every ~20 us whether the
// stream failed or drained.  Once the word arrives the call returns without a stream wait:
// everything the host reads next is in the pinned reply, and everything it writes next (the
// staging's CheckRefs) was read by k_verify_checks, which ran before the reply.  A fault
// surfaces at the runtime's query; a wait past 50 ms (a slow segment, a shared GPU) stops
// burning the core and blocks.  One GPU only (row strips wait through their transport).
static int reply_wait(pgmg_ctx *c, const unsigned *hseq, unsigned seq)
{
    if (c->comm == nullptr && !(c->cfg.flags & PGMG_FLAG_NO_SPIN)) {
        const auto t0 = std::chrono::steady_clock::now();
        auto next = t0 + std::chrono::microseconds(20);
        for (;;) {
            if (__atomic_load_n(hseq, __ATOMIC_ACQUIRE) == seq) return PGMG_OK;
            const auto now = std::chrono::steady_clock::now();
            if (now < next) continue;
            next = now + std::chrono::microseconds(20);
            const hipError_t q = hipStreamQuery(c->s);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) PGMG_HIPC(q);
            if (now - t0 > std::chrono::milliseconds(50)) break;
        }
    }
    return stream_wait(c);
}

static int spec_reserve(pgmg_ctx *c, long long dbl, long long nchk)
{
    if (dbl > c->plog_cap || nchk > c->chk_cap) {
        PGMG_TRY(stream_wait(c));
        if (dbl > c->plog_cap) {
            if (c->plog) HIPC(hipFree(c->plog));
            c->plog = nullptr;
            HIPC(hipMalloc((void **)&c->plog, dbl * sizeof(double)));
            c->plog_cap = dbl;
        }
        if (nchk > c->chk_cap) {
            if (c->uflags) HIPC(hipFree(c->uflags));
            if (c->chk_norm) HIPC(hipFree(c->chk_norm));
            c->uflags = nullptr;
            c->chk_norm = nullptr;
            HIPC(hipMalloc((void **)&c->uflags, (nchk + 1) * sizeof(unsigned)));
            HIPC(hipMalloc((void **)&c->chk_norm, nchk * sizeof(double)));
            if (c->pin) HIPC(hipHostFree(c->pin));
            c->pin = nullptr;
            HIPC(hipHostMalloc((void **)&c->pin, pin_bytes(nchk), hipHostMallocCoherent));
            // (a fresh staging area: its sequence word must not already hold the next seq)
            std::memset(c->pin, 0, pin_bytes(nchk));
            c->pin_seq = 0;
            c->chk_cap = nchk;
        }
    }
    if (!c->stats_bk) HIPC(hipMalloc((void **)&c->stats_bk, 4 * sizeof(unsigned long long)));
    if (c->comm && !c->mark_dev) HIPC(hipMalloc((void **)&c->mark_dev, (c->nb + 1) * sizeof(unsigned)));
    return PGMG_OK;
}

// last norm and decay of level l's checks (spec_mark_levels' prediction); false without history
static bool spec_level_trend(const pgmg_ctx *c, int l, double *last, double *rho)
{
    const std::vector<double> &h = c->lvl_hist[l];
    const size_t m = h.size();
    if (m < 2) return false;
    *last = std::min(h[m - 1], h[m - 2]);
    *rho = 0.4;
    if (m >= 4) {
        const double prev = std::min(h[m - 3], h[m - 4]);
        if (prev > 0.0) *rho = std::min(*rho, std::max(1e-3, *last / prev));
    }
    return true;
}

// Per-level policy.  Residual norms of a level fall geometrically over the V-cycles (after
// a few cycles of growth from phi = 0) until they level off, and on the reference problem
// the levels just above the tail reach eps after ~27 cycles at every N >= 2049
// (scripts/spec_fire_probe.py, spec_trace.py: 0.32-0.35 per cycle in the steady phase).
// A rollback costs a whole segment, so a coarse level whose checks are predicted to fire
// within the next segment -- last norm x rho^cycles < 100 eps with rho = min(0.4, its
// measured decay) -- or did fire decides in-stream from then on (its two fix-ups per visit
// come back); the others keep speculating.  The finest
// level is not predicted (its norm levels off far above eps at these sizes: round-off of
// 1/h^2-scaled sums); if one of its checks does fire the context stops speculating.
// Row strips: each rank predicts from its own partials (a lower bound of the global norm,
// so earlier), then the ranks agree on the union of the marks (one allreduce).
//
// Predicted to fire (one GPU): a level whose last two visits' checks all had norms below
// eps / 4 -- it converged and fires at every check -- is enqueued with its checks decided
// "fires" (k_pre1 / k_post1: the one-sweep passes the in-stream rare paths would run, one
// launch each instead of two) and recorded the other way round: the validation flags a
// check that could NOT fire (sqrt(s) >= eps (1 - 1e-12)), the call is rolled back, and the
// level decides in-stream for the rest of the problem.  A level in that mode whose norm
// comes back above eps / 4 returns to in-stream decisions.
static int spec_mark_levels(pgmg_ctx *c, int cycles)
{
    const double lim = c->cfg.eps * 100.0;
    if (c->comm == nullptr && !(c->cfg.flags & PGMG_FLAG_NO_SPEC_FIRE) && c->spec_gamma == 1) {
        const double flim = c->cfg.eps * 0.25;
        for (int l = 1; l < c->nb; ++l) {
            const std::vector<double> &h = c->lvl_hist[l];
            const size_t m = h.size();
            const size_t need = c->lvl_fire[l] ? 2 : 4;
            bool below = !c->lvl_fire_block[l] && m >= need;
            for (size_t i = m - std::min(m, need); i < m && below; ++i) below = h[i] < flim;
            c->lvl_fire[l] = below ? 1 : 0;
            if (below) c->lvl_exact[l] = 0;
            else if (m >= 2 && h[m - 1] < c->cfg.eps) c->lvl_exact[l] = 1;   // fired: in-stream
        }
    }
    if (tuning_int("PGMG_SPEC_TRACE", 0))
        for (int l = 1; l < c->nb; ++l) {
            fprintf(stderr, "spec level %d N=%d exact %d fire %d block %d hist/eps", l, c->lv[l].N,
                    (int)c->lvl_exact[l], (int)c->lvl_fire[l], (int)c->lvl_fire_block[l]);
            for (double v : c->lvl_hist[l]) fprintf(stderr, " %.3g", v / c->cfg.eps);
            fprintf(stderr, "\n");
        }
    // keep[l]: the segment's first cycles in which level l records "does not fire" (its
    // predicted norm last * rho^k stays at or above 100 eps); 0: in-stream from the start
    std::vector<unsigned> keep(c->nb + 1, (unsigned)cycles);
    for (int l = 1; l < c->nb && c->spec_gamma == 1; ++l) {
        double last, rho;   // min over the last visit; decay per cycle
        if (c->lvl_exact[l] || c->lvl_fire[l] || !spec_level_trend(c, l, &last, &rho)) continue;
        const double k = last >= lim ? std::floor(std::log(lim / last) / std::log(rho)) : 0.0;
        keep[l] = (unsigned)std::max(0.0, std::min((double)cycles, k));
        // (PGMG_FLAG_NO_SPEC_FIRE, the r02 policy: in-stream for the whole segment instead)
        if ((c->cfg.flags & PGMG_FLAG_NO_SPEC_FIRE) && keep[l] < (unsigned)cycles) keep[l] = 0u;
        if (tuning_int("PGMG_SPEC_TRACE", 0))
            fprintf(stderr, "spec level %d N=%d last %.3e rho %.3f: speculates %u of %d cycles\n", l,
                    c->lv[l].N, last, rho, keep[l], cycles);
    }
    if (c->comm) {
        HIPC(hipMemcpyAsync(c->mark_dev, keep.data(), (c->nb + 1) * sizeof(unsigned),
                            hipMemcpyHostToDevice, c->s));
        int e = c->comm->allreduce_min_u32(c->mark_dev, c->nb + 1, c->s);
        if (e) return e;
        HIPC(hipMemcpyAsync(keep.data(), c->mark_dev, (c->nb + 1) * sizeof(unsigned),
                            hipMemcpyDeviceToHost, c->s));
        PGMG_TRY(stream_wait(c));
    }
    for (int l = 1; l < c->nb; ++l) {
        if (!keep[l]) c->lvl_exact[l] = 1;
        c->lvl_kx[l] = (int)keep[l];
    }
    return PGMG_OK;
}

// Segment planning (one GPU).  A level that decides in-stream (two launches of ~5 us per
// visit) can be predicted to fire -- one launch per visit -- only from the norms of a
// validated segment, so a long call (the 3 + 40 cycles of BASELINE configs[1] at N = 4097:
// the coarse levels cross eps at ~27 cycles) would keep it in-stream to its end.  The segment
// ends where such levels can be predicted to fire when that pays for the split: ~10 us per
// level and cycle saved against one more finest-level pass (the cross-fused call restarts:
// k_post + k_pre instead of one k_postpre, 16 B per fine point at ~5 TB/s) and one host
// round trip of the validation.  (A speculating level's crossing of 100 eps needs no split:
// spec_mark_levels gives it its speculating cycles within the segment.)
static int spec_plan_segment(pgmg_ctx *c, int seg)
{
    if (seg < 4 || (c->cfg.flags & PGMG_FLAG_NO_SPEC_FIRE) || c->spec_gamma > 1) return seg;
    // a new problem: a short first segment gathers every level's trend (without one, a long
    // first call speculated blind and rolled back at the first firing check, ~27 cycles in
    // on the reference problem); history sizes are the same on every rank
    if (seg > 8)
        for (int l = 1; l < c->nb; ++l)
            if (c->lvl_hist[l].size() < 2 && !c->lvl_exact[l]) return 3;
    if (c->comm != nullptr) return seg;   // (strips: every rank must agree)
    const double lim = c->cfg.eps * 100.0, flim = c->cfg.eps * 0.25;
    // cycles until last * rho^k falls below t
    auto cycles_to = [](double last, double rho, double t) {
        return last > t ? (int)std::floor(std::log(t / last) / std::log(rho)) : 0;
    };
    // candidate split points: a level's last cycle before it can be predicted to fire (its
    // norm under eps / 4 for two visits)
    struct Cand {
        int k, level;   // predicted to fire from cycle k
        double norm;
    };
    std::vector<Cand> cand;
    for (int l = 1; l < c->nb; ++l) {
        double last, rho;
        if (c->lvl_fire[l] || !spec_level_trend(c, l, &last, &rho)) continue;
        bool exact = c->lvl_exact[l] != 0;
        if (!exact) {
            // a speculating level records "does not fire" up to its crossing of 100 eps within
            // the segment anyway (spec_mark_levels); what a split can give it is the firing
            // prediction, from a segment that ends after its steep decay took it under eps / 4
            const int k = cycles_to(last, rho, lim);
            if (k >= seg) continue;
            if (k >= 2) {
                const int kf = k + cycles_to(lim, rho, flim) + 2;
                if (kf < seg && !c->lvl_fire_block[l])
                    cand.push_back({kf, l, last * std::pow(rho, (double)kf)});
                continue;
            }
            exact = true;   // in-stream from this segment on
        }
        if (exact && !c->lvl_fire_block[l]) {
            // the fire test looks at the LARGER check norm of a visit: its decay; a level whose
            // norm stagnates (the one above the finest typically hovers at 0.5-1 eps for good)
            // or that already had a split at a similar norm gets none
            const std::vector<double> &h = c->lvl_hist[l];
            const size_t m = h.size();
            const double ml = std::max(h[m - 1], h[m - 2]);
            const double mp = m >= 4 ? std::max(h[m - 3], h[m - 4]) : 0.0;
            const double rm = mp > 0.0 ? ml / mp : 1.0;
            if (rm > 0.9 || (c->lvl_fire_try[l] > 0.0 && ml > 0.5 * c->lvl_fire_try[l])) continue;
            // (the decay slows near eps: ~0.7 per cycle on the reference problem, where the
            // steep phase shows ~0.33; a split that comes too early costs without paying)
            const int k = cycles_to(ml, std::max(rm, 0.7), flim) + 2;
            if (k < seg) cand.push_back({std::max(k, 2), l, ml});
        }
    }
    // level-cycles that avoid two in-stream launches (~10 us each) if the segment ends at
    // k: a level that can be predicted to fire by k does so for seg - k
    int best_k = seg;
    double best = 0.0;
    for (const auto &q : cand) {
        const int k = q.k;
        double saved = 0.0;
        for (const auto &p : cand) saved += p.k <= k ? seg - k : 0;
        if (saved > best) {
            best = saved;
            best_k = k;
        }
    }
    const double N0 = (double)c->lv[0].N;
    const double cost = 16.0 * N0 * N0 / 5e12 + 60e-6;
    if (tuning_int("PGMG_SPEC_TRACE", 0))
        fprintf(stderr, "spec plan: seg %d, %zu candidates, best split %d saves %.0f us vs %.0f us\n",
                seg, cand.size(), best_k, best * 10.0, cost * 1e6);
    if (!(best * 10e-6 > cost)) return seg;
    for (const auto &p : cand)
        if (p.k <= best_k) c->lvl_fire_try[p.level] = p.norm;
    return best_k;
}

static void spec_record_norms(pgmg_ctx *c, int n)
{
    for (int i = 0; i < n; ++i) {
        std::vector<double> &h = c->lvl_hist[c->chks[i].level];
        h.push_back(c->hnorm[i]);
        if (h.size() > 8) h.erase(h.begin(), h.end() - 4);
    }
    if (c->spec_gamma <= 1) return;
    // W-cycle plan: the norms of the segment's last cycle, per visit
    const int nv = c->wvisit, seg = c->wseg;
    const std::vector<double> pmin = c->wplan_gamma == c->spec_gamma ? c->wmin : std::vector<double>();
    const int pseg = c->wplan_seg;
    c->wmax.clear();
    c->wmin.clear();
    c->wrho.clear();
    c->wplan_gamma = 0;
    if (nv == 0 || seg <= 0 || nv % seg != 0 || (int)c->chk_visit.size() != n) return;
    const int vc = nv / seg, v0 = nv - vc;
    c->wmax.assign(vc, -1.0);
    c->wmin.assign(vc, HUGE_VAL);
    for (int i = 0; i < n; ++i) {
        const int v = c->chk_visit[i];
        if (v < v0) continue;
        c->wmax[v - v0] = std::max(c->wmax[v - v0], c->hnorm[i]);
        c->wmin[v - v0] = std::min(c->wmin[v - v0], c->hnorm[i]);
    }
    // per-cycle decay of each visit's smaller norm since the previous plan (0: unknown; the
    // first cycles of a problem fall by orders of magnitude, so no "does not fire" without it)
    c->wrho.assign(vc, 0.0);
    if ((int)pmin.size() == vc && pseg > 0)
        for (int i = 0; i < vc; ++i)
            if (pmin[i] > 0.0 && pmin[i] < HUGE_VAL && c->wmin[i] < HUGE_VAL)
                c->wrho[i] = std::min(1.0, std::pow(c->wmin[i] / pmin[i], 1.0 / seg));
    c->wplan_gamma = c->spec_gamma;
    c->wplan_seg = seg;
    if (tuning_int("PGMG_SPEC_TRACE", 0)) {
        int f = 0, q = 0;
        for (int i = 0; i < vc; ++i) {
            f += c->wmax[i] >= 0.0 && c->wmax[i] < 0.25 * c->cfg.eps;
            q += c->wrho[i] > 0.0 && c->wmin[i] * c->wrho[i] * 0.01 >= c->cfg.eps;
        }
        fprintf(stderr, "W plan: %d visits per cycle, %d predicted to fire, %d not (1 cycle)\n",
                vc, f, q);
        // per level: visits, both checks < eps/4, max < eps, and the first visits (in cycle
        // order) whose max norm is >= eps/4 (measurement trace)
        std::vector<int> vlev(vc, -1);
        for (int i = 0; i < n; ++i)
            if (c->chk_visit[i] >= v0) vlev[c->chk_visit[i] - v0] = c->chks[i].level;
        for (int l = 1; l < 32; ++l) {
            int tot = 0, f4 = 0, f1 = 0;
            std::string nf;
            for (int i = 0; i < vc; ++i) {
                if (vlev[i] != l) continue;
                const bool a = c->wmax[i] >= 0.0 && c->wmax[i] < 0.25 * c->cfg.eps;
                f4 += a;
                f1 += c->wmax[i] >= 0.0 && c->wmax[i] < c->cfg.eps;
                if (!a && nf.size() < 400) nf += " " + std::to_string(tot) + ":" + std::to_string(c->wmax[i] / c->cfg.eps);
                ++tot;
            }
            if (tot) fprintf(stderr, "  level %d: %d visits, %d < eps/4, %d < eps; others (index:max/eps):%s\n",
                             l, tot, f4, f1, nf.c_str());
        }
    }
}

// Validation of a speculative call's check log (one host round trip): every recorded check
// re-reduced and compared with its recorded decision (k_verify_checks; row strips: the ranks
// agree by allreduce(min)).  *h = 1 when some check could not be confirmed -- the call must
// be rolled back -- or the log overflowed; per-check norms and verdicts land in hnorm / hflag.
// Only the first n_any checks decide the rollback (the carry pass logs one more).
static int spec_validate(pgmg_ctx *c, unsigned *h_out, bool *overflow_out, int n_any)
{
    const int n = (int)c->chks.size();
    bool overflow = false;
    for (const CheckRef &k : c->chks) overflow |= k.np < 0;
    unsigned h = overflow ? 1u : 0u;
    c->hnorm.assign(n, 0.0);
    c->hflag.assign(n, 1u);
    if (n > 0 && !overflow) {
        // through the pinned (coherent) staging area: k_verify_checks reads the CheckRefs from
        // it and k_spec_reply writes the verdicts, the norms and their OR into it -- two
        // kernels and one stream wait, no copy operations
        CheckRef *hc = reinterpret_cast<CheckRef *>(c->pin);
        double *hn = reinterpret_cast<double *>(c->pin + pin_norm_off(c->chk_cap));
        unsigned *hf = reinterpret_cast<unsigned *>(c->pin + pin_flag_off(c->chk_cap));
        std::memcpy(hc, c->chks.data(), n * sizeof(CheckRef));
        launch_verify_checks(hc, n, c->cfg.eps, c->uflags, c->chk_norm, c->s);
        int e;
        if (c->comm && (e = c->comm->allreduce_min_u32(c->uflags, n, c->s))) return e;
        // (the checks past n_any -- the carried pre-smooth's -- never roll the call back)
        unsigned *hseq = reinterpret_cast<unsigned *>(c->pin + pin_seq_off(c->chk_cap));
        const unsigned seq = ++c->pin_seq;
        launch_spec_reply(c->uflags, c->chk_norm, n, n_any, hf + c->chk_cap, hn, hf, hseq, seq, c->s);
        PGMG_TRY(reply_wait(c, hseq, seq));
        h = hf[c->chk_cap];
        std::memcpy(c->hnorm.data(), hn, n * sizeof(double));
        std::memcpy(c->hflag.data(), hf, n * sizeof(unsigned));
    } else {
        PGMG_TRY(stream_wait(c));
    }
    *h_out = h;
    *overflow_out = overflow;
    return PGMG_OK;
}

static int run_cycles_spec(pgmg_ctx *c, int ncycles, int gamma)
{
    Level &L0 = c->lv[0];
    const int np0 = fused_blocks(L0.N, L0.lo / 2, (L0.hi < L0.N ? L0.hi : L0.N - 1) / 2);
    // (k_postpre's partials, in any form: the recompute form's tiles are narrower)
    const int npp = c->cross ? std::max(postpre_blocks(L0.N, L0.lo / 2, (L0.hi < L0.N ? L0.hi : L0.N - 1) / 2),
                                        postpre_blocks(L0.N, L0.lo / 2, (L0.hi < L0.N ? L0.hi : L0.N - 1) / 2, true))
                             : 0;
    long long d1, k1;
    spec_need_level(c, 1, gamma, &d1, &k1);
    // (level 0 visits level 1 gamma times per cycle)
    const long long per_dbl = 2LL * std::max(np0, npp) + gamma * d1, per_chk = 2 + gamma * k1;
    // segments of at most 2^27 logged doubles (1 GiB) / 2^22 checks
    long long seg_max = std::min(((1LL << 27) - 2LL * std::max(np0, npp)) / per_dbl, ((1LL << 22) - 2) / per_chk);
    if (c->cfg.spec_segment > 0) seg_max = std::min<long long>(seg_max, c->cfg.spec_segment);
    if (seg_max < 1) return run_cycles_plain(c, ncycles, gamma);
    // the cross-fused cycles keep A intact (rotation through S); otherwise copy it
    const bool rotate = c->cross && c->S.base != nullptr;
    // an in-place device call (run_cycles_ext): the first segment reads the caller's phi, the
    // last writes it -- that final k_post only after the validation, since it overwrites the
    // call's input (a rollback reruns from it)
    const void *const ext_in = c->x_in;
    void *const ext_out = c->x_out;
    bool first = true;
    c->spec_gamma = gamma;
    c->wcount[0] = c->wcount[1] = c->wcount[2] = 0;
    while (ncycles > 0) {
        const int seg = spec_plan_segment(c, (int)std::min<long long>(ncycles, seg_max));
        c->x_in = first ? ext_in : nullptr;
        c->x_out = ext_out;
        int e = spec_reserve(c, seg * per_dbl + 2LL * std::max(np0, npp) + 64, seg * per_chk + 4);
        if (e) return e;
        if ((e = spec_mark_levels(c, seg))) return e;
        if (c->spec_off) return run_cycles_plain(c, ncycles, gamma, first);
        const bool last = seg == ncycles;
        const bool seg_first = first;
        const Grid A0 = L0.A, B0 = L0.B, S0 = c->S;
        if (!rotate) {
            if (!c->bk.base && (e = alloc_grid(c->bk, L0))) return e;
            HIPC(hipMemcpyAsync(c->bk.base, L0.A.base, L0.A.bytes, hipMemcpyDeviceToDevice, c->s));
        }
        // stats backup + the coarse levels' "pre-smooth fired" flags (written by the skipped
        // fix-ups) = 0, one launch
        launch_spec_open(c->stats, c->stats_bk, c->flags, (int)(c->lv.size() + 1) * 2 * kMaxSweeps, c->s);
        c->lean = true;
        c->plog_used = 0;
        c->chks.clear();
        c->chk_visit.clear();
        c->wvisit = 0;
        c->wseg = seg;
        std::fill(c->lvl_vis.begin(), c->lvl_vis.end(), 0);
        if (!last) c->x_out = nullptr;   // intermediate segments end in the level-0 grids
        c->defer_post = ext_out != nullptr && last;
        // the carry: the last segment of a V call on the context's own grids ends with the
        // carry pass (enqueue_cross_cycles, "carry"); c->carry_use was set by run_cycles for
        // the first segment
        c->carry_make = last && gamma == 1 && ext_out == nullptr &&
                        !(c->cfg.flags & PGMG_FLAG_NO_CARRY) &&
                        tuning_int("PGMG_CARRY_MAKE", 1) != 0;   // (measurement build: 0 never makes)
        c->carry_chk = -1;
        e = run_cycles_plain(c, seg, gamma, first);
        c->defer_post = false;
        c->carry_make = false;
        c->carry_use = false;
        c->x_out = ext_out;
        c->lean = false;
        first = false;
        if (e) return e;
        int n = (int)c->chks.size();
        const bool made = c->carry_made && c->carry_chk == n - 1;
        if (c->carry_made && !made) return set_err(PGMG_ERR_STATE, "carry check out of place");
        c->carry_made = false;
        unsigned h = 0;
        bool overflow = false;
        if ((e = spec_validate(c, &h, &overflow, made ? n - 1 : n))) return e;
        if (h) {
            // some check could fire: roll back this segment, rerun the rest of the call with
            // in-stream decisions; the levels whose checks could fire stay in-stream
            ++c->rollbacks;
            if (gamma > 1) {   // a W plan's prediction failed
                c->wplan_off = true;
                c->wmax.clear();
                c->wmin.clear();
                c->wrho.clear();
            }
            for (int i = 0; i < n; ++i)
                if (c->hflag[i] || overflow) {
                    const int l = c->chks[i].level;
                    if (l == 0) {
                        c->spec_off = true;
                    } else {
                        c->lvl_exact[l] = 1;
                        if (c->chks[i].expect == 1) {   // a "fires" prediction failed
                            c->lvl_fire[l] = 0;
                            c->lvl_fire_block[l] = 1;
                        }
                    }
                }
            L0.A = A0;
            L0.B = B0;
            c->S = S0;
            c->carry = false;
            if (!rotate)
                HIPC(hipMemcpyAsync(L0.A.base, c->bk.base, L0.A.bytes, hipMemcpyDeviceToDevice, c->s));
            HIPC(hipMemcpyAsync(c->stats, c->stats_bk, 4 * sizeof(unsigned long long),
                                hipMemcpyDeviceToDevice, c->s));
            c->x_in = seg_first ? ext_in : nullptr;
            c->pend_pr = nullptr;
            return run_cycles_plain(c, ncycles, gamma, false);
        }
        if (seg_first && c->carry_took) ++c->carry_n[0];
        c->carry_took = false;
        if (made) {
            // the carried pre-smooth: usable unless its check could fire (then dropped: the
            // next call runs its own k_pre); not one of this call's checks
            const bool ok = !overflow && c->hflag[n - 1] == 0u;
            c->carry = ok;
            ++c->carry_n[ok ? 1 : 2];
            --n;
            c->chks.pop_back();
            c->chk_visit.pop_back();
            c->hnorm.pop_back();
            c->hflag.pop_back();
        }
        spec_record_norms(c, n);
        if (ext_out != nullptr && last) {
            e = c->fp32 ? enqueue_last_post<float>(c) : enqueue_last_post<double>(c);
            if (e) return e;
        }
        ncycles -= seg;
    }
    return PGMG_OK;
}

static int run_cycles_core(pgmg_ctx *c, int ncycles, int gamma)
{
    // W-cycles revisit the coarse levels until their checks fire (the reference's W-cycle at
    // 129 exits 147 times in its first cycle): their speculative calls decide those checks
    // in-stream (chk_mode) and only predict converged levels to fire (one GPU, any N: a W-cycle
    // is never a captured graph, so the smaller grids gain as much)
    const bool w_spec = gamma > 1 && c->fused && c->comm == nullptr &&
                        !(c->cfg.flags & (PGMG_FLAG_NO_SPEC_FIRE | PGMG_FLAG_EXACT_DIST));
    if (!c->spec_off && (gamma == 1 ? c->spec : w_spec)) return run_cycles_spec(c, ncycles, gamma);
    return run_cycles_plain(c, ncycles, gamma);
}

// a call on a device-bound problem (pgmg_set_problem_device): synchronous, as the reference's
// v_cycle is (the caller reads phi when it returns)
static int run_cycles_ext(pgmg_ctx *c, int ncycles, int gamma)
{
    const bool inplace = c->ext_inplace;
    PGMG_TRY(ext_stage_in(c, inplace));
    if (inplace) {
        c->x_in = c->ext_phi;
        c->x_out = c->ext_phi;
        c->ext_P = c->lv[0].N;
    }
    const int e = run_cycles_core(c, ncycles, gamma);
    c->x_in = nullptr;
    c->x_out = nullptr;
    c->defer_post = false;
    c->pend_pr = nullptr;
    if (e) return e;
    if (!inplace) PGMG_TRY(ext_stage_out(c));
    PGMG_TRY(stream_wait(c));
    return PGMG_OK;
}

static int run_cycles(pgmg_ctx *c, int ncycles, int gamma)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    if (!c->have_problem) return set_err(PGMG_ERR_STATE, "pgmg_set_problem first");
    if (ncycles <= 0) return PGMG_OK;
    // the carry is this call's to take (a V call on the context's own problem: the first
    // speculative segment starts from it) or gone; a call that runs in-stream drops it
    c->carry_use = c->carry && gamma == 1 && c->ext_phi == nullptr &&
                   tuning_int("PGMG_CARRY_TAKE", 1) != 0;   // (measurement build: 0 never takes)
    c->carry = false;
    c->carry_took = false;
    const int e = c->ext_phi ? run_cycles_ext(c, ncycles, gamma) : run_cycles_core(c, ncycles, gamma);
    c->carry_use = false;
    return e;
}

int pgmg_comm_stats(pgmg_ctx *c, long long *groups, double *ms)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    if (!c->comm) {
        PGMG_TRY(stream_wait(c));
        if (groups) *groups = 0;
        if (ms) *ms = 0.0;
        return PGMG_OK;
    }
    return c->comm->comm_stats(c->s, groups, ms);
}

int pgmg_comm_ranks(pgmg_ctx *c, int *ranks)
{
    if (!c || !ranks) return set_err(PGMG_ERR_ARG, "null argument");
    if (!c->comm) return *ranks = 1, PGMG_OK;
    return c->comm->comm_ranks(ranks);
}

int pgmg_carry_info(pgmg_ctx *c, long long out[3])
{
    if (!c || !out) return set_err(PGMG_ERR_ARG, "null argument");
    for (int i = 0; i < 3; ++i) out[i] = c->carry_n[i];
    return PGMG_OK;
}

// JacobiSmoother(eps) (Smoother.hpp:38): a new threshold for the following calls.  The carried
// pre-smooth was checked against the old one, and the speculation history's predictions are
// relative to eps: both go (the statistics continue)
int pgmg_set_eps(pgmg_ctx *c, double eps)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    if (!(eps >= 0.0) || !std::isfinite(eps)) return set_err(PGMG_ERR_ARG, "eps must be finite and >= 0");
    PGMG_TRY(stream_wait(c));
    c->cfg.eps = eps;
    c->carry = false;
    if (c->gexec) {   // a captured cycle holds the old eps in its kernel arguments
        HIPC(hipGraphExecDestroy(c->gexec));
        c->gexec = nullptr;
    }
    c->spec_off = false;
    c->fspec_off = false;
    c->lvl_exact.assign(c->nb + 1, 0);
    c->lvl_fire.assign(c->nb + 1, 0);
    c->lvl_fire_block.assign(c->nb + 1, 0);
    c->lvl_fire_try.assign(c->nb + 1, 0.0);
    c->lvl_kx.assign(c->nb + 1, 0);
    c->lvl_vis.assign(c->nb + 1, 0);
    c->wmax.clear();
    c->wmin.clear();
    c->wrho.clear();
    c->wplan_gamma = 0;
    c->wplan_off = false;
    c->lvl_hist.assign(c->nb + 1, std::vector<double>());
    return PGMG_OK;
}

int pgmg_dist_info(pgmg_ctx *c, int *speculative, long long *rollbacks)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    if (speculative) *speculative = c->spec ? 1 : 0;
    if (rollbacks) *rollbacks = c->rollbacks;
    return PGMG_OK;
}

int pgmg_spec_levels(pgmg_ctx *c, unsigned long long *in_stream)
{
    if (!c || !in_stream) return set_err(PGMG_ERR_ARG, "null argument");
    unsigned long long m = (!c->spec || c->spec_off) ? 1ull : 0ull;
    for (int l = 1; l < (int)c->lvl_exact.size() && l < 64; ++l)
        if (c->lvl_exact[l] || c->lvl_fire[l]) m |= 1ull << l;
    *in_stream = m;
    return PGMG_OK;
}

int pgmg_spec_visit_modes(pgmg_ctx *c, long long counts[3])
{
    if (!c || !counts) return set_err(PGMG_ERR_ARG, "null argument");
    for (int i = 0; i < 3; ++i) counts[i] = c->wcount[i];
    return PGMG_OK;
}

int pgmg_spec_fire_levels(pgmg_ctx *c, unsigned long long *fire)
{
    if (!c || !fire) return set_err(PGMG_ERR_ARG, "null argument");
    unsigned long long m = 0;
    for (int l = 1; l < (int)c->lvl_fire.size() && l < 64; ++l)
        if (c->lvl_fire[l]) m |= 1ull << l;
    *fire = m;
    return PGMG_OK;
}

int pgmg_vcycle(pgmg_ctx *c, int ncycles) { return run_cycles(c, ncycles, 1); }
int pgmg_wcycle(pgmg_ctx *c, int ncycles) { return run_cycles(c, ncycles, c ? c->cfg.alpha : 1); }

// h of an N-point grid in the F-cycle's chain: 1/(n_coarse-1) halved once per level
// (MultiGridTestRunner.hpp:195, MultiGrid.hpp:171) — differs from a/(N-1) when a != 1
static double fmg_h(const pgmg_config &cfg, int N)
{
    double h = 1.0 / (cfg.n_coarse - 1);
    for (int n = cfg.n_coarse; n < N; n = 2 * n - 1) h /= 2;
    return h;
}

// sine tables of every level the F-cycle visits: bulk 0..nb-1, then the tail levels
static int fmg_tables(pgmg_ctx *c)
{
    if (c->fmg_tab) return PGMG_OK;
    std::vector<int> Ns;
    for (int l = 0; l < c->nb; ++l) Ns.push_back(c->lv[l].N);
    for (int N = c->lv[c->nb].N;; N = (N - 1) / 2 + 1) {
        Ns.push_back(N);
        if (N <= c->cfg.n_coarse) break;
    }
    std::vector<double> tab;
    c->fmg_off.clear();
    for (int N : Ns) {
        std::vector<double> sx, sy;
        double factor;
        sine_tables(c->cfg, N, fmg_h(c->cfg, N), sx, sy, factor);
        c->fmg_off.push_back((int)tab.size());
        tab.insert(tab.end(), sx.begin(), sx.end());
        tab.insert(tab.end(), sy.begin(), sy.end());
    }
    HIPC(hipMalloc((void **)&c->fmg_tab, tab.size() * sizeof(double)));
    HIPC(hipMemcpy(c->fmg_tab, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice));
    // the RHS of the FMG chain on every bulk level, regenerated in that level's passes like
    // set_problem's level-0 RHS: per level [8 | factor*sx (N) | 1024 | 8 | sy (N) | 16]
    if (c->nb > 0) {
        std::vector<double> g;
        c->fmg_goff.assign(c->nb, 0);
        for (int l = 0; l < c->nb; ++l) {
            const int N = c->lv[l].N;
            std::vector<double> sx, sy;
            double factor;
            sine_tables(c->cfg, N, fmg_h(c->cfg, N), sx, sy, factor);
            const size_t o = g.size(), nx = 8 + N + 1024, ny = 8 + N + 16;
            c->fmg_goff[l] = o;
            g.resize(o + nx + ny, 0.0);
            for (int i = 0; i < N; ++i) g[o + 8 + i] = factor * sx[i];
            for (int j = 0; j < N; ++j) g[o + nx + 8 + j] = sy[j];
        }
        HIPC(hipMalloc((void **)&c->fmg_gtab, g.size() * sizeof(double)));
        HIPC(hipMemcpy(c->fmg_gtab, g.data(), g.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    return PGMG_OK;
}

// One outer F-cycle (MultiGridTestRunner.hpp:192-205 -> MultigridSolver::f_cycle,
// MultiGrid.hpp:138-183) on the current solution A_0:
//   restrict phi to n_coarse (compute_coarsest_grid); then from the coarsest level up:
//   smooth(3); phi_fine = 0 + P phi; f_fine = analytic RHS; one V-cycle on the finer level.
// The levels at or below the tail's top run inside one k_tail launch; the bulk levels use
// the V-cycle kernels with the level's F replaced by the analytic RHS of the FMG chain.
}  // extern "C"

// smooth(3) of the F-cycle climb (MultiGrid.hpp:153) on a bulk level, fused: four sweeps in
// one pass into L.B with the three checks summed speculatively, the decision, the exact
// rare path (x_k from the untouched x0), then L.A and L.B trade places (both frames zero)
template <class T>
static int enqueue_smooth3_fused(pgmg_ctx *c, int l)
{
    Level &L = c->lv[l];
    const bool dist = is_dist(c, l);
    int e;
    // x0 is read 6 rows past the strip (the pass's pipeline), f is local (analytic)
    if (dist && (e = c->comm->halo(L.A, L, 6, c->s))) return e;
    PostPreArgsT<T> q{};
    q.phi = G<T>(L.A);
    q.f = G<T>(L.F);
    q.x4 = G<T>(L.B);
    q.gfx = l == c->gen_level ? c->lgfx : nullptr;   // the climb's level: f regenerated
    q.gsy = l == c->gen_level ? c->lgsy : nullptr;
    q.partials1 = c->partials;
    q.partials2 = c->partials2;
    q.partials3 = c->partials3;
    q.hh = (T)L.hh;
    q.ih = (T)L.ih;
    q.N = L.N;
    q.P = L.P;
    q.Nc = c->lv[l + 1].N;
    q.Pc = c->lv[l + 1].P;
    q.jc0 = L.lo / 2;
    q.jc1 = (L.hi < L.N ? L.hi : L.N - 1) / 2;
    q.row_lo = L.u0;
    q.row_hi = L.u1;
    q.rc_lo = 1;
    q.rc_hi = 1;
    const int np = postpre_blocks(L.N, q.jc0, q.jc1);
    if (c->lean && c->fspec) {
        // speculative F-cycles: the three checks recorded "does not fire" (the pass books its
        // four sweeps), no decision or rare-path launch
        q.partials1 = chk_log(c, np, l, 0);
        q.partials2 = chk_log(c, np, l, 0);
        q.partials3 = chk_log(c, np, l, 0);
        q.stats = c->stats;
        if ((e = launch_smooth4(q, c->s))) return e;
        std::swap(L.A, L.B);
        c->fsmooth_swapped = true;
        return PGMG_OK;
    }
    if ((e = launch_smooth4(q, c->s))) return e;
    const double *g3 = nullptr;
    if (dist) {
        launch_sum_partials(q.partials1, np, c->scalar, c->s);
        launch_sum_partials(q.partials2, np, c->scalar + 1, c->s);
        launch_sum_partials(q.partials3, np, c->scalar + 2, c->s);
        if ((e = c->comm->allreduce_sum(c->scalar, 3, c->s))) return e;
        g3 = c->scalar;
    }
    launch_smooth4_finish(q, np, g3, c->cfg.eps, c->ppflags, c->stats, c->s);
    std::swap(L.A, L.B);
    c->fsmooth_swapped = true;
    return PGMG_OK;
}

// opt: kFSaveTop -- keep a copy of the tail top's restricted grid (a speculative call's first
// F-cycle); kFFromTop -- skip the restriction, start the climb from that copy (its rerun);
// kFR2Next -- another F-cycle follows: the finest k_post forms level 2's restriction
// (k_post_r2); kFR2Done -- the previous F-cycle did: start the restriction at level 2
constexpr int kFSaveTop = 1, kFFromTop = 2, kFR2Next = 4, kFR2Done = 8;

template <class T>
static int enqueue_fcycle(pgmg_ctx *c, int opt = 0)
{
    const int nb = c->nb;
    double factor;
    {
        std::vector<double> sx, sy;
        sine_tables(c->cfg, 1, 1.0, sx, sy, factor);
    }
    int e;
    const bool use_r2 = !(c->cfg.flags & PGMG_FLAG_NO_R2);   // two restriction steps per pass
    if (opt & kFFromTop)
        HIPC(hipMemcpyAsync(c->lv[nb].A.base, c->ftop.base, c->ftop.bytes, hipMemcpyDeviceToDevice, c->s));
    // level 2's values already formed by the previous F-cycle's finest k_post (k_post_r2:
    // the pair 0 -> 2 below, bitwise)
    const bool from2 = (opt & kFR2Done) && c->fr2_made && use_r2 && nb >= 2 && !is_dist(c, 0) &&
                       !is_dist(c, 1);
    c->fr2_made = false;
    for (int l = (opt & kFFromTop) ? nb : (from2 ? 2 : 0); l < nb; ++l) {
        Level &L = c->lv[l], &C = c->lv[l + 1];
        if (!is_dist(c, l)) {
            // the intermediate level's restricted values are dead (the climb overwrites that
            // level's grid before reading it), so two levels go in one pass
            if (use_r2 && l + 2 <= nb && !is_dist(c, l + 1)) {
                const Level &C2 = c->lv[l + 2];
                launch_restrict2_values(G<T>(L.A), L.P, G<T>(C2.A), C2.N, C2.P, c->s);
                ++l;
                continue;
            }
            launch_restrict_values(G<T>(L.A), L.N, L.P, G<T>(C.A), C.N, C.P, c->s);
            continue;
        }
        // row strips: the rank's coarse rows from its fine rows and one halo row each side
        const StripRows sr = strip_rows(L, C);
        if ((e = c->comm->halo(L.A, L, 1, c->s))) return e;
        launch_restrict_values(G<T>(L.A), L.N, L.P, G<T>(C.A), C.N, C.P, c->s, sr.rc_lo, sr.rc_hi);
        // first replicated level: every rank's rows to every rank
        if (!is_dist(c, l + 1) && (e = c->comm->allgather_rows(c, l + 1, C.A))) return e;
    }
    if (opt & kFSaveTop)
        HIPC(hipMemcpyAsync(c->ftop.base, c->lv[nb].A.base, c->ftop.bytes, hipMemcpyDeviceToDevice, c->s));
    {
        Level &Lt = c->lv[nb];
        TailArgsT<T> t{};
        t.f_top = G<T>(Lt.F);
        t.e_top = G<T>(Lt.A);
        t.P_top = Lt.P;
        t.N_top = Lt.N;
        t.h_top = Lt.h;
        t.x0_from_global = 1;
        t.v1 = c->cfg.v1;
        t.v2 = c->cfg.v2;
        t.coarse_iter = c->cfg.coarse_iter;
        t.n_coarse = c->cfg.n_coarse;
        t.eps = c->cfg.eps;
        t.stats = c->stats;
        t.fmg = 1;
        t.fmg_smooth_top = nb > 0 ? 1 : 0;
        t.fmg_tab = c->fmg_tab;
        for (int k = 0; k < 8 && nb + k < (int)c->fmg_off.size(); ++k)
            t.fmg_tab_off[k] = c->fmg_off[nb + k];
        t.fmg_factor = factor;
        HIPC(launch_tail_gamma(t, 1, c->s));
    }
    for (int l = nb - 1; l >= 0; --l) {
        Level &L = c->lv[l];
        Level &C = c->lv[l + 1];
        const double *sx = c->fmg_tab + c->fmg_off[l];
        const bool dist = is_dist(c, l);
        // rows this rank holds: all, or (row strips) its strip and the halo rows, where the
        // analytic RHS is computed locally instead of exchanged
        const int r0 = dist ? std::max(0, L.lo - kHalo) : 0;
        const int r1 = dist ? std::min(L.N, L.hi + kHalo) : L.N;
        // the level's analytic RHS of the FMG h chain is the same on every call: computed
        // once into its own grid (Ffmg for level 0, Ffmg_l[l] below), which stands in for
        // L.F while this level runs (the V-cycle's restriction writes the coarser level's
        // own F, not its cached RHS)
        if (l > 0) {
            std::swap(L.F, c->Ffmg_l[l]);
            c->fmg_f_swapped = l;
        }
        if (!c->fmg_rhs_ready)
            launch_rhs(G<T>(L.F), sx, sx + L.N, factor, L.N, L.P, r0, r1, c->s);
        // this level's passes regenerate its analytic f (bitwise the stored one); its
        // rare paths and the coarser levels read theirs from memory
        // (PGMG_FLAG_STORED_RHS: rgfx is null, every level streams its RHS)
        if (l > 0 && c->rgfx != nullptr) {
            c->gen_level = l;
            c->lgfx = c->fmg_gtab + c->fmg_goff[l] + 8;
            c->lgsy = c->fmg_gtab + c->fmg_goff[l] + (8 + L.N + 1024) + 8;
        }
        // phi_fine = 0 + P phi_coarse (MultiGrid.hpp:159-164): the prolongation assigns the
        // interior, the frame (boundary, and row/column 1 the reference never corrects) is
        // zeroed; the ping-pong buffer's frame mirrors it
        launch_zero_frame(G<T>(L.A), L.P, L.N, c->s, r0, r1);
        launch_zero_frame(G<T>(L.B), L.P, L.N, c->s, r0, r1);
        if (l == 0 && c->S.base) launch_zero_frame(G<T>(c->S), L.P, L.N, c->s, r0, r1);   // S mirrors too
        const bool use_pin = !(c->cfg.flags & PGMG_FLAG_NO_PIN);
        if (c->fused && use_pin) {
            // the V-cycle's k_pre computes the prolongation on the fly (PIN): no separate
            // pass writing the zeroed fine grid; it reads 3 coarse rows past the strip
            if (dist && is_dist(c, l + 1) && (e = c->comm->halo(C.A, C, 3, c->s))) return e;
            c->fr2_want = l == 0 && (opt & kFR2Next) && use_r2;
            e = enqueue_fused_level<T>(c, l, 1, false, true);
            c->fr2_want = false;
            if (e) return e;
            if (l > 0 && (e = enqueue_smooth3_fused<T>(c, l))) return e;
            c->gen_level = 0;
            c->lgfx = c->lgsy = nullptr;
            if (l > 0) std::swap(L.F, c->Ffmg_l[l]);
            c->fmg_f_swapped = -1;
            continue;
        }
        // the prolongation of the rank's rows reads one coarse row past its strip
        if (dist && is_dist(c, l + 1) && (e = c->comm->halo(C.A, C, 1, c->s))) return e;
        ProlongArgsT<T> p{};
        p.c = G<T>(C.A);
        p.fine = G<T>(L.A);
        p.Wf = L.N;
        p.Pf = L.P;
        p.Wc = C.N;
        p.Pc = C.P;
        p.row0 = dist ? std::max(L.u0, 2) : 2;
        p.row1 = dist ? std::min(L.u1, L.N - 1) : L.N - 1;
        p.assign = 1;
        if (p.row1 > p.row0) launch_prolong(p, c->s);
        e = enqueue_cycle_t<T>(c, l, 1, false);
        if (e) return e;
        // the V-cycle above regenerated this level's f where its passes are fused; the
        // general smooth(3) below streams the cached RHS
        c->gen_level = 0;
        c->lgfx = c->lgsy = nullptr;
        if (l > 0 && (e = enqueue_smooth<T>(c, l, 0, 3, false))) return e;
        if (l > 0) std::swap(L.F, c->Ffmg_l[l]);
        c->fmg_f_swapped = -1;
    }
    return PGMG_OK;
}

// Speculative F-cycles (one GPU).  The climb's V-cycles and smooth(3) passes decide their
// early-exit checks in-stream by default: a decision launch after every bulk pass and every
// fused smooth(3), ~86 launches of ~5 us per F-cycle at N = 16385 (9 % of it), while on the
// reference problem no bulk check of an F-cycle fires (the F goldens: 0 exits).  A call of F
// cycles is therefore enqueued with every bulk check recorded "does not fire" (the V-cycles'
// mode 0; smooth(3)'s three checks too, its pass booking the four sweeps) and validated once
// after the call, like the V-cycles' speculative calls.  A rollback needs no copy of the
// level-0 solution: an F-cycle reads phi only through the restriction chain, whose one live
// result is the tail top's grid (the intermediate levels' values are dead, the climb
// overwrites them), so the first F-cycle's tail-top grid is kept (kFSaveTop) and the rerun --
// every F-cycle of the call decided in-stream, bitwise the in-stream call -- starts its first
// climb from it (kFFromTop).  The level buffers the smooth(3) passes swap and the statistics
// are restored first.  A rolled-back problem keeps its F-cycles in-stream (fspec_off).
template <class T>
static int run_fcycles_spec(pgmg_ctx *c, int ncycles)
{
    const int nb = c->nb;
    // log: per F-cycle, every climb level's V-cycle (the level and all below it) and the three
    // smooth(3) checks of the levels below the finest
    long long dbl = 64, nchk = 4;
    for (int l = 0; l < nb; ++l) {
        long long d, k;
        spec_need_level(c, l, 1, &d, &k);
        dbl += (long long)ncycles * d;
        nchk += (long long)ncycles * k;
        if (l == 0) {   // the finest k_post as k_post_r2 (more workgroups than k_post)
            const Level &L = c->lv[0];
            dbl += (long long)ncycles * post_r2_blocks(L.N, L.lo / 2, (L.hi < L.N ? L.hi : L.N - 1) / 2);
        }
        if (l > 0) {
            const Level &L = c->lv[l];
            dbl += 3LL * ncycles * postpre_blocks(L.N, L.lo / 2, (L.hi < L.N ? L.hi : L.N - 1) / 2);
            nchk += 3LL * ncycles;
        }
    }
    int e = spec_reserve(c, dbl, nchk);
    if (e) return e;
    if (!c->ftop.base && (e = alloc_grid(c->ftop, c->lv[nb]))) return e;
    std::vector<Grid> A0(nb + 1), B0(nb + 1);
    for (int l = 0; l <= nb; ++l) {
        A0[l] = c->lv[l].A;
        B0[l] = c->lv[l].B;
    }
    // stats backup + the coarse levels' "pre-smooth fired" flags (written by the skipped rare
    // paths) = 0
    launch_spec_open(c->stats, c->stats_bk, c->flags, (int)(c->lv.size() + 1) * 2 * kMaxSweeps, c->s);
    c->lean = true;
    c->fspec = true;
    c->spec_gamma = 1;
    c->plog_used = 0;
    c->chks.clear();
    c->chk_visit.clear();
    c->wvisit = 0;
    c->cur_visit = -1;
    c->fr2_made = false;
    for (int k = 0; k < ncycles && !e; ++k) {
        // consecutive F-cycles: the finest k_post of one forms the next one's level 2
        const int opt = (k == 0 ? kFSaveTop : kFR2Done) | (k + 1 < ncycles ? kFR2Next : 0);
        e = enqueue_fcycle<T>(c, opt);
        if (!e) c->fmg_rhs_ready = true;
    }
    c->lean = false;
    c->fspec = false;
    c->fr2_made = false;
    if (e) return e;
    unsigned h = 0;
    bool overflow = false;
    if ((e = spec_validate(c, &h, &overflow, (int)c->chks.size()))) return e;
    if (!h) return PGMG_OK;
    ++c->rollbacks;
    c->fspec_off = true;
    for (int l = 0; l <= nb; ++l) {
        c->lv[l].A = A0[l];
        c->lv[l].B = B0[l];
    }
    HIPC(hipMemcpyAsync(c->stats, c->stats_bk, 4 * sizeof(unsigned long long),
                        hipMemcpyDeviceToDevice, c->s));
    // (in-stream: no k_post_r2, every F-cycle restricts from level 0)
    for (int k = 0; k < ncycles && !e; ++k) e = enqueue_fcycle<T>(c, k == 0 ? kFFromTop : 0);
    return e;
}

extern "C" {

int pgmg_fcycle(pgmg_ctx *c, int ncycles)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    if (!c->have_problem) return set_err(PGMG_ERR_STATE, "pgmg_set_problem first");
    if (ncycles <= 0) return PGMG_OK;
    c->carry = false;   // an F-cycle starts from phi itself
    int e = fmg_tables(c);
    if (e) return e;
    Level &L0 = c->lv[0];
    if (c->nb > 0 && !c->Ffmg.base && (e = alloc_grid(c->Ffmg, L0))) return e;
    if ((int)c->Ffmg_l.size() < c->nb) {
        c->Ffmg_l.resize(c->nb);
        for (int l = 1; l < c->nb; ++l)
            if ((e = alloc_grid(c->Ffmg_l[l], c->lv[l]))) return e;
    }
    // the F-cycle's levels use the FMG h chain and (level 0) the analytic RHS of that chain
    // (every level including the tail's top, whose h enqueue_tail passes on).  Everything
    // the F-cycle changes on the context is undone by the guard on EVERY exit path (an
    // error half-way through the climb included), so later V/W-cycles see the user's f,
    // h and no regenerated-RHS level.
    struct Restore {
        pgmg_ctx *c;
        std::vector<Level> saved;
        const double *sgx, *sgy;
        bool f0_swapped = false;
        ~Restore()
        {
            if (c->fmg_f_swapped > 0) {
                std::swap(c->lv[c->fmg_f_swapped].F, c->Ffmg_l[c->fmg_f_swapped]);
                c->fmg_f_swapped = -1;
            }
            if (f0_swapped) std::swap(c->lv[0].F, c->Ffmg);
            c->gen_level = 0;
            c->lgfx = c->lgsy = nullptr;
            c->rgfx = sgx;
            c->rgsy = sgy;
            for (int l = 0; l <= c->nb; ++l) {
                c->lv[l].h = saved[l].h;
                c->lv[l].hh = saved[l].hh;
                c->lv[l].ih = saved[l].ih;
            }
        }
    } guard{c, c->lv, c->rgfx, c->rgsy};
    for (int l = 0; l <= c->nb; ++l) {
        Level &L = c->lv[l];
        const double h = fmg_h(c->cfg, L.N);
        L.h = h;
        L.hh = h * h;
        L.ih = 1.0 / (h * h);
    }
    if (c->nb > 0) {
        std::swap(L0.F, c->Ffmg);
        guard.f0_swapped = true;
    }
    const bool gen = c->nb > 0 && !(c->cfg.flags & PGMG_FLAG_STORED_RHS);
    c->rgfx = gen ? c->fmg_gtab + 8 : nullptr;
    c->rgsy = gen ? c->fmg_gtab + (8 + L0.N + 1024) + 8 : nullptr;
    // a device-bound problem (pgmg_set_problem_device): the F-cycle restricts and climbs on
    // the level-0 grids, so the caller's phi is staged into L.A first (after in-place V/W
    // calls L.A is stale: those calls read and write the caller's array) and the result is
    // copied back; synchronous, like the V/W calls on a bound problem
    const bool ext = c->ext_phi != nullptr;
    if (ext) PGMG_TRY(ext_stage_in(c, false));
    HIPC(hipEventRecord(c->ev0, c->s));
    // speculative F-cycles: one GPU, the fused climb (PIN), not EXACT_DIST, not after a rollback
    const bool fspec = c->nb > 0 && c->fused && c->comm == nullptr && !c->fspec_off &&
                       !(c->cfg.flags & (PGMG_FLAG_EXACT_DIST | PGMG_FLAG_NO_PIN));
    if (fspec) {
        e = c->fp32 ? run_fcycles_spec<float>(c, ncycles) : run_fcycles_spec<double>(c, ncycles);
    } else {
        for (int k = 0; k < ncycles && !e; ++k) {
            e = c->fp32 ? enqueue_fcycle<float>(c) : enqueue_fcycle<double>(c);
            if (!e) c->fmg_rhs_ready = true;
        }
    }
    if (c->fsmooth_swapped && c->gexec) {   // its level buffers traded places: recapture
        PGMG_TRY(stream_wait(c));
        HIPC(hipGraphExecDestroy(c->gexec));
        c->gexec = nullptr;
    }
    c->fsmooth_swapped = false;
    if (e) return e;
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(c->ev1, c->s));
    if (ext) {
        PGMG_TRY(ext_stage_out(c));
        PGMG_TRY(stream_wait(c));
    }
    return PGMG_OK;
}

int pgmg_sync(pgmg_ctx *c)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    PGMG_TRY(stream_wait(c));
    return PGMG_OK;
}

int pgmg_last_elapsed_ms(pgmg_ctx *c, double *ms)
{
    if (!c || !ms) return set_err(PGMG_ERR_ARG, "null argument");
    HIPC(hipEventSynchronize(c->ev1));
    float f = 0.f;
    HIPC(hipEventElapsedTime(&f, c->ev0, c->ev1));
    *ms = f;
    return PGMG_OK;
}

int pgmg_get_solution(pgmg_ctx *c, double *phi)
{
    return pgmg_gather_solution(c, -1, phi);
}

int pgmg_gather_solution(pgmg_ctx *c, int root, double *phi)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    const int me = c->comm ? c->comm->rank() : 0;
    if (root >= c->cfg.world) return set_err(PGMG_ERR_ARG, "root >= world");
    // without strips every rank holds the whole solution: every root means this rank
    if (!phi && (root < 0 || root == me || !c->comm))
        return set_err(PGMG_ERR_ARG, "null phi on a receiving rank");
    if (c->comm) {
        int e = c->comm->wait(c->s);
        if (e) return e;
        return c->comm->gather_solution(c, phi, root);
    }
    PGMG_TRY(stream_wait(c));
    Level &L = c->lv[0];
    if (c->ext_phi) {   // a device-bound problem: the solution is the caller's array
        HIPC(hipMemcpy(phi, c->ext_phi, (size_t)L.N * L.N * sizeof(double), hipMemcpyDeviceToHost));
        return PGMG_OK;
    }
    return download_grid(c, L.A.o, L.P, L.N, phi);
}

// FNV-64 over the IEEE words of phi in the reference layout: the checksum the golden
// fixtures of the reference's runs carry (bench.py verifies the run it timed with it)
int pgmg_solution_hash(pgmg_ctx *c, int root, unsigned long long *out)
{
    if (!c || !out) return set_err(PGMG_ERR_ARG, "null argument");
    const int me = c->comm ? c->comm->rank() : 0;
    if (root >= c->cfg.world) return set_err(PGMG_ERR_ARG, "root >= world");
    const bool want = root < 0 || root == me || !c->comm;
    const long long n = (long long)c->lv[0].N * c->lv[0].N;
    std::vector<double> phi(want ? (size_t)n : 0);
    int e = pgmg_gather_solution(c, root, want ? phi.data() : nullptr);
    if (e) return e;
    unsigned long long h = 1469598103934665603ULL;
    if (want) {
        for (long long i = 0; i < n; ++i) {
            unsigned long long w;
            std::memcpy(&w, &phi[(size_t)i], 8);
            h = (h ^ w) * 1099511628211ULL;
        }
    }
    *out = want ? h : 0ULL;
    return PGMG_OK;
}

int pgmg_residual_norm(pgmg_ctx *c, double *out)
{
    if (!c || !out) return set_err(PGMG_ERR_ARG, "null argument");
    Level &L = c->lv[0];
    int nbk = c->partials_cap < 1024 ? c->partials_cap : 1024;
    // a device-bound problem: its phi (and a caller's f) into the level-0 grids first (the
    // analytic f is in L.F since pgmg_set_problem_device)
    if (c->ext_phi) PGMG_TRY(ext_stage_in(c, false));
    if (c->comm) {
        int e = c->comm->halo(L.A, L, 1, c->s);
        if (e) return e;
    }
    if (c->fp32)
        launch_resnorm_partials(G<float>(L.A), G<float>(L.F), c->partials, (float)L.ih, L.N, L.P,
                                L.u0, L.u1, nbk, c->s);
    else
        launch_resnorm_partials(G<double>(L.A), G<double>(L.F), c->partials, L.ih, L.N, L.P, L.u0,
                                L.u1, nbk, c->s);
    launch_sum_partials(c->partials, nbk, c->scalar, c->s);
    if (c->comm) {
        int e = c->comm->allreduce_sum(c->scalar, 1, c->s);
        if (e) return e;
    }
    double s = 0.0;
    HIPC(hipMemcpyAsync(&s, c->scalar, sizeof(double), hipMemcpyDeviceToHost, c->s));
    PGMG_TRY(stream_wait(c));
    *out = std::sqrt(s);
    return PGMG_OK;
}

int pgmg_stats(pgmg_ctx *c, long long *sweeps, long long *exits)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    unsigned long long h[4];
    PGMG_TRY(stream_wait(c));
    HIPC(hipMemcpy(h, c->stats, sizeof(h), hipMemcpyDeviceToHost));
    if (sweeps) *sweeps = (long long)h[0];
    if (exits) *exits = (long long)h[1];
    return PGMG_OK;
}

int pgmg_stats_detail(pgmg_ctx *c, long long *out4)
{
    if (!c || !out4) return set_err(PGMG_ERR_ARG, "null argument");
    unsigned long long h[4];
    PGMG_TRY(stream_wait(c));
    HIPC(hipMemcpy(h, c->stats, sizeof(h), hipMemcpyDeviceToHost));
    for (int i = 0; i < 4; ++i) out4[i] = (long long)h[i];
    out4[2] = c->cross ? out4[2] : -1;
    return PGMG_OK;
}

int pgmg_levels(pgmg_ctx *c, int *bulk, int *tail_top)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    if (bulk) *bulk = c->nb;
    if (tail_top) *tail_top = c->lv[c->nb].N;
    return PGMG_OK;
}

// algorithmic bytes of one V-cycle on this rank (DESIGN.md "Roofline accounting")
int pgmg_vcycle_bytes(pgmg_ctx *c, double *bytes)
{
    if (!c || !bytes) return set_err(PGMG_ERR_ARG, "null argument");
    double b = 0.0;
    for (int l = 0; l < c->nb; ++l) {
        const Level &L = c->lv[l];
        const Level &C = c->lv[l + 1];
        const double n = (double)(L.u1 - L.u0) * (L.N - 2);
        const double nc = (double)(C.u1 - C.u0) * (C.N - 2);
        if (c->fused) {
            if (l == 0 && c->cross) {                     // steady state: one k_postpre
                b += (c->rgfx ? 16.0 : 24.0) * n + 16.0 * nc;     // phi, (f,) ec in; x4, rc out
                continue;
            }
            if (l > 0 && c->recompute) {                  // x0 = 0, x2 recomputed
                b += 8.0 * n + 8.0 * nc;                  // k_pre: f in; rc out
                b += 16.0 * n + 8.0 * nc;                 // k_post: f, ec in; x2 out
                continue;
            }
            const double fb = (l == 0 && c->rgfx) ? 0.0 : 8.0;  // level 0: f regenerated
            b += (l == 0 ? 16.0 + fb : 16.0) * n + 8.0 * nc;   // k_pre: x0, f in; x2, rc out
            b += (16.0 + fb) * n + 8.0 * nc;                    // k_post: phi, f, ec in; x2 out
            continue;
        }
        const int S1 = c->cfg.v1 + 1, S2 = c->cfg.v2 + 1;
        b += (l == 0 ? 24.0 : 16.0) * n + 24.0 * n * (S1 - 1);  // pre-smooth
        b += 16.0 * n + 8.0 * nc;                                // residual + restriction
        b += 16.0 * n + 8.0 * nc;                                // prolongation (RMW fine)
        b += 24.0 * n * S2;                                      // post-smooth
        if (S1 & 1) b += 16.0 * n;
        if (S2 & 1) b += 16.0 * n;
    }
    const Level &Lt = c->lv[c->nb];
    b += 16.0 * (double)Lt.N * Lt.N;                             // tail: f in, e out
    *bytes = b * (c->lv[0].es / 8.0);                            // per-point figures are fp64
    return PGMG_OK;
}

int pgmg_fine_pass_bytes(pgmg_ctx *c, int pass, double *bytes)
{
    if (!c || !bytes || pass < 0 || pass > 5) return set_err(PGMG_ERR_ARG, "bad argument");
    if (c->nb == 0) return set_err(PGMG_ERR_STATE, "no bulk level");
    const Level &L = c->lv[0], &C = c->lv[1];
    const double n = (double)(L.u1 - L.u0) * (L.N - 2);
    const StripRows sr = strip_rows(L, C);
    const double nc = (double)(sr.rc_hi > sr.rc_lo ? sr.rc_hi - sr.rc_lo : 0) * (C.N - 2);
    double b = 0.0;
    // f is regenerated in-kernel (not read) by the level-0 passes
    const double fb = c->rgfx != nullptr ? 0.0 : 8.0;
    switch (pass) {
    case 0: b = 24.0 * n; break;                               // x, f in; x out
    case 1: b = (16.0 + fb) * n + 8.0 * nc; break;             // x0, (f) in; x2, rc out
    case 2: b = (16.0 + fb) * n + 8.0 * nc; break;             // phi, (f,) ec in; x2 out
    case 3: b = (16.0 + fb) * n + 16.0 * nc; break;            // phi, (f,) ec; x4, rc
    case 4: b = (16.0 + fb) * n + 16.0 * nc; break;            // carry pass: x2 for x4
    case 5: b = (16.0 + fb) * n + 16.0 * nc; break;            // recompute form: phi = x2
    }
    *bytes = b * (L.es / 8.0);
    return PGMG_OK;
}

int pgmg_precision(pgmg_ctx *c, int *precision, int *elem_bytes)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    if (precision) *precision = c->fp32 ? PGMG_PRECISION_FP32 : PGMG_PRECISION_FP64;
    if (elem_bytes) *elem_bytes = c->lv[0].es;
    return PGMG_OK;
}

int pgmg_check_span(const void *origin, long long pitch, int elem_bytes, long long row0,
                    long long row1, long long col0, long long col1)
{
    if (!origin || pitch <= 0 || elem_bytes <= 0 || row1 < row0 || col1 < col0)
        return set_err(PGMG_ERR_ARG, "pgmg_check_span: bad arguments");
    return check_span(origin, pitch, elem_bytes, row0, row1, col0, col1, "pgmg_check_span");
}

int pgmg_phi_device(pgmg_ctx *c, double **ptr, int *pitch, int *row0, int *rows)
{
    if (!c) return set_err(PGMG_ERR_ARG, "null ctx");
    Level &L = c->lv[0];
    c->carry = false;   // the pointer allows writes to phi
    if (ptr) *ptr = static_cast<double *>(L.A.o);
    if (pitch) *pitch = L.P;
    if (row0) *row0 = L.lo;
    if (rows) *rows = L.hi - L.lo;
    return PGMG_OK;
}

}  // extern "C"

template <class T>
static void bench_sweeps(pgmg_ctx *c, int reps)
{
    Level &L = c->lv[0];
    SweepArgsT<T> a{};
    a.f = G<T>(L.F);
    a.hh = (T)L.hh;
    a.inv_hh = (T)L.ih;
    a.W = L.N;
    a.P = L.P;
    a.row0 = L.u0;
    a.row1 = L.u1;
    for (int k = 0; k < reps; ++k) {
        a.xin = G<T>((k & 1) ? L.B : L.A);
        a.xout = G<T>((k & 1) ? L.A : L.B);
        launch_sweep(a, false, true, c->s);
    }
}

extern "C" {

int pgmg_bench_sweep(pgmg_ctx *c, int reps, double *ms)
{
    if (!c || !ms || reps <= 0) return set_err(PGMG_ERR_ARG, "bad argument");
    if (c->nb == 0) return set_err(PGMG_ERR_STATE, "no bulk level");
    c->carry = false;   // the sweeps overwrite phi
    auto run = [&](int n) { c->fp32 ? bench_sweeps<float>(c, n) : bench_sweeps<double>(c, n); };
    run(2);  // warm
    HIPC(hipEventRecord(c->ev0, c->s));
    run(reps);
    HIPC(hipEventRecord(c->ev1, c->s));
    HIPC(hipEventSynchronize(c->ev1));
    float f = 0.f;
    HIPC(hipEventElapsedTime(&f, c->ev0, c->ev1));
    *ms = f / reps;
    return PGMG_OK;
}

int pgmg_fine_pass_time(pgmg_ctx *c, int pass, int *count, double *mean_ms)
{
    if (!c || pass < 0 || pass > 5) return set_err(PGMG_ERR_ARG, "bad argument");
    PGMG_TRY(stream_wait(c));
    auto &pool = c->tpool[pass];
    double tot = 0.0;
    const int n = pool.used / 2;
    for (int i = 0; i < n; ++i) {
        float f = 0.f;
        HIPC(hipEventElapsedTime(&f, pool.ev[2 * i], pool.ev[2 * i + 1]));
        tot += f;
    }
    if (count) *count = n;
    if (mean_ms) *mean_ms = n ? tot / n : 0.0;
    pool.used = 0;
    c->info_bytes[pass] = n ? c->tbytes[pass] / n : 0.0;
    c->info_kern[pass] = n ? c->tkern[pass] : nullptr;
    c->tbytes[pass] = 0.0;
    c->tkern[pass] = nullptr;
    return PGMG_OK;
}

int pgmg_fine_pass_info(pgmg_ctx *c, int pass, char *symbol, int len, double *bytes)
{
    if (!c || pass < 0 || pass > 5 || (symbol && len < 1)) return set_err(PGMG_ERR_ARG, "bad argument");
    if (bytes) *bytes = c->info_bytes[pass];
    if (symbol) {
        std::string name;
        if (c->info_kern[pass]) {
            const char *m = hipKernelNameRefByPtr(c->info_kern[pass], c->s);
            if (m) {
                int st = 0;
                char *d = abi::__cxa_demangle(m, nullptr, nullptr, &st);
                name = (st == 0 && d) ? d : m;
                std::free(d);
            }
        }
        std::snprintf(symbol, (size_t)len, "%s", name.c_str());
    }
    return PGMG_OK;
}

int pgmg_fine_sweep_time(pgmg_ctx *c, int *count, double *mean_ms)
{
    return pgmg_fine_pass_time(c, 0, count, mean_ms);
}

int pgmg_fused(pgmg_ctx *c, int *fused)
{
    if (!c || !fused) return set_err(PGMG_ERR_ARG, "bad argument");
    *fused = c->fused ? 1 : 0;
    return PGMG_OK;
}

}  // extern "C"
