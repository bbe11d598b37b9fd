// pgmg_ops.hip — op-level C ABI on caller-owned device arrays (reference layout)
// mirroring Parallel::ComputeJacobi / ComputeResidual / ComputeRestriction /
// ComputeProlungator (3_part_parallel/Parallel_Method.cu:144-199), plus device
// memory helpers so host code can drive the library without HIP headers.
//
// Like the reference's, the Jacobi op updates the caller's x in place -- but race-free: its
// passes defer every tile-edge output another workgroup reads (pgmg_gops.hip "In-place
// sweeps"; the reference's jacobi_kernel races), so each sweep is exactly the
// out-of-place Jacobi sweep; with eps >= 0 it applies the CPU smoother's residual-norm early
// exit, so its result equals JacobiSmoother::smooth bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>

#include <cmath>
#include <map>
#include <mutex>
#include <vector>

#include "pgmg_ctx.h"

using namespace pgmg;

#define HIPC(expr) PGMG_HIPC(expr)

namespace {

struct OpScratch {
    double *partials = nullptr;
    unsigned *flags = nullptr;
    unsigned long long *stats = nullptr;
    double *scalar = nullptr;
    double *tmp = nullptr;
    size_t tmp_elems = 0;
    double *side = nullptr;   // the in-place passes' deferred tile-edge outputs
    size_t side_elems = 0;
};

// One scratch set per stream: ops enqueued on different streams never share partial sums,
// flags or the ping-pong buffer (the reference's ops are synchronous on the default stream;
// these are asynchronous on the caller's).  A set lives until pgmg_ops_release(stream).
std::mutex g_op_mu;
std::map<hipStream_t, OpScratch> g_ops;

int ensure_scratch(hipStream_t s, size_t tmp_elems, OpScratch **out)
{
    std::lock_guard<std::mutex> lk(g_op_mu);
    OpScratch &o = g_ops[s];
    if (!o.partials) {
        HIPC(hipMalloc((void **)&o.partials, kOpPartialsCap * sizeof(double)));
        HIPC(hipMalloc((void **)&o.flags, (kMaxSweeps + 2) * 128 * sizeof(unsigned)));
        HIPC(hipMalloc((void **)&o.stats, 4 * sizeof(unsigned long long)));
        HIPC(hipMalloc((void **)&o.scalar, 4 * sizeof(double)));
    }
    if (tmp_elems > o.tmp_elems) {
        if (o.tmp) {
            HIPC(hipStreamSynchronize(s));   // the old buffer may still be in use on s
            HIPC(hipFree(o.tmp));
        }
        o.tmp = nullptr;
        o.tmp_elems = 0;
        HIPC(hipMalloc((void **)&o.tmp, tmp_elems * sizeof(double)));
        o.tmp_elems = tmp_elems;
    }
    *out = &o;
    return PGMG_OK;
}

int ensure_side(hipStream_t s, OpScratch &o, size_t elems)
{
    std::lock_guard<std::mutex> lk(g_op_mu);
    if (elems <= o.side_elems) return PGMG_OK;
    if (o.side) {
        HIPC(hipStreamSynchronize(s));
        HIPC(hipFree(o.side));
    }
    o.side = nullptr;
    o.side_elems = 0;
    HIPC(hipMalloc((void **)&o.side, elems * sizeof(double)));
    o.side_elems = elems;
    return PGMG_OK;
}

}  // namespace

extern "C" {

int pgmg_jacobi(double *d_x, double *d_tmp, const double *d_f, int H, int W, double h, int v,
                double eps, int *sweeps_done, void *stream)
{
    if (!d_x || !d_f || H < 3 || W < 3 || v < 0) return set_err(PGMG_ERR_ARG, "pgmg_jacobi: bad argument");
    hipStream_t s = (hipStream_t)stream;
    const size_t L = (size_t)H * W;
    const int S = v + 1;
    const bool check = eps >= 0.0;
    // every sweep runs in place; only a checked call with v >= 1 needs a ping-pong buffer
    const bool need_tmp = check && S >= 2;
    OpScratch *op = nullptr;
    int e = ensure_scratch(s, (d_tmp || !need_tmp) ? 0 : L, &op);
    if (e) return e;
    OpScratch &g_op = *op;
    // the deferred-edge side buffer: only the passes that sweep in place use it (an unchecked
    // call, or the first sweep of a checked call with an odd count; an even checked count is
    // the ping-pong below)
    if ((!check || (S & 1)) && (e = ensure_side(s, g_op, g_defer_elems(H, W)))) return e;
    double *tmp = d_tmp ? d_tmp : g_op.tmp;
    // flag slots: a fresh block of S+1 words per call would need a ring; the op is
    // synchronous w.r.t. its own flags because every launch is stream-ordered.
    unsigned *D = g_op.flags;
    // the sweep counter is read back only for a caller that asks for it
    if (sweeps_done) HIPC(hipMemsetAsync(g_op.stats, 0, 4 * sizeof(unsigned long long), s));
    const double hh = h * h, ih = 1.0 / (h * h);
    const int nb = g_blocks(H, W);
    if (nb > kOpPartialsCap) return set_err(PGMG_ERR_STATE, "pgmg_jacobi: too many blocks");
    if (check && S >= (kMaxSweeps + 2) * 128)
        return set_err(PGMG_ERR_ARG, "pgmg_jacobi: v too large for the early-exit flags");
    auto finish = [&]() -> int {
        HIPC(hipGetLastError());
        if (sweeps_done) {
            unsigned long long st[4];
            HIPC(hipMemcpyAsync(st, g_op.stats, sizeof(st), hipMemcpyDeviceToHost, s));
            HIPC(hipStreamSynchronize(s));
            *sweeps_done = (int)st[0];
        }
        return PGMG_OK;
    };
    if (!check) {
        // the reference GPU op (ComputeJacobi decides nothing between its v+1 sweeps,
        // Parallel_Method.cu:144-160): every sweep on d_x itself, in pairs (k_op_sweep2_ip)
        // with an odd count's single sweep first (k_op_sweep_ip); no tmp, no copy-back
        int left = S;
        if (left & 1) {
            launch_g_sweep_ip(d_x, d_f, g_op.side, &D[1], g_op.stats, hh, H, W, s);
            left -= 1;
        }
        for (; left > 0; left -= 2) launch_g_sweep2_ip(d_x, d_f, g_op.side, g_op.stats, hh, H, W, s);
        return finish();
    }
    if (S & 1) {
        // JacobiSmoother::smooth's checks (Smoother.hpp:59-88) with an odd sweep count: sweep
        // 1 has no check and runs in place; sweeps k = 2 .. S alternate x -> tmp -> x, each
        // deciding the previous sweep's check (k_g_fixup undoes the sweep after a firing
        // check) and ending in x; the first of them also writes x's boundary into tmp (no
        // seed copy).  An even count is the ping-pong below, which ends in x by itself.
        launch_g_sweep_ip(d_x, d_f, g_op.side, &D[1], g_op.stats, hh, H, W, s);
        for (int k = 2; k <= S; ++k) {
            const double *in = (k & 1) ? tmp : d_x;
            double *out = (k & 1) ? d_x : tmp;
            launch_g_sweep(in, d_f, out, g_op.partials, &D[k - 1], nullptr, g_op.stats, hh, ih,
                           H, W, k == 2, s);
            launch_g_fixup(g_op.partials, nb, eps, &D[k - 1], &D[k], in, out, g_op.stats, H, W, s);
        }
        return finish();
    }
    // ping-pong (an even checked count): sweeps alternate x -> tmp -> x and end in x.  No
    // seed copy of tmp (Smoother.hpp:47 copies the whole grid into its output buffer): the first
    // sweep writes x's boundary into tmp besides the interior, which is all a later sweep reads
    for (int k = 1; k <= S; ++k) {
        const double *in = (k & 1) ? d_x : tmp;
        double *out = (k & 1) ? tmp : d_x;
        const bool with_check = check && k >= 2;
        launch_g_sweep(in, d_f, out, with_check ? g_op.partials : nullptr,
                       with_check ? &D[k - 1] : nullptr, k == 1 ? &D[1] : nullptr, g_op.stats, hh,
                       ih, H, W, k == 1, s);
        if (with_check)
            launch_g_fixup(g_op.partials, nb, eps, &D[k - 1], &D[k], in, out, g_op.stats, H, W, s);
    }
    return finish();
}

int pgmg_residual(double *d_r, const double *d_x, const double *d_f, int H, int W, double h,
                  void *stream)
{
    if (!d_r || !d_x || !d_f || H < 3 || W < 3) return set_err(PGMG_ERR_ARG, "pgmg_residual: bad argument");
    launch_g_residual(d_r, d_x, d_f, 1.0 / (h * h), H, W, (hipStream_t)stream);
    HIPC(hipGetLastError());
    return PGMG_OK;
}

int pgmg_restrict(const double *d_fine, double *d_coarse, int Nf, int Nc, void *stream)
{
    if (!d_fine || !d_coarse || Nc < 3 || Nf != 2 * Nc - 1)
        return set_err(PGMG_ERR_ARG, "pgmg_restrict: need Nf == 2*Nc - 1");
    launch_g_restrict(d_fine, d_coarse, Nf, Nc, (hipStream_t)stream);
    HIPC(hipGetLastError());
    return PGMG_OK;
}

int pgmg_prolong(const double *d_coarse, double *d_fine, int Nc, int Nf, int mode, void *stream)
{
    return pgmg_prolong_grid(d_coarse, d_fine, Nc, Nf, mode, 0, stream);
}

int pgmg_prolong_grid(const double *d_coarse, double *d_fine, int Nc, int Nf, int mode,
                      int num_thread, void *stream)
{
    if (!d_fine || !d_coarse || Nc < 3 || Nf != 2 * Nc - 1 || (mode != 0 && mode != 1) ||
        num_thread < 0)
        return set_err(PGMG_ERR_ARG, "pgmg_prolong: need Nf == 2*Nc - 1, mode 0|1, num_thread >= 0");
    // ComputeProlungator's launch: max(1, fine_N / num_thread) blocks of num_thread per side
    const int ext = num_thread > 0 ? std::max(1, Nf / num_thread) * num_thread : Nf;
    launch_g_prolong(d_coarse, d_fine, Nc, Nf, mode, ext, (hipStream_t)stream);
    HIPC(hipGetLastError());
    return PGMG_OK;
}

int pgmg_norm(const double *d_v, long long n, double *result, void *stream)
{
    if (!d_v || n < 0 || !result) return set_err(PGMG_ERR_ARG, "pgmg_norm: bad argument");
    hipStream_t s = (hipStream_t)stream;
    OpScratch *op = nullptr;
    int e = ensure_scratch(s, 0, &op);
    if (e) return e;
    OpScratch &g_op = *op;
    long long nb = (n + kBlock - 1) / kBlock;
    if (nb > 1024) nb = 1024;   // <= kOpPartialsCap
    if (nb < 1) nb = 1;
    launch_g_sumsq(d_v, n, g_op.partials, (int)nb, s);
    launch_sum_partials(g_op.partials, (int)nb, g_op.scalar, s);
    double sum = 0.0;
    HIPC(hipMemcpyAsync(&sum, g_op.scalar, sizeof(double), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    *result = std::sqrt(sum);
    return PGMG_OK;
}

int pgmg_rhs(double *d_f, int W, int H, double h, double a, double p, double q, void *stream)
{
    if (!d_f || W < 1 || H < 1) return set_err(PGMG_ERR_ARG, "pgmg_rhs: bad argument");
    hipStream_t s = (hipStream_t)stream;
    const double factor = (M_PI * M_PI / (a * a)) * (p * p + q * q);  // DynamicGridUtils.hpp:113
    std::vector<double> t(W + H);
    for (int i = 0; i < W; ++i) t[i] = std::sin(p * M_PI * (i * h) / a);
    for (int j = 0; j < H; ++j) t[W + j] = std::sin(q * M_PI * (j * h) / a);
    double *d = nullptr;
    HIPC(hipMalloc((void **)&d, t.size() * sizeof(double)));
    HIPC(hipMemcpy(d, t.data(), t.size() * sizeof(double), hipMemcpyHostToDevice));
    launch_g_rhs(d_f, d, d + W, factor, W, H, s);
    HIPC(hipStreamSynchronize(s));
    HIPC(hipFree(d));
    return PGMG_OK;
}

int pgmg_ops_release(void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    OpScratch o;
    {
        std::lock_guard<std::mutex> lk(g_op_mu);
        auto it = g_ops.find(s);
        if (it == g_ops.end()) return PGMG_OK;
        o = it->second;
        g_ops.erase(it);
    }
    HIPC(hipStreamSynchronize(s));   // ops still queued on s may use the set
    for (void *p : {(void *)o.partials, (void *)o.flags, (void *)o.stats, (void *)o.scalar,
                    (void *)o.tmp, (void *)o.side})
        if (p) HIPC(hipFree(p));
    return PGMG_OK;
}

int pgmg_device_alloc(void **ptr, size_t bytes)
{
    if (!ptr) return set_err(PGMG_ERR_ARG, "null ptr");
    if (hipMalloc(ptr, bytes) != hipSuccess) return set_err(PGMG_ERR_NOMEM, "hipMalloc failed");
    return PGMG_OK;
}

int pgmg_device_free(void *ptr)
{
    HIPC(hipFree(ptr));
    return PGMG_OK;
}

int pgmg_memcpy_h2d(void *dst, const void *src, size_t bytes)
{
    HIPC(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return PGMG_OK;
}

int pgmg_memcpy_d2h(void *dst, const void *src, size_t bytes)
{
    HIPC(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return PGMG_OK;
}

int pgmg_device_sync(void)
{
    HIPC(hipDeviceSynchronize());
    return PGMG_OK;
}

int pgmg_device_count(int *n)
{
    if (!n) return set_err(PGMG_ERR_ARG, "null n");
    hipError_t e = hipGetDeviceCount(n);
    if (e != hipSuccess) {
        *n = 0;
        return set_err(PGMG_ERR_HIP, hipGetErrorString(e));
    }
    return PGMG_OK;
}

}  // extern "C"
