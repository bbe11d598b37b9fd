// pgmg_gops.hip — op-level kernels on caller-owned arrays in the reference layout
// (row-major, pitch = W, no alignment guarantee).  These back the C-ABI entries
// that mirror Parallel::Compute* (3_part_parallel/Parallel_Method.cu:144-199);
// the V-cycle itself uses the aligned, row-marching kernels of pgmg_kernels.hip.
// One thread per point, grid-stride with a fixed grid so the per-block partial
// sums (and thus any early-exit decision) are deterministic run to run.
#include "pgmg_internal.h"

namespace pgmg {

template <int NT>
__device__ __forceinline__ double gblock_sum(double v, double *red)
{
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0) {
        #pragma unroll
        for (int i = 0; i < NT / 64; ++i) s += red[i];
    }
    return s;
}

int g_blocks(int H, int W)
{
    const long long n = (long long)(H - 2) * (W - 2);
    long long nb = (n + kBlock - 1) / kBlock;
    if (nb > 2048) nb = 2048;
    if (nb < 1) nb = 1;
    return (int)nb;
}

// Smoother.hpp:63-70 (sweep) and :75-76 (residual of the input, for the check)
__global__ __launch_bounds__(kBlock) void k_g_sweep(const double *x, const double *f, double *out,
                                                    double *partials, const unsigned *skip,
                                                    unsigned *reset, unsigned long long *stats,
                                                    double hh, double ih, int H, int W)
{
    __shared__ double red[kBlock / 64];
    if (skip != nullptr && *skip != 0u) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (reset != nullptr) *reset = 0u;
        if (stats != nullptr) atomicAdd(&stats[0], 1ull);
    }
    const long long n = (long long)(H - 2) * (W - 2);
    double acc = 0.0;
    for (long long k = (long long)blockIdx.x * kBlock + threadIdx.x; k < n;
         k += (long long)gridDim.x * kBlock) {
        const long long j = 1 + k / (W - 2);
        const long long i = 1 + k % (W - 2);
        const long long q = j * W + i;
        out[q] = 0.25 * ((hh * f[q]) + x[q - 1] + x[q + 1] + x[q - W] + x[q + W]);
        if (partials != nullptr) {
            const double r = f[q] - ih * (4 * x[q] - x[q - 1] - x[q + 1] - x[q - W] - x[q + W]);
            acc += r * r;
        }
    }
    if (partials != nullptr) {
        const double s = gblock_sum<kBlock>(acc, red);
        if (threadIdx.x == 0) partials[blockIdx.x] = s;
    }
}

void launch_g_sweep(const double *xin, const double *f, double *xout, double *partials,
                    const unsigned *skip, unsigned *reset, unsigned long long *stats, double hh,
                    double inv_hh, int H, int W, int nblocks, hipStream_t s)
{
    k_g_sweep<<<dim3(nblocks), dim3(kBlock), 0, s>>>(xin, f, xout, partials, skip, reset, stats,
                                                      hh, inv_hh, H, W);
}

__global__ __launch_bounds__(kBlock) void k_g_fixup(const double *partials, int np, double eps,
                                                    const unsigned *done_prev, unsigned *done_next,
                                                    const double *src, double *dst,
                                                    unsigned long long *stats, int H, int W)
{
    __shared__ double red[kBlock / 64];
    __shared__ int trig;
    const bool leader = blockIdx.x == 0 && threadIdx.x == 0;
    if (*done_prev != 0u) {
        if (leader) *done_next = 1u;
        return;
    }
    double s = 0.0;
    for (int k = threadIdx.x; k < np; k += kBlock) s += partials[k];
    s = gblock_sum<kBlock>(s, red);
    if (threadIdx.x == 0) trig = (sqrt(s) < eps) ? 1 : 0;
    __syncthreads();
    if (leader) {
        *done_next = trig ? 1u : 0u;
        if (trig && stats != nullptr) {
            atomicAdd(&stats[0], (unsigned long long)-1LL);
            atomicAdd(&stats[1], 1ull);
        }
    }
    if (!trig) return;
    const long long n = (long long)(H - 2) * (W - 2);
    for (long long k = (long long)blockIdx.x * kBlock + threadIdx.x; k < n;
         k += (long long)gridDim.x * kBlock) {
        const long long q = (1 + k / (W - 2)) * W + 1 + k % (W - 2);
        dst[q] = src[q];
    }
}

void launch_g_fixup(const double *partials, int np, double eps, const unsigned *done_prev,
                    unsigned *done_next, const double *src, double *dst,
                    unsigned long long *stats, int H, int W, hipStream_t s)
{
    k_g_fixup<<<dim3(256), dim3(kBlock), 0, s>>>(partials, np, eps, done_prev, done_next, src,
                                                  dst, stats, H, W);
}

__global__ void k_g_copy(const double *src, double *dst, long long n)
{
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (long long)gridDim.x * blockDim.x)
        dst[k] = src[k];
}

void launch_g_copy(const double *src, double *dst, long long n, hipStream_t s)
{
    long long nb = (n + 255) / 256;
    if (nb > 4096) nb = 4096;
    if (nb < 1) nb = 1;
    k_g_copy<<<dim3((unsigned)nb), dim3(256), 0, s>>>(src, dst, n);
}

// DynamicGridUtils.hpp:59-69; boundary of r untouched
__global__ void k_g_residual(double *r, const double *x, const double *f, double ih, int H, int W)
{
    const long long n = (long long)(H - 2) * (W - 2);
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (long long)gridDim.x * blockDim.x) {
        const long long q = (1 + k / (W - 2)) * W + 1 + k % (W - 2);
        r[q] = f[q] - ih * (4 * x[q] - x[q - 1] - x[q + 1] - x[q - W] - x[q + W]);
    }
}

void launch_g_residual(double *r, const double *x, const double *f, double inv_hh, int H, int W,
                       hipStream_t s)
{
    k_g_residual<<<dim3(g_blocks(H, W)), dim3(kBlock), 0, s>>>(r, x, f, inv_hh, H, W);
}

// MultiGrid.hpp:187-205; coarse boundary untouched
__global__ void k_g_restrict(const double *Fn, double *C, int Nf, int Nc)
{
    const long long n = (long long)(Nc - 2) * (Nc - 2);
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (long long)gridDim.x * blockDim.x) {
        const long long jc = 1 + k / (Nc - 2), ic = 1 + k % (Nc - 2);
        const long long q = (2 * jc) * Nf + 2 * ic;
        C[jc * Nc + ic] = 0.25 * Fn[q] + 0.125 * (Fn[q + 1] + Fn[q - 1] + Fn[q + Nf] + Fn[q - Nf]) +
                          0.0625 * (Fn[q - Nf - 1] + Fn[q - Nf + 1] + Fn[q + Nf - 1] + Fn[q + Nf + 1]);
    }
}

void launch_g_restrict(const double *fine, double *coarse, int Nf, int Nc, hipStream_t s)
{
    k_g_restrict<<<dim3(g_blocks(Nc, Nc)), dim3(kBlock), 0, s>>>(fine, coarse, Nf, Nc);
}

// mode 0: MultiGrid.hpp:208-226 (fine row/col 1 uncorrected);
// mode 1: prolungator_kernel, Parallel_Method.cu:79-138 (symmetric, boundary := 0).
// Only fine points (y, x) with y, x < ext are touched: the reference's thread grid
// (ComputeProlungator, Parallel_Method.cu:191-197) covers max(1, Nf / num_thread) * num_thread
// rows and columns, so for Nf = 2^k + 1 its last fine row and column are never written.
__global__ void k_g_prolong(const double *C, double *Fn, int Nc, int Nf, int mode, int ext)
{
    const int E = ext < Nf ? ext : Nf;
    const long long n = (long long)E * E;
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (long long)gridDim.x * blockDim.x) {
        const int y = (int)(k / E), x = (int)(k % E);
        const long long kk = (long long)y * Nf + x;
        if (mode == 1) {
            if (y == 0 || y == Nf - 1 || x == 0 || x == Nf - 1) {
                Fn[kk] = 0.0;
                continue;
            }
            const int cx = x / 2, cy = y / 2;
            const long long c = (long long)cy * Nc + cx;
            double v = 0.0;
            if (x % 2 == 0 && y % 2 == 0) {
                v = C[c];
            } else if (x % 2 == 1 && y % 2 == 1) {
                if (cx + 1 < Nc && cy + 1 < Nc) v = 0.25 * (C[c] + C[c + 1] + C[c + Nc] + C[c + Nc + 1]);
            } else if (x % 2 == 1 && y % 2 == 0) {
                if (cx + 1 < Nc) v = 0.5 * (C[c] + C[c + 1]);
            } else {
                if (cy + 1 < Nc) v = 0.5 * (C[c] + C[c + Nc]);
            }
            Fn[kk] += v;
        } else {
            if (x < 2 || y < 2 || x > Nf - 2 || y > Nf - 2) continue;
            const long long jc = y >> 1, ic = x >> 1;
            const double *C0 = C + jc * Nc;
            double v;
            if ((y & 1) == 0) {
                v = ((x & 1) == 0) ? C0[ic] : 0.5 * (C0[ic] + C0[ic + 1]);
            } else {
                const double *C1 = C0 + Nc;
                v = ((x & 1) == 0) ? 0.5 * (C0[ic] + C1[ic])
                                   : 0.25 * (C0[ic] + C0[ic + 1] + C1[ic] + C1[ic + 1]);
            }
            Fn[kk] = Fn[kk] + v;
        }
    }
}

void launch_g_prolong(const double *coarse, double *fine, int Nc, int Nf, int mode, int ext,
                      hipStream_t s)
{
    long long nb = ((long long)Nf * Nf + 255) / 256;
    if (nb > 4096) nb = 4096;
    k_g_prolong<<<dim3((unsigned)nb), dim3(256), 0, s>>>(coarse, fine, Nc, Nf, mode, ext);
}

__global__ __launch_bounds__(kBlock) void k_g_sumsq(const double *v, long long n, double *partials)
{
    __shared__ double red[kBlock / 64];
    double acc = 0.0;
    for (long long k = (long long)blockIdx.x * kBlock + threadIdx.x; k < n;
         k += (long long)gridDim.x * kBlock)
        acc += v[k] * v[k];
    const double s = gblock_sum<kBlock>(acc, red);
    if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

void launch_g_sumsq(const double *v, long long n, double *partials, int nblocks, hipStream_t s)
{
    k_g_sumsq<<<dim3(nblocks), dim3(kBlock), 0, s>>>(v, n, partials);
}

__global__ void k_g_rhs(double *f, const double *sx, const double *sy, double factor, int W, int H)
{
    const long long n = (long long)W * H;
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (long long)gridDim.x * blockDim.x) {
        const int j = (int)(k / W), i = (int)(k % W);
        f[k] = factor * sx[i] * sy[j];
    }
}

void launch_g_rhs(double *f, const double *sx, const double *sy, double factor, int W, int H,
                  hipStream_t s)
{
    long long nb = ((long long)W * H + 255) / 256;
    if (nb > 4096) nb = 4096;
    k_g_rhs<<<dim3((unsigned)nb), dim3(256), 0, s>>>(f, sx, sy, factor, W, H);
}

}  // namespace pgmg
