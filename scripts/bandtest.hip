// bandtest.hip — the memory pattern of k_postpre_lds without its arithmetic: what does the
// HBM deliver for "read a band of rows of one 2.15 GB grid, write the same band of another"
// at N = 16385, as a function of the tile shape, the staging and the prefetch depth?
//
//   block = WAVES waves; a wave owns 116 columns, the block loads a window of
//   WAVES*116 + 12 columns per row (lanes t < npairs, one 16-byte load each);
//   the band is RB fine rows + 12 halo rows; grid = column blocks x bands.
//   LDS=1: each row pair goes through LDS (one barrier per pair), as in k_postpre_lds;
//   LDS=0: each wave loads its own 128-column window (no barrier).
//   D: row pairs of loads in flight (register sets).
// Output: ms per launch and the algorithmic rate (16 B per interior point, like the pass's
// 8 B read + 8 B write), best of 5, per configuration.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/bandtest.hip -o scripts/bandtest
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            printf("%s: %s\n", #x, hipGetErrorString(e));                           \
            return 1;                                                               \
        }                                                                           \
    } while (0)

constexpr int kStride = 116, kMargin = 6;
typedef double v2d __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_nt(double *p, double2 v)
{
    v2d w;
    w.x = v.x;
    w.y = v.y;
    __builtin_nontemporal_store(w, reinterpret_cast<v2d *>(p));
}

template <int NT>
__device__ __forceinline__ double2 bload(const double *base, int n, int t)
{
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(base), (short)0, n * 16, 0x00020000);
    return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, t * 16, 0, NT ? 2 : 0));
}

// ALT: odd bands march upward (their halo rows are then read at the same time as the
// neighbouring bands read the same rows: second reads hit a cache)
template <int WAVES, int LDS, int NTL, int ALT = 0>
__global__ __launch_bounds__(64 * WAVES) void k_band(const double *__restrict__ in,
                                                     double *__restrict__ out, int N, long long P,
                                                     int rb, double *sink)
{
    constexpr int W = WAVES * kStride + 2 * kMargin + 4;
    __shared__ __attribute__((aligned(16))) double sx[2][2][W];
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int L0 = kStride * WAVES * blockIdx.x + 1 - kMargin;
    const int npairs = (kStride * WAVES + 2 * kMargin) / 2;
    const int nv = max(0, min(npairs, (N - 1 - L0) / 2 + 1));
    const int r0 = blockIdx.y * rb - 6;
    const int r1 = min(r0 + rb + 12, N + 6);
    const int c = L0 + kStride * w + 2 * lane;             // this lane's column pair
    const bool own = lane >= kMargin / 2 && lane < kMargin / 2 + kStride / 2 && c <= N - 2 && c >= 1;
    double acc = 0.0;
    if (LDS) {
        double2 pa0, pa1, pb0, pb1;
        const bool up = ALT && (blockIdx.y & 1);
        const int np = (r1 - r0) / 2;
        // pair starting at logical row r (r0, r0 + 2, ..) -> physical first row of the pair
        auto phys = [&](int r) { return up ? r0 + 2 * (np - 1 - (r - r0) / 2) : r; };
        auto ld = [&](int r, double2 &a, double2 &b) {
            const int pr = phys(r);
            a = bload<NTL>(in + (long long)pr * P + L0, nv, t);
            b = bload<NTL>(in + (long long)(pr + 1) * P + L0, nv, t);
        };
        ld(r0, pa0, pa1);
        if (t < npairs) {
            *reinterpret_cast<double2 *>(&sx[0][0][2 * t]) = pa0;
            *reinterpret_cast<double2 *>(&sx[0][1][2 * t]) = pa1;
        }
        ld(r0 + 2, pb0, pb1);
        ld(r0 + 4, pa0, pa1);
        __syncthreads();
        int slot = 0;
        for (int r = r0; r < r1; r += 4) {
            for (int h = 0; h < 2; ++h) {
                const int rr = r + 2 * h;
                if (rr >= r1) break;
                double2 &q0 = h ? pa0 : pb0, &q1 = h ? pa1 : pb1;
                if (rr + 2 < r1 && t < npairs) {
                    *reinterpret_cast<double2 *>(&sx[slot ^ 1][0][2 * t]) = q0;
                    *reinterpret_cast<double2 *>(&sx[slot ^ 1][1][2 * t]) = q1;
                }
                if (rr + 6 < r1) ld(rr + 6, q0, q1);
                for (int s = 0; s < 2; ++s) {
                    const double2 v = *reinterpret_cast<const double2 *>(&sx[slot][s][kStride * w + 2 * lane]);
                    const int row = phys(rr) + s;
                    if (own && row >= r0 + 6 && row < r1 - 6 && row < N - 1)
                        st_nt(out + row * P + c, v);
                    acc += v.x;
                }
                slot ^= 1;
                __syncthreads();
            }
        }
    } else {
        // each wave loads its own 128-column window (overlapping the neighbours' by 12)
        const int nw = max(0, min(64, (N - 1 - (L0 + kStride * w)) / 2 + 1));
        const double *base = in + L0 + kStride * w;
        double2 q[4];
        for (int k = 0; k < 4; ++k) q[k] = bload<NTL>(base + (long long)(r0 + k) * P, nw, lane);
        for (int r = r0; r < r1; r += 4) {
            double2 cq[4];
            for (int k = 0; k < 4; ++k) cq[k] = q[k];
            if (r + 4 < r1)
                for (int k = 0; k < 4; ++k) q[k] = bload<NTL>(base + (long long)(r + 4 + k) * P, nw, lane);
            for (int k = 0; k < 4; ++k) {
                const int row = r + k;
                if (own && row >= r0 + 6 && row < r1 - 6 && row < N - 1)
                    st_nt(out + row * P + c, cq[k]);
                acc += cq[k].x;
            }
        }
    }
    if (acc == 12345.678) *sink = acc;
}

template <int WAVES, int LDS, int NTL, int ALT = 0>
int run(const double *in, double *out, int N, long long P, int blocks, double *sink)
{
    const int cols = (N - 2 + kStride * WAVES - 1) / (kStride * WAVES);
    const int rows = N - 2;
    int bands = blocks / cols;
    if (bands < 1) bands = 1;
    int rb = (rows + bands - 1) / bands;
    rb = (rb + 1) / 2 * 2;
    bands = (rows + rb - 1) / rb;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(e0));
        k_band<WAVES, LDS, NTL, ALT><<<dim3(cols, bands), dim3(64 * WAVES)>>>(in + 1 * P, out + 1 * P, N, P, rb, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
    }
    const double pts = (double)(N - 2) * (N - 2);
    printf("{\"waves\": %d, \"lds\": %d, \"ntl\": %d, \"alt\": %d, \"blocks\": %d, \"band_rows\": %d, \"ms\": %.4f, "
           "\"alg_GBps\": %.1f}\n",
           WAVES, LDS, NTL, ALT, cols * bands, rb, best, 16.0 * pts / (best * 1e-3) / 1e9);
    fflush(stdout);
    return 0;
}

int main(int argc, char **argv)
{
    const int N = 16385;
    const long long Pmax = 16384 + 1024;
    const size_t bytes = (size_t)(N + 24) * Pmax * 8;
    double *in0, *out0, *sink;
    CK(hipMalloc(&in0, bytes));
    CK(hipMalloc(&out0, bytes));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(in0, 0, bytes));
    CK(hipMemset(out0, 0, bytes));
    const int bl[] = {512, 1024, 2048, 3072, 4096, 6144};
    if (argc > 1 && argv[1][0] == 'a') {   // alternating band direction
        const long long P = 16400;
        double *in = in0 + 10 * P, *out = out0 + 10 * P;
        for (int rep = 0; rep < 2; ++rep)
            for (int b : {512, 1024, 3072, 6144}) {
                run<4, 1, 0, 0>(in, out, N, P, b, sink);
                run<4, 1, 0, 1>(in, out, N, P, b, sink);
            }
        return 0;
    }
    if (argc > 1) {   // pitch sweep at fixed shape
        const long long pitches[] = {16400, 16384 + 16, 16384 + 32, 16384 + 64, 16384 + 128, 16384 + 256,
                                     16384 + 512, 16384 + 48, 16384 + 80, 16384 + 144};
        for (long long P : pitches) {
            printf("{\"pitch\": %lld}\n", P);
            for (int b : {512, 3072}) run<4, 1, 0>(in0 + 10 * P, out0 + 10 * P, N, P, b, sink);
        }
        return 0;
    }
    const long long P = 16400;
    double *in = in0 + 10 * P, *out = out0 + 10 * P;   // halo rows above row 0
    for (int b : bl) run<4, 1, 0>(in, out, N, P, b, sink);
    for (int b : bl) run<4, 1, 1>(in, out, N, P, b, sink);
    for (int b : bl) run<8, 1, 1>(in, out, N, P, b, sink);
    for (int b : bl) run<4, 0, 1>(in, out, N, P, b, sink);
    for (int b : bl) run<2, 0, 1>(in, out, N, P, b, sink);
    for (int b : bl) run<1, 0, 1>(in, out, N, P, b, sink);
    return 0;
}
