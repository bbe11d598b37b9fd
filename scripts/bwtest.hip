// bwtest.hip — practical HBM bandwidth of streaming patterns on MI355X (gfx950).
// Establishes the achievable ceiling for the stencils' read/write mixes:
//   copy  1R:1W, add  2R:1W (the Jacobi sweep's mix), read 1R (reduction), write 1W,
//   3R:1W.  16-B per lane (dwordx4), grid-stride over 2 GiB arrays.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/bwtest.hip -o scripts/bwtest
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef double v2d __attribute__((ext_vector_type(2)));

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            printf("%s: %s\n", #x, hipGetErrorString(e));                             \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

template <int NR, bool NT>
__global__ __launch_bounds__(256) void k_stream(const v2d *__restrict__ a,
                                                const v2d *__restrict__ b,
                                                const v2d *__restrict__ c,
                                                v2d *__restrict__ o, long long n, double *sink)
{
    double acc = 0.0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        v2d v = a[i];
        if (NR >= 2) v += b[i];
        if (NR >= 3) v += c[i];
        if (o) {
            if (NT) __builtin_nontemporal_store(v, &o[i]);
            else o[i] = v;
        } else {
            acc += v.x + v.y;
        }
    }
    if (!o && acc == 12345.678) *sink = acc;
}

__global__ __launch_bounds__(256) void k_write(v2d *__restrict__ o, long long n)
{
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        o[i] = v2d{1.0, 2.0};
}

int main()
{
    const long long n = (2LL << 30) / 16;  // 2 GiB per array
    v2d *a, *b, *c, *o;
    double *sink;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&b, n * 16));
    CK(hipMalloc(&c, n * 16));
    CK(hipMalloc(&o, n * 16));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(a, 0, n * 16));
    CK(hipMemset(b, 0, n * 16));
    CK(hipMemset(c, 0, n * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grids[] = {1024, 2048, 4096, 8192, 16384};
    struct T {
        const char *name;
        int nr;
        bool wr, nt;
    } tests[] = {{"read1", 1, false, false}, {"write1", 0, true, false},
                 {"copy_1R1W", 1, true, false}, {"copy_1R1W_nt", 1, true, true},
                 {"add_2R1W", 2, true, false}, {"add_2R1W_nt", 2, true, true},
                 {"add_3R1W", 3, true, false}};
    for (auto &t : tests) {
        double best = 0;
        int bestg = 0;
        for (int g : grids) {
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipEventRecord(e0));
                if (t.nr == 0) k_write<<<g, 256>>>(o, n);
                else if (t.nr == 1 && !t.nt) k_stream<1, false><<<g, 256>>>(a, b, c, t.wr ? o : nullptr, n, sink);
                else if (t.nr == 1) k_stream<1, true><<<g, 256>>>(a, b, c, o, n, sink);
                else if (t.nr == 2 && !t.nt) k_stream<2, false><<<g, 256>>>(a, b, c, o, n, sink);
                else if (t.nr == 2) k_stream<2, true><<<g, 256>>>(a, b, c, o, n, sink);
                else k_stream<3, false><<<g, 256>>>(a, b, c, o, n, sink);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double bytes = (double)n * 16 * (t.nr + (t.wr ? 1 : 0));
                const double gbs = bytes / (ms * 1e-3) / 1e9;
                if (rep > 0 && gbs > best) {
                    best = gbs;
                    bestg = g;
                }
            }
        }
        printf("{\"pattern\": \"%s\", \"best_GBps\": %.1f, \"grid\": %d}\n", t.name, best, bestg);
    }
    return 0;
}
