// bwtest.hip — practical HBM bandwidth of streaming patterns on MI355X (gfx950).
// Establishes the achievable ceiling for the stencils' read/write mixes
//   read 1R, write 1W, copy 1R:1W, add 2R:1W (the Jacobi sweep's mix), 3R:1W
// over 2 GiB arrays (far past the 256 MiB Infinity Cache), for several load schedules:
//   gs    grid-stride, one 16-B load per lane per stream per iteration (round 1's form)
//   gsU   grid-stride, U independent 16-B loads per lane per stream in flight
//   chU   each workgroup streams one contiguous chunk, U 16-B loads per lane in flight
// each with plain or non-temporal (nt) loads/stores, 256- or 512-thread workgroups and
// grids of 1..16 rounds of the resident workgroups.  Prints one JSON line per pattern
// and schedule (best over grids, 3 timed repetitions each).
// Build: hipcc -O3 --offload-arch=gfx950 scripts/bwtest.hip -o scripts/bwtest
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

typedef double v2d __attribute__((ext_vector_type(2)));

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            printf("%s: %s\n", #x, hipGetErrorString(e));                             \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

template <bool NT>
__device__ __forceinline__ v2d ld(const v2d *p)
{
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st(v2d v, v2d *p)
{
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// NR input streams (0..3), W: write the sum, CH: contiguous chunk per workgroup,
// U loads per lane per stream in flight, NTL/NTS non-temporal loads/stores.
template <int NR, bool W, bool CH, int U, bool NTL, bool NTS>
__global__ void k_stream(const v2d *__restrict__ a, const v2d *__restrict__ b,
                         const v2d *__restrict__ c, v2d *__restrict__ o, long long n,
                         double *sink)
{
    double acc = 0.0;
    const long long bs = blockDim.x;
    long long i0, i1, step;
    if (CH) {  // workgroup g streams [g*n/G, (g+1)*n/G), U*bs elements per iteration
        const long long per = (n + gridDim.x - 1) / gridDim.x;
        i0 = (long long)blockIdx.x * per;
        i1 = i0 + per < n ? i0 + per : n;
        i0 += threadIdx.x;
        step = U * bs;
    } else {
        i0 = (long long)blockIdx.x * bs + threadIdx.x;
        i1 = n;
        step = U * (long long)gridDim.x * bs;
    }
    const long long sub = CH ? bs : (long long)gridDim.x * bs;
    for (long long i = i0; i < i1; i += step) {
        v2d va[U], vb[U], vc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long k = i + u * sub;
            const bool ok = k < i1;
            if (NR >= 1) va[u] = ok ? ld<NTL>(a + k) : v2d{0, 0};
            if (NR >= 2) vb[u] = ok ? ld<NTL>(b + k) : v2d{0, 0};
            if (NR >= 3) vc[u] = ok ? ld<NTL>(c + k) : v2d{0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long k = i + u * sub;
            v2d v = v2d{1.0, 2.0};
            if (NR >= 1) v = va[u];
            if (NR >= 2) v += vb[u];
            if (NR >= 3) v += vc[u];
            if (W) {
                if (k < i1) st<NTS>(v, o + k);
            } else {
                acc += v.x + v.y;
            }
        }
    }
    if (!W && acc == 12345.678) *sink = acc;
}

typedef void (*kfn)(const v2d *, const v2d *, const v2d *, v2d *, long long, double *);

struct Sched {
    const char *name;
    kfn f[5];  // read1, write1, copy, add2, add3
};

#define ROW(CH, U, NTL, NTS)                                                                  \
    {k_stream<1, false, CH, U, NTL, NTS>, k_stream<0, true, CH, U, NTL, NTS>,                 \
     k_stream<1, true, CH, U, NTL, NTS>, k_stream<2, true, CH, U, NTL, NTS>,                  \
     k_stream<3, true, CH, U, NTL, NTS>}

int main(int argc, char **argv)
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
    Sched sch[] = {
        {"gs1", ROW(false, 1, false, false)},     {"gs1_nt", ROW(false, 1, true, true)},
        {"gs4", ROW(false, 4, false, false)},     {"gs4_nts", ROW(false, 4, false, true)},
        {"gs4_nt", ROW(false, 4, true, true)},    {"gs8_nt", ROW(false, 8, true, true)},
        {"ch4", ROW(true, 4, false, false)},      {"ch4_nts", ROW(true, 4, false, true)},
        {"ch4_nt", ROW(true, 4, true, true)},     {"ch8_nt", ROW(true, 8, true, true)},
        {"ch2_nt", ROW(true, 2, true, true)},     {"ch8_ntl", ROW(true, 8, true, false)},
        {"ch16_nt", ROW(true, 16, true, true)},   {"ch16_ntl", ROW(true, 16, true, false)},
        {"ch8", ROW(true, 8, false, false)},
    };
    const char *pname[5] = {"read1", "write1", "copy_1R1W", "add_2R1W", "add_3R1W"};
    const int nrw[5] = {1, 1, 2, 3, 4};
    const int blocks[] = {256, 512, 1024};
    const int rounds[] = {1, 2, 4, 8, 16, 32};
    for (int p = 0; p < 5; ++p) {
        for (auto &s : sch) {
            double best = 0;
            int bestg = 0, bestb = 0;
            for (int bs : blocks) {
                for (int r : rounds) {
                    const int g = (256 * (2048 / bs) * r / 2) > 0 ? 256 * (2048 / bs) * r / 2 : 256;  // r half-occupancy rounds
                    for (int rep = 0; rep < 4; ++rep) {
                        CK(hipEventRecord(e0));
                        s.f[p]<<<g, bs>>>(a, b, c, o, n, sink);
                        CK(hipEventRecord(e1));
                        CK(hipEventSynchronize(e1));
                        float ms;
                        CK(hipEventElapsedTime(&ms, e0, e1));
                        const double gbs = (double)n * 16 * nrw[p] / (ms * 1e-3) / 1e9;
                        if (rep > 0 && gbs > best) {
                            best = gbs;
                            bestg = g;
                            bestb = bs;
                        }
                    }
                }
            }
            printf("{\"pattern\": \"%s\", \"sched\": \"%s\", \"best_GBps\": %.1f, \"grid\": %d, "
                   "\"block\": %d}\n",
                   pname[p], s.name, best, bestg, bestb);
            fflush(stdout);
        }
    }
    return 0;
}
