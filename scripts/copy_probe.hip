// copy_probe.hip -- what a streaming pass over a 16385^2 fp64 grid in the reference layout
// (pitch 16385: odd rows start 8 bytes off a 16-byte boundary) can reach on MI355X, by access
// shape.  Each variant copies the interior (rows 1..N-2, columns 1..N-2) of src into dst
// (16 B per interior point: 4.29 GB), timed with hipEvents (best of 5 after 2 warmups), and
// reports TB/s of the algorithmic bytes.  Shapes:
//   flat_*      the whole array as one contiguous run (a ceiling: no row structure)
//   cols_*      the op kernels' shape: lane t owns the column pair (1 + 2t, 2 + 2t), a
//               workgroup marches a band of rows with U rows of loads in flight
//   rows_*      a workgroup walks whole rows: each wave takes 1 KiB chunks of one row in turn
// suffixes: _nt non-temporal stores, _pl plain stores; _g<G> workgroup count.
//   hipcc -O3 --offload-arch=gfx950 scripts/copy_probe.hip -o scripts/bin/copy_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef double dpair_u __attribute__((ext_vector_type(2), aligned(8)));

template <bool NT>
__device__ __forceinline__ void st2(double *p, dpair_u v)
{
    if (NT) __builtin_nontemporal_store(v, (dpair_u *)p);
    else *(dpair_u *)p = v;
}
__device__ __forceinline__ dpair_u ld2(const double *p) { return *(const dpair_u *)p; }

// flat: element range [lo, hi) of the array as pairs, grid-stride, U pairs per lane in flight
template <bool NT, int U>
__global__ __launch_bounds__(256) void k_flat(const double *__restrict__ s, double *__restrict__ d,
                                              long long npairs)
{
    const long long stride = (long long)gridDim.x * 256;
    for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < npairs; p += stride * U) {
        dpair_u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long q = p + u * stride;
            v[u] = q < npairs ? ld2(s + 2 * q) : dpair_u{0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long q = p + u * stride;
            if (q < npairs) st2<NT>(d + 2 * q, v[u]);
        }
    }
}

// cols: the op kernels' geometry (k_op_copy_interior)
template <bool NT, int U>
__global__ __launch_bounds__(256) void k_cols(const double *__restrict__ s, double *__restrict__ d,
                                              int N, int rpb)
{
    const int npairs = (N - 1) >> 1;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= npairs) return;
    const int c = 1 + 2 * t;
    const bool second = c + 1 <= N - 2;
    const int jb = 1 + blockIdx.y * rpb;
    const int je = min(jb + rpb, N - 1);
    for (int j = jb; j < je; j += U) {
        dpair_u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld2(s + (long long)min(j + u, je - 1) * N + c);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (j + u >= je) break;
            double *q = d + (long long)(j + u) * N + c;
            if (second) st2<NT>(q, v[u]);
            else q[0] = v[u].x;
        }
    }
}

// rows: workgroup b takes rows b, b + G, ...; its 4 waves sweep the row in 1 KiB chunks, U
// chunks of loads in flight per wave
template <bool NT, int U>
__global__ __launch_bounds__(256) void k_rows(const double *__restrict__ s, double *__restrict__ d,
                                              int N)
{
    const int npairs = (N - 1) >> 1;   // pairs (1 + 2t, 2 + 2t) of a row's interior
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int chunks = (npairs + 63) / 64;
    for (int j = 1 + blockIdx.x; j < N - 1; j += gridDim.x) {
        const long long row = (long long)j * N;
        for (int c0 = w; c0 < chunks; c0 += 4 * U) {
            dpair_u v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = (c0 + 4 * u) * 64 + lane;
                v[u] = t < npairs ? ld2(s + row + 1 + 2 * t) : dpair_u{0, 0};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = (c0 + 4 * u) * 64 + lane;
                if (t < npairs) {
                    double *q = d + row + 1 + 2 * t;
                    if (1 + 2 * t + 1 <= N - 2) st2<NT>(q, v[u]);
                    else q[0] = v[u].x;
                }
            }
        }
    }
}

template <class F>
static void run(const char *name, double bytes, F launch)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 2; ++i) launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int t = 0; t < 5; ++t) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    CK(hipGetLastError());
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"tbps\": %.3f}\n", name, best, bytes / (best * 1e-3) / 1e12);
    fflush(stdout);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main(int argc, char **argv)
{
    const int N = argc > 1 ? atoi(argv[1]) : 16385;
    const long long n = (long long)N * N;
    double *s, *d;
    CK(hipMalloc(&s, n * sizeof(double) + 64));
    CK(hipMalloc(&d, n * sizeof(double) + 64));
    CK(hipMemset(s, 0, n * sizeof(double)));
    CK(hipMemset(d, 0, n * sizeof(double)));
    const double interior = 16.0 * (double)(N - 2) * (double)(N - 2);
    const double flat = 16.0 * (double)(n / 2 * 2);
    char nm[64];
    for (int G : {1024, 2048, 4096, 8192}) {
        snprintf(nm, sizeof nm, "flat_nt_u4_g%d", G);
        run(nm, flat, [&] { k_flat<true, 4><<<G, 256>>>(s, d, n / 2); });
        snprintf(nm, sizeof nm, "flat_pl_u4_g%d", G);
        run(nm, flat, [&] { k_flat<false, 4><<<G, 256>>>(s, d, n / 2); });
    }
    const int npairs = (N - 1) / 2, gx = (npairs + 255) / 256;
    for (int G : {1024, 2048, 4096}) {
        const int gymax = G / gx > 0 ? G / gx : 1;
        const int rpb = (N - 2 + gymax - 1) / gymax;
        const int gy = (N - 2 + rpb - 1) / rpb;
        snprintf(nm, sizeof nm, "cols_nt_u8_g%d", gx * gy);
        run(nm, interior, [&] { k_cols<true, 8><<<dim3(gx, gy), 256>>>(s, d, N, rpb); });
        snprintf(nm, sizeof nm, "cols_pl_u8_g%d", gx * gy);
        run(nm, interior, [&] { k_cols<false, 8><<<dim3(gx, gy), 256>>>(s, d, N, rpb); });
        snprintf(nm, sizeof nm, "cols_nt_u4_g%d", gx * gy);
        run(nm, interior, [&] { k_cols<true, 4><<<dim3(gx, gy), 256>>>(s, d, N, rpb); });
    }
    for (int G : {1024, 2048, 4096}) {
        snprintf(nm, sizeof nm, "rows_nt_u4_g%d", G);
        run(nm, interior, [&] { k_rows<true, 4><<<G, 256>>>(s, d, N); });
        snprintf(nm, sizeof nm, "rows_pl_u4_g%d", G);
        run(nm, interior, [&] { k_rows<false, 4><<<G, 256>>>(s, d, N); });
        snprintf(nm, sizeof nm, "rows_nt_u8_g%d", G);
        run(nm, interior, [&] { k_rows<true, 8><<<G, 256>>>(s, d, N); });
    }
    CK(hipFree(s));
    CK(hipFree(d));
    return 0;
}
