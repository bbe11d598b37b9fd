// launch_probe.hip — where a latency-bound coarse pass's time goes.
//
// Chains of dependent launches on one stream, each variant 400 launches, host-paired
// (hipEvents around the chain, per-launch average) and, under
//   rocprofv3 --kernel-trace --stats -- ./launch_probe
// per-kernel trace durations.  Variants, 256-thread workgroups:
//   null<G>          empty kernel, G workgroups (G = 1, 64, 512, 2048)
//   null_args        empty, 512 WGs, a 512-byte kernarg block (the fused passes pass ~200 B)
//   null_lds         empty, 512 WGs, 48 KiB of LDS allocated (the tail's 125 KiB at 1 WG)
//   touch            512 WGs; each loads one double its predecessor launch wrote and writes
//                    one: a dependent global-memory round trip per launch
//   touch_sum        the same + a block reduction through LDS (one barrier), like the
//                    rare-path decision kernels re-reducing partials
//   stream4k         512 WGs, each reads 4 KiB and writes 4 KiB (2 MiB per launch: a level-513
//                    array) with one load per lane in flight
//   stream4k_x3      the same with three dependent rounds of loads per workgroup (a band
//                    marching 3 row iterations, each waiting for its loads)
//
//   hipcc -O3 --offload-arch=gfx950 scripts/launch_probe.hip -o /tmp/launch_probe
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

struct BigArgs {
    double *p;
    double pad[63];
};

__global__ __launch_bounds__(256) void k_null(double *) {}
__global__ __launch_bounds__(256) void k_null_args(BigArgs a)
{
    if (a.pad[5] == 12345.0 && threadIdx.x == 999) a.p[0] = 1.0;
}
__global__ __launch_bounds__(256) void k_null_lds(double *p)
{
    __shared__ double s[6144];
    if (threadIdx.x == 999) {
        s[threadIdx.x] = 1.0;
        p[0] = s[threadIdx.x ^ 1];
    }
}
__global__ __launch_bounds__(256) void k_touch(const double *in, double *out)
{
    if (threadIdx.x == 0) out[blockIdx.x * 16] = in[blockIdx.x * 16] + 1.0;
}
__global__ __launch_bounds__(256) void k_touch_sum(const double *in, double *out)
{
    __shared__ double red[4];
    double v = in[blockIdx.x * 256 + threadIdx.x];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x * 256] = red[0] + red[1] + red[2] + red[3];
}
template <int ROUNDS>
__global__ __launch_bounds__(256) void k_stream(const double2 *in, double2 *out)
{
    // 4 KiB per workgroup = 256 lanes x 16 B; ROUNDS dependent rounds over 4 KiB / ROUNDS
    const int base = blockIdx.x * 256;
    double2 acc = make_double2(0.0, 0.0);
    #pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        const double2 v = in[base + ((threadIdx.x + r * 85) & 255)];
        acc.x += v.x;
        acc.y += v.y;
        if (ROUNDS > 1) __builtin_amdgcn_s_waitcnt(0);
        in = (const double2 *)((const char *)in + (acc.x == 1e300 ? 8 : 0));  // data-dependent
    }
    out[base + threadIdx.x] = acc;
}

template <class F>
static void run(const char *name, F launch, int reps = 400)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 20; ++i) launch(i);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int t = 0; t < 3; ++t) {
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < reps; ++i) launch(i);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    printf("{\"variant\": \"%s\", \"us_per_launch\": %.3f}\n", name, best * 1e3 / reps);
    fflush(stdout);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main()
{
    double *p0, *p1;
    const size_t n = 2 << 20;   // 2 Mi doubles = 16 MiB each
    CK(hipMalloc(&p0, n * sizeof(double)));
    CK(hipMalloc(&p1, n * sizeof(double)));
    CK(hipMemset(p0, 0, n * sizeof(double)));
    CK(hipMemset(p1, 0, n * sizeof(double)));
    for (int G : {1, 64, 512, 2048}) {
        char nm[32];
        snprintf(nm, sizeof nm, "null%d", G);
        run(nm, [&](int) { k_null<<<G, 256>>>(p0); });
    }
    BigArgs ba{};
    ba.p = p0;
    run("null_args", [&](int) { k_null_args<<<512, 256>>>(ba); });
    run("null_lds", [&](int) { k_null_lds<<<512, 256>>>(p0); });
    run("touch", [&](int i) {
        if (i & 1) k_touch<<<512, 256>>>(p1, p0);
        else k_touch<<<512, 256>>>(p0, p1);
    });
    run("touch_sum", [&](int i) {
        if (i & 1) k_touch_sum<<<512, 256>>>(p1, p0);
        else k_touch_sum<<<512, 256>>>(p0, p1);
    });
    run("stream4k", [&](int i) {
        if (i & 1) k_stream<1><<<512, 256>>>((const double2 *)p1, (double2 *)p0);
        else k_stream<1><<<512, 256>>>((const double2 *)p0, (double2 *)p1);
    });
    run("stream4k_x3", [&](int i) {
        if (i & 1) k_stream<3><<<512, 256>>>((const double2 *)p1, (double2 *)p0);
        else k_stream<3><<<512, 256>>>((const double2 *)p0, (double2 *)p1);
    });
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipFree(p0));
    CK(hipFree(p1));
    return 0;
}
