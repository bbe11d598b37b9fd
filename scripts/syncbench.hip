// Microbenchmark: back-to-back launch cost of small kernels vs grid-wide barriers inside
// one cooperative launch (cooperative_groups grid.sync and a hand-rolled atomic barrier),
// on MI355X.  Informs whether the latency-bound coarse levels should be one persistent
// kernel.  Build: hipcc -O3 --offload-arch=gfx950 syncbench.hip -o syncbench
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <cstdio>
namespace cg = cooperative_groups;

__global__ void k_small(float *p, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1.0f;
}

__global__ void k_coop(float *p, int n, int iters)
{
    cg::grid_group g = cg::this_grid();
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = 0; k < iters; ++k) {
        if (i < n) p[i] += 1.0f;
        g.sync();
    }
}

__device__ void atomic_barrier(unsigned *cnt, unsigned *gen, unsigned nb)
{
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __atomic_thread_fence(__ATOMIC_RELEASE);   // agent scope default for device
        if (atomicAdd(cnt, 1u) == nb - 1) {
            __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g)
                __builtin_amdgcn_s_sleep(1);
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
    }
    __syncthreads();
}

__global__ void k_atomic(float *p, int n, int iters, unsigned *bar)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = 0; k < iters; ++k) {
        if (i < n) p[i] += 1.0f;
        atomic_barrier(bar, bar + 1, gridDim.x);
    }
}

int main()
{
    const int n = 1 << 20, iters = 2000;
    float *p;
    unsigned *bar;
    hipMalloc(&p, n * sizeof(float));
    hipMalloc(&bar, 64);
    hipMemset(p, 0, n * sizeof(float));
    hipMemset(bar, 0, 64);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float ms;
    for (int blocks : {256, 512, 1024}) {
        for (int w = 0; w < 2; ++w) {
            hipEventRecord(a);
            for (int k = 0; k < iters; ++k) k_small<<<blocks, 256>>>(p, n);
            hipEventRecord(b);
            hipEventSynchronize(b);
        }
        hipEventElapsedTime(&ms, a, b);
        printf("{\"test\": \"launch\", \"blocks\": %d, \"us_per\": %.3f}\n", blocks, ms * 1e3 / iters);
        int maxb = 0;
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&maxb, k_coop, 256, 0);
        int cus = 0;
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
        if (blocks > maxb * cus) continue;
        int it = iters;
        void *args[] = {&p, (void *)&n, &it};
        for (int w = 0; w < 2; ++w) {
            hipEventRecord(a);
            hipError_t e = hipLaunchCooperativeKernel((void *)k_coop, dim3(blocks), dim3(256), args, 0, 0);
            hipEventRecord(b);
            hipEventSynchronize(b);
            if (e != hipSuccess) printf("coop launch error %s\n", hipGetErrorString(e));
        }
        hipEventElapsedTime(&ms, a, b);
        printf("{\"test\": \"grid.sync\", \"blocks\": %d, \"us_per\": %.3f}\n", blocks, ms * 1e3 / iters);
        void *args2[] = {&p, (void *)&n, &it, &bar};
        for (int w = 0; w < 2; ++w) {
            hipEventRecord(a);
            hipError_t e = hipLaunchCooperativeKernel((void *)k_atomic, dim3(blocks), dim3(256), args2, 0, 0);
            hipEventRecord(b);
            hipEventSynchronize(b);
            if (e != hipSuccess) printf("coop launch error %s\n", hipGetErrorString(e));
        }
        hipEventElapsedTime(&ms, a, b);
        printf("{\"test\": \"atomic_barrier\", \"blocks\": %d, \"us_per\": %.3f}\n", blocks, ms * 1e3 / iters);
    }
    // graph of launches
    {
        hipStream_t s;
        hipStreamCreate(&s);
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int k = 0; k < 200; ++k) k_small<<<256, 256, 0, s>>>(p, n);
        hipStreamEndCapture(s, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        for (int w = 0; w < 2; ++w) {
            hipEventRecord(a, s);
            for (int r = 0; r < 10; ++r) hipGraphLaunch(ge, s);
            hipEventRecord(b, s);
            hipEventSynchronize(b);
        }
        hipEventElapsedTime(&ms, a, b);
        printf("{\"test\": \"graph_launch\", \"blocks\": 256, \"us_per\": %.3f}\n", ms * 1e3 / 2000);
    }
    return 0;
}
