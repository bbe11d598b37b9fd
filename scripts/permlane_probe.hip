// Semantics probe of gfx950's v_permlane16_swap / v_permlane32_swap and DPP row_ror:8 as the
// clang builtins expose them (which element of the returned pair is which operand).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *o)
{
    const unsigned l = threadIdx.x;
    const unsigned a = l, b = 100 + l;
    auto p = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    auto q = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    o[l] = p[0];
    o[64 + l] = p[1];
    o[128 + l] = q[0];
    o[192 + l] = q[1];
    o[256 + l] = (unsigned)__builtin_amdgcn_mov_dpp((int)a, 0x128, 0xF, 0xF, true);
}
int main()
{
    unsigned *d, h[320];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
    k<<<1, 64>>>(d);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char *nm[5] = {"p16[0]", "p16[1]", "p32[0]", "p32[1]", "ror8"};
    for (int t = 0; t < 5; ++t) {
        printf("%s:", nm[t]);
        for (int l = 0; l < 64; l += 4) printf(" %u", h[t * 64 + l]);
        printf("\n");
    }
    return 0;
}
