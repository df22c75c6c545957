// probe_permlane.hip -- semantics of v_permlane32_swap / v_permlane16_swap (gfx950) as the
// k_ladder5 V-store transpose uses them: prints, for a = lane, b = 100 + lane, the
// results of each swap at lanes 0, 16, 32, 48.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_permlane tools/probe_permlane.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned *o)
{
    const unsigned a = threadIdx.x, b = 100 + threadIdx.x;
    auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    auto q = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    o[threadIdx.x * 4 + 0] = r[0];
    o[threadIdx.x * 4 + 1] = r[1];
    o[threadIdx.x * 4 + 2] = q[0];
    o[threadIdx.x * 4 + 3] = q[1];
}

int main()
{
    unsigned *d, h[256];
    hipMalloc(&d, sizeof h);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; l += 16)
        printf("lane %2d: swap32 -> (%3u, %3u)  swap16 -> (%3u, %3u)\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2],
               h[4 * l + 3]);
    return 0;
}
