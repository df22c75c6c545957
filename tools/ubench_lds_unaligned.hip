// Does gfx950 LDS serve unaligned ds_read_b32 / ds_read_b64 correctly, and at what cost?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int MODE>   // 0 aligned b32, 1 unaligned b32, 2 unaligned b64 (2 dwords), 3 aligned b64
__global__ void __launch_bounds__(256) k(uint32_t *out, int iters, int stride)
{
    __shared__ uint8_t lds[8192 + 64];
    for (int i = threadIdx.x; i < 8192 + 64; i += 256) lds[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    const int lane = threadIdx.x;
    int off = (lane * stride) % 8000;
    if (MODE == 0 || MODE == 3) off &= ~7;
    else off |= 1;                       // odd byte address
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        const int o = (off + it * 13) % 8000 | (MODE == 0 || MODE == 3 ? 0 : 1);
        const int oo = (MODE == 0 || MODE == 3) ? (o & ~7) : o;
        if (MODE <= 1) {
            uint32_t v;
            __builtin_memcpy(&v, lds + oo, 4);
            acc += v;
        } else {
            uint2 v;
            __builtin_memcpy(&v, lds + oo, 8);
            acc += v.x ^ v.y;
        }
    }
    out[blockIdx.x * 256 + lane] = acc;
    if (blockIdx.x == 0 && iters == 1) {   // correctness probe: return the raw dword read at `off`
        uint32_t v;
        __builtin_memcpy(&v, lds + off, 4);
        out[1 << 20 | lane] = v;
        uint32_t want = 0;
        for (int b = 0; b < 4; ++b) want |= (uint32_t)(uint8_t)((off + b) * 7 + 3) << (8 * b);
        out[(1 << 20) + 256 + lane] = want;
    }
}
int main()
{
    uint32_t *o;
    hipMalloc(&o, (2 << 20) * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // correctness (MODE 1 with iters=1)
    hipLaunchKernelGGL(k<1>, 1, 256, 0, 0, o, 1, 3);
    hipDeviceSynchronize();
    uint32_t h[512];
    hipMemcpy(h, o + (1 << 20), 512 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += h[i] != h[256 + i];
    printf("unaligned ds_read_b32 correctness: %d bad of 256 (err=%s)\n", bad, hipGetErrorString(hipGetLastError()));
    const char *names[] = {"aligned b32", "unaligned b32", "unaligned b64", "aligned b64"};
    for (int m = 0; m < 4; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (m == 0) hipLaunchKernelGGL(k<0>, 4096, 256, 0, 0, o, 2000, 3);
            if (m == 1) hipLaunchKernelGGL(k<1>, 4096, 256, 0, 0, o, 2000, 3);
            if (m == 2) hipLaunchKernelGGL(k<2>, 4096, 256, 0, 0, o, 2000, 3);
            if (m == 3) hipLaunchKernelGGL(k<3>, 4096, 256, 0, 0, o, 2000, 3);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep) printf("%-14s %.3f ms\n", names[m], ms);
        }
    }
    printf("err=%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
