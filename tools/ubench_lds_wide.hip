// Microbenchmark: cost of 16-B / 8-B LDS reads at 4-byte (not 16-byte) aligned
// addresses, the access shape of the ladder's horizontal FIR (lane = output
// column, window start = 4-aligned byte position that advances 2..5 bytes per lane).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// MODE 0: 4x ds_read_b32   1: ds_read_b128 (16-B aligned)   2: ds_read_b128 (4-B aligned)
//      3: 2x ds_read_b64 (4-B aligned)   4: ds_read_b96 (4-B aligned) + b32
template <int MODE>
__global__ void __launch_bounds__(256) k(uint32_t *out, int iters, int step_x2)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[16384 + 256];
    for (int i = threadIdx.x; i < (16384 + 256) / 4; i += 256) reinterpret_cast<uint32_t *>(lds)[i] = i * 2654435761u;
    __syncthreads();
    const int lane = threadIdx.x;
    // window start: lane * step/2 bytes, rounded down to 4 (or 16)
    int base = ((threadIdx.x & 63) * step_x2 / 2 + (threadIdx.x >> 6) * 2048) & ~3;
    if (MODE == 1) base &= ~15;
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        const int o = (base + ((it * 256) & 8191));
        const uint8_t *p = lds + o;
        u32x4 v;
        if (MODE == 0) {
            const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
            v = u32x4{q[0], q[1], q[2], q[3]};
        } else if (MODE == 1 || MODE == 2) {
            asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)p));
        } else if (MODE == 3) {
            u32x2 a, b;
            asm volatile("ds_read_b64 %0, %2\n ds_read_b64 %1, %2 offset:8\n s_waitcnt lgkmcnt(0)"
                         : "=v"(a), "=v"(b) : "v"((uint32_t)(uintptr_t)p));
            v = u32x4{a.x, a.y, b.x, b.y};
        } else {
            typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
            u32x3 a;
            asm volatile("ds_read_b96 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(a) : "v"((uint32_t)(uintptr_t)p));
            v = u32x4{a.x, a.y, a.z, 0};
        }
        acc += v.x ^ (v.y * 3) ^ (v.z * 5) ^ (v.w * 7);
    }
    out[blockIdx.x * 256 + lane] = acc;
    if (blockIdx.x == 0 && iters == 1) {
        // correctness: compare against byte-wise read of the same address
        const uint8_t *p = lds + base;
        uint32_t w[4];
        for (int d = 0; d < 4; ++d) {
            w[d] = 0;
            for (int b = 0; b < 4; ++b) w[d] |= (uint32_t)p[4 * d + b] << (8 * b);
        }
        const uint32_t want = w[0] ^ (w[1] * 3) ^ (w[2] * 5) ^ (w[3] * 7);
        const uint32_t want3 = w[0] ^ (w[1] * 3) ^ (w[2] * 5);
        out[(1 << 20) + lane] = (MODE == 4) ? (acc != want3) : (acc != want);
    }
}

int main()
{
    uint32_t *o;
    hipMalloc(&o, (2 << 20) * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"4x b32", "b128 a16", "b128 a4", "2x b64 a4", "b96 a4"};
    void (*fns[])(uint32_t *, int, int) = {k<0>, k<1>, k<2>, k<3>, k<4>};
    for (int step : {4, 6, 9}) {
        for (int m = 0; m < 5; ++m) {
            hipLaunchKernelGGL(fns[m], 1, 256, 0, 0, o, 1, step);
            hipDeviceSynchronize();
            uint32_t h[256];
            hipMemcpy(h, o + (1 << 20), 256 * 4, hipMemcpyDeviceToHost);
            int bad = 0;
            for (int i = 0; i < 256; ++i) bad += h[i] != 0;
            float best = 1e9;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                hipLaunchKernelGGL(fns[m], 4096, 256, 0, 0, o, 4000, step);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            // wave-instructions per CU: 4096 WG * 4 waves * 4000 iters / 256 CUs
            const double wi = 4096.0 * 4 * 4000 / 256;
            printf("lane step %.1f B  %-10s  bad=%d  %.3f ms  %.2f ns/wave-iter/CU\n", step / 2.0, names[m], bad, best,
                   best * 1e6 / wi);
        }
    }
    printf("err=%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
