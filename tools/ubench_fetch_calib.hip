// FETCH_SIZE calibration for k_ladder7's staging pattern (MI355X_MICROARCH.md:
// "calibrate on a known byte count in your own access pattern").  Every 64-byte
// row segment of a 4K-like plane stack (pitch 3840, far larger than the 256 MB
// Infinity Cache) is read exactly once by LDS-DMA pieces shaped as in ladder7.hip:
// a piece = 16 rows x 64 bytes, lane l -> row l >> 2, chunk (l & 3) ^ (2 ((row >> 3) & 1)).
// Mode 1 reads the same bytes with plain 16-B-per-lane streaming loads (the guide's
// calibrated case) for comparison.  Run under rocprofv3 --pmc FETCH_SIZE; the
// program prints the byte count it read.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

constexpr int kPitch = 3840, kRows = 2160;            // one "plane"
constexpr int kPieceCols = kPitch / 64;               // 60 pieces per 16-row band

__global__ __launch_bounds__(256) void k_dma(const uint8_t *src, int nplanes, int *sink)
{
    __shared__ __attribute__((aligned(1024))) uint8_t lds[4 * 1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int bands = kRows / 16;
    const int total = nplanes * bands * kPieceCols;            // pieces
    const int r = lane >> 2, ch = (lane & 3) ^ (2 * ((r >> 3) & 1));
    for (int p = blockIdx.x * 4 + w; p < total; p += gridDim.x * 4) {
        const int plane = p / (bands * kPieceCols), rem = p % (bands * kPieceCols);
        const int band = rem / kPieceCols, pc = rem % kPieceCols;
        const uint8_t *a = src + (size_t)plane * kPitch * kRows + (size_t)(16 * band + r) * kPitch + 64 * pc + 16 * ch;
        __builtin_amdgcn_global_load_lds((const void *)a, (__attribute__((address_space(3))) void *)(lds + 1024 * w),
                                         16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (threadIdx.x == 0 && lds[0] == 0xA5 && lds[1] == 0x5A) sink[0] = 1;   // keep the loads
}

__global__ __launch_bounds__(256) void k_stream(const uint4 *src, size_t n16, int *sink)
{
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char **argv)
{
    const int nplanes = argc > 1 ? atoi(argv[1]) : 64;      // 64 x 8.3 MB = 531 MB > 256 MB MALL
    const int mode = argc > 2 ? atoi(argv[2]) : 0;
    const size_t bytes = (size_t)nplanes * kPitch * kRows;
    uint8_t *src;
    int *sink;
    if (hipMalloc(&src, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    hipMemset(src, 1, bytes);
    hipDeviceSynchronize();
    for (int it = 0; it < 3; ++it) {
        if (mode == 0)
            hipLaunchKernelGGL(k_dma, dim3(4096), dim3(256), 0, 0, src, nplanes, sink);
        else
            hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, (const uint4 *)src, bytes / 16, sink);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("mode %d: %zu bytes read per launch (%d planes)\n", mode, bytes, nplanes);
    hipFree(src);
    hipFree(sink);
    return 0;
}
