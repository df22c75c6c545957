// ubench_vstore.hip -- cost of the V epilogue's store shapes on gfx950 (diagnostic).
// Every wave writes NT tiles of 16 rows x 16 bytes into a plane with pitch P:
//   A: dword per lane, lane (n, g) -> row n, bytes 4g..4g+3      (64 lanes, 16 lines / instr)
//   B: dwordx4 per lane for lanes g == 0 (16 lanes, one 16-B row segment each)
//   C: dwordx4, 4 adjacent tiles per instruction: lane (n, t) -> row n, bytes 16t..16t+15
//   D: dwordx4, fully contiguous 1 KB per instruction
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_vstore tools/ubench_vstore.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(256) k_store(uint8_t *plane, int pitch, int tiles_per_wave, int rows_per_block)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n = lane & 15, g = lane >> 4;
    const int gw = blockIdx.x * 4 + wave;
    uint8_t *base = plane + (size_t)(blockIdx.x * rows_per_block) * pitch;
    const uint32_t v = 0x01010101u * (uint32_t)lane;
    for (int t = 0; t < tiles_per_wave; ++t) {
        const int col = ((wave * tiles_per_wave + t) * 16) % (pitch - 64);
        const int row0 = (t * 16) % (rows_per_block - 16);
        if (MODE == 0) {
            *reinterpret_cast<uint32_t *>(base + (size_t)(row0 + n) * pitch + col + 4 * g) = v;
        } else if (MODE == 1) {
            if (g == 0) *reinterpret_cast<u32x4 *>(base + (size_t)(row0 + n) * pitch + col) = (u32x4){v, v, v, v};
        } else if (MODE == 2) {
            if ((t & 3) == 0)
                *reinterpret_cast<u32x4 *>(base + (size_t)(row0 + n) * pitch + (col & ~63) + 16 * g) = (u32x4){v, v, v, v};
        } else {
            if ((t & 3) == 0)
                *reinterpret_cast<u32x4 *>(base + (size_t)row0 * pitch + (col & ~1023) % pitch + 16 * lane) = (u32x4){v, v, v, v};
        }
    }
    (void)gw;
}

int main()
{
    const int pitch = 2048, blocks = 2048, rows_per_block = 64, tiles = 256;
    uint8_t *plane;
    hipMalloc(&plane, (size_t)pitch * rows_per_block * blocks);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *name[4] = {"A dword x64 lanes (16 lines/instr)", "B dwordx4 x16 lanes", "C dwordx4 x64, 4 tiles wide",
                           "D dwordx4 x64 contiguous"};
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            switch (mode) {
            case 0: hipLaunchKernelGGL(k_store<0>, dim3(blocks), dim3(256), 0, 0, plane, pitch, tiles, rows_per_block); break;
            case 1: hipLaunchKernelGGL(k_store<1>, dim3(blocks), dim3(256), 0, 0, plane, pitch, tiles, rows_per_block); break;
            case 2: hipLaunchKernelGGL(k_store<2>, dim3(blocks), dim3(256), 0, 0, plane, pitch, tiles, rows_per_block); break;
            default: hipLaunchKernelGGL(k_store<3>, dim3(blocks), dim3(256), 0, 0, plane, pitch, tiles, rows_per_block); break;
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double bytes = (double)blocks * 4 * tiles * 256;   // tile bytes written (same for every mode)
            if (rep) printf("%-40s %8.3f ms  %7.1f GB/s of tile bytes\n", name[mode], ms, bytes / ms / 1e6);
        }
    }
    hipFree(plane);
    return 0;
}
