// probe_mfma_i8.hip -- checks the two facts k_ladder5 relies on for
// v_mfma_i32_16x16x64_i8 (gfx950):
//  (1) pairing: lane l's A byte j (row m = l & 15, lane group g = l >> 4)
//      multiplies lane l' = n + 16 g's B byte j (column n) and the products
//      of all (g, j) are summed, whatever K order the hardware uses inside;
//  (2) C/D layout: lane l register i holds C[row 4 (l >> 4) + i][col l & 15].
// Also times back-to-back issue (cycles per MFMA on one SIMD).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_mfma_i8 tools/probe_mfma_i8.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_probe(const int8_t *A, const int8_t *B, int *C, long long *cyc)
{
    const int l = threadIdx.x;
    v4i a, b;
    for (int r = 0; r < 4; ++r) {
        int wa = 0, wb = 0;
        for (int k = 0; k < 4; ++k) {
            wa |= (int)(uint8_t)A[l * 16 + 4 * r + k] << (8 * k);
            wb |= (int)(uint8_t)B[l * 16 + 4 * r + k] << (8 * k);
        }
        a[r] = wa;
        b[r] = wb;
    }
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int i = 0; i < 4; ++i) C[l * 4 + i] = c[i];
    // timing: 4 independent chains of 256 MFMAs
    v4i d0 = c, d1 = c, d2 = c, d3 = c;
    long long t0 = clock64();
    for (int it = 0; it < 256; ++it) {
        d0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, a, d1, 0, 0, 0);
        d2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, d2, 0, 0, 0);
        d3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, b, d3, 0, 0, 0);
    }
    long long t1 = clock64();
    if (l == 0) cyc[0] = t1 - t0;
    if (d0[0] + d1[1] + d2[2] + d3[3] == 123456789) C[0] = 0;
}

int main()
{
    int8_t hA[64 * 16], hB[64 * 16];
    srand(7);
    for (int i = 0; i < 64 * 16; ++i) {
        hA[i] = (int8_t)(rand() & 255);
        hB[i] = (int8_t)(rand() & 255);
    }
    int8_t *dA, *dB;
    int *dC;
    long long *dcyc;
    hipMalloc(&dA, sizeof hA);
    hipMalloc(&dB, sizeof hB);
    hipMalloc(&dC, 64 * 4 * sizeof(int));
    hipMalloc(&dcyc, sizeof(long long));
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dcyc);
    int hC[256];
    long long cyc = 0;
    hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    hipMemcpy(&cyc, dcyc, sizeof cyc, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 4; ++i) {
            const int row = 4 * (l >> 4) + i, col = l & 15;
            long long want = 0;
            for (int g = 0; g < 4; ++g)
                for (int j = 0; j < 16; ++j)
                    want += (long long)hA[(row + 16 * g) * 16 + j] * hB[(col + 16 * g) * 16 + j];
            if (want != hC[l * 4 + i]) ++bad;
        }
    printf("mfma_i32_16x16x64_i8 pairing+layout: %s (%d of 256 wrong); %.1f cycles per MFMA (4 chains)\n",
           bad ? "MISMATCH" : "ok", bad, cyc / 1024.0);
    return bad ? 1 : 0;
}
