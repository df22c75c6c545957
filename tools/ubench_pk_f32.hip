// ubench_pk_f32: does gfx950's packed f32 VALU (v_pk_fma_f32, two f32 FMAs per lane per
// instruction) raise the f32 FMA rate over v_fma_f32?  (VERDICT r05 item 2 proposed moving
// k_tonemap_w's float chain to it.)  Every kernel does the same number of f32 FMAs per lane:
//   fma:  16 independent chains of v_fma_f32,
//   pk:    8 independent chains of v_pk_fma_f32 (2 FMAs each),
//   mix:   8 chains of v_fma_f32 + 4 of v_pk_fma_f32,
// over a grid that fills every SIMD with 8 waves.  Prints the FMA rate of each.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_pk_f32.hip -o tools/ubench_pk_f32
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                             \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

constexpr int kIters = 4096;

__global__ void __launch_bounds__(256) k_fma(float *out, float a, float b)
{
    float x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * 1e-3f + i;
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) k_pk(float *out, float a, float b)
{
    f2 x[8];
    const f2 va = {a, a}, vb = {b, b};
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (f2){threadIdx.x * 1e-3f + i, threadIdx.x * 1e-3f - i};
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(va), "v"(vb));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_mix(float *out, float a, float b)
{
    float x[8];
    f2 y[4];
    const f2 va = {a, a}, vb = {b, b};
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3f + i;
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = (f2){threadIdx.x * 1e-3f + i, threadIdx.x * 1e-3f - i};
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[2 * i]) : "v"(a), "v"(b));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(y[i]) : "v"(va), "v"(vb));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[2 * i + 1]) : "v"(a), "v"(b));
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) s += y[i].x + y[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main()
{
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int blocks = prop.multiProcessorCount * 8;     // 8 four-wave workgroups per CU: 8 waves per SIMD
    float *out;
    CHK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const double fmas = (double)blocks * 256 * kIters * 16;   // per kernel (every variant)
    const char *names[3] = {"v_fma_f32 x16", "v_pk_fma_f32 x8", "mixed 8 + 4 pk"};
    for (int rep = 0; rep < 2; ++rep)
        for (int k = 0; k < 3; ++k) {
            CHK(hipEventRecord(e0, 0));
            if (k == 0) hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-4f);
            if (k == 1) hipLaunchKernelGGL(k_pk, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-4f);
            if (k == 2) hipLaunchKernelGGL(k_mix, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-4f);
            CHK(hipGetLastError());
            CHK(hipEventRecord(e1, 0));
            CHK(hipEventSynchronize(e1));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            std::printf("%-18s %8.3f ms  %7.1f TFLOP/s f32 (2 per FMA)\n", names[k], ms, 2 * fmas / (ms * 1e-3) / 1e12);
        }
    CHK(hipFree(out));
    return 0;
}
