// Micro-benchmark: throughput of the VALU ops the ladder kernel is built from.
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 4096
template <int OP>
__global__ void __launch_bounds__(256) k(unsigned *out, unsigned seed)
{
    unsigned a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
    const unsigned b = seed * 0x01010101u;
    int c0 = 0, c1 = 1, c2 = 2, c3 = 3, c4 = 4, c5 = 5, c6 = 6, c7 = 7;
    for (int i = 0; i < N; ++i) {
#define STEP(A, C) \
        if (OP == 0) C = __builtin_amdgcn_sdot4((int)A, (int)b, C, false); \
        else if (OP == 1) { typedef short s2 __attribute__((ext_vector_type(2))); C = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, A), __builtin_bit_cast(s2, b), C, false); } \
        else if (OP == 2) C = C; \
        else if (OP == 3) C = C * (int)A + (int)b; \
        else C = (C + (int)A) ^ (int)b;
        STEP(a0, c0) STEP(a1, c1) STEP(a2, c2) STEP(a3, c3) STEP(a4, c4) STEP(a5, c5) STEP(a6, c6) STEP(a7, c7)
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}
int main()
{
    unsigned *o;
    hipMalloc(&o, 256 * 256 * 16 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"v_dot4c_i32_i8", "v_dot2c_i32_i16", "(unused)", "v_mul_lo+add", "v_add+xor"};
    for (int op : {0, 1, 3, 4}) {
        for (int rep = 0; rep < 2; ++rep) {
            const int blocks = 256 * 16;
            hipEventRecord(e0);
            if (op == 0) hipLaunchKernelGGL(k<0>, blocks, 256, 0, 0, o, 3u);
            if (op == 1) hipLaunchKernelGGL(k<1>, blocks, 256, 0, 0, o, 3u);
            if (op == 3) hipLaunchKernelGGL(k<3>, blocks, 256, 0, 0, o, 3u);
            if (op == 4) hipLaunchKernelGGL(k<4>, blocks, 256, 0, 0, o, 3u);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double wave_instr = (double)blocks * 4 * N * 8;     // 4 waves per block, 8 ops per iter
            const double per_cu_clk = wave_instr / (ms * 1e-3) / 256 / 2.4e9;
            if (rep) printf("%-18s %.3f ms  %.3f wave-instr/clk/CU (x%s)\n", names[op], ms, per_cu_clk,
                            op == 3 ? "2 instr" : op == 4 ? "2 instr" : "1");
        }
    }
    return 0;
}
