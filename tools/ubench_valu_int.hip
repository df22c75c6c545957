// ubench_valu_int.hip -- SIMD issue throughput of the integer VALU instructions the yadif / ladder
// arithmetic leans on (v_sad_u8, v_perm_b32, packed 16-bit ops, SDWA byte selects, ...).
// Every thread runs ITERS x 8 independent chains of one instruction (inline asm, so nothing is
// folded); 8 waves per SIMD on every CU.  Prints cycles per wave-instruction per SIMD at the
// measured clock (s_memtime ticks around the loop, wave 0 of each workgroup).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_valu_int tools/ubench_valu_int.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define ITERS 4096

#define OP8(stmt) stmt(0) stmt(1) stmt(2) stmt(3) stmt(4) stmt(5) stmt(6) stmt(7)

template <int K>
__global__ void __launch_bounds__(256) kern(uint32_t *out, unsigned long long *ticks, uint32_t seed)
{
    uint32_t a[8], b = seed ^ threadIdx.x, c = seed * 3u + 7u, sel = 0x07050301u;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = seed + i * 0x01010101u + threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#define S_ADD(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define S_SAD(i) asm volatile("v_sad_u8 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
#define S_PERM(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(sel));
#define S_PKADD(i) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define S_PKMAX(i) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define S_SDWA(i) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2" : "+v"(a[i]) : "v"(b));
#define S_MAX3(i) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
#define S_BFE(i) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a[i]));
#define S_CND(i) asm volatile("v_cmp_lt_i32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b) : "vcc");
#define S_LSHLOR(i) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a[i]) : "v"(b));
        if constexpr (K == 0) { OP8(S_ADD) }
        if constexpr (K == 1) { OP8(S_SAD) }
        if constexpr (K == 2) { OP8(S_PERM) }
        if constexpr (K == 3) { OP8(S_PKADD) }
        if constexpr (K == 4) { OP8(S_PKMAX) }
        if constexpr (K == 5) { OP8(S_SDWA) }
        if constexpr (K == 6) { OP8(S_MAX3) }
        if constexpr (K == 7) { OP8(S_BFE) }
        if constexpr (K == 8) { OP8(S_CND) }
        if constexpr (K == 9) { OP8(S_LSHLOR) }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x == 0) ticks[blockIdx.x] = t1 - t0;
}

template <int K>
static void run(const char *name, int ninst, int cus, int waves_per_simd = 8)
{
    const int blocks = cus * waves_per_simd;   // 256 threads = 4 waves = one per SIMD
    uint32_t *out;
    unsigned long long *ticks;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipMalloc(&ticks, (size_t)blocks * 8);
    hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), 0, 0, out, ticks, 12345u);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), 0, 0, out, ticks, 777u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> t(blocks);
    hipMemcpy(t.data(), ticks, (size_t)blocks * 8, hipMemcpyDeviceToHost);
    double avg = 0;
    for (auto v : t) avg += (double)v;
    avg /= blocks;
    // per SIMD: waves_per_simd waves x ITERS x 8 x ninst wave-instructions during avg ticks
    const double per = avg / ((double)waves_per_simd * ITERS * 8 * ninst);
    printf("%-10s %6.2f ticks per wave-instruction per SIMD (%d waves/SIMD), kernel %.3f ms\n", name, per,
           waves_per_simd, ms);
    hipFree(out);
    hipFree(ticks);
}

int main()
{
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    printf("%s, %d CUs\n", p.gcnArchName, cus);
    run<0>("v_add_u32", 1, cus);
    run<1>("v_sad_u8", 1, cus);
    run<2>("v_perm_b32", 1, cus);
    run<3>("v_pk_add", 1, cus);
    run<4>("v_pk_max", 1, cus);
    run<5>("add_sdwa", 1, cus);
    run<6>("v_max3", 1, cus);
    run<7>("v_bfe", 1, cus);
    run<8>("cmp+cnd", 2, cus);
    run<9>("lshl_or", 1, cus);
    for (int w : {1, 2, 4}) {
        run<1>("v_sad_u8", 1, cus, w);
        run<0>("v_add_u32", 1, cus, w);
        run<8>("cmp+cnd", 2, cus, w);
    }
    return 0;
}
