// ladder_mfma.h -- device helpers of k_ladder7 (ladder7.hip): wave-uniform table reads,
// the H epilogue pack, the row-segment stores and the permlane transposes of the V
// epilogue, the walk's shape per variant.  Arithmetic: ladder7.hip header.
#pragma once
#include "dts_internal.h"

#ifndef DTS_L7_COMPACT_EDGE
#define DTS_L7_COMPACT_EDGE 0   // 1: partial-row stores as a byte loop (smaller walk code; A/B)
#endif
#ifndef DTS_NT_STORES
#define DTS_NT_STORES 0     // 1: non-temporal output row stores (ladder7 A/B)
#endif

namespace dts {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(4))) const uint32_t k_u32;
typedef __attribute__((address_space(1))) const v4i g_cv4i;
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
typedef __attribute__((address_space(1))) u32x2 g_u32x2;
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) uint8_t g_u8;
#define GP6(T, p) ((T *)(uintptr_t)(p))

// wave-uniform struct read through the constant address space (s_load)
template <class T>
__device__ __forceinline__ T kld6(const T *p)
{
    static_assert(sizeof(T) % 4 == 0, "dword data only");
    struct W { uint32_t w[sizeof(T) / 4]; } w;
    k_u32 *q = GP6(k_u32, p);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) w.w[i] = q[i];
    return __builtin_bit_cast(T, w);
}

// FFMIN(((256 hi + lo) >> 7), 32767) of two rows, as int16x2 (even row low)
__device__ __forceinline__ uint32_t pack_h6(int hi, int lo, int hi2, int lo2)
{
    const int a = ((hi << 8) + lo) >> 7, b = ((hi2 << 8) + lo2) >> 7;
    return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(a, b));
}

// NB bytes (4, 8, 16) at byte `at` of an output row with `room` bytes left from `at`
template <int NB>
__device__ __forceinline__ void put_row6(uint64_t rowp, int at, int room, const uint32_t (&w)[NB / 4])
{
    g_u8 *p = GP6(g_u8, rowp + (uint64_t)(int64_t)at);
    if (room >= NB) {
#if DTS_NT_STORES
        // diagnostic: non-temporal output stores (keep L2 / Infinity Cache for the source)
        if (NB == 16)
            __builtin_nontemporal_store((u32x4){w[0], w[1], w[2 % (NB / 4)], w[3 % (NB / 4)]}, GP6(g_u32x4, p));
        else if (NB == 8)
            __builtin_nontemporal_store((u32x2){w[0], w[1 % (NB / 4)]}, GP6(g_u32x2, p));
        else
            __builtin_nontemporal_store(w[0], GP6(g_u32, p));
#else
        if (NB == 16)
            *GP6(g_u32x4, p) = (u32x4){w[0], w[1], w[2 % (NB / 4)], w[3 % (NB / 4)]};
        else if (NB == 8)
            *GP6(g_u32x2, p) = (u32x2){w[0], w[1 % (NB / 4)]};
        else
            *GP6(g_u32, p) = w[0];
#endif
    } else {
#if DTS_L7_COMPACT_EDGE
        // the plane's last columns (right-edge units only): a byte loop, not unrolled -- the
        // unrolled form put NB predicated stores with their exec-mask sequences into every
        // row-block store site of every walk variant, code the whole CU pair's instruction
        // cache carries for a path few waves take
        asm volatile("" : "+v"(room));
#pragma unroll 1
        for (int i = 0; i < NB && i < room; ++i) {
            const int q = i >> 2;
            const uint32_t d = q == 0 ? w[0] : q == 1 ? w[1 % (NB / 4)] : q == 2 ? w[2 % (NB / 4)] : w[3 % (NB / 4)];
            p[i] = (uint8_t)(d >> (8 * (i & 3)));
        }
#else
        // the plane's last columns: predicated byte stores.  room goes through an empty asm
        // so the per-byte lane masks are formed here, not hoisted out of the walk (16 SGPR
        // pairs live across every granule)
        asm volatile("" : "+v"(room));
#pragma unroll
        for (int i = 0; i < NB; ++i)
            if (i < room) p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
#endif
    }
}

// tiles a, b, c, d (lane group G holds columns 4G..4G+3 of each) -> lane group G holds
// columns 0..15 of tile G
__device__ __forceinline__ void transpose4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t (&o)[4])
{
    const auto r = __builtin_amdgcn_permlane32_swap(a, c, false, false);   // [a0 a1 c0 c1], [a2 a3 c2 c3]
    const auto s = __builtin_amdgcn_permlane32_swap(b, d, false, false);   // [b0 b1 d0 d1], [b2 b3 d2 d3]
    const auto x = __builtin_amdgcn_permlane16_swap(r[0], s[0], false, false);   // [a0 b0 c0 d0], [a1 b1 c1 d1]
    const auto z = __builtin_amdgcn_permlane16_swap(r[1], s[1], false, false);   // [a2 b2 c2 d2], [a3 b3 c3 d3]
    o[0] = x[0];
    o[1] = x[1];
    o[2] = z[0];
    o[3] = z[1];
}

// tiles a, b -> lane group G holds columns 8G..8G+7 of the pair
__device__ __forceinline__ void transpose2(uint32_t a, uint32_t b, uint32_t (&o)[2])
{
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);   // [a0 a1 b0 b1], [a2 a3 b2 b3]
    const auto x = __builtin_amdgcn_permlane16_swap(r[0], r[1], false, false);   // [a0 a2 b0 b2], [a1 a3 b1 b3]
    o[0] = x[0];
    o[1] = x[1];
}

template <int VAR>
struct Walk6 {
    static constexpr int CT = l6_ct(VAR), NP = l6_np(VAR), HKB = l6_hkb(VAR), VKB = l6_vkb(VAR);
    static constexpr int T = CT * NP, R = 4 * VKB;
};

} // namespace
} // namespace dts
