// ladder_mfma.h -- device helpers shared by k_ladder6 (ladder6.hip) and k_ladder7
// (ladder7.hip): wave-uniform table reads, the H epilogue pack, the V row block (out^T =
// H^T C^T on v_mfma_i32_16x16x64_i8 over the register ring, av_clip_uint8(v >> 19), the
// permlane transposes and the coalesced row stores through a per-wave LDS exchange),
// counted vmcnt waits.  Arithmetic: ladder6.hip header.
#pragma once
#include "dts_internal.h"

#ifndef DTS_L6_ABLATE
#define DTS_L6_ABLATE 0     // diagnostic builds only (ladder6.hip)
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
        // the plane's last columns: predicated byte stores.  room goes through an empty asm
        // so the per-byte lane masks are formed here, not hoisted out of the walk (16 SGPR
        // pairs live across every granule)
        asm volatile("" : "+v"(room));
#pragma unroll
        for (int i = 0; i < NB; ++i)
            if (i < room) p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
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

// Stores of one row block: lane (m, g) holds NB bytes of output row y0 + m at byte
// at0 + NB g.  Through a 1-KB LDS scratch they move to lane 4 m + g, so four consecutive
// lanes hold one row's 4 NB contiguous bytes (one cache access per row segment instead
// of one per lane), then the store of rows < dstH, bytes < rowbytes.
template <int NB>
__device__ __forceinline__ void put6(uint8_t *scr, uint64_t base, uint32_t pitch, int y0, int dstH, int at0,
                                     int rowbytes, const uint32_t (&w)[NB / 4], int m, int g, int lane)
{
    // the exchange needs every lane: the stores of a previous call (some lanes skip
    // them) are done before this write (a convergent point)
    __builtin_amdgcn_wave_barrier();
    uint32_t v[NB / 4];
    if (NB == 16) {
        *reinterpret_cast<u32x4 *>(scr + 16 * (4 * m + g)) = (u32x4){w[0], w[1 % (NB / 4)], w[2 % (NB / 4)], w[3 % (NB / 4)]};
        const u32x4 x = *reinterpret_cast<const u32x4 *>(scr + 16 * lane);
        v[0] = x.x;
        v[1 % (NB / 4)] = x.y;
        v[2 % (NB / 4)] = x.z;
        v[3 % (NB / 4)] = x.w;
    } else if (NB == 8) {
        *reinterpret_cast<u32x2 *>(scr + 8 * (4 * m + g)) = (u32x2){w[0], w[1 % (NB / 4)]};
        const u32x2 x = *reinterpret_cast<const u32x2 *>(scr + 8 * lane);
        v[0] = x.x;
        v[1 % (NB / 4)] = x.y;
    } else {
        *reinterpret_cast<uint32_t *>(scr + 4 * (4 * m + g)) = w[0];
        v[0] = *reinterpret_cast<const uint32_t *>(scr + 4 * lane);
    }
    const int y = y0 + (lane >> 2);
    const int at = at0 + NB * (lane & 3);
    if (y < dstH) put_row6<NB>(base + (uint64_t)y * pitch, at, rowbytes - at, v);
    __builtin_amdgcn_wave_barrier();
}

template <int VAR>
struct Walk6 {
    static constexpr int CT = l6_ct(VAR), NP = l6_np(VAR), HKB = l6_hkb(VAR), VKB = l6_vkb(VAR);
    static constexpr int T = CT * NP, R = 4 * VKB;
};

// one row block: V over the whole ring, then the stores of output row 16 j + m
// V of one row block over the whole ring: w[t] = 4 consecutive output bytes of row
// 16 j + m (lane (m, g): columns 4 g .. 4 g + 3 of tile t)
template <int VAR>
__device__ __forceinline__ void vcalc(const v4i (&rh)[Walk6<VAR>::VKB][Walk6<VAR>::T],
                                      const v4i (&rl)[Walk6<VAR>::VKB][Walk6<VAR>::T],
                                      const v4i (&vh)[Walk6<VAR>::VKB], const v4i (&vl)[Walk6<VAR>::VKB],
                                      uint32_t (&w)[Walk6<VAR>::T])
{
    using W = Walk6<VAR>;
    // 65536 hh + 256 (hl + lh) + ll + bias as three chained accumulations: the hh chain
    // starts at bias >> 16 (the bias is 12 << 16), each next chain starts at the previous
    // one << 8 -- two shifts per value instead of a three-term combine
    static_assert(kL5VBias == 12 << 16, "V bias folded into the hh chain");
    const v4i vb = {12, 12, 12, 12};
    v4i acc[W::T];
#pragma unroll
    for (int t = 0; t < W::T; ++t) acc[t] = vb;
#pragma unroll
    for (int kb = 0; kb < W::VKB; ++kb)
#pragma unroll
        for (int t = 0; t < W::T; ++t) acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(rh[kb][t], vh[kb], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < W::T; ++t) acc[t] <<= 8;
#pragma unroll
    for (int kb = 0; kb < W::VKB; ++kb)
#pragma unroll
        for (int t = 0; t < W::T; ++t) {
            acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(rh[kb][t], vl[kb], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(rl[kb][t], vh[kb], acc[t], 0, 0, 0);
        }
#pragma unroll
    for (int t = 0; t < W::T; ++t) acc[t] <<= 8;
#pragma unroll
    for (int kb = 0; kb < W::VKB; ++kb)
#pragma unroll
        for (int t = 0; t < W::T; ++t) acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(rl[kb][t], vl[kb], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < W::T; ++t) {
        // av_clip_uint8(val >> 19) of 4 columns, packed
        // (the builtin, not inline asm: the hazard recognizer does not pad an asm statement
        // that reads an MFMA result)
        const uint32_t lo = __builtin_amdgcn_ashr_pk_u8_i32(acc[t][0], acc[t][1], 19);
        const uint32_t hi = __builtin_amdgcn_ashr_pk_u8_i32(acc[t][2], acc[t][3], 19);
        w[t] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
    }
}

template <int VAR, class UT>
__device__ __forceinline__ int vblock(const UT &U, int j, const v4i (&rh)[Walk6<VAR>::VKB][Walk6<VAR>::T],
                                       const v4i (&rl)[Walk6<VAR>::VKB][Walk6<VAR>::T],
                                       const v4i (&vh)[Walk6<VAR>::VKB], const v4i (&vl)[Walk6<VAR>::VKB],
                                       const uint64_t (&ob)[2], const uint32_t (&op)[2], int m, int g,
                                       uint8_t *scr)
{
    using W = Walk6<VAR>;
    uint32_t w[W::T];
    vcalc<VAR>(rh, rl, vh, vl, w);
    if (DTS_L6_ABLATE & 4) {
#pragma unroll
        for (int t = 0; t < W::T; ++t) asm volatile("" ::"v"(w[t]));
        return 0;
    }
    const int y0 = 16 * j, lane = 16 * g + m;
    if (W::NP == 1) {                                      // luma
        if (W::CT == 4) {
            uint32_t o[4];
            transpose4(w[0], w[1 % W::T], w[2 % W::T], w[3 % W::T], o);
            put6<16>(scr, ob[0], op[0], y0, U.dstH, U.col0, U.dstW, o, m, g, lane);
        } else {
            uint32_t o[2];
            transpose2(w[0], w[1 % W::T], o);
            put6<8>(scr, ob[0], op[0], y0, U.dstH, U.col0, U.dstW, o, m, g, lane);
        }
    } else if (U.fmt == DTS_FMT_NV12) {                    // chroma, U V interleaved
#pragma unroll
        for (int c = 0; c < W::CT; ++c) {
            const uint32_t u = w[c], v = w[W::CT + c];
            const uint32_t o[2] = {__builtin_amdgcn_perm(v, u, 0x05010400u), __builtin_amdgcn_perm(v, u, 0x07030602u)};
            put6<8>(scr, ob[0], op[0], y0, U.dstH, 2 * U.col0 + 32 * c, 2 * U.dstW, o, m, g, lane);
        }
    } else {                                               // chroma, U and V planes
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            if (W::CT == 2) {
                uint32_t o[2];
                transpose2(w[2 * p], w[(2 * p + 1) % W::T], o);
                put6<8>(scr, ob[p], op[p], y0, U.dstH, U.col0, U.dstW, o, m, g, lane);
            } else {
                const uint32_t o[1] = {w[p % W::T]};
                put6<4>(scr, ob[p], op[p], y0, U.dstH, U.col0, U.dstW, o, m, g, lane);
            }
        }
    }
    // store instructions issued (one per put6; edge units' byte stores are not counted,
    // which only makes the next source wait longer)
    return W::NP == 1 ? 1 : (U.fmt == DTS_FMT_NV12 ? W::CT : 2);
}

// s_waitcnt vmcnt(min(n, LO + 15)) for a run-time n >= LO (a switch of 16 immediates):
// waiting for fewer outstanding instructions than were issued is never too short
template <int LO>
__device__ __forceinline__ void vm_wait_n6(int n)
{
    static_assert(LO >= 0 && LO + 15 < 64, "vmcnt is 6 bits");
#define DTS_W6(k) \
    case k: __builtin_amdgcn_s_waitcnt(((LO + k) & 15) | (7 << 4) | (15 << 8) | (((LO + k) >> 4) << 14)); break;
    switch (min(max(n - LO, 0), 15)) {
        DTS_W6(0) DTS_W6(1) DTS_W6(2) DTS_W6(3) DTS_W6(4) DTS_W6(5) DTS_W6(6) DTS_W6(7)
        DTS_W6(8) DTS_W6(9) DTS_W6(10) DTS_W6(11) DTS_W6(12) DTS_W6(13) DTS_W6(14)
    default: DTS_W6(15)
    }
#undef DTS_W6
}

// s_waitcnt vmcnt(N) through the builtin, so the compiler's own wait insertion sees it
// (it does not order the LDS-DMA writes with the ds_reads of the same LDS)
template <int N>
__device__ __forceinline__ void vm_wait6()
{
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

} // namespace
} // namespace dts
