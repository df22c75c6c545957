// ladder6.hip -- k_ladder6, the v6 ladder kernel: 8-bit 4:2:0 planar sources
// to 8-bit renditions, both FIR passes on the matrix cores
// (v_mfma_i32_16x16x64_i8), the H outputs never leaving the VGPRs.
//
// Same arithmetic as libswscale hScale8To15_c -> yuv2planeX_8_c /
// yuv2nv12cX_c under SWS_BITEXACT|SWS_ACCURATE_RND (FFmpeg 4.4; bit-exact,
// DESIGN.md "Oracle"), and the same integer identities as k_ladder5
// (ladder5.hip header), organised so that nothing is shared between waves:
//
//  * one wave = one work unit: CT 16-column tiles of one rendition of one plane
//    kind (chroma: the same columns of U and V) of one frame, walked top to
//    bottom in granules of 16 source rows.  Workgroups are single waves; the
//    units of frame f all run on XCD f % 8 (workgroup ids go round robin over
//    the XCDs), so a frame's source rows are fetched from HBM into one L2 and
//    re-read from there by the other units of the frame;
//  * H of a granule: per tile one MFMA per K block and tap half.  A = 16 source
//    rows x 64 columns straight from memory (one 16-B load per lane, the bytes
//    x0 + 64 kb + 16 g .. + 15 of row m), xor 0x80; B = the tile's taps, held in
//    VGPRs for the whole walk (plan6.cpp K order);
//  * the H result of a tile is, per lane, 4 consecutive source rows of one
//    output column -- exactly a V A-operand dword once split into y >> 8 and
//    (y & 255) ^ 0x80 bytes.  The last 4 VKB granules of every tile stay in a
//    register ring (slot = granule mod 4 VKB; the walk is unrolled by the ring
//    length so every slot is a fixed register);
//  * V of a row block (16 output rows) runs right after the granule that
//    completes its window: out^T = H^T C^T over the whole ring, 4 MFMAs per K
//    block, the fragment laid out for where each granule sits in the ring;
//  * stores: each lane holds 4 consecutive columns of one output row per tile;
//    v_permlane32/16_swap transpose the tiles so a lane holds 16 (CT 4) or 8
//    consecutive bytes of its row (nv12: U and V interleaved by v_perm).
#include "dts_internal.h"

#ifndef DTS_L6_NS
#define DTS_L6_NS 2         // LDS stages per wave: source granules in flight (DMA'd NS granules ahead)
#endif
#ifndef DTS_L6_ABLATE
#define DTS_L6_ABLATE 0     // diagnostic builds only: 1 skip the source loads, 2 skip the V blocks, 8 load
                            // one (tile, K block) of source per granule and feed it to every tile,
                            // 4 skip the V stores
#endif
#ifndef DTS_L6_LDSPAD
#define DTS_L6_LDSPAD 0     // diagnostic builds only: extra LDS per wave (fewer waves per CU)
#endif
#ifndef DTS_L6_WPE
#define DTS_L6_WPE 0        // > 0: ask the compiler for at least this many waves per SIMD
#endif

#ifndef DTS_L6_STAMP
#define DTS_L6_STAMP 0      // diagnostic builds only: per-variant, per-phase s_memtime sums (tools/stamp6.py)
#endif

namespace dts {

#if DTS_L6_STAMP
// [variant][phase]: cycles summed over every wave; [variant][6]: granules, [variant][7]: waves
__device__ unsigned long long g_l6_stamp[kL6Variants][8];
#define L6_STAMP(k)                                                        \
    do {                                                                   \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();        \
        st_acc[k] += t_ - st_last;                                         \
        st_last = t_;                                                      \
    } while (0)
#else
#define L6_STAMP(k) (void)0
#endif

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
        if (NB == 16)
            *GP6(g_u32x4, p) = (u32x4){w[0], w[1], w[2 % (NB / 4)], w[3 % (NB / 4)]};
        else if (NB == 8)
            *GP6(g_u32x2, p) = (u32x2){w[0], w[1 % (NB / 4)]};
        else
            *GP6(g_u32, p) = w[0];
    } else {
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
template <int VAR>
__device__ __forceinline__ int vblock(const Unit6 &U, int j, const v4i (&rh)[Walk6<VAR>::VKB][Walk6<VAR>::T],
                                       const v4i (&rl)[Walk6<VAR>::VKB][Walk6<VAR>::T],
                                       const v4i (&vh)[Walk6<VAR>::VKB], const v4i (&vl)[Walk6<VAR>::VKB],
                                       const uint64_t (&ob)[2], const uint32_t (&op)[2], int m, int g,
                                       uint8_t *scr)
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
    uint32_t w[W::T];
#pragma unroll
    for (int t = 0; t < W::T; ++t) {
        // av_clip_uint8(val >> 19) of 4 columns, packed
        const uint32_t lo = __builtin_amdgcn_ashr_pk_u8_i32(acc[t][0], acc[t][1], 19);
        const uint32_t hi = __builtin_amdgcn_ashr_pk_u8_i32(acc[t][2], acc[t][3], 19);
        w[t] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
    }
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

template <int VAR>
__device__ __forceinline__ void walk6(const Ladder6Params &P, const Unit6 &U, int f)
{
    using W = Walk6<VAR>;
    constexpr int CT = W::CT, NP = W::NP, HKB = W::HKB, VKB = W::VKB, T = W::T, R = W::R;
    const int lane = (int)threadIdx.x, m = lane & 15, g = lane >> 4;
    // source planes of this frame (luma: plane 0; chroma: planes 1 and 2)
    // (the plane tables are read from the kernarg segment by s_load: indexing the by-value
    // parameter with a run-time index would copy it to scratch)
    const uint8_t *ka = (const uint8_t *)__builtin_amdgcn_kernarg_segment_ptr();
    const DevPlanes S = kld6(reinterpret_cast<const DevPlanes *>(ka + offsetof(Ladder6Params, src)));
    uint64_t sb[NP];
    uint32_t sp[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        sb[p] = (U.kind ? S.data[1 + p] : S.data[0]) + (uint64_t)f * (uint64_t)S.fstride;
        sp[p] = (uint32_t)(U.kind ? S.pitch[1 + p] : S.pitch[0]);
    }
    // output planes: luma plane 0; nv12 chroma plane 1; yuv420p chroma planes 1 and 2
    uint64_t ob[2];
    uint32_t op[2];
    {
        const DevPlanes D = kld6(reinterpret_cast<const DevPlanes *>(ka + offsetof(Ladder6Params, dst)) + U.rung);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            ob[p] = (U.kind ? D.data[1 + p] : D.data[0]) + (uint64_t)f * (uint64_t)D.fstride;
            op[p] = (uint32_t)(U.kind ? D.pitch[1 + p] : D.pitch[0]);
        }
    }
    (void)P;
    const uint64_t fr = (uint64_t)(uintptr_t)P.frag + 16u * (uint32_t)lane;
    // H B operands of the walk
    v4i bh[CT][HKB], bl[CT][HKB];
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int kb = 0; kb < HKB; ++kb) {
            const uint64_t o = fr + (uint64_t)(U.hfrag + (uint32_t)(c * HKB + kb)) * 2048u;
            bh[c][kb] = *GP6(g_cv4i, o);
            bl[c][kb] = *GP6(g_cv4i, o + 1024);
        }
    // V: the next row block to run and its fire granule; the next one whose fragments are
    // to be DMA'd and its fire granule
    k_u32 *fire = GP6(k_u32, P.fire + U.fire);
    int j = 0, jf = 0;
    int fg = U.nrb > 0 ? (int)fire[0] : 0x7fffffff, fgf = fg;
    v4i vh[VKB], vl[VKB];
    const v4i zero = {0, 0, 0, 0}, hbias = {kL5Bias, kL5Bias, kL5Bias, kL5Bias};
    // the ring: slot s of tile t is dword s % 4 of rh[s / 4][t] (hi bytes) and rl (lo bytes)
    v4i rh[VKB][T], rl[VKB][T];
#pragma unroll
    for (int kb = 0; kb < VKB; ++kb)
#pragma unroll
        for (int t = 0; t < T; ++t) rh[kb][t] = rl[kb][t] = zero;
    const int ngran = U.ngran, srcH1 = U.srcH - 1;
#if DTS_L6_STAMP
    unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif
    // A operands: the 16 rows x 64 bytes of every (plane, tile, K block) reach this wave's
    // LDS by LDS-DMA, NS granules ahead (stage q % NS).  DMA lane l loads row l >> 2, chunk
    // (l & 3) ^ ((l >> 4) & 3) of the 64 bytes: four lanes cover one row's 64 contiguous
    // bytes (one cache access instead of four), and the A read of lane (m, g) -- row m,
    // chunk g -- is a conflict-free ds_read_b128 at 16 (4 m + (g ^ ((m >> 2) & 3))).
    constexpr int NS = DTS_L6_NS, ND = T * HKB;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds6[];
    const int dr = lane >> 2, dch = (lane & 3) ^ ((dr >> 2) & 3);
    uint32_t dcol[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) dcol[c] = (uint32_t)U.x0[c] + 16u * (uint32_t)dch;
    const uint32_t roff = 16u * (uint32_t)(4 * m + (g ^ ((m >> 2) & 3)));
    // V fragment slots after the stages: row block j's fragments in slot j % fs, DMA'd right
    // after the source of its fire granule, so the source wait covers them too
    uint8_t *fb = lds6 + NS * ND * 1024;
    const int FS = U.fs;
    int fsi = 0, fsu = 0;
    int ops = 0;                                           // VMEM instructions issued so far
    int oend[NS];                                          // ops after the batch of granule q (slot q % NS)
    auto frags = [&](int upto) {
        while (fgf <= upto) {
            ops += 2 * VKB;
            uint8_t *dst = fb + (uint32_t)fsi * (uint32_t)(VKB * 2048);
            const uint64_t src = fr + (uint64_t)(U.vfrag + (uint32_t)(jf * VKB)) * 2048u;
#pragma unroll
            for (int h = 0; h < 2 * VKB; ++h)
                __builtin_amdgcn_global_load_lds((const void *)(uintptr_t)(src + 1024u * h),
                                                 (__attribute__((address_space(3))) void *)(dst + 1024 * h), 16, 0, 0);
            fsi = fsi + 1 == FS ? 0 : fsi + 1;
            ++jf;
            fgf = jf < U.nrb ? (int)fire[jf] : 0x7fffffff;
        }
    };
    // one batch: the fragments of the row blocks firing at granule q, then granule q's source
    auto dma = [&](int q) {
        frags(q);
        if (DTS_L6_ABLATE & 1) return;
        const uint32_t row = (uint32_t)min(kL6Gran * q + dr, srcH1);
        uint8_t *st = lds6 + (uint32_t)(q % NS) * (uint32_t)(ND * 1024);
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const uint64_t rp = sb[p] + (uint64_t)(row * sp[p]);
#pragma unroll
            for (int c = 0; c < CT; ++c)
#pragma unroll
                for (int kb = 0; kb < HKB; ++kb)
                    if (!(DTS_L6_ABLATE & 8) || (p * CT + c) * HKB + kb == 0)
                    {
                        __builtin_amdgcn_global_load_lds(
                            (const void *)(uintptr_t)(rp + dcol[c] + 64u * kb),
                            (__attribute__((address_space(3))) void *)(st + 1024 * ((p * CT + c) * HKB + kb)), 16, 0, 0);
                        ++ops;
                    }
        }
    };
#pragma unroll
    for (int i = 0; i < NS - 1; ++i) {
        dma(i);
        oend[i] = ops;
    }
    // the walk is unrolled by the ring length, so ring slot q % R and stage q % NS are
    // fixed registers / offsets in each copy; granules past the plane (to a whole ring
    // period) are computed and never used
    static_assert(R % NS == 0, "the stages cycle within a ring period");
    const int ngp = (ngran + R - 1) / R * R;
    for (int q0 = 0; q0 < ngp; q0 += R) {
#pragma unroll
        for (int s = 0; s < R; ++s) {
            const int q = q0 + s;
            // granule q + NS - 1 into the stage granule q - 1 was read from (its ds_reads
            // completed before its MFMAs); past the plane: clamped rows, unused, which keeps
            // the count uniform
            L6_STAMP(4);
            dma(q + NS - 1);
            oend[(s + NS - 1) % NS] = ops;
            L6_STAMP(0);
            // granule q's batch (its source and the fragments of the row blocks firing at
            // q) has landed: every VMEM instruction issued after it may still be in flight
            vm_wait_n6<(NS - 1) * ((DTS_L6_ABLATE & (1 | 8)) ? (DTS_L6_ABLATE & 1 ? 0 : 1) : ND)>(ops - oend[s % NS]);
            L6_STAMP(1);
            {
                const uint8_t *st = lds6 + (s % NS) * (ND * 1024) + roff;
                v4i a[T][HKB];
#pragma unroll
                for (int t = 0; t < T; ++t)
#pragma unroll
                    for (int kb = 0; kb < HKB; ++kb)
                        a[t][kb] = *reinterpret_cast<const v4i *>(st + ((DTS_L6_ABLATE & 8) ? 0 : 1024 * (t * HKB + kb))) ^
                                   (int)0x80808080u;
                v4i ah[T], al[T];
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    ah[t] = zero;
                    al[t] = hbias;
                }
#pragma unroll
                for (int kb = 0; kb < HKB; ++kb)
#pragma unroll
                    for (int t = 0; t < T; ++t) {
                        ah[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[t][kb], bh[t % CT][kb], ah[t], 0, 0, 0);
                        al[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[t][kb], bl[t % CT][kb], al[t], 0, 0, 0);
                    }
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    const uint32_t p0 = pack_h6(ah[t].x, al[t].x, ah[t].y, al[t].y);   // rows 4g, 4g+1
                    const uint32_t p1 = pack_h6(ah[t].z, al[t].z, ah[t].w, al[t].w);   // rows 4g+2, 4g+3
                    rh[s / 4][t][s % 4] = (int)__builtin_amdgcn_perm(p1, p0, 0x07050301u);
                    rl[s / 4][t][s % 4] = (int)(__builtin_amdgcn_perm(p1, p0, 0x06040200u) ^ 0x80808080u);
                }
            }
            L6_STAMP(2);
            while (fg == q) {
                {
                    const uint8_t *fu = fb + (uint32_t)fsu * (uint32_t)(VKB * 2048) + 16u * (uint32_t)lane;
#pragma unroll
                    for (int kb = 0; kb < VKB; ++kb) {
                        vh[kb] = *reinterpret_cast<const v4i *>(fu + 2048 * kb);
                        vl[kb] = *reinterpret_cast<const v4i *>(fu + 2048 * kb + 1024);
                    }
                    fsu = fsu + 1 == FS ? 0 : fsu + 1;
                }
                if (!(DTS_L6_ABLATE & 2)) {
                    ops += vblock<VAR>(U, j, rh, rl, vh, vl, ob, op, m, g, fb + FS * VKB * 2048);
                } else {
#pragma unroll
                    for (int kb = 0; kb < VKB; ++kb)
#pragma unroll
                        for (int t = 0; t < T; ++t)
                            asm volatile("" ::"v"(rh[kb][t]), "v"(rl[kb][t]), "v"(vh[kb]), "v"(vl[kb]));
                }
                ++j;
                fg = j < U.nrb ? (int)fire[j] : 0x7fffffff;
                L6_STAMP(3);
            }
        }
    }
    // the DMAs past the plane still write this workgroup's LDS: drain them before the
    // wave (and its LDS allocation) ends
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if DTS_L6_STAMP
    L6_STAMP(5);
    if (lane == 0) {
        for (int k = 0; k < 6; ++k) atomicAdd(&g_l6_stamp[VAR][k], st_acc[k]);
        atomicAdd(&g_l6_stamp[VAR][6], (unsigned long long)ngp);
        atomicAdd(&g_l6_stamp[VAR][7], 1ull);
    }
#endif
}

__global__ __launch_bounds__(64)
#if DTS_L6_WPE > 0
__attribute__((amdgpu_waves_per_eu(DTS_L6_WPE)))
#endif
void k_ladder6(Ladder6Params P)
{
    // workgroup b: XCD b % 8; frame 8 (k / nunits) + b % 8, unit k % nunits (k = b / 8)
    const int b = (int)blockIdx.x, k = b >> 3;
    const int fq = k / P.nunits;
    const int f = 8 * fq + (b & 7);
    if (f >= P.nframes) return;
    const Unit6 U = kld6(P.units + (k - fq * P.nunits));
    switch (U.variant) {
    case 0: walk6<0>(P, U, f); break;
    case 1: walk6<1>(P, U, f); break;
    case 2: walk6<2>(P, U, f); break;
    case 3: walk6<3>(P, U, f); break;
    case 4: walk6<4>(P, U, f); break;
    case 5: walk6<5>(P, U, f); break;
    case 6: walk6<6>(P, U, f); break;
    default: walk6<7>(P, U, f); break;
    }
}

} // namespace

#if DTS_L6_STAMP
int ladder6_stamps(unsigned long long *out, bool reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_l6_stamp), sizeof(g_l6_stamp)) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[kL6Variants * 8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_l6_stamp), z, sizeof z) != hipSuccess) return -1;
    }
    return kL6Variants * 8;
}
#endif

static_assert(DTS_L6_NS <= kL6Stages, "the planner sizes the fragment slots for kL6Stages granules");

int ladder6_lds_bytes(const Unit6 &u)
{
    const int v = u.variant;
    return DTS_L6_NS * l6_ct(v) * l6_np(v) * l6_hkb(v) * 1024 + u.fs * l6_vkb(v) * 2048 + 1024 +   // + store scratch
           DTS_L6_LDSPAD;
}

hipError_t launch_ladder6(const Ladder6Params &p, int grid, int lds_bytes, hipStream_t s)
{
    hipLaunchKernelGGL(k_ladder6, dim3(grid), dim3(64), lds_bytes, s, p);
    return hipGetLastError();
}

} // namespace dts
