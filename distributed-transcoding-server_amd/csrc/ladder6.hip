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
#define DTS_L6_ABLATE 0     // diagnostic builds only: 1 skip the source loads, 2 skip the V blocks,
                            // 4 skip the V stores
#endif
#ifndef DTS_L6_WPE
#define DTS_L6_WPE 0        // > 0: ask the compiler for at least this many waves per SIMD
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

// av_clip_uint8((65536 hh + 256 (hl + lh) + ll + bias) >> 19) of 4 columns, packed
__device__ __forceinline__ uint32_t vcombine6(const v4i &hh, const v4i &hl, const v4i &ll)
{
    int v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (((hh[i] << 8) + hl[i]) << 8) + ll[i];
    const uint32_t lo = __builtin_amdgcn_ashr_pk_u8_i32(v[0], v[1], 19);
    const uint32_t hi = __builtin_amdgcn_ashr_pk_u8_i32(v[2], v[3], 19);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
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

template <int VAR>
struct Walk6 {
    static constexpr int CT = l6_ct(VAR), NP = l6_np(VAR), HKB = l6_hkb(VAR), VKB = l6_vkb(VAR);
    static constexpr int T = CT * NP, R = 4 * VKB;
};

// one row block: V over the whole ring, then the stores of output row 16 j + m
template <int VAR>
__device__ __forceinline__ void vblock(const Unit6 &U, int j, const v4i (&rh)[Walk6<VAR>::VKB][Walk6<VAR>::T],
                                       const v4i (&rl)[Walk6<VAR>::VKB][Walk6<VAR>::T],
                                       const v4i (&vh)[Walk6<VAR>::VKB], const v4i (&vl)[Walk6<VAR>::VKB],
                                       const uint64_t (&ob)[2], const uint32_t (&op)[2], int m, int g)
{
    using W = Walk6<VAR>;
    const v4i zero = {0, 0, 0, 0}, vbias = {kL5VBias, kL5VBias, kL5VBias, kL5VBias};
    v4i hh[W::T], hl[W::T], ll[W::T];
#pragma unroll
    for (int t = 0; t < W::T; ++t) {
        hh[t] = zero;
        hl[t] = zero;
        ll[t] = vbias;
    }
#pragma unroll
    for (int kb = 0; kb < W::VKB; ++kb)
#pragma unroll
        for (int t = 0; t < W::T; ++t) {
            const v4i ah = rh[kb][t], al = rl[kb][t];
            hh[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, vh[kb], hh[t], 0, 0, 0);
            hl[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, vl[kb], hl[t], 0, 0, 0);
            ll[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, vl[kb], ll[t], 0, 0, 0);
            hl[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, vh[kb], hl[t], 0, 0, 0);
        }
    uint32_t w[W::T];
#pragma unroll
    for (int t = 0; t < W::T; ++t) w[t] = vcombine6(hh[t], hl[t], ll[t]);
    if (DTS_L6_ABLATE & 4) {
#pragma unroll
        for (int t = 0; t < W::T; ++t) asm volatile("" ::"v"(w[t]));
        return;
    }
    const int y = 16 * j + m;
    if (y >= U.dstH) return;
    if (W::NP == 1) {                                      // luma
        const uint64_t rowp = ob[0] + (uint64_t)y * op[0];
        if (W::CT == 4) {
            uint32_t o[4];
            transpose4(w[0], w[1 % W::T], w[2 % W::T], w[3 % W::T], o);
            const int at = U.col0 + 16 * g;
            put_row6<16>(rowp, at, U.dstW - at, o);
        } else {
            uint32_t o[2];
            transpose2(w[0], w[1 % W::T], o);
            const int at = U.col0 + 8 * g;
            put_row6<8>(rowp, at, U.dstW - at, o);
        }
    } else if (U.fmt == DTS_FMT_NV12) {                    // chroma, U V interleaved
        const uint64_t rowp = ob[0] + (uint64_t)y * op[0];
#pragma unroll
        for (int c = 0; c < W::CT; ++c) {
            const uint32_t u = w[c], v = w[W::CT + c];
            const uint32_t o[2] = {__builtin_amdgcn_perm(v, u, 0x05010400u), __builtin_amdgcn_perm(v, u, 0x07030602u)};
            const int at = 2 * U.col0 + 32 * c + 8 * g;
            put_row6<8>(rowp, at, 2 * U.dstW - at, o);
        }
    } else {                                               // chroma, U and V planes
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const uint64_t rowp = ob[p] + (uint64_t)y * op[p];
            if (W::CT == 2) {
                uint32_t o[2];
                transpose2(w[2 * p], w[(2 * p + 1) % W::T], o);
                const int at = U.col0 + 8 * g;
                put_row6<8>(rowp, at, U.dstW - at, o);
            } else {
                const uint32_t o[1] = {w[p % W::T]};
                const int at = U.col0 + 4 * g;
                put_row6<4>(rowp, at, U.dstW - at, o);
            }
        }
    }
}

// s_waitcnt vmcnt(N) through the builtin, so the compiler's own wait insertion sees it
// (it does not order the LDS-DMA writes with the ds_reads of the same LDS)
template <int N>
__device__ __forceinline__ void vm_wait6()
{
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// ring slot s <- this granule's (hi, lo) dwords of every tile (s wave-uniform)
template <int S, int R, int T>
__device__ __forceinline__ void ring_put(v4i (&rh)[R / 4][T], v4i (&rl)[R / 4][T], int s, const uint32_t (&hi)[T],
                                         const uint32_t (&lo)[T])
{
    if constexpr (S < R) {
        if (s == S) {
#pragma unroll
            for (int t = 0; t < T; ++t) {
                rh[S / 4][t][S % 4] = (int)hi[t];
                rl[S / 4][t][S % 4] = (int)lo[t];
            }
            return;
        }
        ring_put<S + 1, R, T>(rh, rl, s, hi, lo);
    }
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
    auto frags = [&](int upto) {
        while (fgf <= upto) {
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
    auto dma = [&](int q) {
        if (DTS_L6_ABLATE & 1) {
            frags(q);
            return;
        }
        const uint32_t row = (uint32_t)min(kL6Gran * q + dr, srcH1);
        uint8_t *st = lds6 + (uint32_t)(q % NS) * (uint32_t)(ND * 1024);
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const uint64_t rp = sb[p] + (uint64_t)(row * sp[p]);
#pragma unroll
            for (int c = 0; c < CT; ++c)
#pragma unroll
                for (int kb = 0; kb < HKB; ++kb)
                    __builtin_amdgcn_global_load_lds(
                        (const void *)(uintptr_t)(rp + dcol[c] + 64u * kb),
                        (__attribute__((address_space(3))) void *)(st + 1024 * ((p * CT + c) * HKB + kb)), 16, 0, 0);
        }
        frags(q);
    };
#pragma unroll
    for (int i = 0; i < NS - 1; ++i) dma(i);
    int s = 0;                                             // ring slot of granule q
    for (int q = 0; q < ngran; ++q) {
        {
            // granule q + NS - 1 into the stage granule q - 1 was read from (its ds_reads
            // completed before its MFMAs); past the plane: clamped rows, unused, which keeps
            // the count uniform
            dma(q + NS - 1);
            // granule q's DMAs have landed: only the (NS - 1) ND DMAs issued after them may
            // be outstanding (younger V stores / fragment loads only make this wait longer)
            vm_wait6<(NS - 1) * ND>();
            const uint8_t *st = lds6 + (uint32_t)(q % NS) * (uint32_t)(ND * 1024) + roff;
            v4i a[T][HKB];
#pragma unroll
            for (int t = 0; t < T; ++t)
#pragma unroll
                for (int kb = 0; kb < HKB; ++kb)
                    a[t][kb] = *reinterpret_cast<const v4i *>(st + 1024 * (t * HKB + kb)) ^ (int)0x80808080u;
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
            uint32_t hi[T], lo[T];
#pragma unroll
            for (int t = 0; t < T; ++t) {
                const uint32_t p0 = pack_h6(ah[t].x, al[t].x, ah[t].y, al[t].y);   // rows 4g, 4g+1
                const uint32_t p1 = pack_h6(ah[t].z, al[t].z, ah[t].w, al[t].w);   // rows 4g+2, 4g+3
                hi[t] = __builtin_amdgcn_perm(p1, p0, 0x07050301u);
                lo[t] = __builtin_amdgcn_perm(p1, p0, 0x06040200u) ^ 0x80808080u;
            }
            ring_put<0, R, T>(rh, rl, s, hi, lo);
            s = s + 1 == R ? 0 : s + 1;
        }
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
                vblock<VAR>(U, j, rh, rl, vh, vl, ob, op, m, g);
            } else {
#pragma unroll
                for (int kb = 0; kb < VKB; ++kb)
#pragma unroll
                    for (int t = 0; t < T; ++t) asm volatile("" ::"v"(rh[kb][t]), "v"(rl[kb][t]), "v"(vh[kb]), "v"(vl[kb]));
            }
            ++j;
            fg = j < U.nrb ? (int)fire[j] : 0x7fffffff;
        }
    }
    // the DMAs past the plane still write this workgroup's LDS: drain them before the
    // wave (and its LDS allocation) ends
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

static_assert(DTS_L6_NS <= kL6Stages, "the planner sizes the fragment slots for kL6Stages granules");

int ladder6_lds_bytes(const Unit6 &u)
{
    const int v = u.variant;
    return DTS_L6_NS * l6_ct(v) * l6_np(v) * l6_hkb(v) * 1024 + u.fs * l6_vkb(v) * 2048;
}

hipError_t launch_ladder6(const Ladder6Params &p, int grid, int lds_bytes, hipStream_t s)
{
    hipLaunchKernelGGL(k_ladder6, dim3(grid), dim3(64), lds_bytes, s, p);
    return hipGetLastError();
}

} // namespace dts
