// kernels.hip -- gfx950 kernels of the per-segment pixel filtergraph.
//
//  k_ladder   : fused separable polyphase scale + pixel-format convert for
//               every rendition of a graph in ONE launch (libswscale
//               hScale8To15/hScale16To15 -> yuv2planeX_8 / yuv2nv12cX under
//               SWS_BITEXACT|SWS_ACCURATE_RND, bit-exact).
//  k_quality  : vf_psnr SSE + vf_ssim 4x4-block / 8x8-window SSIM partials.
//  k_qreduce  : fixed-order reduction of the quality partials per frame.
//  k_synth    : deterministic testsrc2-like source frames.
//
// Design (DESIGN.md "Kernels"): one workgroup = one (frame, rendition, plane
// kind, column strip).  It walks the source rows top to bottom in steps of
// 8 rows: the strip's source window is staged into LDS with 16-B coalesced
// loads (prefetched one step ahead in registers), each thread produces the
// 15-bit horizontal intermediates of its output column for the 8 rows with
// v_dot4_i32_i8 (u8) / v_dot2_i32_i16 (p010) from per-thread coefficient
// registers, row pairs are packed int16x2 into an LDS ring, and the vertical
// FIR (v_dot2_i32_i16 with wave-uniform coefficients) emits every output row
// whose window is complete.  No intermediate touches HBM; each source byte is
// fetched from HBM once per rendition strip (re-reads of the same frame by
// the other renditions hit the XCD L2 / Infinity Cache).
#include "dts_internal.h"

#ifndef DTS_ABLATE
#define DTS_ABLATE 0
#endif
#ifndef DTS_V_UNROLL
#define DTS_V_UNROLL 1
#endif

namespace dts {

__constant__ uint8_t c_dither[8][8] = DTS_DITHER_8X8_128;

typedef short short2v __attribute__((ext_vector_type(2)));
// global (address space 1) views: keeps VMEM traffic off the flat path so LDS
// waits (lgkmcnt) and global waits (vmcnt) stay independent
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_cu32x4;
typedef __attribute__((address_space(1))) const uint32_t g_cu32;
typedef __attribute__((address_space(1))) const int32_t g_ci32;
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) uint16_t g_u16;
typedef __attribute__((address_space(1))) uint8_t g_u8;
#define GPTR(T, p) ((T *)(uintptr_t)(p))

__device__ __forceinline__ int dot4(uint32_t a, uint32_t b, int c)
{
    return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

__device__ __forceinline__ int dot2(uint32_t a, uint32_t b, int c)
{
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, a), __builtin_bit_cast(short2v, b), c, false);
}

__device__ __forceinline__ uint32_t clip8(int v)
{
    v >>= 19;
    return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// output.c p010 output_pixel: av_clip_uintp2(val >> 17, 10) << 6
__device__ __forceinline__ uint16_t clip10s(int v)
{
    v >>= 17;
    return (uint16_t)((v < 0 ? 0 : (v > 1023 ? 1023 : v)) << 6);
}

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel)
{
    return __builtin_amdgcn_perm(hi, lo, sel);
}

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// ---------------------------------------------------------------------------
// k_ladder
// ---------------------------------------------------------------------------
constexpr int kVPre = 4;     // output rows per wave whose V data is prefetched per step

// Horizontal FIR of one thread's output column over the kBlkRows staged rows,
// packed as int16x2 row pairs.  ND is a compile-time tap-dword count so all
// LDS reads of a row issue before the first dot product consumes them.
// v_cvt_pk_i16_i32 saturates, which is exactly FFMIN(val, 32767) here (val >=
// -32768 always holds for normalised filters on 8/10-bit samples).
template <int SRC, int ND, int NDMAX>
__device__ __forceinline__ void hrows(const uint8_t *s, int swb, const uint32_t (&ch)[NDMAX],
                                      const uint32_t (&cl)[NDMAX], int bias, uint32_t (&hp)[kBlkRows / 2])
{
#pragma unroll
    for (int pr = 0; pr < kBlkRows / 2; ++pr) {
        int val[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint32_t *rp = reinterpret_cast<const uint32_t *>(s + (2 * pr + q) * swb);
            uint32_t v[ND];
#pragma unroll
            for (int k = 0; k < ND; ++k) v[k] = rp[k];
            if (SRC == kSrcP010) {
                int a = 0;
#pragma unroll
                for (int k = 0; k < ND; ++k) a = dot2(v[k], ch[k], a);
                val[q] = a >> 9;                            // hScale16To15: sh = depth - 1
            } else {
                int a = 0, c = bias;
#pragma unroll
                for (int k = 0; k < ND; ++k) {
                    a = dot4(v[k], ch[k], a);
                    c = dot4(v[k], cl[k], c);
                }
                val[q] = (a * 256 + c) >> 7;                // hScale8To15 (src ^ 0x80 bias folded in c)
            }
        }
        hp[pr] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(val[0], val[1]));
    }
}

// Vertical FIR of one output row for one wave.  Luma: each lane owns 4
// consecutive columns (one ds_read_b128 per row pair); chroma: 2 columns of U
// and of V.  NV row pairs, tap pair k read from lane k of cq by v_readlane.
template <int KIND, int NV>
__device__ __forceinline__ void vtaps(const uint32_t *ring, int RP, int q0, int lane, uint32_t cq, int (&acc)[4])
{
    constexpr int cols = KIND ? kChromaCols : kLumaCols;
    const int s0 = q0 & (RP - 1);
    if (s0 + NV <= RP) {                     // no wrap: one base address, immediate offsets
        const uint32_t *b = ring + s0 * cols;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const uint32_t c = __builtin_amdgcn_readlane(cq, k);
            if (KIND == 0) {
                const uint4 v = *reinterpret_cast<const uint4 *>(b + k * cols + 4 * lane);
                acc[0] = dot2(v.x, c, acc[0]);
                acc[1] = dot2(v.y, c, acc[1]);
                acc[2] = dot2(v.z, c, acc[2]);
                acc[3] = dot2(v.w, c, acc[3]);
            } else {
                const uint2 u = *reinterpret_cast<const uint2 *>(b + k * cols + 2 * lane);
                const uint2 w = *reinterpret_cast<const uint2 *>(b + (RP + k) * cols + 2 * lane);
                acc[0] = dot2(u.x, c, acc[0]);
                acc[1] = dot2(u.y, c, acc[1]);
                acc[2] = dot2(w.x, c, acc[2]);
                acc[3] = dot2(w.y, c, acc[3]);
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int sl = (s0 + k) & (RP - 1);
            const uint32_t c = __builtin_amdgcn_readlane(cq, k);
            if (KIND == 0) {
                const uint4 v = *reinterpret_cast<const uint4 *>(ring + sl * cols + 4 * lane);
                acc[0] = dot2(v.x, c, acc[0]);
                acc[1] = dot2(v.y, c, acc[1]);
                acc[2] = dot2(v.z, c, acc[2]);
                acc[3] = dot2(v.w, c, acc[3]);
            } else {
                const uint2 u = *reinterpret_cast<const uint2 *>(ring + sl * cols + 2 * lane);
                const uint2 w = *reinterpret_cast<const uint2 *>(ring + (RP + sl) * cols + 2 * lane);
                acc[0] = dot2(u.x, c, acc[0]);
                acc[1] = dot2(u.y, c, acc[1]);
                acc[2] = dot2(w.x, c, acc[2]);
                acc[3] = dot2(w.y, c, acc[3]);
            }
        }
    }
}

template <int KIND>
__device__ __forceinline__ void vtaps_any(const uint32_t *ring, int RP, int q0, int lane, int nv, uint32_t cq,
                                          int (&acc)[4])
{
#if DTS_V_UNROLL
    switch (nv) {                                            // wave-uniform
#define DTS_VCASE(N) \
    case N: vtaps<KIND, N>(ring, RP, q0, lane, cq, acc); return;
        DTS_VCASE(1) DTS_VCASE(2) DTS_VCASE(3) DTS_VCASE(4) DTS_VCASE(5) DTS_VCASE(6) DTS_VCASE(7) DTS_VCASE(8)
        DTS_VCASE(9) DTS_VCASE(10) DTS_VCASE(11) DTS_VCASE(12) DTS_VCASE(13) DTS_VCASE(14) DTS_VCASE(15) DTS_VCASE(16)
#undef DTS_VCASE
    default:
        break;
    }
#endif
    // wide vertical filters (> 32 taps): generic loop (the pair table is
    // read from registers of up to 64 lanes)
    constexpr int cols = KIND ? kChromaCols : kLumaCols;
    for (int k = 0; k < nv; ++k) {
        const int sl = ((q0 + k) & (RP - 1));
        const uint32_t c = __builtin_amdgcn_readlane(cq, k);
        if (KIND == 0) {
            const uint4 v = *reinterpret_cast<const uint4 *>(ring + sl * cols + 4 * lane);
            acc[0] = dot2(v.x, c, acc[0]);
            acc[1] = dot2(v.y, c, acc[1]);
            acc[2] = dot2(v.z, c, acc[2]);
            acc[3] = dot2(v.w, c, acc[3]);
        } else {
            const uint2 u = *reinterpret_cast<const uint2 *>(ring + sl * cols + 2 * lane);
            const uint2 w = *reinterpret_cast<const uint2 *>(ring + (RP + sl) * cols + 2 * lane);
            acc[0] = dot2(u.x, c, acc[0]);
            acc[1] = dot2(u.y, c, acc[1]);
            acc[2] = dot2(w.x, c, acc[2]);
            acc[3] = dot2(w.y, c, acc[3]);
        }
    }
}

// One work item: a (frame, rung, plane kind, column strip) walked top to bottom.
template <int SRC, int NDMAX>
__device__ __forceinline__ void ladder_item(const LadderParams &P, int frame, int jid, uint8_t *smem)
{
    const int t = threadIdx.x;
    const Job J = P.jobs[jid];
    const int kind = J.kind;
    const RungKind K = P.rk[J.rung * 2 + kind];
    const int RP = P.ring_pairs;
    const int pcols = kind ? kChromaCols : kLumaCols;
    const int srcH = kind ? P.chrH : P.srcH;
    const int swb = J.swb;
    const int plane_stage = kBlkRows * swb;         // bytes of one plane in a stage buffer

    uint8_t *const stage0 = smem;
    uint8_t *const stage1 = smem + P.stage_bytes;
    uint32_t *const ring = reinterpret_cast<uint32_t *>(smem + 2 * P.stage_bytes);

    // ---- staging item decode (fixed per thread for the whole walk) --------
    const int n16 = swb >> 4;                        // 16-B chunks per row per plane
    const bool inter_chroma = kind && (SRC != kSrcPlanar8);
    const int per_row = inter_chroma ? 2 * n16 : n16;
    const int pln = kind ? 1 : 0;
    const int64_t pitch = P.src.pitch[pln];
    const int64_t fbase = (int64_t)frame * P.src.fstride;
    uint64_t gaddr[kMaxLoads];
    int srow[kMaxLoads], sofs[kMaxLoads];
    bool sok[kMaxLoads];
#pragma unroll
    for (int k = 0; k < kMaxLoads; ++k) {
        const int i = t + k * kThreads;
        int plane = pln, row = 0, c = 0;
        if (inter_chroma) {
            row = i / per_row;
            c = i - row * per_row;
        } else {
            const int pr = i / n16;
            c = i - pr * n16;
            plane += pr / kBlkRows;
            row = pr % kBlkRows;
        }
        if (plane > 2) plane = 2;
        const int64_t boff = (int64_t)J.sx0 * (inter_chroma ? (SRC == kSrcP010 ? 4 : 2) : (SRC == kSrcP010 ? 2 : 1)) +
                             16 * c;
        gaddr[k] = P.src.data[plane] + fbase + row * P.src.pitch[plane] + boff;
        srow[k] = row;
        sok[k] = (i < J.nload) && (boff + 16 <= P.src.pitch[plane]);
        sofs[k] = inter_chroma ? row * swb + 8 * c : (plane - pln) * plane_stage + row * swb + 16 * c;
    }
    const int64_t rowstep = (int64_t)kBlkRows * pitch;

    uint4 pre[kMaxLoads];
    auto issue = [&](int b) {
#pragma unroll
        for (int k = 0; k < kMaxLoads; ++k) {
            pre[k] = make_uint4(0, 0, 0, 0);
            if (sok[k] && b * kBlkRows + srow[k] < srcH) {
                const u32x4 v = *GPTR(g_cu32x4, gaddr[k] + b * rowstep);
                pre[k] = make_uint4(v.x, v.y, v.z, v.w);
            }
        }
    };
    auto commit = [&](uint8_t *stage) {
#pragma unroll
        for (int k = 0; k < kMaxLoads; ++k) {
            if (t + k * kThreads >= J.nload) continue;
            uint4 v = pre[k];
            if (!inter_chroma) {
                if (SRC == kSrcP010) {
                    v.x = (v.x >> 6) & 0x03ff03ffu;
                    v.y = (v.y >> 6) & 0x03ff03ffu;
                    v.z = (v.z >> 6) & 0x03ff03ffu;
                    v.w = (v.w >> 6) & 0x03ff03ffu;
                } else {
                    v.x ^= 0x80808080u;
                    v.y ^= 0x80808080u;
                    v.z ^= 0x80808080u;
                    v.w ^= 0x80808080u;
                }
                *reinterpret_cast<uint4 *>(stage + sofs[k]) = v;
            } else if (SRC == kSrcNV12) {
                uint2 u, w;
                u.x = perm(v.y, v.x, 0x06040200u) ^ 0x80808080u;
                u.y = perm(v.w, v.z, 0x06040200u) ^ 0x80808080u;
                w.x = perm(v.y, v.x, 0x07050301u) ^ 0x80808080u;
                w.y = perm(v.w, v.z, 0x07050301u) ^ 0x80808080u;
                *reinterpret_cast<uint2 *>(stage + sofs[k]) = u;
                *reinterpret_cast<uint2 *>(stage + plane_stage + sofs[k]) = w;
            } else { // p010 interleaved UV: dword = U16 | V16 << 16
                uint2 u, w;
                u.x = (perm(v.y, v.x, 0x05040100u) >> 6) & 0x03ff03ffu;
                u.y = (perm(v.w, v.z, 0x05040100u) >> 6) & 0x03ff03ffu;
                w.x = (perm(v.y, v.x, 0x07060302u) >> 6) & 0x03ff03ffu;
                w.y = (perm(v.w, v.z, 0x07060302u) >> 6) & 0x03ff03ffu;
                *reinterpret_cast<uint2 *>(stage + sofs[k]) = u;
                *reinterpret_cast<uint2 *>(stage + plane_stage + sofs[k]) = w;
            }
        }
    };

    // ---- horizontal lane: one output column, coefficients in registers ----
    const int hplane = kind ? (t >> 7) : 0;
    const int hcol = kind ? (t & (kChromaCols - 1)) : t;
    const bool hact = hcol < J.ncols;
    const int hx = J.x0 + (hact ? hcol : 0);
    const int nd = K.nd;
    uint32_t chv[NDMAX], clv[NDMAX];
    int bias = 0, lofs = 0;
    {
        const int p = GPTR(g_ci32, K.hpos)[hx];
        bias = SRC == kSrcP010 ? 0 : GPTR(g_ci32, K.hbias)[hx];
        lofs = hplane * plane_stage + (p - J.sx0) * (SRC == kSrcP010 ? 2 : 1);
#pragma unroll
        for (int k = 0; k < NDMAX; ++k) {
            chv[k] = k < nd ? GPTR(g_cu32, K.hch)[(int64_t)k * K.dstW + hx] : 0u;
            clv[k] = (SRC != kSrcP010 && k < nd) ? GPTR(g_cu32, K.hcl)[(int64_t)k * K.dstW + hx] : 0u;
        }
    }

    auto hpass = [&](int b, const uint8_t *stage) {
        if (!hact) return;
#if DTS_ABLATE & 1      // diagnostic builds only: skip the H arithmetic
        {
#pragma unroll
            for (int pr = 0; pr < kBlkRows / 2; ++pr)
                ring[(hplane * RP + ((b * (kBlkRows / 2) + pr) & (RP - 1))) * pcols + hcol] = (uint32_t)b;
            return;
        }
#endif
        uint32_t hp[kBlkRows / 2];
        const uint8_t *s = stage + lofs;
        switch (nd) {                                        // wave-uniform
#define DTS_HCASE(N)                                                           \
    case N:                                                                    \
        if (N <= NDMAX) hrows<SRC, (N <= NDMAX ? N : 1), NDMAX>(s, swb, chv, clv, bias, hp); \
        break;
            DTS_HCASE(1) DTS_HCASE(2) DTS_HCASE(3) DTS_HCASE(4) DTS_HCASE(5) DTS_HCASE(6) DTS_HCASE(7)
            DTS_HCASE(8) DTS_HCASE(10) DTS_HCASE(12) DTS_HCASE(14) DTS_HCASE(16)
#undef DTS_HCASE
        default:
            break;
        }
#pragma unroll
        for (int pr = 0; pr < kBlkRows / 2; ++pr) {
            const int slot = (b * (kBlkRows / 2) + pr) & (RP - 1);
            ring[(hplane * RP + slot) * pcols + hcol] = hp[pr];
        }
    };

    // ---- vertical: one output row per wave, taps via v_readlane -----------
    const int wave = uniform(t >> 6);
    const int lane = t & 63;
    const int rung = J.rung;
    DevPlanes dst = P.dst[0];
    int dfmt = P.dst_fmt[0];
    if (rung == 1) { dst = P.dst[1]; dfmt = P.dst_fmt[1]; }
    if (rung == 2) { dst = P.dst[2]; dfmt = P.dst_fmt[2]; }
    if (rung == 3) { dst = P.dst[3]; dfmt = P.dst_fmt[3]; }
    const int64_t dbase = (int64_t)frame * dst.fstride;
    const bool hidepth = SRC == kSrcP010;
    const bool d16 = dfmt == DTS_FMT_P010LE;
    const int nv = K.nv;
    const int nvl = lane < nv ? lane : nv - 1;

    auto vrow = [&](int y, int q0, uint32_t cq) {
#if DTS_ABLATE & 2      // diagnostic builds only: skip the V arithmetic and stores
        return;
#endif
        int acc[4];
        if (kind == 0) {
            const int c0 = 4 * lane;
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] = d16 ? 1 << 16 : (hidepth ? c_dither[y & 7][(c0 + i) & 7] : 64) << 12;
            vtaps_any<0>(ring, RP, q0, lane, nv, cq, acc);
            if (d16) {      // output.c yuv2p010lX_c
                const uint64_t row = dst.data[0] + dbase + (int64_t)y * dst.pitch[0] + 2 * J.x0;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (c0 + i < J.ncols) *GPTR(g_u16, row + 2 * (c0 + i)) = clip10s(acc[i]);
                return;
            }
            const uint32_t o = clip8(acc[0]) | (clip8(acc[1]) << 8) | (clip8(acc[2]) << 16) | (clip8(acc[3]) << 24);
            const uint64_t row = dst.data[0] + dbase + (int64_t)y * dst.pitch[0] + J.x0;
            if (c0 + 3 < J.ncols) {
                *GPTR(g_u32, row + c0) = o;
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (c0 + i < J.ncols) *GPTR(g_u8, row + c0 + i) = (uint8_t)(o >> (8 * i));
            }
        } else {
            const int c0 = 2 * lane;
            if (hidepth) {     // vscale.c: U dither offset 0, V offset 3 (x0 is a multiple of 8)
                acc[0] = c_dither[y & 7][(c0) & 7] << 12;
                acc[1] = c_dither[y & 7][(c0 + 1) & 7] << 12;
                acc[2] = c_dither[y & 7][(c0 + 3) & 7] << 12;
                acc[3] = c_dither[y & 7][(c0 + 4) & 7] << 12;
            } else {
                acc[0] = acc[1] = acc[2] = acc[3] = 64 << 12;
            }
            if (d16) acc[0] = acc[1] = acc[2] = acc[3] = 1 << 16;
            vtaps_any<1>(ring, RP, q0, lane, nv, cq, acc);
            if (d16) {      // output.c yuv2p010cX_c: U16,V16 pairs
                const uint64_t row = dst.data[1] + dbase + (int64_t)y * dst.pitch[1] + 4 * J.x0;
                if (c0 < J.ncols) {
                    *GPTR(g_u16, row + 4 * c0) = clip10s(acc[0]);
                    *GPTR(g_u16, row + 4 * c0 + 2) = clip10s(acc[2]);
                }
                if (c0 + 1 < J.ncols) {
                    *GPTR(g_u16, row + 4 * c0 + 4) = clip10s(acc[1]);
                    *GPTR(g_u16, row + 4 * c0 + 6) = clip10s(acc[3]);
                }
                return;
            }
            const uint32_t U0 = clip8(acc[0]), U1 = clip8(acc[1]), V0 = clip8(acc[2]), V1 = clip8(acc[3]);
            if (dfmt == DTS_FMT_NV12) {
                const uint64_t row = dst.data[1] + dbase + (int64_t)y * dst.pitch[1] + 2 * J.x0;
                const uint32_t o = U0 | (V0 << 8) | (U1 << 16) | (V1 << 24);
                if (c0 + 1 < J.ncols)
                    *GPTR(g_u32, row + 2 * c0) = o;
                else if (c0 < J.ncols)
                    *GPTR(g_u16, row + 2 * c0) = (uint16_t)o;
            } else {
                const uint64_t ru = dst.data[1] + dbase + (int64_t)y * dst.pitch[1] + J.x0;
                const uint64_t rv = dst.data[2] + dbase + (int64_t)y * dst.pitch[2] + J.x0;
                if (c0 + 1 < J.ncols) {
                    *GPTR(g_u16, ru + c0) = (uint16_t)(U0 | (U1 << 8));
                    *GPTR(g_u16, rv + c0) = (uint16_t)(V0 | (V1 << 8));
                } else if (c0 < J.ncols) {
                    *GPTR(g_u8, ru + c0) = (uint8_t)U0;
                    *GPTR(g_u8, rv + c0) = (uint8_t)V0;
                }
            }
        }
    };

    // ---- the walk ---------------------------------------------------------
    // step b: commit the rows of step b+1 (loaded during step b-1) to the
    // other stage buffer, issue the rows of step b+2 and the V data of the
    // output rows step b+1 finishes, run H(b), barrier, run V(b) (data
    // fetched during step b-1), barrier.  Every global load has one whole step
    // to land before it is consumed.
    const int nb = K.nblocks;
    g_ci32 *vlim = GPTR(g_ci32, K.vlim);
    g_ci32 *vposg = GPTR(g_ci32, K.vpos);
    g_cu32 *vcg = GPTR(g_cu32, K.vcoef);
    uint32_t cqA[kVPre], cqB[kVPre];
    int qpA[kVPre], qpB[kVPre];
    auto vfetch = [&](int lo, int hi, uint32_t (&cq)[kVPre], int (&qp)[kVPre]) {
#pragma unroll
        for (int i = 0; i < kVPre; ++i) {
            const int y = lo + wave + 4 * i;
            cq[i] = 0;
            qp[i] = 0;
            if (y < hi) {
                cq[i] = vcg[(int64_t)y * nv + nvl];
                qp[i] = vposg[y];
            }
        }
    };
    issue(0);
    commit(stage0);
    if (nb > 1) issue(1);
    int vlo = 0;
    int vhi = uniform(vlim[0]);
    int vhi_next = nb > 1 ? vlim[1] : vhi;
    vfetch(0, vhi, cqA, qpA);
    __syncthreads();
    for (int b = 0; b < nb; ++b) {
        const uint8_t *cur = (b & 1) ? stage1 : stage0;
        uint8_t *nxt = (b & 1) ? stage0 : stage1;
        const int vhn = uniform(vhi_next);
        if (b + 1 < nb) {
            commit(nxt);
            if (b + 2 < nb) {
                issue(b + 2);
                vhi_next = vlim[b + 2];
            }
            vfetch(vhi, vhn, cqB, qpB);
        }
        hpass(b, cur);
        __syncthreads();
        for (int y = vlo + wave, i = 0; y < vhi; y += 4, ++i) {   // one call site keeps the code small
            int q;
            uint32_t cq;
            if (i < kVPre) {
                q = i == 0 ? qpA[0] : i == 1 ? qpA[1] : i == 2 ? qpA[2] : qpA[3];
                cq = i == 0 ? cqA[0] : i == 1 ? cqA[1] : i == 2 ? cqA[2] : cqA[3];
            } else {                                                // rare: > kVPre rows per wave (upscaling)
                q = vposg[y];
                cq = vcg[(int64_t)y * nv + nvl];
            }
            vrow(y, uniform(q) >> 1, cq);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kVPre; ++i) {
            cqA[i] = cqB[i];
            qpA[i] = qpB[i];
        }
        vlo = vhi;
        vhi = vhn;
    }
}

// Persistent workgroups pull (frame, strip) items from a device counter:
// frame-major so the renditions of a frame run together (source re-reads
// hit L2 / MALL), heaviest strips first within a frame (short tail).
template <int SRC, int NDMAX>
__global__ void __launch_bounds__(kThreads) k_ladder(const LadderParams P)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t *slot = reinterpret_cast<uint32_t *>(smem + 2 * P.stage_bytes);   // ring word 0, free between items
    for (;;) {
        if (threadIdx.x == 0) *slot = atomicAdd(P.queue, 1u);
        __syncthreads();
        const int item = uniform((int)*slot);
        __syncthreads();
        if (item >= P.nitems) return;
        ladder_item<SRC, NDMAX>(P, item / P.njobs, item % P.njobs, smem);
        __syncthreads();
    }
}

int ladder_ndmax_for(int nd)
{
    static const int buckets[] = {4, 8, 16};
    for (int b : buckets)
        if (nd <= b) return b;
    return 0;
}

template <int SRC, int N>
static hipError_t launch_one(const LadderParams &p, int grid, int lds, hipStream_t s)
{
    hipLaunchKernelGGL((k_ladder<SRC, N>), dim3((unsigned)grid), dim3(kThreads), lds, s, p);
    return hipGetLastError();
}

template <int SRC>
static hipError_t launch_ladder_src(const LadderParams &p, int ndmax, int lds, int grid, hipStream_t s)
{
    switch (ndmax) {
    case 4: return launch_one<SRC, 4>(p, grid, lds, s);
    case 8: return launch_one<SRC, 8>(p, grid, lds, s);
    case 16: return launch_one<SRC, 16>(p, grid, lds, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_ladder(const LadderParams &p, int ndmax, int lds_bytes, int grid, hipStream_t s)
{
    switch (p.src_kind) {
    case kSrcPlanar8: return launch_ladder_src<kSrcPlanar8>(p, ndmax, lds_bytes, grid, s);
    case kSrcNV12: return launch_ladder_src<kSrcNV12>(p, ndmax, lds_bytes, grid, s);
    case kSrcP010: return launch_ladder_src<kSrcP010>(p, ndmax, lds_bytes, grid, s);
    default: return hipErrorInvalidValue;
    }
}

template <int SRC, int N>
static int occ_one(int lds)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void *>(&k_ladder<SRC, N>), kThreads,
                                                     (size_t)lds) != hipSuccess)
        return 0;
    return n;
}

template <int SRC>
static int occ_src(int ndmax, int lds)
{
    switch (ndmax) {
    case 4: return occ_one<SRC, 4>(lds);
    case 8: return occ_one<SRC, 8>(lds);
    case 16: return occ_one<SRC, 16>(lds);
    default: return 0;
    }
}

int ladder_blocks_per_cu(int src_kind, int ndmax, int lds_bytes)
{
    switch (src_kind) {
    case kSrcPlanar8: return occ_src<kSrcPlanar8>(ndmax, lds_bytes);
    case kSrcNV12: return occ_src<kSrcNV12>(ndmax, lds_bytes);
    case kSrcP010: return occ_src<kSrcP010>(ndmax, lds_bytes);
    default: return 0;
    }
}

// ---------------------------------------------------------------------------
// k_quality: vf_psnr + vf_ssim partials.  One workgroup per (frame, plane, walk):
// a column strip of TBX 4x4 blocks (64; nv12 chroma 32 -- 256 bytes of a row either
// way) walked down kQWalk tiles of 16 block rows.  Per tile a thread owns one item: 4
// (nv12 chroma 2) blocks of one block row, loaded as one 16-byte segment per pixel row
// and image a tile ahead of their use; the blocks' sums (s1, s2, ss, s12) go to a
// circular LDS image of 17 block rows (the previous tile's last row is carried, never
// re-read); each owned block adds ss - 2*s12 = sum((a-b)^2) to the SSE; each 8x8
// window (2x2 blocks at stride 4) whose top block row lies in the walk evaluates
// ssim_end1 in f32 exactly as vf_ssim.c and accumulates in f64.  The strip's right
// apron column and the walk's bottom apron row are read once.  Pixels outside whole
// blocks (plane width/height not multiples of 4) add to the SSE directly.  An nv12
// chroma workgroup scores U and V from one read of the interleaved rows (two block
// images side by side in LDS; its partials go to the tile of plane 1 and of plane 2).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float ssim_end1(int s1, int s2, int ss, int s12)
{
    const int c1 = (int)(.01 * .01 * 255 * 255 * 64 + .5);
    const int c2 = (int)(.03 * .03 * 255 * 255 * 64 * 63 + .5);
    const int vars = ss * 64 - s1 * s1 - s2 * s2;
    const int covar = s12 * 64 - s1 * s2;
    return (float)(2 * s1 * s2 + c1) * (float)(2 * covar + c2) /
           ((float)(s1 * s1 + s2 * s2 + c1) * (float)(vars + c2));
}

__device__ __forceinline__ uint32_t load4(const uint8_t *row, int x, bool inter, int comp)
{
    if (!inter) return *reinterpret_cast<const uint32_t *>(row + x);
    const uint2 v = *reinterpret_cast<const uint2 *>(row + 2 * x);
    return perm(v.y, v.x, comp ? 0x07050301u : 0x06040200u);
}

__device__ __forceinline__ int load1(const uint8_t *row, int x, bool inter, int comp)
{
    return inter ? row[2 * x + comp] : row[x];
}

__device__ __forceinline__ int4 sums4(const uint32_t (&va)[4], const uint32_t (&vb)[4])
{
    uint32_t s1 = 0, s2 = 0, ss = 0, s12 = 0;
#pragma unroll
    for (int yy = 0; yy < 4; ++yy) {
        s1 = __builtin_amdgcn_udot4(va[yy], 0x01010101u, s1, false);
        s2 = __builtin_amdgcn_udot4(vb[yy], 0x01010101u, s2, false);
        ss = __builtin_amdgcn_udot4(va[yy], va[yy], ss, false);
        ss = __builtin_amdgcn_udot4(vb[yy], vb[yy], ss, false);
        s12 = __builtin_amdgcn_udot4(va[yy], vb[yy], s12, false);
    }
    return make_int4((int)s1, (int)s2, (int)ss, (int)s12);
}

#ifndef DTS_BOUNDS_CHECK
// 1 (diagnostic builds, tools/build_qvar.sh): every k_quality global access is checked against the
// scored plane's rows and row bytes; an access outside is skipped and poisons the tile's partials
// (SSE all ones, SSIM NaN), so a parity test fails on it instead of the GPU faulting
#define DTS_BOUNDS_CHECK 0
#endif
#ifndef DTS_BCHK_SHRINK
#define DTS_BCHK_SHRINK 0   // > 0: the check's row bytes shrunk (a negative control: the tests must fail)
#endif

#ifndef DTS_Q_PREFETCH
#define DTS_Q_PREFETCH 1    // 0: a tile's rows loaded when the tile starts (fewer VGPRs; A/B knob)
#endif

// INTER: nv12 chroma workgroups (tiles of plane 1 scoring U and V); else one plane each
template <bool INTER>
__global__ void __launch_bounds__(kThreads) k_quality(const QualityParams P, int gt0, int ngt)
{
    constexpr int RB = kQTileBY + 1;                // circular block rows: the carried row + one tile
    constexpr int BW = kQTileBX + 2;                // columns: TBX + 1 (nv12 chroma: 2 x (TBX + 1))
    __shared__ int4 bs[RB + 1][BW];                 // + the walk's apron row below (row RB)
    __shared__ double red_s[2][kThreads / 64];
    __shared__ unsigned long long red_e[2][kThreads / 64];
    const int t = threadIdx.x;
    const int total = P.tile_base[3];
    // XCD-aware order (round 5): workgroup b runs on XCD b % 8, and item e = (b % 8) per + b / 8
    // gives each XCD a contiguous run of (frame, tile) items, so a strip's neighbours run beside it
    // on the same L2 and its apron column (the first block of the next strip: a 128-byte line per
    // row read for 4 bytes) is an L2 hit rather than a third line fetched per 256-byte strip row
    const int nitems = P.nframes * ngt, per = (nitems + 7) >> 3;
    const int e = ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);
    if (e >= nitems) return;
    const int frame = e / ngt;
    const int gt = gt0 + e % ngt;
    const int plane = gt >= P.tile_base[2] ? 2 : (gt >= P.tile_base[1] ? 1 : 0);
    const int tile = gt - P.tile_base[plane];
    const int tx = tile % P.tiles_x[plane], tw = tile / P.tiles_x[plane];
    const int w = P.pw[plane], h = P.ph[plane];
    const int W4 = w >> 2, H4 = h >> 2;
    const int TBX = P.tbx[plane];
    const int bx0 = tx * TBX;
    constexpr bool inter = INTER;
    constexpr int NC = INTER ? 2 : 1;               // components scored: U and V of nv12 chroma
    const int dp = inter ? 1 : plane;
    const uint8_t *A = reinterpret_cast<const uint8_t *>(P.a.data[dp]) + (int64_t)frame * P.a.fstride;
    const uint8_t *B = reinterpret_cast<const uint8_t *>(P.b.data[dp]) + (int64_t)frame * P.b.fstride;
    const int64_t pa = P.a.pitch[dp], pb = P.b.pitch[dp];
    const bool vec16 = (((uintptr_t)A | (uintptr_t)B | (uint64_t)pa | (uint64_t)pb) & 15) == 0;
    constexpr int NB = INTER ? 2 : 4;               // blocks per item: 16 bytes of an image row
    const int iby = t >> 4, iq = t & 15;            // item: blocks NB iq .. NB iq + NB - 1 of block row iby
    const int by00 = tw * P.walk[plane] * kQTileBY; // first block row of the walk
    const int nk = min(P.walk[plane], (h - 4 * by00 + 4 * kQTileBY - 1) / (4 * kQTileBY));

    unsigned long long sse[2] = {0, 0};
    double ssim[2] = {0.0, 0.0};
    bool oob = false;                               // DTS_BOUNDS_CHECK: an access outside the plane
    const int rowb = (inter ? 2 * w : w) - DTS_BCHK_SHRINK;   // bytes of a scored row
    auto outside = [&](int y, int xb, int nb) {
        if (!DTS_BOUNDS_CHECK) return false;
        const bool o = y < 0 || y >= h || xb < 0 || xb + nb > rowb;
        oob |= o;
        return o;
    };
    // one block by 4-byte loads (edges, the apron column, unaligned planes); zero outside
    auto block = [&](int gx, int gy, int comp) {
        if (gx >= W4 || gy >= H4 || gx < 0) return make_int4(0, 0, 0, 0);
        uint32_t va[4], vb[4];
#pragma unroll
        for (int yy = 0; yy < 4; ++yy) {
            if (outside(4 * gy + yy, (inter ? 2 : 1) * 4 * gx, inter ? 8 : 4)) return make_int4(0, 0, 0, 0);
            va[yy] = load4(A + (int64_t)(4 * gy + yy) * pa, 4 * gx, inter, comp);
            vb[yy] = load4(B + (int64_t)(4 * gy + yy) * pb, 4 * gx, inter, comp);
        }
        return sums4(va, vb);
    };
    // the item's 4 pixel rows, both images, one 16-byte load each (when the item is whole)
    uint4 ra[4], rb[4];
    auto fetch = [&](int by0) {
        const int gx = bx0 + NB * iq, gy = by0 + iby;
        if (vec16 && gy < H4 && gx + NB <= W4) {
#pragma unroll
            for (int yy = 0; yy < 4; ++yy) {
                if (outside(4 * gy + yy, 4 * (inter ? 2 : 1) * gx, 16)) continue;
                ra[yy] = *reinterpret_cast<const uint4 *>(A + (int64_t)(4 * gy + yy) * pa + 4 * (inter ? 2 : 1) * gx);
                rb[yy] = *reinterpret_cast<const uint4 *>(B + (int64_t)(4 * gy + yy) * pb + 4 * (inter ? 2 : 1) * gx);
            }
        }
    };
    // the item's block sums into LDS row `row` (+ SSE of blocks inside the plane); slot
    // k of 4: block NB iq + (k mod NB) of component k / NB (nv12 chroma: U U V V)
    auto put = [&](int by0, int row) {
        const int gx = bx0 + NB * iq, gy = by0 + iby;
        if (vec16 && gy < H4 && gx + NB <= W4) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int c = inter ? k >> 1 : 0, kb = inter ? k & 1 : k;
                const uint32_t sel = c ? 0x07050301u : 0x06040200u;
                uint32_t va[4], vb[4];
#pragma unroll
                for (int yy = 0; yy < 4; ++yy) {
                    if (inter) {
                        va[yy] = perm(kb ? ra[yy].w : ra[yy].y, kb ? ra[yy].z : ra[yy].x, sel);
                        vb[yy] = perm(kb ? rb[yy].w : rb[yy].y, kb ? rb[yy].z : rb[yy].x, sel);
                    } else {
                        va[yy] = k == 0 ? ra[yy].x : k == 1 ? ra[yy].y : k == 2 ? ra[yy].z : ra[yy].w;
                        vb[yy] = k == 0 ? rb[yy].x : k == 1 ? rb[yy].y : k == 2 ? rb[yy].z : rb[yy].w;
                    }
                }
                const int4 r = sums4(va, vb);
                bs[row][c * (TBX + 1) + NB * iq + kb] = r;
                sse[c] += (unsigned long long)(r.z - 2 * r.w);
            }
        } else {
#pragma unroll 1
            for (int k = 0; k < 4; ++k) {
                const int c = inter ? k >> 1 : 0, kb = inter ? k & 1 : k;
                const int4 r = block(gx + kb, gy, c + (plane == 2));
                bs[row][c * (TBX + 1) + NB * iq + kb] = r;
                if (gx + kb < W4 && gy < H4) sse[c] += (unsigned long long)(r.z - 2 * r.w);
            }
        }
    };
    // pixels outside whole blocks, inside the tile's pixel rectangle
    auto strips = [&](int py0) {
        const int px0 = 4 * bx0;
        const int px1 = min(w, px0 + 4 * TBX), py1 = min(h, py0 + 4 * kQTileBY);
        const int ax0 = max(px0, 4 * W4), ay1 = min(py1, 4 * H4);     // right strip: x >= 4 W4, y < 4 H4
        const int aw = max(0, px1 - ax0), ah = max(0, ay1 - py0);
        for (int i = t; i < aw * ah; i += kThreads) {
            const int y = py0 + i / aw, x = ax0 + i % aw;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                if (outside(y, inter ? 2 * x + c + (plane == 2) : x, 1)) continue;
                const int d = load1(A + (int64_t)y * pa, x, inter, c + (plane == 2)) -
                              load1(B + (int64_t)y * pb, x, inter, c + (plane == 2));
                sse[c] += (unsigned long long)(d * d);
            }
        }
        const int by0p = max(py0, 4 * H4);                             // bottom strip: y >= 4 H4
        const int bw = max(0, px1 - px0), bh = max(0, py1 - by0p);
        for (int i = t; i < bw * bh; i += kThreads) {
            const int y = by0p + i / bw, x = px0 + i % bw;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                if (outside(y, inter ? 2 * x + c + (plane == 2) : x, 1)) continue;
                const int d = load1(A + (int64_t)y * pa, x, inter, c + (plane == 2)) -
                              load1(B + (int64_t)y * pb, x, inter, c + (plane == 2));
                sse[c] += (unsigned long long)(d * d);
            }
        }
    };
    // windows with top rows r0 .. r1 - 1 of the circular image (base b: top block row by0 - 1 + r)
    auto windows = [&](int by0, int b, int r0, int r1, bool apron_row) {
        const int rw = NC * TBX, nw = (r1 - r0) * rw;
#pragma unroll 1
        for (int i = t; i < nw; i += kThreads) {
            const int r = r0 + i / rw, cx = i % rw, c = cx >= TBX, wx = cx - c * TBX;
            if (bx0 + wx < W4 - 1 && by0 - 1 + r < H4 - 1) {
                const int l0 = (b + r) % RB, l1 = apron_row ? RB : (b + r + 1) % RB, x = c * (TBX + 1) + wx;
                const int4 p = bs[l0][x], q = bs[l0][x + 1], u = bs[l1][x], v = bs[l1][x + 1];
                const double e = (double)ssim_end1(p.x + q.x + u.x + v.x, p.y + q.y + u.y + v.y,
                                                   p.z + q.z + u.z + v.z, p.w + q.w + u.w + v.w);
                if (NC == 1) {
                    ssim[0] += e;
                } else {
                    ssim[0] += c ? 0.0 : e;
                    ssim[1] += c ? e : 0.0;
                }
            }
        }
    };
    if (DTS_Q_PREFETCH) fetch(by00);
    int b = 0;                                      // circular base: the carried row
    for (int k = 0; k < nk; ++k) {
        const int by0 = by00 + k * kQTileBY;
        if (!DTS_Q_PREFETCH) fetch(by0);
        if (k) __syncthreads();                     // the previous windows are done with the rows
        put(by0, (b + 1 + iby) % RB);
        if (t < NC * kQTileBY) {                    // the apron column: block TBX of block row t
            const int c = t >= kQTileBY, r = t - c * kQTileBY;
            bs[(b + 1 + r) % RB][c * (TBX + 1) + TBX] = block(bx0 + TBX, by0 + r, c + (plane == 2));
        }
        strips(4 * by0);
        __syncthreads();
        if (DTS_Q_PREFETCH && k + 1 < nk) fetch(by0 + kQTileBY);   // the next tile's rows fly during the windows
        windows(by0, b, k ? 0 : 1, kQTileBY, false);
        b = (b + kQTileBY) % RB;                    // this tile's last row is the next tile's carried row
    }
    {   // the apron row below the walk: windows with top row at the walk's last block row
        const int by0 = by00 + nk * kQTileBY;       // (b now holds that row)
        if (by0 < H4) {
            __syncthreads();
            for (int i = t; i < NC * (TBX + 1); i += kThreads) {
                const int c = i > TBX, x = i - c * (TBX + 1);
                bs[RB][i] = block(bx0 + x, by0, c + (plane == 2));
            }
            __syncthreads();
            windows(by0, b, 0, 1, true);    // top block row by0 - 1 (held at b), bottom by0 (row RB)
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            ssim[c] += __shfl_xor(ssim[c], o);
            sse[c] += __shfl_xor(sse[c], o);
        }
        if ((t & 63) == 0) {
            red_s[c][t >> 6] = ssim[c];
            red_e[c][t >> 6] = sse[c];
        }
    }
    const bool poison = DTS_BOUNDS_CHECK && __syncthreads_or(oob);
    if (!DTS_BOUNDS_CHECK) __syncthreads();
    if (t < NC) {
        double s = 0;
        unsigned long long e = 0;
        for (int i = 0; i < kThreads / 64; ++i) {
            s += red_s[t][i];
            e += red_e[t][i];
        }
        const int g = gt + t * (P.tile_base[2] - P.tile_base[1]);      // V: the same tile of plane 2
        if (DTS_BOUNDS_CHECK && (g < 0 || g >= total || frame >= P.nframes)) return;
        P.partial_ssim[(int64_t)frame * total + g] = poison ? __builtin_nan("") : s;
        P.partial_sse[(int64_t)frame * total + g] = poison ? ~0ull : e;
    }
}

// one workgroup per (frame, plane); fixed-order tree reduction
__global__ void __launch_bounds__(kThreads) k_qreduce(const QualityParams P)
{
    __shared__ double rs[kThreads];
    __shared__ unsigned long long re[kThreads];
    const int frame = blockIdx.x / 3, plane = blockIdx.x % 3, t = threadIdx.x;
    const int total = P.tile_base[3];
    const int lo = P.tile_base[plane], hi = P.tile_base[plane + 1];
    double s = 0;
    unsigned long long e = 0;
    for (int i = lo + t; i < hi; i += kThreads) {
        s += P.partial_ssim[(int64_t)frame * total + i];
        e += P.partial_sse[(int64_t)frame * total + i];
    }
    rs[t] = s;
    re[t] = e;
    __syncthreads();
    for (int o = kThreads / 2; o > 0; o >>= 1) {
        if (t < o) {
            rs[t] += rs[t + o];
            re[t] += re[t + o];
        }
        __syncthreads();
    }
    if (t == 0) {
        P.out[frame].sse[plane] = re[0];
        P.out[frame].ssim_sum[plane] = rs[0];
    }
}

// One segment's record: the n per-frame records summed (u64 SSE exact; the f64 SSIM
// window sums in a fixed order: thread t takes frames t, t + kThreads, ... in order,
// then the tree; the same n always gives the same bits).  One workgroup per record
// field: 3 SSE + 3 SSIM sums.  vf_psnr / vf_ssim keep exactly these running sums
// across a stream (uninit: mse_comp / nb_frames, ssim / nb_frames).
__global__ void __launch_bounds__(kThreads) k_qsum(const dts_qraw *raw, int n, dts_qraw *sum)
{
    __shared__ double rs[kThreads];
    __shared__ unsigned long long re[kThreads];
    const int c = blockIdx.x % 3, t = threadIdx.x;
    const bool ssim = blockIdx.x >= 3;
    double s = 0;
    unsigned long long e = 0;
    for (int i = t; i < n; i += kThreads) {
        if (ssim)
            s += raw[i].ssim_sum[c];
        else
            e += raw[i].sse[c];
    }
    rs[t] = s;
    re[t] = e;
    __syncthreads();
    for (int o = kThreads / 2; o > 0; o >>= 1) {
        if (t < o) {
            rs[t] += rs[t + o];
            re[t] += re[t + o];
        }
        __syncthreads();
    }
    if (t == 0) {
        if (ssim)
            sum->ssim_sum[c] = rs[0];
        else
            sum->sse[c] = re[0];
    }
}

hipError_t launch_qsum(const dts_qraw *raw, int n, dts_qraw *sum, hipStream_t s)
{
    hipLaunchKernelGGL(k_qsum, dim3(6), dim3(kThreads), 0, s, raw, n, sum);
    return hipGetLastError();
}

hipError_t launch_quality(const QualityParams &p, int total_tiles, hipStream_t s)
{
    auto grid = [&](int ngt) { return dim3((unsigned)(8 * ((ngt * p.nframes + 7) / 8))); };   // (k_quality: XCD order)
    if (!p.interleaved) {
        hipLaunchKernelGGL(k_quality<false>, grid(total_tiles), dim3(kThreads), 0, s, p, 0, total_tiles);
    } else {                                        // nv12: plane 1's workgroups score plane 2 as well
        const int nl = p.tile_base[1], nc = p.tile_base[2] - p.tile_base[1];
        hipLaunchKernelGGL(k_quality<false>, grid(nl), dim3(kThreads), 0, s, p, 0, nl);
        if (nc > 0 && hipPeekAtLastError() == hipSuccess)
            hipLaunchKernelGGL(k_quality<true>, grid(nc), dim3(kThreads), 0, s, p, nl, nc);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_qreduce, dim3((unsigned)(3 * p.nframes)), dim3(kThreads), 0, s, p);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// k_synth: one thread per 4 samples of one plane row
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) k_synth(int w, int h, int fmt, int pattern, uint32_t seed,
                                                    int64_t first, DevPlanes dst, int quads_y, int quads_c)
{
    const int64_t frame = blockIdx.y;
    const int64_t f = first + frame;
    const int cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    int64_t q = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const bool ten = fmt == DTS_FMT_P010LE;
    uint8_t *base0 = reinterpret_cast<uint8_t *>(dst.data[0]) + frame * dst.fstride;
    if (q < quads_y) {
        const int qw = (w + 3) >> 2;
        const int y = (int)(q / qw), x0 = (int)(q % qw) * 4;
        uint8_t *row = base0 + (int64_t)y * dst.pitch[0];
        for (int i = 0; i < 4 && x0 + i < w; ++i) {
            const int v = synth_sample(pattern, seed, x0 + i, y, f, 0, w, h, ten);
            if (ten) {
                const int s = v << 6;
                row[2 * (x0 + i)] = (uint8_t)s;
                row[2 * (x0 + i) + 1] = (uint8_t)(s >> 8);
            } else {
                row[x0 + i] = (uint8_t)v;
            }
        }
        return;
    }
    q -= quads_y;
    if (q >= quads_c) return;
    const int qw = (cw + 3) >> 2;
    const int y = (int)(q / qw), x0 = (int)(q % qw) * 4;
    for (int i = 0; i < 4 && x0 + i < cw; ++i) {
        const int x = x0 + i;
        const int u = synth_sample(pattern, seed, x, y, f, 1, cw, ch, ten);
        const int v = synth_sample(pattern, seed, x, y, f, 2, cw, ch, ten);
        if (fmt == DTS_FMT_YUV420P) {
            reinterpret_cast<uint8_t *>(dst.data[1])[frame * dst.fstride + (int64_t)y * dst.pitch[1] + x] = (uint8_t)u;
            reinterpret_cast<uint8_t *>(dst.data[2])[frame * dst.fstride + (int64_t)y * dst.pitch[2] + x] = (uint8_t)v;
        } else if (fmt == DTS_FMT_NV12) {
            uint8_t *row = reinterpret_cast<uint8_t *>(dst.data[1]) + frame * dst.fstride + (int64_t)y * dst.pitch[1];
            row[2 * x] = (uint8_t)u;
            row[2 * x + 1] = (uint8_t)v;
        } else {
            uint8_t *row = reinterpret_cast<uint8_t *>(dst.data[1]) + frame * dst.fstride + (int64_t)y * dst.pitch[1];
            const int su = u << 6, sv = v << 6;
            row[4 * x] = (uint8_t)su;
            row[4 * x + 1] = (uint8_t)(su >> 8);
            row[4 * x + 2] = (uint8_t)sv;
            row[4 * x + 3] = (uint8_t)(sv >> 8);
        }
    }
}

hipError_t launch_synth(int w, int h, int fmt, int pattern, uint32_t seed, int64_t first, const DevPlanes &dst,
                        int nframes, hipStream_t s)
{
    const int cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    const int quads_y = ((w + 3) >> 2) * h;
    const int quads_c = ((cw + 3) >> 2) * ch;
    const int blocks = (quads_y + quads_c + kThreads - 1) / kThreads;
    hipLaunchKernelGGL(k_synth, dim3((unsigned)blocks, (unsigned)nframes), dim3(kThreads), 0, s, w, h, fmt, pattern,
                       seed, first, dst, quads_y, quads_c);
    return hipGetLastError();
}

} // namespace dts
