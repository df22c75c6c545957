// ladder5.hip -- k_ladder5, the v5 ladder kernel: every rendition of an
// 8-bit 4:2:0 source in one persistent launch, both FIR passes on the
// matrix cores (v_mfma_i32_16x16x64_i8).
//
// Same arithmetic as libswscale hScale8To15_c -> yuv2planeX_8_c /
// yuv2nv12cX_c under SWS_BITEXACT|SWS_ACCURATE_RND (FFmpeg 4.4; bit-exact,
// DESIGN.md "Oracle"), organised for CDNA4:
//
//  * one work item = (frame, plane kind, column strip): a strip of the luma
//    plane, or the same columns of both chroma planes, for ALL renditions,
//    walked top to bottom in steps of 16 source rows.  Each step's rows are
//    staged once in LDS (src ^ 0x80, i.e. the sample - 128 as i8) and read by
//    every rendition, so the source is fetched from HBM once per frame;
//  * H: a 16-output tile of one rendition over 16 source rows is one MFMA per
//    64-column K block and tap half: the int16 taps c = 256 hi + lo (signed
//    bytes) are the B operands (held in VGPRs for the whole walk), the staged
//    rows the A operand, so sum(src * c) = 256 sum(src' hi) + sum(src' lo) +
//    128 * 16384 exactly in i32; FFMIN(val >> 7, 32767) (v_cvt_pk_i16_i32),
//    and the int16 result y goes to the rendition's ring as two column-major
//    byte planes, y >> 8 and (y & 255) ^ 0x80;
//  * V: 16 output rows x 16 columns of a rendition are out^T = H^T C^T: the
//    ring bytes (A: 16 columns x 64 source rows) times the V taps split the
//    same way (B: 64 source rows x 16 output rows), four MFMAs per K block,
//      sum(c y) = 65536 hh + 256 (hl + lh) + ll + 128 * 4096,
//    then + 64 << 12 (flat dither), v_ashr_pk_u8_i32 (>> 19, clip to u8): each
//    lane holds 4 consecutive columns of one row, one dword store (nv12
//    chroma: U and V interleaved, 8 bytes);
//  * one barrier per step: H(b+1) of one wave overlaps V(b) of another (the
//    planner sizes each ring so their rows never meet).
#include "dts_internal.h"

#ifndef DTS_L5_ABLATE
#define DTS_L5_ABLATE 0     // diagnostic builds only: 1 skip H, 2 skip V, 4 skip source loads, 8 skip V stores,
                            // 16 skip the H epilogue (MFMAs kept)
#endif

#ifndef DTS_L5_STAMP
#define DTS_L5_STAMP 0      // diagnostic builds only: per-phase s_memtime sums (tools/stamp5.py)
#endif

namespace dts {

#if DTS_L5_STAMP
// [phase]: cycles summed over every wave and step; [15]: steps
__device__ unsigned long long g_l5_stamp[16];
#define L5_STAMP(k)                                                        \
    do {                                                                   \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();        \
        st_acc[k] += t_ - st_last;                                         \
        st_last = t_;                                                      \
    } while (0)
#else
#define L5_STAMP(k) (void)0
#endif

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef short short2v __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(4))) const uint32_t k_u32;
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) uint16_t g_u16;
typedef __attribute__((address_space(1))) uint8_t g_u8;
#define GP5(T, p) ((T *)(uintptr_t)(p))

__device__ __forceinline__ int uni5(int v) { return __builtin_amdgcn_readfirstlane(v); }


// wave-uniform struct / field read through the constant address space (s_load)
template <class T>
__device__ __forceinline__ T kld(const T *p)
{
    static_assert(sizeof(T) % 4 == 0, "dword data only");
    struct W { uint32_t w[sizeof(T) / 4]; } w;
    k_u32 *q = GP5(k_u32, p);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) w.w[i] = q[i];
    return __builtin_bit_cast(T, w);
}

// LDS access by byte address (the addresses below are computed as integers)
__device__ __forceinline__ u32x2 lds_rd64(const uint32_t *lds, uint32_t byte)
{
    return *reinterpret_cast<const u32x2 *>(reinterpret_cast<const uint8_t *>(lds) + byte);
}
__device__ __forceinline__ uint32_t *lds_at(uint32_t *lds, uint32_t byte)
{
    return reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(lds) + byte);
}

__device__ __forceinline__ uint32_t pack_h(int hi, int lo, int hi2, int lo2)
{
    // FFMIN(((256 hi + lo) >> 7), 32767) of two rows, as int16x2 (even row low)
    const int a = ((hi << 8) + lo) >> 7, b = ((hi2 << 8) + lo2) >> 7;
    return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(a, b));
}

struct Walk5 {
    int nplanes, nsteps, srcH, Pb, stage_b;
    int L, cpr, ne;
    int lane, wave, t;
};

// This thread's staging loads of a step: kL5MaxLoads 16-B source chunks.
struct Loads5 {
    __amdgpu_buffer_rsrc_t rs[2];   // load planes (planar chroma: U, V)
    uint32_t pitch[2];
    uint32_t col[kL5MaxLoads];      // byte offset of the chunk in its source row
    int row[kL5MaxLoads];           // staged row (0..15), -1 = no chunk
    uint32_t dst[kL5MaxLoads];      // LDS byte offset of the chunk in stage buffer 0
    int nlp;                        // load planes
};

__device__ __forceinline__ void issue_loads(const Loads5 &ld, int b, const Walk5 &W, u32x4 (&pre)[kL5MaxLoads])
{
    if (b >= W.nsteps || (DTS_L5_ABLATE & 4)) return;
#pragma unroll
    for (int k = 0; k < kL5MaxLoads; ++k) {
        const int lp = ld.nlp == 2 ? (k >> 1) : 0;
        if (ld.row[k] >= 0) {
            const int r = min(kL5Rows * b + ld.row[k], W.srcH - 1);
            const uint32_t off = (uint32_t)r * ld.pitch[lp] + ld.col[k];
            pre[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(lp ? ld.rs[1] : ld.rs[0], off, 0, 0));
        }
    }
}

// prefetched chunks -> stage buffer (b & 1), as src ^ 0x80 (nv12 chroma: de-interleaved into U, V)
template <int SRC>
__device__ __forceinline__ void store_stage(uint32_t *lds, const Loads5 &ld, int b, const Walk5 &W,
                                            const u32x4 (&pre)[kL5MaxLoads], bool nv12c)
{
    const uint32_t boff = (uint32_t)((b & 1) * W.nplanes * kL5Rows * W.Pb);
#pragma unroll
    for (int k = 0; k < kL5MaxLoads; ++k) {
        if (ld.row[k] < 0) continue;
        const u32x4 v = pre[k];
        if (SRC == kSrcNV12 && nv12c) {
            const uint32_t u0 = __builtin_amdgcn_perm(v.y, v.x, 0x06040200u) ^ 0x80808080u;
            const uint32_t u1 = __builtin_amdgcn_perm(v.w, v.z, 0x06040200u) ^ 0x80808080u;
            const uint32_t v0 = __builtin_amdgcn_perm(v.y, v.x, 0x07050301u) ^ 0x80808080u;
            const uint32_t v1 = __builtin_amdgcn_perm(v.w, v.z, 0x07050301u) ^ 0x80808080u;
            *reinterpret_cast<u32x2 *>(lds_at(lds, ld.dst[k] + boff)) = (u32x2){u0, u1};
            *reinterpret_cast<u32x2 *>(lds_at(lds, ld.dst[k] + boff + kL5Rows * W.Pb)) = (u32x2){v0, v1};
        } else {
            *reinterpret_cast<u32x4 *>(lds_at(lds, ld.dst[k] + boff)) = v ^ 0x80808080u;
        }
    }
}

// H(b) of this wave: NE entries (K blocks), straight-line -- every A read, then
// every MFMA, then the epilogues -- so the reads and the matrix pipe overlap.
// A K block continuing a tile adds the previous block's sums (the lo MFMAs all
// start at the bias: the continuation subtracts the extra one).  An epilogue
// writes 4 rows of one column: their y >> 8 and (y & 255) ^ 0x80 bytes.
template <int I0, int NE>
__device__ __forceinline__ void hpart(uint32_t *lds, const v4i (&bh)[kL5Ent], const v4i (&bl)[kL5Ent],
                                      const uint32_t (&aad)[kL5Ent], const uint32_t (&whi)[kL5Ent],
                                      const uint32_t (&wlo)[kL5Ent], const uint32_t (&pos)[kL5Ent], uint32_t fl,
                                      uint32_t boff, v4i &ch, v4i &cl)
{
    const v4i zero = {0, 0, 0, 0}, bias = {kL5Bias, kL5Bias, kL5Bias, kL5Bias};
    v4i a[NE], ah[NE], al[NE];
#pragma unroll
    for (int i = 0; i < NE; ++i) {
        const u32x2 x = lds_rd64(lds, aad[I0 + i] + boff), y = lds_rd64(lds, aad[I0 + i] + boff + 32);
        a[i] = __builtin_bit_cast(v4i, (u32x4){x.x, x.y, y.x, y.y});
    }
    __builtin_amdgcn_sched_barrier(0);                     // every A read in flight before the first MFMA
#pragma unroll
    for (int i = 0; i < NE; ++i) {
        ah[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], bh[I0 + i], zero, 0, 0, 0);
        al[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], bl[I0 + i], bias, 0, 0, 0);
    }
    if (DTS_L5_ABLATE & 16) {
#pragma unroll
        for (int i = 0; i < NE; ++i) asm volatile("" ::"v"(ah[i]), "v"(al[i]));
        return;
    }
#pragma unroll
    for (int i = 0; i < NE; ++i) {
        const uint32_t f = (fl >> (2 * (I0 + i))) & 3u;
        if (!(f & 1u)) {                                   // continues the previous K block's tile
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                ah[i][r] += ch[r];
                al[i][r] = al[i][r] + cl[r] - kL5Bias;
            }
        }
        if (f & 2u) {
            const uint32_t p0 = pack_h(ah[i].x, al[i].x, ah[i].y, al[i].y);    // rows 4g, 4g+1
            const uint32_t p1 = pack_h(ah[i].z, al[i].z, ah[i].w, al[i].w);    // rows 4g+2, 4g+3
            *lds_at(lds, whi[I0 + i] + pos[I0 + i]) = __builtin_amdgcn_perm(p1, p0, 0x07050301u);
            *lds_at(lds, wlo[I0 + i] + pos[I0 + i]) = __builtin_amdgcn_perm(p1, p0, 0x06040200u) ^ 0x80808080u;
        } else {
            ch = ah[i];
            cl = al[i];
        }
    }
}

// H(b) of this wave: NE entries (K blocks) in halves of up to 4 -- every A read
// of a half, then its MFMAs, then its epilogues -- so the reads and the matrix
// pipe overlap.  A K block continuing a tile adds the previous block's sums
// (the lo MFMAs all start at the bias: the continuation subtracts the extra
// one).  An epilogue writes 4 rows of one column: their y >> 8 and
// (y & 255) ^ 0x80 bytes.
template <int NE>
__device__ __forceinline__ void hstep(uint32_t *lds, const v4i (&bh)[kL5Ent], const v4i (&bl)[kL5Ent],
                                      const uint32_t (&aad)[kL5Ent], const uint32_t (&whi)[kL5Ent],
                                      const uint32_t (&wlo)[kL5Ent], const uint32_t (&pos)[kL5Ent], uint32_t fl,
                                      uint32_t boff)
{
    v4i ch = {0, 0, 0, 0}, cl = {0, 0, 0, 0};
    hpart<0, (NE < 4 ? NE : 4)>(lds, bh, bl, aad, whi, wlo, pos, fl, boff, ch, cl);
    if (NE > 4) hpart<4, (NE > 4 ? NE - 4 : 1)>(lds, bh, bl, aad, whi, wlo, pos, fl, boff, ch, cl);
}

// V of one (row group, 16-column tile, plane): 4 MFMAs per K block, then the
// 4 output bytes (columns 4g..4g+3 of output row lane & 15) packed in a dword
__device__ __forceinline__ uint32_t vtile(const uint32_t *lds, const Ring5 &g, int col, int w0m, int nkb,
                                          const v4i (&vh)[kL5MaxVkb], const v4i (&vl)[kL5MaxVkb], int lane)
{
    const v4i zero = {0, 0, 0, 0}, vbias = {kL5VBias, kL5VBias, kL5VBias, kL5VBias};
    v4i hh = zero, hl = zero, ll = vbias;
    const uint32_t cb = (uint32_t)(col * g.CP);
    const int rr = g.RR;
#pragma unroll
    for (int kb = 0; kb < kL5MaxVkb; ++kb) {
        if (kb < nkb) {
            int r0 = w0m + 64 * kb + 8 * (lane >> 4), r1 = r0 + 32;
            r0 = r0 >= rr ? r0 - rr : r0;
            r1 = r1 >= rr ? r1 - rr : r1;
            const u32x2 h0 = lds_rd64(lds, (uint32_t)g.hi + cb + (uint32_t)r0);
            const u32x2 h1 = lds_rd64(lds, (uint32_t)g.hi + cb + (uint32_t)r1);
            const u32x2 l0 = lds_rd64(lds, (uint32_t)g.lo + cb + (uint32_t)r0);
            const u32x2 l1 = lds_rd64(lds, (uint32_t)g.lo + cb + (uint32_t)r1);
            const v4i ahi = __builtin_bit_cast(v4i, (u32x4){h0.x, h0.y, h1.x, h1.y});
            const v4i alo = __builtin_bit_cast(v4i, (u32x4){l0.x, l0.y, l1.x, l1.y});
            hh = __builtin_amdgcn_mfma_i32_16x16x64_i8(ahi, vh[kb], hh, 0, 0, 0);
            hl = __builtin_amdgcn_mfma_i32_16x16x64_i8(ahi, vl[kb], hl, 0, 0, 0);
            hl = __builtin_amdgcn_mfma_i32_16x16x64_i8(alo, vh[kb], hl, 0, 0, 0);
            ll = __builtin_amdgcn_mfma_i32_16x16x64_i8(alo, vl[kb], ll, 0, 0, 0);
        }
    }
    int v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (((hh[i] << 8) + hl[i]) << 8) + ll[i];
    // av_clip_uint8(val >> 19) of 4 columns, packed
    const uint32_t lo = __builtin_amdgcn_ashr_pk_u8_i32(v[0], v[1], 19);
    const uint32_t hi = __builtin_amdgcn_ashr_pk_u8_i32(v[2], v[3], 19);
    return (lo & 0xffffu) | (hi << 16);
}

// One output store of 4 bytes at byte column x of a row (fewer at the plane's right edge).
__device__ __forceinline__ void store4(uint64_t row, int x, int ncols, uint32_t w)
{
    if (DTS_L5_ABLATE & 8) {
        asm volatile("" ::"v"(w));
        return;
    }
    if (ncols >= 4) {
        *GP5(g_u32, row + x) = w;
    } else {
        for (int i = 0; i < ncols; ++i) GP5(g_u8, row + x)[i] = (uint8_t)(w >> (8 * i));
    }
}

// V work of one step, fetched before the barrier it runs after: the fragments
// of its first row group (their latency hides under the barrier wait)
struct VPrep5 {
    int e0, e1;
    v4i vh[kL5MaxVkb], vl[kL5MaxVkb];
};

__device__ __forceinline__ void vfrags(const uint32_t *bf, int frag, int nkb, int lane, v4i (&vh)[kL5MaxVkb],
                                       v4i (&vl)[kL5MaxVkb])
{
    const u32x4 *f = reinterpret_cast<const u32x4 *>(bf + (size_t)frag * 512);
    vh[0] = __builtin_bit_cast(v4i, f[lane]);
    vl[0] = __builtin_bit_cast(v4i, f[64 + lane]);
    vh[1] = vl[1] = (v4i){0, 0, 0, 0};
    if (nkb > 1) {
        vh[1] = __builtin_bit_cast(v4i, f[128 + lane]);
        vl[1] = __builtin_bit_cast(v4i, f[192 + lane]);
    }
}

// Kernel arguments are read through the kernarg segment pointer with scalar
// loads: indexing the by-value parameter with a runtime rendition or plane
// makes the compiler copy it to scratch.
__device__ __forceinline__ const Ladder5Params *kargs()
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (const Ladder5Params *)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
#else
    return nullptr;
#endif
}

// Per-item rendition table (LDS bytes 16..): wave r < nrungs fills rendition r's
// 16 dwords {x0, nct, pitch Y/U/V, 0, plane base lo/hi Y/U/V of this frame, 0...}
__device__ __forceinline__ void rung_table(uint32_t *lds, const Strip5 *S, int nrungs, int frame, const Walk5 &W)
{
    const int r = W.wave;
    if (r >= nrungs || W.lane >= 16) return;
    const DevPlanes d = kld(&kargs()->dst[r]);
    const uint64_t fb = (uint64_t)frame * d.fstride;
    const uint64_t b0 = d.data[0] + fb, b1 = d.data[1] + fb, b2 = d.data[2] + fb;
    const int k = W.lane;
    uint32_t v = 0;
    v = k == 0 ? (uint32_t)kld(&S->x0[r]) : v;
    v = k == 1 ? (uint32_t)kld(&S->nct[r]) : v;
    v = k == 2 ? (uint32_t)d.pitch[0] : v;
    v = k == 3 ? (uint32_t)d.pitch[1] : v;
    v = k == 4 ? (uint32_t)d.pitch[2] : v;
    v = k == 6 ? (uint32_t)b0 : v;
    v = k == 7 ? (uint32_t)(b0 >> 32) : v;
    v = k == 8 ? (uint32_t)b1 : v;
    v = k == 9 ? (uint32_t)(b1 >> 32) : v;
    v = k == 10 ? (uint32_t)b2 : v;
    v = k == 11 ? (uint32_t)(b2 >> 32) : v;
    lds[4 + 16 * r + k] = v;
}

// V of one row group: its 16-column tiles dealt round robin over the 4 waves
// (pitches and plane bases of this frame from the rendition table)
__device__ __forceinline__ void vgroup(const uint32_t *lds, const Walk5 &W, const VEnt5 &VE, const v4i (&vh)[kL5MaxVkb],
                                       const v4i (&vl)[kL5MaxVkb], int first, int nct, int x0, uint32_t pY,
                                       uint32_t pU, uint32_t pV, uint64_t bY, uint64_t bU, uint64_t bV)
{
    const int n = W.lane & 15, g = W.lane >> 4;
    const int y = 16 * VE.G + n;
    const bool rowok = n < VE.rows;
    if (W.nplanes == 1) {
        const uint64_t orow = bY + (uint64_t)y * pY;
        for (int ct = first; ct < nct; ct += 4) {
            const uint32_t w = vtile(lds, VE.ring0, 16 * ct + n, VE.w0, VE.nkb, vh, vl, W.lane);
            const int x = x0 + 16 * ct + 4 * g;
            if (rowok) store4(orow, x, VE.dstW - x, w);
        }
    } else {
        const Ring5 g1 = {VE.hi1, VE.lo1, VE.ring0.CP, VE.ring0.RR};
        const bool nv = VE.fmt == DTS_FMT_NV12;
        const uint64_t urow = bU + (uint64_t)y * pU;
        const uint64_t vrow = bV + (uint64_t)y * pV;
        for (int ct = first; ct < nct; ct += 4) {
            const uint32_t wu = vtile(lds, VE.ring0, 16 * ct + n, VE.w0, VE.nkb, vh, vl, W.lane);
            const uint32_t wv = vtile(lds, g1, 16 * ct + n, VE.w0, VE.nkb, vh, vl, W.lane);
            const int x = x0 + 16 * ct + 4 * g;
            if (!rowok) continue;
            if (!nv) {
                store4(urow, x, VE.dstW - x, wu);
                store4(vrow, x, VE.dstW - x, wv);
            } else {
                // yuv2nv12cX: U0 V0 U1 V1 U2 V2 U3 V3
                const uint32_t q0 = __builtin_amdgcn_perm(wv, wu, 0x05010400u);
                const uint32_t q1 = __builtin_amdgcn_perm(wv, wu, 0x07030602u);
                store4(urow, 2 * x, 2 * (VE.dstW - x), q0);
                store4(urow, 2 * x + 4, 2 * (VE.dstW - x) - 4, q1);
            }
        }
    }
}

// V of a step for this wave; the first group's fragments came from vprep
__device__ __forceinline__ void vrun(const uint32_t *lds, const Kind5 *K, const Walk5 &W, const uint32_t *bf,
                                     VPrep5 &V)
{
    int rot = 0;
    for (int e = V.e0; e < V.e1; ++e) {
        const VEnt5 VE = kld(K->vsched + e);
        const uint32_t *tb = lds + 4 + 16 * VE.rung;
        const u32x4 t0 = *reinterpret_cast<const u32x4 *>(tb);        // x0, nct, pitch Y, pitch U
        const u32x4 t1 = *reinterpret_cast<const u32x4 *>(tb + 4);    // pitch V, 0, base Y
        const u32x4 t2 = *reinterpret_cast<const u32x4 *>(tb + 8);    // base U, base V
        const int nct = uni5((int)t0.y);
        const int first = (W.wave - rot) & 3;
        rot += nct;
        if (first >= nct) continue;
        if (e != V.e0) vfrags(bf, VE.bfrag, VE.nkb, W.lane, V.vh, V.vl);
        auto u64 = [](uint32_t lo, uint32_t hi) {
            return ((uint64_t)(uint32_t)uni5((int)hi) << 32) | (uint32_t)uni5((int)lo);
        };
        vgroup(lds, W, VE, V.vh, V.vl, first, nct, uni5((int)t0.x), (uint32_t)uni5((int)t0.z),
               (uint32_t)uni5((int)t0.w), (uint32_t)uni5((int)t1.x), u64(t1.z, t1.w), u64(t2.x, t2.y),
               u64(t2.z, t2.w));
    }
}

template <int SRC>
__device__ __forceinline__ void run5(const Ladder5Params &P, int frame, const Job5 &J, uint32_t *lds)
{
    const Kind5 *K = P.kinds + J.kind;
    Walk5 W;
    W.t = threadIdx.x;
    W.lane = W.t & 63;
    W.wave = uni5(W.t >> 6);
    W.nplanes = kld(&K->nplanes);
    W.nsteps = kld(&K->nsteps);
    W.srcH = kld(&K->srcH);
    W.Pb = kld(&K->P);
    W.stage_b = kld(&K->stage);
    const Strip5 *S = kld(&K->strips) + J.strip;
    W.L = kld(&S->L);
    W.cpr = kld(&S->cpr);
    W.ne = kld(&S->nent[W.wave]);
    const Ent5 *ents = kld(&K->ents) + kld(&S->ent0[W.wave]);
    const uint32_t *bf = kld(&K->bfrag);
    const bool chroma = W.nplanes == 2;
    const bool nv12c = SRC == kSrcNV12 && chroma;

    // ---- this wave's H entries: B fragments in VGPRs, per-lane LDS addresses ----
    const int g = W.lane >> 4, n = W.lane & 15;
    v4i bh[kL5Ent], bl[kL5Ent];
    uint32_t aad[kL5Ent], whi[kL5Ent], wlo[kL5Ent], pos[kL5Ent], rr[kL5Ent];
    uint32_t fl = 0;
#pragma unroll
    for (int i = 0; i < kL5Ent; ++i) {
        bh[i] = bl[i] = (v4i){0, 0, 0, 0};
        aad[i] = whi[i] = wlo[i] = pos[i] = 0;
        rr[i] = 16;
        if (i < W.ne) {
            const Ent5 E = kld(ents + i);
            const u32x4 *f = reinterpret_cast<const u32x4 *>(bf + (size_t)E.bfrag * 512);
            bh[i] = __builtin_bit_cast(v4i, f[W.lane]);
            bl[i] = __builtin_bit_cast(v4i, f[64 + W.lane]);
            aad[i] = (uint32_t)(W.stage_b + E.plane * kL5Rows * W.Pb + n * W.Pb + E.soff + 8 * g);
            const Ring5 rg = kld(K->ring + E.ring);
            const uint32_t cb = (uint32_t)((E.col0 + n) * rg.CP + 4 * g);
            whi[i] = (uint32_t)rg.hi + cb;
            wlo[i] = (uint32_t)rg.lo + cb;
            rr[i] = (uint32_t)rg.RR;
            fl |= (uint32_t)(E.flags & 3) << (2 * i);
        }
    }
    fl = (uint32_t)uni5((int)fl);
    // ring row of each entry's step: kept in VGPRs (the SGPRs are the scarce file here)
#pragma unroll
    for (int i = 0; i < kL5Ent; ++i) {
        asm volatile("v_mov_b32 %0, %1" : "=v"(pos[i]) : "v"(pos[i]));
        asm volatile("v_mov_b32 %0, %1" : "=v"(rr[i]) : "v"(rr[i]));
    }
    // make the B fragments resident here: otherwise the compiler's wait for them sits
    // inside the step loop, where it would also drain every prefetch load each step
#pragma unroll
    for (int i = 0; i < kL5Ent; ++i) asm volatile("" ::"v"(bh[i]), "v"(bl[i]));

    // ---- this thread's staging loads ----
    Loads5 ld;
    {
        const int nlp = (SRC == kSrcPlanar8 && chroma) ? 2 : 1;
        ld.nlp = nlp;
        const int bps = nv12c ? 2 : 1;
        for (int lp = 0; lp < 2; ++lp) {
            const int spl = chroma ? (nv12c ? 1 : 1 + lp) : 0;           // source plane
            const int sp = lp < nlp ? spl : 0;
            const uint64_t base = kld(&kargs()->src.data[sp]) + (uint64_t)frame * kld(&kargs()->src.fstride);
            const int64_t pitch = kld(&kargs()->src.pitch[sp]);
            const uint32_t lo = (uint32_t)uni5((int)(uint32_t)base), hi = (uint32_t)uni5((int)(uint32_t)(base >> 32));
            ld.rs[lp] = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), 0,
                                                          uni5((int)(pitch * W.srcH)), 0x00020000);
            ld.pitch[lp] = (uint32_t)pitch;
        }
        const int per = kL5Rows * W.cpr;                                  // chunks per load plane
        const float rc = 1.0f / (float)W.cpr;
#pragma unroll
        for (int k = 0; k < kL5MaxLoads; ++k) {
            const int lp = nlp == 2 ? (k >> 1) : 0;
            const int c = W.t + 256 * (nlp == 2 ? (k & 1) : k);
            ld.row[k] = -1;
            ld.col[k] = 0;
            ld.dst[k] = 0;
            if (c < per) {
                const int row = (int)(((float)c + 0.5f) * rc), cc = c - row * W.cpr;
                ld.row[k] = row;
                ld.col[k] = (uint32_t)(W.L * bps + 16 * cc);
                ld.dst[k] = (uint32_t)(W.stage_b + lp * kL5Rows * W.Pb + row * W.Pb + (nv12c ? 8 : 16) * cc);
            }
        }
    }

    rung_table(lds, S, kld(&K->nrungs), frame, W);

    // ---- prologue: block 0 -> stage 0; block 1 in flight ----
    u32x4 pre[kL5MaxLoads];
#pragma unroll
    for (int k = 0; k < kL5MaxLoads; ++k) pre[k] = (u32x4){0, 0, 0, 0};
    issue_loads(ld, 0, W, pre);
    store_stage<SRC>(lds, ld, 0, W, pre, nv12c);
    issue_loads(ld, 1, W, pre);
    __syncthreads();

    // iteration b (after barrier b - 1: stage b written, H(b - 1) done): V(b - 1), whose
    // fragments were fetched before the barrier; H(b); stage block b + 1 and issue the
    // loads of b + 2 (the wait for the previous loads comes after H(b), so it does not
    // wait on V's stores, which count in the same vmcnt); fetch V(b)'s fragments (its
    // step record came one iteration earlier); barrier b.  V(b - 1) reads rows H(b) may
    // be writing elsewhere in the ring: the planner's RR keeps them apart.
    VPrep5 V;
    V.e0 = V.e1 = 0;
    int4 vs = kld(kld(&K->vstep));                          // step 0's record
#if DTS_L5_STAMP
    unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_last = __builtin_amdgcn_s_memtime();
#endif
    for (int b = 0; b <= W.nsteps; ++b) {
        if (b > 0 && !(DTS_L5_ABLATE & 2)) vrun(lds, K, W, bf, V);
        L5_STAMP(0);
        if (b == W.nsteps) break;
        {
            const uint32_t boff = (uint32_t)((b & 1) * W.nplanes * kL5Rows * W.Pb);
            switch ((DTS_L5_ABLATE & 1) ? 0 : W.ne) {
#define DTS_H5(k) \
    case k: hstep<k>(lds, bh, bl, aad, whi, wlo, pos, fl, boff); break;
                DTS_H5(1) DTS_H5(2) DTS_H5(3) DTS_H5(4) DTS_H5(5) DTS_H5(6) DTS_H5(7) DTS_H5(8)
#undef DTS_H5
            default:
                break;
            }
#pragma unroll
            for (int i = 0; i < kL5Ent; ++i) {                 // next step's rows: ring row (16 b) % RR
                const uint32_t np = pos[i] + 16;
                pos[i] = np >= rr[i] ? 0 : np;
            }
        }
        L5_STAMP(1);
        if (b + 1 < W.nsteps) store_stage<SRC>(lds, ld, b + 1, W, pre, nv12c);
        L5_STAMP(2);
        issue_loads(ld, b + 2, W, pre);
        L5_STAMP(3);
        if (!(DTS_L5_ABLATE & 2)) {
            V.e0 = vs.x;
            V.e1 = vs.y;
            if (vs.x < vs.y) vfrags(bf, vs.z, vs.w, W.lane, V.vh, V.vl);
            vs = kld(kld(&K->vstep) + b + 1);
        }
        L5_STAMP(4);
        __syncthreads();
        L5_STAMP(5);
    }
#if DTS_L5_STAMP
    if (W.lane == 0) {
        for (int k = 0; k < 6; ++k) atomicAdd(&g_l5_stamp[k], st_acc[k]);
        atomicAdd(&g_l5_stamp[15], (unsigned long long)W.nsteps);
    }
#endif
}

} // namespace

// Persistent workgroups pull (frame, item) pairs from one counter per XCD
// (workgroup b serves queue b % nq, which holds the frames f = x mod nq), so
// every strip of a frame -- and the source halos neighbouring strips share --
// stays in one XCD's L2.
template <int SRC>
__global__ void __launch_bounds__(256, 2) k_ladder5(const Ladder5Params P)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    volatile int *slot = reinterpret_cast<volatile int *>(lds);
    for (;;) {
        const int x = P.nq > 1 ? (int)(blockIdx.x % (unsigned)P.nq) : 0;
        if (threadIdx.x == 0) *slot = (int)atomicAdd(P.queue + x, 1u);
        __syncthreads();
        const int item = uni5(*slot);
        __syncthreads();
        const int nf = (P.nframes - x + P.nq - 1) / P.nq;
        if (item >= nf * P.njobs) return;
        const int fq = item / P.njobs, jid = item - fq * P.njobs;
        const Job5 J = kld(P.jobs + jid);
        run5<SRC>(P, x + P.nq * fq, J, lds);
    }
}

template <int SRC>
static int occ5(int lds)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void *>(&k_ladder5<SRC>), 256,
                                                     (size_t)lds) != hipSuccess)
        return 0;
    return n;
}

hipError_t launch_ladder5(const Ladder5Params &p, int src_kind, int lds_bytes, int grid, hipStream_t s)
{
    switch (src_kind) {
    case kSrcPlanar8:
        hipLaunchKernelGGL(k_ladder5<kSrcPlanar8>, dim3((unsigned)grid), dim3(256), lds_bytes, s, p);
        break;
    case kSrcNV12:
        hipLaunchKernelGGL(k_ladder5<kSrcNV12>, dim3((unsigned)grid), dim3(256), lds_bytes, s, p);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

#if DTS_L5_STAMP
int ladder5_stamps(unsigned long long *out, bool reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_l5_stamp), sizeof(g_l5_stamp)) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_l5_stamp), z, sizeof z) != hipSuccess) return -1;
    }
    return 16;
}
#endif

int ladder5_blocks_per_cu(int src_kind, int lds_bytes)
{
    switch (src_kind) {
    case kSrcPlanar8: return occ5<kSrcPlanar8>(lds_bytes);
    case kSrcNV12: return occ5<kSrcNV12>(lds_bytes);
    default: return 0;
    }
}

} // namespace dts
