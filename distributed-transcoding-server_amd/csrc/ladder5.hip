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
#define DTS_L5_ABLATE 0     // diagnostic builds only: 1 skip H, 2 skip V, 4 skip every DMA, 8 skip V stores,
                            // 16 skip the H epilogue (MFMAs kept), 32 skip the source DMA (fragments kept)
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
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
typedef __attribute__((address_space(1))) u32x2 g_u32x2;
typedef __attribute__((address_space(1))) uint16_t g_u16;
typedef __attribute__((address_space(1))) uint8_t g_u8;
#define GP5(T, p) ((T *)(uintptr_t)(p))

__device__ __forceinline__ int uni5(int v) { return __builtin_amdgcn_readfirstlane(v); }

// V works two tiles at once (two independent MFMA chains) when the register budget
// allows it: 2 waves per SIMD (256 VGPRs), not 4 (128)
constexpr bool kL5VPair = kL5Waves <= 8;


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
    int nplanes, nsteps, srcH, stage, SB, FA, FB;
    int L, cpr, Pb, PS, nsi, ne;
    int vrank;                      // V tile order: the waves with fewer H entries first
    int lane, wave, t;
};

// This item's LDS-DMA sources: buffer descriptors (SGPRs) of the load planes and
// of the fragment table
struct Dma5 {
    u32x4 rs[2];                    // load planes (planar chroma: U, V)
    u32x4 rf;                       // B fragment pairs (V fragments in step order)
    uint32_t pitch[2];
    uint32_t colb;                  // byte column of the strip's first staged sample
    float rc;                       // 1 / cpr
    int ipp;                        // DMA instructions per load plane (PS / 1 KB)
};

__device__ __forceinline__ u32x4 rsrc5(uint64_t base, uint32_t bytes)
{
    u32x4 r;
    r.x = (uint32_t)uni5((int)(uint32_t)base);
    r.y = (uint32_t)uni5((int)(uint32_t)(base >> 32));      // stride 0
    r.z = (uint32_t)uni5((int)bytes);                        // num_records: offsets past it read 0
    r.w = 0x00020000u;
    return r;
}

// One LDS-DMA instruction: 64 lanes x 16 B from voff (per lane) to LDS m0 + 16 lane.
// M0 is the compiler's: saved and restored inside the statement.
__device__ __forceinline__ void dma16(const u32x4 &rs, uint32_t voff, uint32_t m0)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(rs), "s"(m0)
                 : "memory");
}

// Bundle s -> stage buffer s % kL5Stages: the 16 source rows of step s, as stored
// (row-major, pitch Pb, load plane p at p * PS).  Instruction i of the bundle is
// issued by wave i % kL5Waves; returns how many this wave issued (its vmcnt share).
__device__ __forceinline__ int issue_bundle(const Walk5 &W, const Dma5 &D, int s)
{
    if (DTS_L5_ABLATE & (4 | 32)) return 0;
    const uint32_t buf = (uint32_t)(W.stage + (s % kL5Stages) * W.SB);
    int m = 0;
    for (int i = W.wave; i < W.nsi; i += kL5Waves, ++m) {
        const int p = i >= D.ipp ? 1 : 0;
        const int ii = i - p * D.ipp;
        const int c = 64 * ii + W.lane;
        const int row = (int)(((float)c + 0.5f) * D.rc), cc = c - row * W.cpr;
        const int r = min(kL5StepRows * s + row, W.srcH - 1);
        const uint32_t off = (uint32_t)r * (p ? D.pitch[1] : D.pitch[0]) + D.colb + 16u * (uint32_t)cc;
        dma16(p ? D.rs[1] : D.rs[0], row < kL5StepRows ? off : 0x80000000u,
              buf + (uint32_t)(p * W.PS) + 1024u * (uint32_t)ii);
    }
    return m;
}

// V(b)'s fragments (nfu 1 KB units from fragment pair vf0 on, one contiguous run)
// -> fragment buffer b % kL5FragBufs, dealt over the waves after the source
// instructions; returns how many this wave issued
__device__ __forceinline__ int issue_frags(const Walk5 &W, const Dma5 &D, int b, int vf0, int nfu)
{
    if (DTS_L5_ABLATE & 4) return 0;
    const uint32_t buf = (uint32_t)(W.FA + (b % kL5FragBufs) * W.FB);
    int m = 0;
    for (int j = (W.wave - W.nsi % kL5Waves + kL5Waves) % kL5Waves; j < nfu; j += kL5Waves, ++m)
        dma16(D.rf, (uint32_t)vf0 * 2048u + 1024u * (uint32_t)j + 16u * (uint32_t)W.lane, buf + 1024u * (uint32_t)j);
    return m;
}

// End of a step: every load of this wave except its m youngest memory operations (the
// bundle it issued this step and the V stores after it) has landed, the ring writes
// too; then the barrier.  A raw barrier:
// __syncthreads() would also wait for the DMAs still in flight.
__device__ __forceinline__ void step_wait(int m)
{
#define DTS_W5(k) \
    case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
#define DTS_W5x8(k) DTS_W5(k) DTS_W5(k + 1) DTS_W5(k + 2) DTS_W5(k + 3) DTS_W5(k + 4) DTS_W5(k + 5) DTS_W5(k + 6) DTS_W5(k + 7)
    switch (m < 63 ? m : 63) {                 // fewer than issued: waits longer, never shorter
        DTS_W5x8(0) DTS_W5x8(8) DTS_W5x8(16) DTS_W5x8(24) DTS_W5x8(32) DTS_W5x8(40) DTS_W5x8(48)
        DTS_W5(56) DTS_W5(57) DTS_W5(58) DTS_W5(59) DTS_W5(60) DTS_W5(61) DTS_W5(62) DTS_W5(63)
    default:
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        break;
    }
#undef DTS_W5x8
#undef DTS_W5
}

__device__ __forceinline__ void step_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ u32x4 lds_rd128(const uint32_t *lds, uint32_t byte)
{
    return *reinterpret_cast<const u32x4 *>(reinterpret_cast<const uint8_t *>(lds) + byte);
}

// H(b) of this wave: NE entries, straight-line -- every A read, then every MFMA,
// then the epilogues -- so the reads and the matrix pipe overlap.  An entry is
// 16 (8, 4) outputs over one 64-column K block; its epilogue writes 4 rows of one
// column per lane: their y >> 8 and (y & 255) ^ 0x80 bytes (lanes past the
// entry's outputs hold an out-of-range LDS address: their writes are dropped).
// Per-entry constants (wave-uniform, SGPRs) and the lane's part of the addresses
struct HEnt5 {
    uint32_t ao[kL5Ent];            // stage offset of the entry's K block (+ lane part abase)
    uint32_t hb[kL5Ent];            // ring hi byte plane + col0 * CP
    uint32_t dl[kL5Ent];            // lo - hi byte plane offset
    uint32_t cp[kL5Ent];            // ring column pitch
    uint32_t no[kL5Ent];            // outputs (16, 8, 4): lanes n >= no write nowhere
    uint32_t pos[kL5Ent];           // ring row of this step (16 b % RR)
    uint32_t rr[kL5Ent];
};

// ring write address of entry i for this lane: column col0 + n, rows 4g..4g+3 of row
// block BLK of this step
template <int BLK>
__device__ __forceinline__ uint32_t hwaddr(const HEnt5 &E, int i, int n, int g)
{
    uint32_t p = E.pos[i] + (uint32_t)(kL5Rows * BLK);
    p = p >= E.rr[i] ? p - E.rr[i] : p;
    const uint32_t a = E.hb[i] + (uint32_t)n * E.cp[i] + 4u * (uint32_t)g + p;
    return (uint32_t)n < E.no[i] ? a : 0x40000000u;        // out of range: the write is dropped
}

template <int I0, int NE, bool ILV, int BLK>
__device__ __forceinline__ void hpart(uint32_t *lds, const v4i (&bh)[kL5Ent], const v4i (&bl)[kL5Ent],
                                      const HEnt5 &E, uint32_t abase, int n, int g, uint32_t odd, uint32_t boff)
{
    const v4i zero = {0, 0, 0, 0}, bias = {kL5Bias, kL5Bias, kL5Bias, kL5Bias};
    v4i a[NE], ah[NE], al[NE];
#pragma unroll
    for (int i = 0; i < NE; ++i) {
        if (ILV) {       // nv12 chroma: U V interleaved as stored; even (U) or odd (V) bytes
            const uint32_t ad = abase + E.ao[I0 + i] + boff;
            const u32x4 x = lds_rd128(lds, ad), y = lds_rd128(lds, ad + 64);
            const uint32_t sel = (odd >> (I0 + i)) & 1u ? 0x07050301u : 0x06040200u;
            a[i] = __builtin_bit_cast(v4i, (u32x4){__builtin_amdgcn_perm(x.y, x.x, sel), __builtin_amdgcn_perm(x.w, x.z, sel),
                                                   __builtin_amdgcn_perm(y.y, y.x, sel), __builtin_amdgcn_perm(y.w, y.z, sel)} ^
                                                   0x80808080u);
        } else {
            const uint32_t ad = abase + E.ao[I0 + i] + boff;
            const u32x2 x = lds_rd64(lds, ad), y = lds_rd64(lds, ad + 32);
            a[i] = __builtin_bit_cast(v4i, (u32x4){x.x, x.y, y.x, y.y} ^ 0x80808080u);
        }
    }
    __builtin_amdgcn_sched_barrier(0);                     // every A read in flight before the first MFMA
#pragma unroll
    for (int i = 0; i < NE; ++i) {
        ah[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], bh[I0 + i], zero, 0, 0, 0);
        al[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], bl[I0 + i], bias, 0, 0, 0);
        if (!kL5VPair) {        // 128-VGPR budget: finish each entry before the next one's MFMAs
            const uint32_t p0 = pack_h(ah[i].x, al[i].x, ah[i].y, al[i].y);
            const uint32_t p1 = pack_h(ah[i].z, al[i].z, ah[i].w, al[i].w);
            if (!(DTS_L5_ABLATE & 16)) {
                const uint32_t w = hwaddr<BLK>(E, I0 + i, n, g);
                *lds_at(lds, w) = __builtin_amdgcn_perm(p1, p0, 0x07050301u);
                *lds_at(lds, w + E.dl[I0 + i]) = __builtin_amdgcn_perm(p1, p0, 0x06040200u) ^ 0x80808080u;
            }
        }
    }
    if (!kL5VPair) return;
    if (DTS_L5_ABLATE & 16) {
#pragma unroll
        for (int i = 0; i < NE; ++i) asm volatile("" ::"v"(ah[i]), "v"(al[i]));
        return;
    }
#pragma unroll
    for (int i = 0; i < NE; ++i) {
        const uint32_t p0 = pack_h(ah[i].x, al[i].x, ah[i].y, al[i].y);    // rows 4g, 4g+1
        const uint32_t p1 = pack_h(ah[i].z, al[i].z, ah[i].w, al[i].w);    // rows 4g+2, 4g+3
        const uint32_t w = hwaddr<BLK>(E, I0 + i, n, g);
        *lds_at(lds, w) = __builtin_amdgcn_perm(p1, p0, 0x07050301u);
        *lds_at(lds, w + E.dl[I0 + i]) = __builtin_amdgcn_perm(p1, p0, 0x06040200u) ^ 0x80808080u;
    }
}

// H(b) of this wave in parts of up to 4 entries
template <int NE, bool ILV, int BLK>
__device__ __forceinline__ void hblock(uint32_t *lds, const v4i (&bh)[kL5Ent], const v4i (&bl)[kL5Ent],
                                       const HEnt5 &E, uint32_t abase, int n, int g, uint32_t odd, uint32_t boff)
{
    hpart<0, (NE < 4 ? NE : 4), ILV, BLK>(lds, bh, bl, E, abase, n, g, odd, boff);
    if (NE > 4) hpart<4, (NE > 4 ? NE - 4 : 1), ILV, BLK>(lds, bh, bl, E, abase, n, g, odd, boff);
}

// H of a step: its kL5Blk row blocks (staged kL5Rows rows apart)
template <int NE, bool ILV>
__device__ __forceinline__ void hstep(uint32_t *lds, const v4i (&bh)[kL5Ent], const v4i (&bl)[kL5Ent],
                                      const HEnt5 &E, uint32_t abase, int n, int g, uint32_t odd, uint32_t boff,
                                      uint32_t blkb)
{
    static_assert(kL5Blk == 2, "two row blocks per step");
    hblock<NE, ILV, 0>(lds, bh, bl, E, abase, n, g, odd, boff);
    hblock<NE, ILV, 1>(lds, bh, bl, E, abase, n, g, odd, boff + blkb);
}

// V of two (row group, 16-column tile, plane) tiles at once -- two independent
// chains, so one's LDS reads overlap the other's MFMAs: 4 MFMAs per K block
// each, then the 4 output bytes (columns 4g..4g+3 of output row lane & 15)
// packed in a dword.  hiX / loX: LDS byte address of the tile's first column
// in its hi / lo ring.
__device__ __forceinline__ uint32_t vcombine(const v4i &hh, const v4i &hl, const v4i &ll)
{
    int v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (((hh[i] << 8) + hl[i]) << 8) + ll[i];
    // av_clip_uint8(val >> 19) of 4 columns, packed
    const uint32_t lo = __builtin_amdgcn_ashr_pk_u8_i32(v[0], v[1], 19);
    const uint32_t hi = __builtin_amdgcn_ashr_pk_u8_i32(v[2], v[3], 19);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

template <int NKB>
__device__ __forceinline__ uint32_t vtile1(const uint32_t *lds, uint32_t hiA, uint32_t loA, int w0m, int rr,
                                           const v4i (&vh)[kL5MaxVkb], const v4i (&vl)[kL5MaxVkb], int lane)
{
    const v4i zero = {0, 0, 0, 0}, vbias = {kL5VBias, kL5VBias, kL5VBias, kL5VBias};
    v4i hh = zero, hl = zero, ll = vbias;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
        int r0 = w0m + 64 * kb + 8 * (lane >> 4), r1 = r0 + 32;
        r0 = r0 >= rr ? r0 - rr : r0;
        r1 = r1 >= rr ? r1 - rr : r1;
        const u32x2 h0 = lds_rd64(lds, hiA + (uint32_t)r0), h1 = lds_rd64(lds, hiA + (uint32_t)r1);
        const u32x2 l0 = lds_rd64(lds, loA + (uint32_t)r0), l1 = lds_rd64(lds, loA + (uint32_t)r1);
        const v4i ah = __builtin_bit_cast(v4i, (u32x4){h0.x, h0.y, h1.x, h1.y});
        const v4i al = __builtin_bit_cast(v4i, (u32x4){l0.x, l0.y, l1.x, l1.y});
        hh = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, vh[kb], hh, 0, 0, 0);
        hl = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, vl[kb], hl, 0, 0, 0);
        ll = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, vl[kb], ll, 0, 0, 0);
        hl = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, vh[kb], hl, 0, 0, 0);
    }
    return vcombine(hh, hl, ll);
}

// two tiles as two independent chains (when registers allow: kL5VPair)
template <int NKB>
__device__ __forceinline__ void vtile2(const uint32_t *lds, uint32_t hiA, uint32_t loA, uint32_t hiB, uint32_t loB,
                                       int w0m, int rr, const v4i (&vh)[kL5MaxVkb], const v4i (&vl)[kL5MaxVkb],
                                       int lane, uint32_t &wa, uint32_t &wb)
{
    const v4i zero = {0, 0, 0, 0}, vbias = {kL5VBias, kL5VBias, kL5VBias, kL5VBias};
    v4i hhA = zero, hlA = zero, llA = vbias, hhB = zero, hlB = zero, llB = vbias;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
        int r0 = w0m + 64 * kb + 8 * (lane >> 4), r1 = r0 + 32;
        r0 = r0 >= rr ? r0 - rr : r0;
        r1 = r1 >= rr ? r1 - rr : r1;
        const u32x2 ha0 = lds_rd64(lds, hiA + (uint32_t)r0), ha1 = lds_rd64(lds, hiA + (uint32_t)r1);
        const u32x2 la0 = lds_rd64(lds, loA + (uint32_t)r0), la1 = lds_rd64(lds, loA + (uint32_t)r1);
        const u32x2 hb0 = lds_rd64(lds, hiB + (uint32_t)r0), hb1 = lds_rd64(lds, hiB + (uint32_t)r1);
        const u32x2 lb0 = lds_rd64(lds, loB + (uint32_t)r0), lb1 = lds_rd64(lds, loB + (uint32_t)r1);
        const v4i ahA = __builtin_bit_cast(v4i, (u32x4){ha0.x, ha0.y, ha1.x, ha1.y});
        const v4i alA = __builtin_bit_cast(v4i, (u32x4){la0.x, la0.y, la1.x, la1.y});
        const v4i ahB = __builtin_bit_cast(v4i, (u32x4){hb0.x, hb0.y, hb1.x, hb1.y});
        const v4i alB = __builtin_bit_cast(v4i, (u32x4){lb0.x, lb0.y, lb1.x, lb1.y});
        hhA = __builtin_amdgcn_mfma_i32_16x16x64_i8(ahA, vh[kb], hhA, 0, 0, 0);
        hlA = __builtin_amdgcn_mfma_i32_16x16x64_i8(ahA, vl[kb], hlA, 0, 0, 0);
        llA = __builtin_amdgcn_mfma_i32_16x16x64_i8(alA, vl[kb], llA, 0, 0, 0);
        hhB = __builtin_amdgcn_mfma_i32_16x16x64_i8(ahB, vh[kb], hhB, 0, 0, 0);
        hlB = __builtin_amdgcn_mfma_i32_16x16x64_i8(ahB, vl[kb], hlB, 0, 0, 0);
        llB = __builtin_amdgcn_mfma_i32_16x16x64_i8(alB, vl[kb], llB, 0, 0, 0);
        hlA = __builtin_amdgcn_mfma_i32_16x16x64_i8(alA, vh[kb], hlA, 0, 0, 0);
        hlB = __builtin_amdgcn_mfma_i32_16x16x64_i8(alB, vh[kb], hlB, 0, 0, 0);
    }
    wa = vcombine(hhA, hlA, llA);
    wb = vcombine(hhB, hlB, llB);
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

// V fragments of a row group from its step's fragment area (fb: LDS byte address)
__device__ __forceinline__ void vfrags(const uint32_t *lds, uint32_t fb, int nkb, int lane, v4i (&vh)[kL5MaxVkb],
                                       v4i (&vl)[kL5MaxVkb])
{
    const uint32_t o = fb + 16u * (uint32_t)lane;
    vh[0] = __builtin_bit_cast(v4i, lds_rd128(lds, o));
    vl[0] = __builtin_bit_cast(v4i, lds_rd128(lds, o + 1024));
    vh[1] = vl[1] = (v4i){0, 0, 0, 0};
    if (nkb > 1) {
        vh[1] = __builtin_bit_cast(v4i, lds_rd128(lds, o + 2048));
        vl[1] = __builtin_bit_cast(v4i, lds_rd128(lds, o + 3072));
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

// V of one row group: its 16-column tiles dealt round robin over the waves,
// two tiles per vtile2 (luma: tiles ct and ct + W; chroma: U and V of tile ct)
// (pitches and plane bases of this frame from the rendition table)
template <int NKB>
__device__ __forceinline__ void vgroup(const uint32_t *lds, const Walk5 &W, const VEnt5 &VE, const v4i (&vh)[kL5MaxVkb],
                                       const v4i (&vl)[kL5MaxVkb], int first, int nct, int x0, uint32_t pY,
                                       uint32_t pU, uint32_t pV, uint64_t bY, uint64_t bU, uint64_t bV, int &nst)
{
    const int n = W.lane & 15, g = W.lane >> 4;
    const int y = 16 * VE.G + n;
    const bool rowok = n < VE.rows;
    const uint32_t CP = (uint32_t)VE.ring0.CP, dlo = (uint32_t)(VE.ring0.lo - VE.ring0.hi);
    if (W.nplanes == 1) {
        const uint64_t orow = bY + (uint64_t)y * pY;
        for (int ct = first; ct < nct; ct += 2 * kL5Waves) {
            const int ct2 = ct + kL5Waves < nct ? ct + kL5Waves : ct;
            const uint32_t ha = (uint32_t)VE.ring0.hi + (uint32_t)(16 * ct + n) * CP;
            const uint32_t hb = (uint32_t)VE.ring0.hi + (uint32_t)(16 * ct2 + n) * CP;
            uint32_t wa, wb;
            if (kL5VPair) {
                vtile2<NKB>(lds, ha, ha + dlo, hb, hb + dlo, VE.w0, VE.ring0.RR, vh, vl, W.lane, wa, wb);
            } else {
                wa = vtile1<NKB>(lds, ha, ha + dlo, VE.w0, VE.ring0.RR, vh, vl, W.lane);
                __builtin_amdgcn_sched_barrier(0);
                wb = ct2 != ct ? vtile1<NKB>(lds, hb, hb + dlo, VE.w0, VE.ring0.RR, vh, vl, W.lane) : wa;
            }
            if (!rowok) continue;
            const int xa = x0 + 16 * ct + 4 * g, xb = x0 + 16 * ct2 + 4 * g;
            if (x0 + 16 * ct2 + 16 <= VE.dstW) {            // both tiles inside the plane (uniform)
                if (!(DTS_L5_ABLATE & 8)) {
                    *GP5(g_u32, orow + xa) = wa;
                    *GP5(g_u32, orow + xb) = wb;
                    nst += 2;                               // counted: the step's vmcnt wait skips them
                }
                continue;
            }
            store4(orow, xa, VE.dstW - xa, wa);
            if (ct2 != ct) store4(orow, xb, VE.dstW - xb, wb);
        }
    } else {
        const bool nv = VE.fmt == DTS_FMT_NV12;
        const uint64_t urow = bU + (uint64_t)y * pU;
        const uint64_t vrow = bV + (uint64_t)y * pV;
        for (int ct = first; ct < nct; ct += kL5Waves) {
            const uint32_t cb = (uint32_t)(16 * ct + n) * CP;
            uint32_t wu, wv;
            if (kL5VPair) {
                vtile2<NKB>(lds, (uint32_t)VE.ring0.hi + cb, (uint32_t)VE.ring0.lo + cb, (uint32_t)VE.hi1 + cb,
                            (uint32_t)VE.lo1 + cb, VE.w0, VE.ring0.RR, vh, vl, W.lane, wu, wv);
            } else {
                wu = vtile1<NKB>(lds, (uint32_t)VE.ring0.hi + cb, (uint32_t)VE.ring0.lo + cb, VE.w0, VE.ring0.RR, vh,
                                 vl, W.lane);
                __builtin_amdgcn_sched_barrier(0);
                wv = vtile1<NKB>(lds, (uint32_t)VE.hi1 + cb, (uint32_t)VE.lo1 + cb, VE.w0, VE.ring0.RR, vh, vl, W.lane);
            }
            const int x = x0 + 16 * ct + 4 * g;
            if (!rowok) continue;
            if (x0 + 16 * ct + 16 <= VE.dstW) {              // the whole tile inside the plane (uniform)
                if (DTS_L5_ABLATE & 8) continue;
                if (!nv) {
                    *GP5(g_u32, urow + x) = wu;
                    *GP5(g_u32, vrow + x) = wv;
                    nst += 2;
                } else {                                    // yuv2nv12cX: U0 V0 U1 V1 U2 V2 U3 V3
                    *GP5(g_u32x2, urow + 2 * x) = (u32x2){__builtin_amdgcn_perm(wv, wu, 0x05010400u),
                                                          __builtin_amdgcn_perm(wv, wu, 0x07030602u)};
                    nst += 1;
                }
                continue;
            }
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

// V of a step for this wave: the row groups vs.x .. vs.y - 1, fragments from the
// fragment area fa (LDS byte address) of the step's bundle
__device__ __forceinline__ void vrun(const uint32_t *lds, const Kind5 *K, const Walk5 &W, const int2 &vs, uint32_t fa,
                                     int &nst)
{
    const VEnt5 *vsched = kld(&K->vsched);
    int rot = 0;
    for (int e = vs.x; e < vs.y; ++e) {
        const VEnt5 VE = kld(vsched + e);
        const uint32_t *tb = lds + 4 + 16 * VE.rung;
        const u32x4 t0 = *reinterpret_cast<const u32x4 *>(tb);        // x0, nct, pitch Y, pitch U
        const u32x4 t1 = *reinterpret_cast<const u32x4 *>(tb + 4);    // pitch V, 0, base Y
        const u32x4 t2 = *reinterpret_cast<const u32x4 *>(tb + 8);    // base U, base V
        const int nct = uni5((int)t0.y);
        const int first = (W.vrank - rot % kL5Waves + kL5Waves) % kL5Waves;
        rot += nct;
        if (first >= nct) continue;
        v4i vh[kL5MaxVkb], vl[kL5MaxVkb];
        vfrags(lds, fa + (uint32_t)VE.foff, VE.nkb, W.lane, vh, vl);
        auto u64 = [](uint32_t lo, uint32_t hi) {
            return ((uint64_t)(uint32_t)uni5((int)hi) << 32) | (uint32_t)uni5((int)lo);
        };
        const int x0 = uni5((int)t0.x);
        const uint32_t pY = (uint32_t)uni5((int)t0.z), pU = (uint32_t)uni5((int)t0.w), pV = (uint32_t)uni5((int)t1.x);
        if (VE.nkb > 1)
            vgroup<2>(lds, W, VE, vh, vl, first, nct, x0, pY, pU, pV, u64(t1.z, t1.w), u64(t2.x, t2.y),
                      u64(t2.z, t2.w), nst);
        else
            vgroup<1>(lds, W, VE, vh, vl, first, nct, x0, pY, pU, pV, u64(t1.z, t1.w), u64(t2.x, t2.y),
                      u64(t2.z, t2.w), nst);
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
    W.stage = kld(&K->stage);
    W.SB = kld(&K->SB);
    W.FA = kld(&K->FA);
    W.FB = kld(&K->FB);
    const Strip5 *S = kld(&K->strips) + J.strip;
    W.L = kld(&S->L);
    W.cpr = kld(&S->cpr);
    W.Pb = kld(&S->Pb);
    W.PS = kld(&S->PS);
    W.nsi = kld(&S->nsi);
    W.ne = kld(&S->nent[W.wave]);
    W.vrank = (W.wave - kld(&S->hextra) + kL5Waves) % kL5Waves;
    const Ent5 *ents = kld(&K->ents) + kld(&S->ent0[W.wave]);
    const uint32_t *bf = kld(&K->bfrag);
    const bool chroma = W.nplanes == 2;
    const bool nv12c = SRC == kSrcNV12 && chroma;
    const int nlp = kld(&K->nlp);

    // ---- this wave's H entries: B fragments in VGPRs, per-lane LDS addresses ----
    const int g = W.lane >> 4, n = W.lane & 15;
    v4i bh[kL5Ent], bl[kL5Ent];
    HEnt5 HE;
    const uint32_t abase = (uint32_t)(n * W.Pb + (nv12c ? 16 : 8) * g);
    uint32_t odd = 0;
#pragma unroll
    for (int i = 0; i < kL5Ent; ++i) {
        bh[i] = bl[i] = (v4i){0, 0, 0, 0};
        HE.ao[i] = HE.hb[i] = HE.dl[i] = HE.cp[i] = HE.no[i] = HE.pos[i] = 0;
        HE.rr[i] = kL5StepRows;
        if (i < W.ne) {
            const Ent5 E = kld(ents + i);
            const g_u32x4 *f = GP5(const g_u32x4, bf + (size_t)E.bfrag * 512);
            bh[i] = __builtin_bit_cast(v4i, f[W.lane]);
            bl[i] = __builtin_bit_cast(v4i, f[64 + W.lane]);
            HE.ao[i] = (uint32_t)(W.stage + (nlp == 2 ? E.plane * W.PS : 0) + E.soff);
            const Ring5 rg = kld(K->ring + E.ring);
            HE.hb[i] = (uint32_t)(rg.hi + E.col0 * rg.CP);
            HE.dl[i] = (uint32_t)(rg.lo - rg.hi);
            HE.cp[i] = (uint32_t)rg.CP;
            HE.no[i] = E.flags & 16 ? 4u : E.flags & 8 ? 8u : 16u;
            HE.rr[i] = (uint32_t)rg.RR;
            odd |= (uint32_t)((E.flags >> 2) & 1) << i;
        }
    }
    odd = (uint32_t)uni5((int)odd);

    // ---- this item's DMA sources ----
    Dma5 D;
    {
        const int bps = nv12c ? 2 : 1;
        for (int lp = 0; lp < 2; ++lp) {
            const int spl = chroma ? (nv12c ? 1 : 1 + lp) : 0;           // source plane
            const int sp = lp < nlp ? spl : 0;
            const uint64_t base = kld(&kargs()->src.data[sp]) + (uint64_t)frame * kld(&kargs()->src.fstride);
            const int64_t pitch = kld(&kargs()->src.pitch[sp]);
            D.rs[lp] = rsrc5(base, (uint32_t)(pitch * W.srcH));
            D.pitch[lp] = (uint32_t)pitch;
        }
        D.rf = rsrc5((uint64_t)(uintptr_t)bf, kld(&K->nbfrag) * 2048u);
        D.colb = (uint32_t)(W.L * bps);
        D.rc = 1.0f / (float)W.cpr;
        D.ipp = W.PS >> 10;
    }

    rung_table(lds, S, kld(&K->nrungs), frame, W);

    // ---- prologue: bundles 0 and 1 ----
    const int4 *vstep = kld(&K->vstep);
    issue_bundle(W, D, 0);
    if (W.nsteps > 1) issue_bundle(W, D, 1);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    // iteration b (after barrier b - 1: bundle b and V(b - 1)'s fragments landed, H(b - 1)
    // done): V(b)'s fragments into buffer b % kL5FragBufs (V(b - 2) read it); V(b - 1);
    // H(b); bundle b + 2 into the buffer H(b - 1) read; wait for all but bundle b + 2 and
    // the counted V stores; barrier b.
    // V(b - 1) reads rows H(b) may be writing elsewhere in the ring: the planner's RR
    // keeps them apart.  Step records come one iteration ahead of their use.
    int2 vsV = {0, 0};                                      // V(b - 1)'s groups
    int2 vsF = kld(reinterpret_cast<const int2 *>(vstep) + 1);       // V(b)'s fragments
#if DTS_L5_STAMP
    unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_last = __builtin_amdgcn_s_memtime();
#endif
    for (int b = 0; b <= W.nsteps; ++b) {
        const int2 nV = kld(reinterpret_cast<const int2 *>(vstep + b));
        const int2 nF = kld(reinterpret_cast<const int2 *>(vstep + b + 1) + 1);
        // V(b)'s fragments first: the oldest loads of the step
        if (b < W.nsteps) issue_frags(W, D, b, vsF.x, vsF.y);
        int nst = 0;                                        // V stores issued (counted)
        if (b > 0 && !(DTS_L5_ABLATE & 2))
            vrun(lds, K, W, vsV, (uint32_t)(W.FA + ((b - 1) % kL5FragBufs) * W.FB), nst);
        L5_STAMP(0);
        if (b == W.nsteps) break;
        const uint32_t boff = (uint32_t)((b % kL5Stages) * W.SB);
        const uint32_t blkb = (uint32_t)(kL5Rows * W.Pb);      // second row block of the step
        if (nv12c) {
            switch ((DTS_L5_ABLATE & 1) ? 0 : W.ne) {
#define DTS_H5(k) \
    case k: hstep<k, true>(lds, bh, bl, HE, abase, n, g, odd, boff, blkb); break;
                DTS_H5(1) DTS_H5(2) DTS_H5(3) DTS_H5(4) DTS_H5(5)
#undef DTS_H5
            default:
                break;
            }
        } else {
            switch ((DTS_L5_ABLATE & 1) ? 0 : W.ne) {
#define DTS_H5(k) \
    case k: hstep<k, false>(lds, bh, bl, HE, abase, n, g, odd, boff, blkb); break;
                DTS_H5(1) DTS_H5(2) DTS_H5(3) DTS_H5(4) DTS_H5(5)
#undef DTS_H5
            default:
                break;
            }
        }
#pragma unroll
        for (int i = 0; i < kL5Ent; ++i) {                  // next step's rows: ring row (32 b) % RR
            const uint32_t np = HE.pos[i] + kL5StepRows;
            HE.pos[i] = np >= HE.rr[i] ? np - HE.rr[i] : np;
        }
        L5_STAMP(1);
        // bundle b + 2 after H: the V stores ahead of it in the memory queue have drained by now
        const int m = b + 2 < W.nsteps ? issue_bundle(W, D, b + 2) : 0;
        L5_STAMP(2);
        vsV = nV;
        vsF = nF;
        L5_STAMP(3);
        // bundle b + 1 and V(b)'s fragments have landed: younger are this step's V stores
        // and bundle b + 2
        step_wait(m);
        (void)nst;
        L5_STAMP(4);
        step_barrier();
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
__global__ void __launch_bounds__(kL5Threads, kL5Waves / 4) k_ladder5(const Ladder5Params P)
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
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void *>(&k_ladder5<SRC>), kL5Threads,
                                                     (size_t)lds) != hipSuccess)
        return 0;
    return n;
}

hipError_t launch_ladder5(const Ladder5Params &p, int src_kind, int lds_bytes, int grid, hipStream_t s)
{
    switch (src_kind) {
    case kSrcPlanar8:
        hipLaunchKernelGGL(k_ladder5<kSrcPlanar8>, dim3((unsigned)grid), dim3(kL5Threads), lds_bytes, s, p);
        break;
    case kSrcNV12:
        hipLaunchKernelGGL(k_ladder5<kSrcNV12>, dim3((unsigned)grid), dim3(kL5Threads), lds_bytes, s, p);
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
