// ladder4.hip -- k_ladder4, the v4 ladder kernel: scale + pixel-format
// convert for every rendition of a graph in one persistent launch.
//
// Same arithmetic as libswscale hScale8To15_c / hScale16To15_c ->
// yuv2planeX_8_c / yuv2nv12cX_c under SWS_BITEXACT|SWS_ACCURATE_RND
// (bit-exact; DESIGN.md "Oracle"), organised for CDNA4:
//
//  * one work item = (frame, rendition, plane Y/U/V, strip of up to 64
//    output columns), walked top to bottom in steps of 128 source rows;
//  * H: lane = source row pair.  Each wave owns a contiguous share of the
//    strip's output columns (an HGroup4); its lanes hold their two rows'
//    window in VGPRs (global_load_dwordx4), widen u8 / p010 samples to
//    int16x2 sample pairs, and evaluate every output whose window starts at a
//    pair position (positions unrolled at compile time; a wave-uniform bit
//    mask says which hold an output).  Taps are wave-uniform: staged in LDS
//    once per item and read with broadcast ds_read_b128; one v_dot2_i32_i16
//    does 2 taps of one row; v_cvt_pk_i16_i32 applies the 15-bit clip and
//    packs the row pair into the int16x2 dword the V pass consumes.  As soon
//    as the walk has converted the last sample pair of a 16-byte load, its
//    registers are refilled with the next step's rows, so the next step's
//    source streams in under the rest of this step's H and V work;
//  * the row-pair dwords go to an LDS ring [slot][column] with an odd column
//    pitch (conflict-free writes down a column, reads across a row);
//  * V: lane = output column, two output rows per wave and iteration,
//    v_dot2_i32_i16 over ring dwords with the rows' tap pairs (staged in LDS
//    one step ahead), then dither/round, >> 19, clip and a byte store (p010
//    output: + 1 << 16, >> 17, 10-bit clip, << 6 and a 16-bit store).
#include "dts_internal.h"

#ifndef DTS_L4_HSMEM
#define DTS_L4_HSMEM 1      // H taps: 1 = scalar loads (s_load) from the global table, 0 = LDS broadcast reads (r01v5)
#endif

#ifndef DTS_L4_HPF
#define DTS_L4_HPF 0        // 1: prefetch the next output's H taps (r01v10: -2 % cfg2, the extra SGPRs spill)
#endif

#ifndef DTS_L4_V2
#define DTS_L4_V2 1         // V: both rows of an iteration share one tap-group loop (LDS reads issued together)
#endif

#ifndef DTS_L4_VSMEM
#define DTS_L4_VSMEM 0      // 1: V taps / ring slots read with scalar loads from the global tables (no LDS staging)
#endif

#ifndef DTS_L4_ABLATE
#define DTS_L4_ABLATE 0     // diagnostic builds only: 1 skip H, 2 skip V, 4 skip source loads, 8 skip V stores
#endif

namespace dts {

__constant__ uint8_t c_dither_l4[8][8] = DTS_DITHER_8X8_128;

namespace {

typedef short short2v __attribute__((ext_vector_type(2)));
typedef unsigned short ushort2v __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_cu32x4;
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) uint16_t g_u16;
// constant address space: wave-uniform reads become s_load
typedef __attribute__((address_space(4))) const uint32_t k_u32;
typedef __attribute__((address_space(4))) const int32_t k_i32;
#define GP(T, p) ((T *)(uintptr_t)(p))

enum : int { kCvtP8 = 0, kCvtNV = 1, kCvtP16 = 2, kCvtP16C = 3 };

__device__ __forceinline__ int dot2(uint32_t a, uint32_t b, int c)
{
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, a), __builtin_bit_cast(short2v, b), c, false);
}

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel)
{
    return __builtin_amdgcn_perm(hi, lo, sel);
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint32_t shr(uint32_t d, uint32_t sh)
{
    ushort2v v = __builtin_bit_cast(ushort2v, d);
    v = v >> (ushort2v){(unsigned short)sh, (unsigned short)sh};
    return __builtin_bit_cast(uint32_t, v);
}

// Conversion kinds (what one row's 8 x 16-byte loads hold):
//   P8  : planar u8, 8 sample pairs per load (the 8-bit planes are read as they are)
//   NV  : nv12 interleaved chroma, 4 pairs per load, sel picks U or V (input.c nv12ToUV_c)
//   P16 : p010 luma, LE16 >> 6, 4 pairs per load (input.c p010LEToY_c)
//   P16C: p010 interleaved chroma (U16,V16 dwords) >> 6, 2 pairs per load, sel picks U or V
//         (input.c p010LEToUV_c)
template <int CVT>
constexpr int pairs_per_load() { return CVT == kCvtP8 ? 8 : (CVT == kCvtP16C ? 2 : 4); }

// sample pairs the 8 loads of one row hold (= api.cpp plan4_for cap)
template <int CVT>
constexpr int cap_pairs() { return 8 * pairs_per_load<CVT>(); }

// Sample pair q (samples 2q, 2q+1 past the window base) of one row as int16x2.
// z is an opaque zero private to each hpass instantiation: without it the
// identical conversions of every tap-count variant are merged and hoisted in
// front of hdispatch's switch, where they all stay live at once.
template <int CVT>
__device__ __forceinline__ uint32_t pair_at(const uint32_t (&r)[32], int q, uint32_t sel, uint32_t z)
{
    if (CVT == kCvtP8) return perm(0u, r[q >> 1], ((q & 1) ? 0x0c030c02u : 0x0c010c00u) ^ z);
    if (CVT == kCvtNV) return perm(0u, r[q], sel ^ z);
    if (CVT == kCvtP16) return shr(r[q], 6u + z);
    return shr(perm(r[2 * q + 1], r[2 * q], sel ^ z), 6u + z);
}

// pair positions the unrolled H code handles (= filters.cpp qmax4)
constexpr int qmax4(int n, int cap)
{
    return (4 * n + 8) < (cap - n + 1) ? ((4 * n + 8) < 64 ? 4 * n + 8 : 64)
                                       : ((cap - n + 1) < 64 ? cap - n + 1 : 64);
}

// One lane's source window (its two rows) for one step, read through a
// buffer descriptor over the source plane: voffsets o0/o1 are the rows' byte
// offsets plus the window offset, load k adds 16k (an immediate).  The range
// check turns every read past the plane (and the wrapped negative offsets of
// row 0 when the window starts left of it) into zeros; a window starting left
// of a later row reads the previous row's tail instead.  Both only ever meet
// zero taps, as do loads k >= nload, which keep whatever the slot held.
struct Window {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t o0, o1;
    int nload;
};

// z: an opaque zero (soffset), keeps the loads of different hpass
// instantiations apart like pair_at's
__device__ __forceinline__ void load_chunk(uint32_t (&ra)[32], uint32_t (&rb)[32], const Window &w, int k,
                                           uint32_t z = 0)
{
    if (DTS_L4_ABLATE & 4) return;
    if (k < w.nload) {                                       // wave-uniform
        const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(w.rs, w.o0 + 16 * k, z, 0));
        const u32x4 x = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(w.rs, w.o1 + 16 * k, z, 0));
        ra[4 * k + 0] = v.x; ra[4 * k + 1] = v.y; ra[4 * k + 2] = v.z; ra[4 * k + 3] = v.w;
        rb[4 * k + 0] = x.x; rb[4 * k + 1] = x.y; rb[4 * k + 2] = x.z; rb[4 * k + 3] = x.w;
    }
}

// Horizontal FIR of one wave over its row pair for every output whose window
// starts at a pair position q < qend with bit q of mask set.  Outputs are
// visited in column order; their N int16x2 tap pairs (rows of NP = N rounded
// up to 4 dwords) follow each other in LDS at cl and are read with wave-wide
// broadcast ds_read_b128; their ring dwords follow each other at wp.  Every
// load slot of ra/rb is refilled from nw (the next step) once its last sample
// pair has been converted; slots the walk never reaches are refilled at its end.
template <int CVT, int N, int QMAX, int SH>
__device__ __forceinline__ void hpass(uint32_t (&ra)[32], uint32_t (&rb)[32], uint32_t sel, uint64_t mask,
                                      int qend, const uint32_t *cl, uint32_t *wp, const Window &nw)
{
    constexpr int NP = (N + 3) & ~3;
    constexpr int PPL = pairs_per_load<CVT>();
    static_assert(QMAX + N - 1 <= 8 * PPL, "window exceeds the 8 loads");
    uint32_t z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    uint32_t pa[QMAX + N + 7], pb[QMAX + N + 7];
#pragma unroll
    for (int q = 0; q < N - 1; ++q) {
        pa[q] = pair_at<CVT>(ra, q, sel, z);
        pb[q] = pair_at<CVT>(rb, q, sel, z);
        if (q % PPL == PPL - 1) load_chunk(ra, rb, nw, q / PPL, z);
    }
#if DTS_L4_HSMEM
    k_u32 *cg = GP(k_u32, cl);
#if DTS_L4_HPF
    uint32_t cn[NP];                                 // the next output's taps (the table is padded by 16 dwords)
#pragma unroll
    for (int i = 0; i < NP; ++i) cn[i] = cg[i];
#endif
#else
    const uint4 *cv = reinterpret_cast<const uint4 *>(cl);
#endif
    // a constant trip count (no early exit) keeps the loop fully unrolled, so
    // every pa/pb/ra/rb index is a compile-time register; qend is tested once
    // per 8 positions, the output mask once per position
#pragma unroll
    for (int q8 = 0; q8 < QMAX; q8 += 8) {
        if (q8 < qend) {
#pragma unroll
            for (int q = q8; q < q8 + 8 && q < QMAX; ++q) {
                const int pn = q + N - 1;                    // the pair this position converts
                pa[pn] = pair_at<CVT>(ra, pn, sel, z);
                pb[pn] = pair_at<CVT>(rb, pn, sel, z);
                if (pn % PPL == PPL - 1) load_chunk(ra, rb, nw, pn / PPL, z);
                if ((((q < 32) ? (uint32_t)mask : (uint32_t)(mask >> 32)) >> (q & 31)) & 1u) {
                    uint32_t c[NP];
#if DTS_L4_HSMEM && DTS_L4_HPF
                    cg += NP;
#pragma unroll
                    for (int i = 0; i < NP; ++i) {
                        c[i] = cn[i];
                        cn[i] = cg[i];
                    }
#elif DTS_L4_HSMEM
#pragma unroll
                    for (int i = 0; i < NP; ++i) c[i] = cg[i];
                    cg += NP;
#else
#pragma unroll
                    for (int i = 0; i < NP / 4; ++i) {
                        const uint4 v = cv[i];
                        c[4 * i + 0] = v.x;
                        c[4 * i + 1] = v.y;
                        c[4 * i + 2] = v.z;
                        c[4 * i + 3] = v.w;
                    }
                    cv += NP / 4;
#endif
                    int a = 0, b = 0;
#pragma unroll
                    for (int t = 0; t < N; ++t) {
                        a = dot2(pa[q + t], c[t], a);
                        b = dot2(pb[q + t], c[t], b);
                    }
                    // FFMIN(val >> sh, 32767) for both rows (val >> sh >= -32768 always holds)
                    *wp++ = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(a >> SH, b >> SH));
                }
            }
        }
    }
    // pairs [0, conv) were converted above; refill the slots holding any later pair
    const int conv = min((qend + 7) & ~7, QMAX) + N - 1;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if ((k + 1) * PPL - 1 >= conv) load_chunk(ra, rb, nw, k, z);
}

// Wave-uniform struct read through the constant address space (s_load).
template <class T>
__device__ __forceinline__ T kload(const T *p)
{
    static_assert(sizeof(T) % 4 == 0, "dword structs only");
    struct W { uint32_t w[sizeof(T) / 4]; } w;
    k_u32 *q = GP(k_u32, p);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) w.w[i] = q[i];
    return __builtin_bit_cast(T, w);
}

constexpr int kCP = kRing4Cols + 1;   // ring column pitch (dwords)

// Vertical FIR of one output row for one lane: ng groups of 4 ring dwords
// (row pairs) from slot s0 on (wrapping at R), with the row's tap pairs in LDS
// at cq (broadcast ds_read_b128; rows are zero-padded to groups of 4, so the
// ring dwords past the window only meet zero taps).  s0 is wave-uniform.
#if DTS_L4_VSMEM
struct KQuad {                                  // 4 wave-uniform tap pairs through s_load
    k_u32 *p;
    __device__ __forceinline__ uint4 operator[](int g) const
    {
        return make_uint4(p[4 * g], p[4 * g + 1], p[4 * g + 2], p[4 * g + 3]);
    }
};
#endif

__device__ __forceinline__ int vtaps(const uint32_t *rl, int R, int s0, int ng, const uint32_t *cq, int acc)
{
#if DTS_L4_VSMEM
    const KQuad c4{GP(k_u32, cq)};
#else
    const uint4 *c4 = reinterpret_cast<const uint4 *>(cq);
#endif
    if (s0 + 4 * ng <= R) {
        const uint32_t *p = rl + s0 * kCP;
        for (int g = 0; g < ng; ++g, p += 4 * kCP) {
            const uint4 c = c4[g];
            acc = dot2(p[0], c.x, acc);
            acc = dot2(p[kCP], c.y, acc);
            acc = dot2(p[2 * kCP], c.z, acc);
            acc = dot2(p[3 * kCP], c.w, acc);
        }
    } else {                                                 // the window wraps round the ring
        for (int g = 0; g < ng; ++g) {
            const uint4 c = c4[g];
            const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                int s = s0 + 4 * g + i;
                if (s >= R) s -= R;
                acc = dot2(rl[s * kCP], cc[i], acc);
            }
        }
    }
    return acc;
}

// Two output rows of one lane at once (slots s0, s1, tap rows cq0, cq1): the
// LDS reads of both rows' groups issue together, so one LDS round trip serves
// both accumulators.  Each accumulator sums in vtaps' order (bit-identical).
__device__ __forceinline__ void vtaps2(const uint32_t *rl, int R, int s0, int s1, int ng, const uint32_t *cq0,
                                       const uint32_t *cq1, int &acc0, int &acc1)
{
#if DTS_L4_V2 && !DTS_L4_VSMEM
    if (s0 + 4 * ng <= R && s1 + 4 * ng <= R) {
        const uint32_t *p = rl + s0 * kCP, *q = rl + s1 * kCP;
        const uint4 *c0 = reinterpret_cast<const uint4 *>(cq0), *c1 = reinterpret_cast<const uint4 *>(cq1);
        for (int g = 0; g < ng; ++g, p += 4 * kCP, q += 4 * kCP) {
            const uint4 a = c0[g], b = c1[g];
            const uint32_t p0 = p[0], p1 = p[kCP], p2 = p[2 * kCP], p3 = p[3 * kCP];
            const uint32_t q0 = q[0], q1 = q[kCP], q2 = q[2 * kCP], q3 = q[3 * kCP];
            acc0 = dot2(p0, a.x, acc0);
            acc1 = dot2(q0, b.x, acc1);
            acc0 = dot2(p1, a.y, acc0);
            acc1 = dot2(q1, b.y, acc1);
            acc0 = dot2(p2, a.z, acc0);
            acc1 = dot2(q2, b.z, acc1);
            acc0 = dot2(p3, a.w, acc0);
            acc1 = dot2(q3, b.w, acc1);
        }
        return;
    }
#endif
    acc0 = vtaps(rl, R, s0, ng, cq0, acc0);
    acc1 = vtaps(rl, R, s1, ng, cq1, acc1);
}

// yuv2planeX_8 / yuv2nv12cX accumulator start for output row y: the dither
// (flat 64 for 8-bit sources, this lane's ff_dither_8x8_128 column, packed in
// dlo/dhi, for >8-bit sources) << 12
template <int SRC>
__device__ __forceinline__ int vinit(int y, uint32_t dlo, uint32_t dhi)
{
    if (SRC != kSrcP010) return 64 << 12;
    const uint32_t dw = (y & 4) ? dhi : dlo;
    return (int)((dw >> (8 * (y & 3))) & 255u) << 12;
}

__device__ __forceinline__ void vstore(uint64_t p, int acc)
{
    int v = acc >> 19;
    v = v < 0 ? 0 : (v > 255 ? 255 : v);
    *GP(g_u8, p) = (uint8_t)v;
}

// output.c yuv2p010lX_c / yuv2p010cX_c: av_clip_uintp2(val >> 17, 10) << 6, LE16
__device__ __forceinline__ void vstore16(uint64_t p, int acc)
{
    int v = acc >> 17;
    v = v < 0 ? 0 : (v > 1023 ? 1023 : v);
    *GP(g_u16, p) = (uint16_t)(v << 6);
}

// Per-item state shared by the H and V halves of a walk.
struct Item {
    const uint32_t *hco;                 // this wave's H taps (LDS)
    uint32_t *vco_base;                  // V taps, 2 step buffers (LDS)
    int *vsl_base;                       // V ring slots, 2 step buffers (LDS)
    const uint32_t *rl;                  // ring column of this lane (V)
    __amdgpu_buffer_rsrc_t rsrc;         // source plane of the frame
    int64_t pitch;
    int64_t opitch;
    uint64_t obase;                      // output sample of this lane in row 0
    uint64_t mask;
    const uint32_t *vcoef;
    const int32_t *vslot;
    const int32_t *vlim;
    uint32_t sel, dlo, dhi;
    bool d16;                            // p010 output (yuv2p010*: 1 << 16 rounding, no dither)
    int R, srcH, nsteps, nvp, lofs, nload, qend, col0, wave, lane, t;
    bool vact;
};

// The output rows step b completes, rows vlo + wave + 4i for this wave, two
// rows per iteration; the step's ring slots and tap pairs are staged in LDS
// (row y at index y - vlo).
template <int SRC>
__device__ __forceinline__ void vpass(const Item &I, int b)
{
    k_i32 *vlim = GP(k_i32, I.vlim);
    const int vlo = b > 0 ? vlim[b - 1] : 0, vhi = vlim[b];
#if DTS_L4_VSMEM
    k_i32 *vsl = GP(k_i32, I.vslot) + vlo;
    const uint32_t *vco = I.vcoef + (int64_t)vlo * I.nvp;
#else
    const int *vsl = I.vsl_base + (b & 1) * kV4SlotMax;
    const uint32_t *vco = I.vco_base + (b & 1) * kV4CoefDw;
#endif
    const int ng = I.nvp >> 2;
    for (int y = vlo + I.wave; y < vhi; y += 8) {
        const int y2 = min(y + 4, vhi - 1);
        const int i0 = y - vlo, i1 = y2 - vlo;
        const int s0 = uni(vsl[i0]), s1 = uni(vsl[i1]);
        int a0 = I.d16 ? 1 << 16 : vinit<SRC>(y, I.dlo, I.dhi);
        int a1 = I.d16 ? 1 << 16 : vinit<SRC>(y2, I.dlo, I.dhi);
        vtaps2(I.rl, I.R, s0, s1, ng, vco + i0 * I.nvp, vco + i1 * I.nvp, a0, a1);
        if (DTS_L4_ABLATE & 8) {                                   // diagnostic: keep V, drop its stores
            asm volatile("" ::"v"(a0), "v"(a1));
        } else if (I.vact) {
            if (I.d16) {
                vstore16(I.obase + (int64_t)y * I.opitch, a0);
                if (y + 4 < vhi) vstore16(I.obase + (int64_t)y2 * I.opitch, a1);
            } else {
                vstore(I.obase + (int64_t)y * I.opitch, a0);
                if (y + 4 < vhi) vstore(I.obase + (int64_t)y2 * I.opitch, a1);
            }
        }
    }
}

// step b's V taps and slots -> LDS buffer b & 1
__device__ __forceinline__ void vstage(const Item &I, int b)
{
    k_i32 *vlim = GP(k_i32, I.vlim);
    const int vlo = b > 0 ? vlim[b - 1] : 0, nr = vlim[b] - vlo;
    uint4 *d4 = reinterpret_cast<uint4 *>(I.vco_base + (b & 1) * kV4CoefDw);
    const uint4 *g4 = reinterpret_cast<const uint4 *>(I.vcoef + (int64_t)vlo * I.nvp);
    for (int i = I.t; i < nr * I.nvp / 4; i += kThreads) d4[i] = g4[i];
    for (int i = I.t; i < nr; i += kThreads) I.vsl_base[(b & 1) * kV4SlotMax + i] = I.vslot[vlo + i];
}

// this lane's two source rows of step b (rows past the plane re-read its last
// row: their H results only meet zero V taps); step nsteps (loaded by the last
// step) reads nothing
__device__ __forceinline__ Window window(const Item &I, int b)
{
    Window w;
    w.rs = I.rsrc;
    const int r0 = min(128 * b + 2 * I.lane, I.srcH - 1), r1 = min(128 * b + 2 * I.lane + 1, I.srcH - 1);
    const bool on = b < I.nsteps;
    w.o0 = on ? (uint32_t)(r0 * I.pitch + I.lofs) : 0x80000000u;
    w.o1 = on ? (uint32_t)(r1 * I.pitch + I.lofs) : 0x80000000u;
    w.nload = I.nload;
    return w;
}

// The walk of one item down its plane with N tap pairs per output.
template <int SRC, int CVT, int N>
__device__ __forceinline__ void walk(const Item &I, uint32_t *ring)
{
    constexpr int SH = SRC == kSrcP010 ? 9 : 7;                    // hScale16To15: sh = depth - 1
    constexpr int QMAX = qmax4(N, cap_pairs<CVT>());
    uint32_t ra[32], rb[32];
    {
        const Window w0 = window(I, 0);
#pragma unroll
        for (int k = 0; k < 8; ++k) load_chunk(ra, rb, w0, k);
    }
    int slot0 = 0;
    for (int b = 0; b <= I.nsteps; ++b) {
        if (!DTS_L4_VSMEM && b < I.nsteps) vstage(I, b);
        if (!(DTS_L4_ABLATE & 2) && b > 0) vpass<SRC>(I, b - 1);
        __syncthreads();
        if (b < I.nsteps) {
            const Window nw = window(I, b + 1);
            int s = slot0 + I.lane;
            if (s >= I.R) s -= I.R;
            // opaque per step: keeps the compiler from hoisting the ~2 x QMAX
            // position tests out of the walk as long-lived SGPR lane masks
            uint64_t mask = I.mask;
            int qend = I.qend;
            asm volatile("" : "+s"(mask), "+s"(qend));
            if (!(DTS_L4_ABLATE & 1)) {
                hpass<CVT, N, QMAX, SH>(ra, rb, I.sel, mask, qend, I.hco, ring + s * kCP + I.col0, nw);
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) load_chunk(ra, rb, nw, k);
            }
            slot0 += 64;
            if (slot0 >= I.R) slot0 -= I.R;
        }
        __syncthreads();
    }
}

// One item: a strip of one plane (Y, U or V) of one rendition of one frame.
// CVT is the plane's source conversion; planar u8 sources share one
// instantiation for all three planes.  The walk is instantiated per tap-pair
// count, so each one's loop holds only its own unrolled H code.
template <int SRC, int CVT>
__device__ __forceinline__ void item4(const Ladder4Params &P, int frame, const Job4 &J, uint32_t *ring)
{
    const int kind = J.kind;
    const int cpl = kind ? J.plane : 0;                            // chroma: 0 = U, 1 = V
    Item I;
    I.sel = CVT == kCvtNV ? (cpl ? 0x0c030c01u : 0x0c020c00u) : (cpl ? 0x07060302u : 0x05040100u);
    I.t = threadIdx.x;
    I.lane = I.t & 63;
    I.wave = uni(I.t >> 6);
    const RungKind4 K = kload(P.rk + J.rk);
    const HGroup4 hg = kload(K.groups + J.group0 + I.wave);
    I.R = P.ring;
    I.srcH = kind ? P.chrH : P.srcH;
    I.nsteps = K.nsteps;
    I.nvp = (K.NV + 3) & ~3;
    I.lofs = hg.lofs;
    I.nload = hg.nload;
    I.qend = hg.qend;
    I.col0 = hg.col0;
    I.mask = hg.mask;
    I.vcoef = K.vcoef;
    I.vslot = K.vslot;
    I.vlim = K.vlim;
    const int spl = kind ? (SRC == kSrcPlanar8 ? 1 + cpl : 1) : 0; // source plane
    I.pitch = spl == 0 ? P.src.pitch[0] : (spl == 1 ? P.src.pitch[1] : P.src.pitch[2]);
    {   // the source plane of this frame as a buffer (descriptor inputs made provably uniform)
        const uint64_t pbase = (spl == 0 ? P.src.data[0] : (spl == 1 ? P.src.data[1] : P.src.data[2])) +
                               (uint64_t)frame * P.src.fstride;
        const uint32_t lo = (uint32_t)uni((int)(uint32_t)pbase), hi = (uint32_t)uni((int)(uint32_t)(pbase >> 32));
        const int bytes = uni((int)(I.pitch * I.srcH));
        I.rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), 0, bytes,
                                                   0x00020000);
    }
    // LDS: [ring][H taps: 4 waves][V taps: 2 step buffers][V slots: 2 step buffers]
    uint32_t *const hco = ring + kRing4Dw + I.wave * kH4CoefDw;
    I.vco_base = ring + kRing4Dw + 4 * kH4CoefDw;
    I.vsl_base = reinterpret_cast<int *>(I.vco_base + 2 * kV4CoefDw);
#if DTS_L4_HSMEM
    I.hco = K.hcoef + hg.coef;                                     // read by s_load in hpass
    (void)hco;
#else
    I.hco = hco;
    {   // this wave's output taps for the whole walk: global -> LDS once per item
        const int ndw = __builtin_popcountll(hg.mask) * ((K.N + 3) & ~3);
        const uint4 *g4 = reinterpret_cast<const uint4 *>(K.hcoef + hg.coef);
        for (int i = I.lane; i < ndw / 4; i += 64) reinterpret_cast<uint4 *>(hco)[i] = g4[i];
    }
#endif

    // V-side constants of this lane
    I.vact = I.lane < J.ncols;
    I.rl = ring + I.lane;
    // indexed by the item's rung: read per item from the kernarg segment, not held in SGPRs
    const DevPlanes dst = P.dst[J.rung];
    const int dfmt = P.dst_fmt[J.rung];
    const uint64_t dfb = (uint64_t)frame * dst.fstride;
    I.d16 = dfmt == DTS_FMT_P010LE;
    if (kind == 0) {
        I.obase = dst.data[0] + dfb + (uint64_t)(J.x0 + I.lane) * (I.d16 ? 2 : 1);
        I.opitch = dst.pitch[0];
    } else if (I.d16) {                                            // p010: U16,V16 pairs
        I.obase = dst.data[1] + dfb + 4 * (J.x0 + I.lane) + 2 * cpl;
        I.opitch = dst.pitch[1];
    } else if (dfmt == DTS_FMT_NV12) {
        I.obase = dst.data[1] + dfb + 2 * (J.x0 + I.lane) + cpl;
        I.opitch = dst.pitch[1];
    } else {
        I.obase = (cpl ? dst.data[2] : dst.data[1]) + dfb + J.x0 + I.lane;
        I.opitch = cpl ? dst.pitch[2] : dst.pitch[1];
    }
    // yuv2planeX_8 / yuv2nv12cX dither for >8-bit sources: ff_dither_8x8_128[y & 7][(x + off) & 7],
    // off = 0 for Y and U, 3 for V; x0 is a multiple of 8
    I.dlo = 0;
    I.dhi = 0;
    if (SRC == kSrcP010) {
        const int dx = (I.lane + (cpl ? 3 : 0)) & 7;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            I.dlo |= (uint32_t)c_dither_l4[r][dx] << (8 * r);
            I.dhi |= (uint32_t)c_dither_l4[r + 4][dx] << (8 * r);
        }
    }
    switch (K.N) {                                                 // wave-uniform, once per item
#define DTS_W4(n) \
    case n: walk<SRC, CVT, n>(I, ring); break;
        DTS_W4(2) DTS_W4(3) DTS_W4(4) DTS_W4(5) DTS_W4(6) DTS_W4(7) DTS_W4(8) DTS_W4(9) DTS_W4(10)
        DTS_W4(11) DTS_W4(12) DTS_W4(14) DTS_W4(16)
#undef DTS_W4
    default:
        break;                                                     // other counts are never planned
    }
}

} // namespace

#ifndef DTS_L4_WAVES
#define DTS_L4_WAVES 3          // waves per SIMD the register budget is cut for (<= 168 VGPRs)
#endif
// Persistent workgroups pull (frame, job) items from a device counter,
// frame-major so the renditions of one frame run together (source re-reads
// across renditions and strip halos hit L2 / the Infinity Cache).
template <int SRC>
__global__ void __launch_bounds__(kThreads, DTS_L4_WAVES) k_ladder4(const Ladder4Params P)
{
    constexpr int kLumaCvt = SRC == kSrcP010 ? kCvtP16 : kCvtP8;
    constexpr int kChromaCvt = SRC == kSrcPlanar8 ? kCvtP8 : (SRC == kSrcNV12 ? kCvtNV : kCvtP16C);
    extern __shared__ __attribute__((aligned(16))) uint32_t ring[];
    volatile int *slot = reinterpret_cast<volatile int *>(ring);   // ring dword 0: idle between items
    for (;;) {
        // nq > 1: one queue per XCD (workgroups are dispatched round-robin over the
        // XCDs), holding the frames f = x (mod nq), so every strip of a frame -- and
        // the source rows its renditions and halos re-read -- stays in one XCD's L2
        const int x = P.nq > 1 ? (int)(blockIdx.x % (unsigned)P.nq) : 0;
        if (threadIdx.x == 0) *slot = (int)atomicAdd(P.queue + x, 1u);
        __syncthreads();
        const int item = uni(*slot);
        __syncthreads();
        const int nf = (P.nframes - x + P.nq - 1) / P.nq;          // frames of this queue
        if (item >= nf * P.njobs) return;
        const int fq = item / P.njobs, jid = item - fq * P.njobs;
        const int frame = x + P.nq * fq;
        const Job4 J = kload(P.jobs + jid);
        if (kLumaCvt == kChromaCvt || J.kind == 0)
            item4<SRC, kLumaCvt>(P, frame, J, ring);
        else
            item4<SRC, kChromaCvt>(P, frame, J, ring);
    }
}

template <int SRC>
static int occ4(int lds)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void *>(&k_ladder4<SRC>), kThreads,
                                                     (size_t)lds) != hipSuccess)
        return 0;
    return n;
}

hipError_t launch_ladder4(const Ladder4Params &p, int lds_bytes, int grid, hipStream_t s)
{
    switch (p.src_kind) {
    case kSrcPlanar8:
        hipLaunchKernelGGL(k_ladder4<kSrcPlanar8>, dim3((unsigned)grid), dim3(kThreads), lds_bytes, s, p);
        break;
    case kSrcNV12:
        hipLaunchKernelGGL(k_ladder4<kSrcNV12>, dim3((unsigned)grid), dim3(kThreads), lds_bytes, s, p);
        break;
    case kSrcP010:
        hipLaunchKernelGGL(k_ladder4<kSrcP010>, dim3((unsigned)grid), dim3(kThreads), lds_bytes, s, p);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

int ladder4_blocks_per_cu(int src_kind, int lds_bytes)
{
    switch (src_kind) {
    case kSrcPlanar8: return occ4<kSrcPlanar8>(lds_bytes);
    case kSrcNV12: return occ4<kSrcNV12>(lds_bytes);
    case kSrcP010: return occ4<kSrcP010>(lds_bytes);
    default: return 0;
    }
}

} // namespace dts
