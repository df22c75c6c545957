// ladder4.hip -- k_ladder4, the v4 ladder kernel: scale + pixel-format
// convert for every rendition of a graph in one persistent launch.
//
// Same arithmetic as libswscale hScale8To15_c / hScale16To15_c ->
// yuv2planeX_8_c / yuv2nv12cX_c under SWS_BITEXACT|SWS_ACCURATE_RND
// (bit-exact; DESIGN.md "Oracle"), organised for CDNA4:
//
//  * one work item = (frame, rendition, plane kind, strip of C output
//    columns), walked top to bottom in steps of 128 source rows;
//  * H: lane = source row pair.  Each wave owns a contiguous share of the
//    strip's output columns (an HGroup4); its lanes load their two rows'
//    window straight into VGPRs (global_load_dwordx4), widen u8 / p010
//    samples to int16x2 sample pairs, and evaluate every output whose window
//    starts at a pair position (positions unrolled at compile time; a
//    wave-uniform bit mask says which hold an output).  The taps are
//    wave-uniform, so they come from SGPRs (s_load) and one v_dot2_i32_i16
//    does 2 taps of one row; v_cvt_pk_i16_i32 applies the 15-bit clip and
//    packs the row pair into the int16x2 dword the V pass consumes;
//  * the row-pair dwords go to an LDS ring [slot][column] with an odd column
//    pitch (conflict-free writes down a column, reads across a row);
//  * V: lane = output column (chroma: lanes 0-31 U, 32-63 V), one output row
//    per wave, v_dot2_i32_i16 over ring dwords with SGPR tap pairs, then
//    dither/round, >> 19, clip and a byte store.
//  The next step's source rows are in flight while V runs on the ring.
#include "dts_internal.h"

#ifndef DTS_L4_ABLATE
#define DTS_L4_ABLATE 0     // diagnostic builds only: 1 skip H, 2 skip V, 4 skip source loads
#endif

namespace dts {

__constant__ uint8_t c_dither_l4[8][8] = DTS_DITHER_8X8_128;

namespace {

typedef short short2v __attribute__((ext_vector_type(2)));
typedef unsigned short ushort2v __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_cu32x4;
typedef __attribute__((address_space(1))) uint8_t g_u8;
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

// Sample pair q (samples 2q, 2q+1 past the window base) of one row as int16x2.
//   P8  : planar u8 (the 8-bit planes are read as they are)
//   NV  : nv12 interleaved chroma, sel picks U or V (input.c nv12ToUV_c)
//   P16 : p010 luma, LE16 >> 6 (input.c p010LEToY_c)
//   P16C: p010 interleaved chroma (U16,V16 dwords) >> 6, sel picks U or V (p010LEToUV_c)
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

// Horizontal FIR of one wave over its row pair for every output whose window
// starts at a pair position q < qend with bit q of mask set.  Outputs are
// visited in column order; their N int16x2 tap pairs (rows of NP = N rounded
// up to 4 dwords) follow each other in LDS at cl and are read with wave-wide
// broadcast ds_read_b128; their ring dwords follow each other at wp.
template <int CVT, int N, int QMAX, int SH>
__device__ __forceinline__ void hpass(const uint32_t (&ra)[32], const uint32_t (&rb)[32], uint32_t sel,
                                      uint64_t mask, int qend, const uint32_t *cl, uint32_t *wp)
{
    constexpr int NP = (N + 3) & ~3;
    uint32_t z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    uint32_t pa[QMAX + N + 7], pb[QMAX + N + 7];
#pragma unroll
    for (int q = 0; q < N - 1; ++q) {
        pa[q] = pair_at<CVT>(ra, q, sel, z);
        pb[q] = pair_at<CVT>(rb, q, sel, z);
    }
    const uint4 *cv = reinterpret_cast<const uint4 *>(cl);
    // a constant trip count (no early exit) keeps the loop fully unrolled, so
    // every pa/pb index is a compile-time register; qend is tested once per 8
    // positions, the output mask once per position
#pragma unroll
    for (int q8 = 0; q8 < QMAX; q8 += 8) {
        if (q8 < qend) {
#pragma unroll
            for (int q = q8; q < q8 + 8 && q < QMAX; ++q) {
                pa[q + N - 1] = pair_at<CVT>(ra, q + N - 1, sel, z);
                pb[q + N - 1] = pair_at<CVT>(rb, q + N - 1, sel, z);
                if ((uint32_t)(mask >> q) & 1u) {
                    uint32_t c[NP];
#pragma unroll
                    for (int i = 0; i < NP / 4; ++i) {
                        const uint4 v = cv[i];
                        c[4 * i + 0] = v.x;
                        c[4 * i + 1] = v.y;
                        c[4 * i + 2] = v.z;
                        c[4 * i + 3] = v.w;
                    }
                    cv += NP / 4;
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

template <int CVT, int CAP, int SH>
__device__ __forceinline__ void hdispatch(int N, const uint32_t (&ra)[32], const uint32_t (&rb)[32], uint32_t sel,
                                          uint64_t mask, int qend, const uint32_t *cp, uint32_t *wp)
{
    switch (N) {                                             // wave-uniform
#define DTS_H4(n) \
    case n: hpass<CVT, n, qmax4(n, CAP), SH>(ra, rb, sel, mask, qend, cp, wp); break;
        DTS_H4(2) DTS_H4(3) DTS_H4(4) DTS_H4(5) DTS_H4(6) DTS_H4(7) DTS_H4(8) DTS_H4(9) DTS_H4(10)
        DTS_H4(11) DTS_H4(12) DTS_H4(14) DTS_H4(16)
#undef DTS_H4
    default:
        break;
    }
}

// Vertical FIR of one output row for one lane: NV ring dwords (row pairs)
// from slot s0 on (wrapping at R), wave-uniform tap pairs in LDS at cq
// (broadcast reads).
template <int CP, int NV>
__device__ __forceinline__ int vtaps(const uint32_t *rl, int R, int s0, const uint32_t *cq, int acc)
{
    constexpr int NVP = (NV + 3) & ~3;
    uint32_t c[NVP];
#pragma unroll
    for (int i = 0; i < NVP / 4; ++i) {
        const uint4 v = reinterpret_cast<const uint4 *>(cq)[i];
        c[4 * i + 0] = v.x;
        c[4 * i + 1] = v.y;
        c[4 * i + 2] = v.z;
        c[4 * i + 3] = v.w;
    }
    if (s0 + NV <= R) {
        const uint32_t *b = rl + s0 * CP;
#pragma unroll
        for (int t = 0; t < NV; ++t) acc = dot2(b[t * CP], c[t], acc);
    } else {
#pragma unroll
        for (int t = 0; t < NV; ++t) {
            int s = s0 + t;
            if (s >= R) s -= R;
            acc = dot2(rl[s * CP], c[t], acc);
        }
    }
    return acc;
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

// The output rows [vlo, vhi) of one V step, rows vlo + wave + 4i for this
// wave, two rows per iteration.  vsl / vco: the step's ring slots and tap
// pairs staged in LDS (row y at index y - vlo).
template <int SRC, int CP, int NV>
__device__ __forceinline__ void vrows(const uint32_t *rl, int R, const int *vsl, const uint32_t *vco, int vlo,
                                      int vhi, int wave, bool vact, uint64_t obase, int64_t opitch, uint32_t dlo,
                                      uint32_t dhi)
{
    constexpr int NVP = (NV + 3) & ~3;
    for (int y = vlo + wave; y < vhi; y += 8) {
        const int y2 = min(y + 4, vhi - 1);
        const int i0 = y - vlo, i1 = y2 - vlo;
        const int a0 = vtaps<CP, NV>(rl, R, vsl[i0], vco + i0 * NVP, vinit<SRC>(y, dlo, dhi));
        const int a1 = vtaps<CP, NV>(rl, R, vsl[i1], vco + i1 * NVP, vinit<SRC>(y2, dlo, dhi));
        if (vact) {
            vstore(obase + (int64_t)y * opitch, a0);
            if (y + 4 < vhi) vstore(obase + (int64_t)y2 * opitch, a1);
        }
    }
}

template <int SRC, int CP>
__device__ __forceinline__ void vpass_any(int nv, const uint32_t *rl, int R, const int *vsl, const uint32_t *vco,
                                          int vlo, int vhi, int wave, bool vact, uint64_t obase, int64_t opitch,
                                          uint32_t dlo, uint32_t dhi)
{
    switch (nv) {                                            // wave-uniform, once per V step
#define DTS_V4(n) \
    case n: vrows<SRC, CP, n>(rl, R, vsl, vco, vlo, vhi, wave, vact, obase, opitch, dlo, dhi); break;
        DTS_V4(1) DTS_V4(2) DTS_V4(3) DTS_V4(4) DTS_V4(5) DTS_V4(6) DTS_V4(7) DTS_V4(8)
        DTS_V4(9) DTS_V4(10) DTS_V4(11) DTS_V4(12) DTS_V4(13) DTS_V4(14) DTS_V4(15) DTS_V4(16)
#undef DTS_V4
    default:
        break;                                               // nv > 16 is rejected at graph creation
    }
}

// One item: a strip of one plane kind of one rendition of one frame.
template <int SRC, int KIND>
__device__ __forceinline__ void item4(const Ladder4Params &P, int frame, const Job4 &J, uint32_t *ring)
{
    constexpr int CVT = KIND == 0 ? (SRC == kSrcP010 ? kCvtP16 : kCvtP8)
                                  : (SRC == kSrcPlanar8 ? kCvtP8 : (SRC == kSrcNV12 ? kCvtNV : kCvtP16C));
    constexpr bool planar2 = KIND == 1 && SRC == kSrcPlanar8;     // U and V in separate planes
    constexpr int CAP = planar2 ? 32 : (CVT == kCvtP8 ? 64 : (CVT == kCvtP16C ? 16 : 32));
    constexpr int CP = KIND ? kRing4ColsC + 1 : kRing4ColsL + 1;
    constexpr int SH = SRC == kSrcP010 ? 9 : 7;                    // hScale16To15: sh = depth - 1
    constexpr uint32_t kSelU = CVT == kCvtNV ? 0x0c020c00u : 0x05040100u;
    constexpr uint32_t kSelV = CVT == kCvtNV ? 0x0c030c01u : 0x07060302u;

    const int t = threadIdx.x, lane = t & 63, wave = uni(t >> 6);
    const RungKind4 K = kload(P.rk + J.rk);
    const HGroup4 hg = kload(K.groups + J.group0 + wave);
    const int R = P.ring;
    const int srcH = KIND ? P.chrH : P.srcH;
    const int pl0 = KIND ? 1 : 0;
    const int64_t pitch = P.src.pitch[pl0];
    const uint64_t fb = (uint64_t)frame * P.src.fstride;
    const uint64_t base0 = P.src.data[pl0] + fb + hg.lofs;
    const uint64_t base1 = P.src.data[2] + fb + hg.lofs;
    const int nload = hg.nload;
    const int lofs = hg.lofs;
    // LDS: [ring][H taps: 4 waves][V taps: 2 step buffers][V slots: 2 step buffers]
    uint32_t *const hco = ring + kRing4Dw + wave * kH4CoefDw;
    uint32_t *const vco_base = ring + kRing4Dw + 4 * kH4CoefDw;
    int *const vsl_base = reinterpret_cast<int *>(vco_base + 2 * kV4CoefDw);
    {   // this wave's output taps for the whole walk: global -> LDS once per item
        const int ndw = __builtin_popcountll(hg.mask) * ((K.N + 3) & ~3);
        const uint4 *g4 = reinterpret_cast<const uint4 *>(K.hcoef + hg.coef);
        for (int i = lane; i < ndw / 4; i += 64) reinterpret_cast<uint4 *>(hco)[i] = g4[i];
    }

    // V-side constants of this lane
    const int vpl = KIND ? (lane >> 5) : 0;
    const int col = KIND ? (lane & 31) : lane;
    const bool vact = col < J.ncols;
    const uint32_t *rl = ring + vpl * (R * CP) + col;
    // indexed by the item's rung: read per item from the kernarg segment, not held in SGPRs
    const DevPlanes dst = P.dst[J.rung];
    const int dfmt = P.dst_fmt[J.rung];
    const uint64_t dfb = (uint64_t)frame * dst.fstride;
    uint64_t obase;
    int64_t opitch;
    if (KIND == 0) {
        obase = dst.data[0] + dfb + J.x0 + col;
        opitch = dst.pitch[0];
    } else if (dfmt == DTS_FMT_NV12) {
        obase = dst.data[1] + dfb + 2 * (J.x0 + col) + vpl;
        opitch = dst.pitch[1];
    } else {
        obase = (vpl ? dst.data[2] : dst.data[1]) + dfb + J.x0 + col;
        opitch = dst.pitch[1];
    }
    // yuv2planeX_8 / yuv2nv12cX dither for >8-bit sources: ff_dither_8x8_128[y & 7][(x + off) & 7],
    // off = 0 for Y and U, 3 for V; x0 is a multiple of 8
    uint32_t dlo = 0, dhi = 0;
    if (SRC == kSrcP010) {
        const int dx = (col + (vpl ? 3 : 0)) & 7;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            dlo |= (uint32_t)c_dither_l4[r][dx] << (8 * r);
            dhi |= (uint32_t)c_dither_l4[r + 4][dx] << (8 * r);
        }
    }
    k_i32 *vlim = GP(k_i32, K.vlim);
    const int nv = K.NV, nvp = (nv + 3) & ~3;

    auto vstage = [&](int b) {                                 // step b's V taps and slots -> LDS buffer b & 1
        const int vlo = b > 0 ? vlim[b - 1] : 0, nr = vlim[b] - vlo;
        uint4 *d4 = reinterpret_cast<uint4 *>(vco_base + (b & 1) * kV4CoefDw);
        const uint4 *g4 = reinterpret_cast<const uint4 *>(K.vcoef + (int64_t)vlo * nvp);
        for (int i = t; i < nr * nvp / 4; i += kThreads) d4[i] = g4[i];
        for (int i = t; i < nr; i += kThreads) vsl_base[(b & 1) * kV4SlotMax + i] = K.vslot[vlo + i];
    };
    auto vpass = [&](int b) {                                  // the output rows step b completes
        const int vlo = b > 0 ? vlim[b - 1] : 0;
        vpass_any<SRC, CP>(nv, rl, R, vsl_base + (b & 1) * kV4SlotMax, vco_base + (b & 1) * kV4CoefDw, vlo,
                           vlim[b], wave, vact, obase, opitch, dlo, dhi);
    };

    const int nsteps = K.nsteps;
    int slot0 = 0;
    for (int b = 0; b <= nsteps; ++b) {
        uint32_t ra[32], rb[32];
        if (b < nsteps) {                                      // this step's source rows -> VGPRs
            // rows past the plane re-read its last row: their H results only meet zero V taps
            const int r0 = min(128 * b + 2 * lane, srcH - 1), r1 = min(128 * b + 2 * lane + 1, srcH - 1);
            const int64_t ro0 = (int64_t)r0 * pitch, ro1 = (int64_t)r1 * pitch;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int kk = planar2 ? (k & 3) : k;
                u32x4 v = {0u, 0u, 0u, 0u}, w = {0u, 0u, 0u, 0u};
                if (!(DTS_L4_ABLATE & 4) && kk < nload && lofs + 16 * kk >= 0) {   // chunks left of the row: zero taps
                    const uint64_t a = (planar2 && k >= 4 ? base1 : base0) + 16 * kk;
                    v = *GP(g_cu32x4, a + ro0);
                    w = *GP(g_cu32x4, a + ro1);
                }
                ra[4 * k + 0] = v.x; ra[4 * k + 1] = v.y; ra[4 * k + 2] = v.z; ra[4 * k + 3] = v.w;
                rb[4 * k + 0] = w.x; rb[4 * k + 1] = w.y; rb[4 * k + 2] = w.z; rb[4 * k + 3] = w.w;
            }
        }
        if (b < nsteps) vstage(b);
        if (!(DTS_L4_ABLATE & 2) && b > 0) vpass(b - 1);
        __syncthreads();
        if (!(DTS_L4_ABLATE & 1) && b < nsteps) {
            int s = slot0 + lane;
            if (s >= R) s -= R;
            uint32_t *wp = ring + s * CP + hg.col0;
#pragma unroll 1
            for (int pass = 0; pass < (KIND ? 2 : 1); ++pass) {
                // opaque per pass: keeps the compiler from hoisting the ~2 x QMAX
                // position tests out of the walk as long-lived SGPR lane masks
                uint64_t mask = hg.mask;
                int qend = hg.qend;
                asm volatile("" : "+s"(mask), "+s"(qend));
                hdispatch<CVT, CAP, SH>(K.N, ra, rb, pass ? kSelV : kSelU, mask, qend, hco,
                                        wp + pass * (R * CP));
                if (planar2) {                                 // the V plane's window moves down
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        ra[i] = ra[i + 16];
                        rb[i] = rb[i + 16];
                    }
                }
            }
            slot0 += 64;
            if (slot0 >= R) slot0 -= R;
        }
        __syncthreads();
    }
}

} // namespace

// Persistent workgroups pull (frame, job) items from a device counter,
// frame-major so the renditions of one frame run together (source re-reads
// across renditions and strip halos hit L2 / the Infinity Cache).
#ifndef DTS_L4_WAVES
#define DTS_L4_WAVES 3          // waves per SIMD the register budget is cut for (<= 168 VGPRs)
#endif
template <int SRC>
__global__ void __launch_bounds__(kThreads, DTS_L4_WAVES) k_ladder4(const Ladder4Params P)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t ring[];
    volatile int *slot = reinterpret_cast<volatile int *>(ring);   // ring dword 0: idle between items
    for (;;) {
        if (threadIdx.x == 0) *slot = (int)atomicAdd(P.queue, 1u);
        __syncthreads();
        const int item = uni(*slot);
        __syncthreads();
        if (item >= P.nitems) return;
        const int frame = item / P.njobs, jid = item - frame * P.njobs;
        const Job4 J = kload(P.jobs + jid);
        if (J.kind == 0)
            item4<SRC, 0>(P, frame, J, ring);
        else
            item4<SRC, 1>(P, frame, J, ring);
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
