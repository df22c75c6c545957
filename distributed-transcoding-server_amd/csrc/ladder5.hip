// ladder5.hip -- k_ladder5, the v5 ladder kernel: every rendition of an
// 8-bit 4:2:0 source in one persistent launch, the horizontal FIR on the
// matrix cores.
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
//  * H: a 16-output tile of one rendition over 16 source rows is one
//    v_mfma_i32_16x16x64_i8 per 64-column K block and tap half: the int16
//    taps c = 256 hi + lo (hi, lo signed bytes) are the B operands (held in
//    VGPRs for the whole walk), the staged rows the A operand, so
//      sum(src * c) = 256 sum(src' hi) + sum(src' lo) + 128 * 16384
//    exactly in i32 (src' = src - 128; every row's taps sum to 1 << 14);
//    then FFMIN(val >> 7, 32767) by v_cvt_pk_i16_i32 into the int16x2 row
//    pairs of a per-rendition LDS ring;
//  * V: lane = 4 output columns of one row (nv12 chroma: 2 columns of U and
//    V), v_dot2_i32_i16 over the ring's row pairs (quad-major ring: the 4
//    columns of a pair are one ds_read_b128, consecutive pairs 16 B apart,
//    so a window is immediate offsets; slots [0, mirror) are also written
//    past the ring's end so no window wraps), then + 64 << 12 (flat dither),
//    v_ashr_pk_u8_i32 (>> 19, clip to u8) and one dword store per lane.
//  * One barrier per step: H(b+1) of one wave overlaps V(b) of another (the
//    planner sizes the ring so their slots never meet).
#include "dts_internal.h"

namespace dts {

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

__device__ __forceinline__ int dot2(uint32_t a, uint32_t b, int c)
{
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, a), __builtin_bit_cast(short2v, b), c, false);
}

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
__device__ __forceinline__ u32x4 lds_rd128(const uint32_t *lds, uint32_t byte)
{
    return *reinterpret_cast<const u32x4 *>(reinterpret_cast<const uint8_t *>(lds) + byte);
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
    int nplanes, nsteps, srcH, Pb, stage_b, R, M, nunits;
    int L, cpr, ne;
    int lane, wave, t;
};

// This thread's staging loads of a step: kL5MaxLoads 16-B chunks.
struct Loads5 {
    __amdgpu_buffer_rsrc_t rs[2];   // load planes (planar chroma: U, V)
    int64_t pitch[2];
    uint32_t col[kL5MaxLoads];      // byte offset of the chunk in its source row
    int row[kL5MaxLoads];           // staged row (0..15), -1 = no chunk
    uint32_t dst[kL5MaxLoads];      // LDS byte offset of the chunk in stage buffer 0
    int nlp;                        // load planes
};

template <int SRC>
__device__ __forceinline__ void issue_loads(const Loads5 &ld, int b, int srcH, u32x4 (&pre)[kL5MaxLoads])
{
#pragma unroll
    for (int k = 0; k < kL5MaxLoads; ++k) {
        const int lp = ld.nlp == 2 ? (k >> 1) : 0;
        if (ld.row[k] >= 0) {
            const int r = min(kL5Rows * b + ld.row[k], srcH - 1);
            const uint32_t off = (uint32_t)r * (uint32_t)ld.pitch[lp] + ld.col[k];
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

// step b's V rows of every unit -> V staging buffer (b & 1): per row its ring slot, then np4 tap pairs
__device__ __forceinline__ void stage_v(uint32_t *lds, const Kind5 *K, const Walk5 &W, int b)
{
    for (int u = 0; u < W.nunits; ++u) {
        const Unit5 *U = K->unit + u;
        const int32_t *vlim = kld(&U->vlim);
        const int vlo = b > 0 ? kld(vlim + b - 1) : 0, vhi = kld(vlim + b);
        const int np4 = kld(&U->np4), vco = kld(&U->vco), vdw = kld(&U->vco_dw);
        const int stride = 4 + np4;
        uint32_t *dst = lds + vco + (b & 1) * vdw;
        const int32_t *vslot = kld(&U->vslot);
        const uint32_t *vcoef = kld(&U->vcoef);
        for (int i = W.t; i < vhi - vlo; i += 256) {
            const int y = vlo + i;
            dst[i * stride] = (uint32_t)vslot[y];
            const u32x4 *c = reinterpret_cast<const u32x4 *>(vcoef + (int64_t)y * np4);
            for (int g = 0; g < np4 / 4; ++g) *reinterpret_cast<u32x4 *>(dst + i * stride + 4 + 4 * g) = c[g];
        }
    }
}

// One output store of 4 bytes at byte column x of a row (fewer at the plane's right edge).
__device__ __forceinline__ void store4(uint64_t row, int x, int ncols, uint32_t w)
{
    if (ncols >= 4) {
        *GP5(g_u32, row + x) = w;
    } else {
        for (int i = 0; i < ncols; ++i) GP5(g_u8, row + x)[i] = (uint8_t)(w >> (8 * i));
    }
}

// V pass of step b for this wave
__device__ __forceinline__ void vpass(uint32_t *lds, const Ladder5Params &P, const Kind5 *K, const Strip5 *S,
                                      const Walk5 &W, int frame, int b)
{
    int rot = 0;                                           // passes handed out so far (round robin over waves)
    for (int u = 0; u < W.nunits; ++u) {
        const Unit5 *U = K->unit + u;
        const int32_t *vlim = kld(&U->vlim);
        const int vlo = b > 0 ? kld(vlim + b - 1) : 0, nr = kld(vlim + b) - vlo;
        if (nr <= 0) continue;
        const int Q = kld(&S->quads[u]);
        const int tasks = nr * Q;
        const int npass = (tasks + 63) >> 6;
        const int first = (W.wave - rot) & 3;
        rot += npass;
        if (first >= npass || Q <= 0) continue;
        const int mode = kld(&U->mode), np4 = kld(&U->np4), vdw = kld(&U->vco_dw);
        const int rung = kld(&U->rung), dstW = kld(&U->dstW), plane = kld(&U->plane);
        const int x0 = kld(&S->x0[rung]);
        const Ring5 *g0 = K->ring + kld(&U->ring0), *g1 = K->ring + kld(&U->ring1);
        const int r0lds = kld(&g0->lds), r0qs = kld(&g0->qstride), r1lds = kld(&g1->lds);
        const uint32_t vbase = (uint32_t)(kld(&U->vco) + (b & 1) * vdw);
        const int stride = 4 + np4;
        const DevPlanes dst = P.dst[rung];
        const uint64_t pbase = (plane == 0 ? dst.data[0] : (plane == 1 ? dst.data[1] : dst.data[2])) +
                               (uint64_t)frame * dst.fstride;
        const int64_t pitch = plane == 0 ? dst.pitch[0] : (plane == 1 ? dst.pitch[1] : dst.pitch[2]);
        const float rq = 1.0f / (float)Q;
        for (int p = first; p < npass; p += 4) {
            const int task = p * 64 + W.lane;
            const int row = (int)(((float)task + 0.5f) * rq);
            const int q = task - row * Q;
            if (task >= tasks) continue;
            const uint32_t vrow = 4u * (vbase + (uint32_t)(row * stride));
            const int slot = (int)lds[vrow / 4];
            int a0 = 64 << 12, a1 = 64 << 12, a2 = 64 << 12, a3 = 64 << 12;
            if (mode == 0) {
                uint32_t ra = 4u * (uint32_t)(r0lds + q * r0qs + slot * 4);
                for (int g = 0; g < np4; g += 4, ra += 64) {
                    const u32x4 c = lds_rd128(lds, vrow + 16 + 4 * g);
                    const u32x4 d0 = lds_rd128(lds, ra), d1 = lds_rd128(lds, ra + 16);
                    const u32x4 d2 = lds_rd128(lds, ra + 32), d3 = lds_rd128(lds, ra + 48);
                    a0 = dot2(d0.x, c.x, a0); a1 = dot2(d0.y, c.x, a1); a2 = dot2(d0.z, c.x, a2); a3 = dot2(d0.w, c.x, a3);
                    a0 = dot2(d1.x, c.y, a0); a1 = dot2(d1.y, c.y, a1); a2 = dot2(d1.z, c.y, a2); a3 = dot2(d1.w, c.y, a3);
                    a0 = dot2(d2.x, c.z, a0); a1 = dot2(d2.y, c.z, a1); a2 = dot2(d2.z, c.z, a2); a3 = dot2(d2.w, c.z, a3);
                    a0 = dot2(d3.x, c.w, a0); a1 = dot2(d3.y, c.w, a1); a2 = dot2(d3.z, c.w, a2); a3 = dot2(d3.w, c.w, a3);
                }
                // av_clip_uint8(val >> 19) of 4 columns, packed
                const uint32_t lo = __builtin_amdgcn_ashr_pk_u8_i32(a0, a1, 19);
                const uint32_t hi = __builtin_amdgcn_ashr_pk_u8_i32(a2, a3, 19);
                const int x = x0 + 4 * q;
                store4(pbase + (uint64_t)((int64_t)(vlo + row) * pitch), x, dstW - x, (lo & 0xffffu) | (hi << 16));
            } else {
                // nv12 chroma: columns 2q', 2q'+1 of U (ring0) and V (ring1); a0/a1 = U, a2/a3 = V
                const uint32_t qo = 4u * (uint32_t)((q >> 1) * r0qs + slot * 4 + 2 * (q & 1));
                uint32_t ru = 4u * (uint32_t)r0lds + qo, rv = 4u * (uint32_t)r1lds + qo;
                for (int g = 0; g < np4; g += 4, ru += 64, rv += 64) {
                    const u32x4 c = lds_rd128(lds, vrow + 16 + 4 * g);
                    const u32x2 u0 = lds_rd64(lds, ru), u1 = lds_rd64(lds, ru + 16);
                    const u32x2 u2 = lds_rd64(lds, ru + 32), u3 = lds_rd64(lds, ru + 48);
                    const u32x2 v0 = lds_rd64(lds, rv), v1 = lds_rd64(lds, rv + 16);
                    const u32x2 v2 = lds_rd64(lds, rv + 32), v3 = lds_rd64(lds, rv + 48);
                    a0 = dot2(u0.x, c.x, a0); a1 = dot2(u0.y, c.x, a1); a2 = dot2(v0.x, c.x, a2); a3 = dot2(v0.y, c.x, a3);
                    a0 = dot2(u1.x, c.y, a0); a1 = dot2(u1.y, c.y, a1); a2 = dot2(v1.x, c.y, a2); a3 = dot2(v1.y, c.y, a3);
                    a0 = dot2(u2.x, c.z, a0); a1 = dot2(u2.y, c.z, a1); a2 = dot2(v2.x, c.z, a2); a3 = dot2(v2.y, c.z, a3);
                    a0 = dot2(u3.x, c.w, a0); a1 = dot2(u3.y, c.w, a1); a2 = dot2(v3.x, c.w, a2); a3 = dot2(v3.y, c.w, a3);
                }
                const uint32_t lo = __builtin_amdgcn_ashr_pk_u8_i32(a0, a2, 19);   // U0 V0
                const uint32_t hi = __builtin_amdgcn_ashr_pk_u8_i32(a1, a3, 19);   // U1 V1
                const int c0 = x0 + 2 * q;
                const uint64_t r = pbase + (uint64_t)((int64_t)(vlo + row) * pitch);
                if (c0 + 2 <= dstW)
                    *GP5(g_u32, r + 2 * c0) = (lo & 0xffffu) | (hi << 16);
                else
                    *GP5(g_u16, r + 2 * c0) = (uint16_t)lo;
            }
        }
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
    W.stage_b = 4 * kld(&K->stage);
    W.R = kld(&K->R);
    W.M = kld(&K->M);
    W.nunits = kld(&K->nunits);
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
    uint32_t aad[kL5Ent], wad[kL5Ent];
    uint32_t fl = 0;
#pragma unroll
    for (int i = 0; i < kL5Ent; ++i) {
        bh[i] = bl[i] = (v4i){0, 0, 0, 0};
        aad[i] = wad[i] = 0;
        if (i < W.ne) {
            const Ent5 E = kld(ents + i);
            const u32x4 *f = reinterpret_cast<const u32x4 *>(bf + (size_t)E.bfrag * 512);
            bh[i] = __builtin_bit_cast(v4i, f[W.lane]);
            bl[i] = __builtin_bit_cast(v4i, f[64 + W.lane]);
            aad[i] = (uint32_t)(W.stage_b + E.plane * kL5Rows * W.Pb + n * W.Pb + E.soff + 8 * g);
            const Ring5 *rg = K->ring + E.ring;
            const int col = E.col0 + n;
            wad[i] = 4u * (uint32_t)(kld(&rg->lds) + (col >> 2) * kld(&rg->qstride) + 8 * g + (col & 3));
            fl |= (uint32_t)(E.flags & 3) << (2 * i);
        }
    }
    fl = (uint32_t)uni5((int)fl);

    // ---- staging loads of this thread ----
    Loads5 ld;
    {
        const int nlp = (SRC == kSrcPlanar8 && chroma) ? 2 : 1;
        ld.nlp = nlp;
        const int bps = nv12c ? 2 : 1;
        for (int lp = 0; lp < 2; ++lp) {
            const int spl = chroma ? (nv12c ? 1 : 1 + lp) : 0;           // source plane
            const int sp = lp < nlp ? spl : 0;
            const uint64_t base = (sp == 0 ? P.src.data[0] : (sp == 1 ? P.src.data[1] : P.src.data[2])) +
                                  (uint64_t)frame * P.src.fstride;
            const int64_t pitch = sp == 0 ? P.src.pitch[0] : (sp == 1 ? P.src.pitch[1] : P.src.pitch[2]);
            const uint32_t lo = (uint32_t)uni5((int)(uint32_t)base), hi = (uint32_t)uni5((int)(uint32_t)(base >> 32));
            ld.rs[lp] = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), 0,
                                                          uni5((int)(pitch * W.srcH)), 0x00020000);
            ld.pitch[lp] = pitch;
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

    // ---- prologue: block 0 -> stage 0, block 1 in flight ----
    u32x4 pre[kL5MaxLoads];
#pragma unroll
    for (int k = 0; k < kL5MaxLoads; ++k) pre[k] = (u32x4){0, 0, 0, 0};
    issue_loads<SRC>(ld, 0, W.srcH, pre);
    store_stage<SRC>(lds, ld, 0, W, pre, nv12c);
    if (W.nsteps > 1) issue_loads<SRC>(ld, 1, W.srcH, pre);
    __syncthreads();

    const v4i zero = {0, 0, 0, 0}, bias = {kL5Bias, kL5Bias, kL5Bias, kL5Bias};
    int sb = 0;                                            // ring slot of step b's first row pair = (8 b) % R
    for (int b = 0; b < W.nsteps; ++b) {
        // ---- H(b): MFMA tiles of this wave -> rings ----
        {
            const uint32_t boff = (uint32_t)((b & 1) * W.nplanes * kL5Rows * W.Pb);
            const uint32_t soff = (uint32_t)(16 * sb);
            const bool mir = sb < W.M;
            const uint32_t moff = (uint32_t)(16 * W.R);
            // every K block starts fresh accumulators (independent MFMA chains); a
            // tile's earlier K blocks are carried in ch / cl and added at its last one
            v4i ch = zero, cl = zero;
#pragma unroll
            for (int i = 0; i < kL5Ent; ++i) {
                if (i < W.ne) {
                    const uint32_t f = (fl >> (2 * i)) & 3u;
                    const u32x2 x = lds_rd64(lds, aad[i] + boff), y = lds_rd64(lds, aad[i] + boff + 32);
                    const v4i a = __builtin_bit_cast(v4i, (u32x4){x.x, x.y, y.x, y.y});
                    v4i ah = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bh[i], zero, 0, 0, 0);
                    v4i al = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bl[i], (f & 1u) ? bias : zero, 0, 0, 0);
                    if (!(f & 1u)) {
                        ah += ch;
                        al += cl;
                    }
                    if (f & 2u) {
                        const uint32_t p0 = pack_h(ah.x, al.x, ah.y, al.y);    // rows 4g, 4g+1
                        const uint32_t p1 = pack_h(ah.z, al.z, ah.w, al.w);    // rows 4g+2, 4g+3
                        uint32_t *w = lds_at(lds, wad[i] + soff);
                        w[0] = p0;
                        w[4] = p1;
                        if (mir) {
                            uint32_t *m = lds_at(lds, wad[i] + soff + moff);
                            m[0] = p0;
                            m[4] = p1;
                        }
                    } else {
                        ch = ah;
                        cl = al;
                    }
                }
            }
        }
        // ---- V taps of step b, the next block's rows, the loads after it ----
        stage_v(lds, K, W, b);
        if (b + 1 < W.nsteps) {
            store_stage<SRC>(lds, ld, b + 1, W, pre, nv12c);
            if (b + 2 < W.nsteps) issue_loads<SRC>(ld, b + 2, W.srcH, pre);
        }
        __syncthreads();
        // ---- V(b) ----
        vpass(lds, P, K, S, W, frame, b);
        sb += 8;
        if (sb >= W.R) sb -= W.R;
    }
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

int ladder5_blocks_per_cu(int src_kind, int lds_bytes)
{
    switch (src_kind) {
    case kSrcPlanar8: return occ5<kSrcPlanar8>(lds_bytes);
    case kSrcNV12: return occ5<kSrcNV12>(lds_bytes);
    default: return 0;
    }
}

} // namespace dts
