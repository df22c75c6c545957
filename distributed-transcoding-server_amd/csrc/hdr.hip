// hdr.hip -- k_tonemap: HDR10 -> SDR bt709 8-bit 4:2:0 at the output size
// (BASELINE config 3), the stage a reference ffmpeg
// worker gets from
//   zscale=t=linear:npl=N,format=gbrpf32le,zscale=p=bt709,
//   tonemap=<mode>:param=P:desat=D:peak=K,zscale=t=bt709:m=bt709:r=tv,format=yuv420p
// after the libswscale scale (which the ladder kernel runs bit-exactly into a
// p010 intermediate).  Float path: the output must match the double-precision
// restatement (oracle/vf_tonemap_ref.c) within +-1 LSB.
//
// Chroma as vf_zscale has zimg resample it by default (bilinear, chroma location
// "left" = MPEG-2 4:2:0 siting; oracle/vf_tonemap_ref.c states the filter): the
// 4:2:0 chroma is interpolated up to every pixel before the bt2020 matrix, and the
// output Cb/Cr are filtered back down 2:1 (taps 1/4 1/2 1/4 x 1/8 3/8 3/8 1/8).
// A workgroup owns 64 chroma columns x kTmCRows chroma rows: it stages the chroma
// samples it needs (+1 each side) in LDS, converts every luma pixel of its tile
// plus a one-pixel ring (the 2:1 filter's support) keeping the full-resolution
// Cb/Cr in LDS, writes the tile's luma, then filters its chroma outputs from LDS.
// The two transfer curves (PQ EOTF, 6 pow per pixel, and the BT.709 OETF, 3 pow
// per pixel) are 1024-interval tables (built in double on the host, 2 x (kTmLutN
// + 1) floats) staged in LDS and linearly interpolated: measured against the exact
// curves, 2e-4 of the 8-bit outputs move by one LSB, inside the +-1 LSB
// tolerance.
#include "dts_internal.h"

#ifndef DTS_TM_OETF_POW
#define DTS_TM_OETF_POW 0   // 1: BT.709 OETF by v_log / v_exp instead of the LDS table (A/B knob)
#endif
#ifndef DTS_TM_ABLATE
#define DTS_TM_ABLATE 0     // diagnostic bits (wrong output): 1 no ring pass, 2 no chroma 2:1 pass, 4 no pixel math
#endif
#ifndef DTS_TM_UNROLL
#define DTS_TM_UNROLL 0     // 1: both block iterations of a lane unrolled (8 pixels in flight; A/B knob)
#endif

namespace dts {

namespace {

__device__ __forceinline__ float pw(float x, float y)
{
    // x >= 0; v_log_f32 / v_exp_f32 (base 2); log2(0) = -inf -> 0
    return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
}

// table t[0..kTmLutN] of a curve on [0, 1] as chords (intercept, slope) in table units,
// linearly interpolated; the argument arrives pre-scaled by kTmLutN (the scale is
// folded into the producing FMA): clamp (v_med3), truncate, one 8-byte LDS read, one
// fma intercept + x slope (api.cpp tonemap_luts: no fract, the intercept absorbs it)
__device__ __forceinline__ float lut(const float2 *t, float xn)
{
    const float x = __builtin_amdgcn_fmed3f(xn, 0.f, (float)kTmLutN);
    const float2 e = t[(int)x];
    return __builtin_fmaf(x, e.y, e.x);
}
// the PQ table (api.cpp tonemap_luts): x already offset by kTmPqOff and inside the table by
// construction (pixel<>), so no clamp
__device__ __forceinline__ float lut_pq(const float2 *t, float x)
{
    const float2 e = t[(int)x];
    return __builtin_fmaf(x, e.y, e.x);
}

#if DTS_TM_OETF_POW
// BT.709 OETF on [0, 1] (the host table's curve, api.cpp tonemap_luts)
__device__ __forceinline__ float oetf709(float v)
{
    const float x = __builtin_amdgcn_fmed3f(v, 0.f, 1.f);
    const float p = __builtin_fmaf(1.09929682680944f, pw(x, 0.45f), -0.09929682680944f);
    return x < 0.018053968510807f ? 4.5f * x : p;
}
#endif

// global (not flat) loads / stores at integer addresses
template <class T> __device__ __forceinline__ T gld(uint64_t a) { return *(__attribute__((address_space(1))) const T *)a; }
template <class T> __device__ __forceinline__ void gst(uint64_t a, T v) { *(__attribute__((address_space(1))) T *)a = v; }

__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }

#if DTS_TM_OETF_POW
__device__ __forceinline__ float hable(float in)
{
    const float a = 0.15f, b = 0.50f, c = 0.10f, d = 0.20f, e = 0.02f, f = 0.30f;
    return (in * (in * a + b * c) + d * e) * rcp(in * (in * a + b) + d * f) - e / f;
}
#endif

__device__ __forceinline__ float mobius(float in, float j, float peak)
{
    if (in <= j) return in;
    const float a = -j * j * (peak - 1.f) / (j * j - 2.f * j + peak);
    const float b = (j * j - 2.f * j * peak + peak) / fmaxf(peak - 1.f, 1e-6f);
    return (b * b + 2.f * b * j + j * j) / (b - a) * (in + a) / (in + b);
}


// One pixel: 10-bit Y code, chroma (Cb', Cr' already centred) -> bt709 (Y', Cb', Cr').
// The curve and the desaturation switch are template parameters: a branch per pixel
// would keep the compiler from interleaving a thread's four pixels (LUT reads in flight).
template <int MODE, bool DESAT>
__device__ __forceinline__ void pixel(const TonemapParams &P, const float2 *tl, float y10, float2 c, float &Y,
                                      float2 &C)
{
    if (DTS_TM_ABLATE & 4) {
        Y = y10 * (219.f / 1024.f) + 16.5f;
        C = c;
        return;
    }
    const float2 *pq = tl, *oetf = tl + kTmPqN;              // pq already scaled by 10000 / npl
    constexpr float N = (float)kTmLutN;
    constexpr float kr2 = 0.2627f, kb2 = 0.0593f, kg2 = 1.f - kr2 - kb2;
    constexpr float kr7 = 0.2126f, kb7 = 0.0722f, kg7 = 1.f - kr7 - kb7;
    // non-linear R'G'B' x N (the table scale) + kTmPqOff (the PQ table's index offset): from
    // 10-bit codes, y' x N in [-74.8, 1120.5] and Cb, Cr in [-512, 511] / 896, so R' in [-938, 1982],
    // B' in [-1176, 2220], G' in [-505, 1552] (x N): the PQ lookups index [104, 3500] of kTmPqN
    const float yy = __builtin_fmaf(y10, N / 876.f, -64.f * N / 876.f + (float)kTmPqOff);
    const float rp = __builtin_fmaf(c.y, 2.f * (1.f - kr2) * N, yy), bp = __builtin_fmaf(c.x, 2.f * (1.f - kb2) * N, yy);
    // g' = (y' - kr r' - kb b') / kg with r' = y' + 2 (1 - kr) Cr, b' = y' + 2 (1 - kb) Cb
    const float gp = __builtin_fmaf(c.x, -2.f * kb2 * (1.f - kb2) / kg2 * N,
                                    __builtin_fmaf(c.y, -2.f * kr2 * (1.f - kr2) / kg2 * N, yy));
    const float r0 = lut_pq(pq, rp), g0 = lut_pq(pq, gp), b0 = lut_pq(pq, bp);
    const float r = P.m[0] * r0 + P.m[1] * g0 + P.m[2] * b0;
    const float g = P.m[3] * r0 + P.m[4] * g0 + P.m[5] * b0;
    const float b = P.m[6] * r0 + P.m[7] * g0 + P.m[8] * b0;
    // vf_tonemap.c tonemap(), desaturation as one affine map per channel (round 6): MIX(x, luma,
    // ob) = u x + ol with u = 1 - ob and ol = ob luma, where ob = max(luma - desat, 1e-6) /
    // max(luma, 1e-6); ol = min(t, luma) for t = max(luma - desat, 1e-6) (luma >= 1e-6: t;
    // below: luma).  u >= 0, so sig = max(r', g', b') = u max(r, g, b) + ol, and the final
    // r' sig / sig0 folds into the OETF argument as one fma per channel: r (u k) + ol k
    float u = 1.f, ol = 0.f, sig0;
    const float mx = __builtin_fmaxf(__builtin_fmaxf(r, g), b);
    if (DESAT) {
        const float luma = kr7 * r + kg7 * g + kb7 * b;
        const float lm = fmaxf(luma, 1e-6f), t = fmaxf(luma - P.desat, 1e-6f);
        u = (lm - t) * rcp(lm);                               // (v_rcp: an IEEE divide is ~10 VALU)
        ol = fminf(t, luma);
        sig0 = fmaxf(__builtin_fmaf(u, mx, ol), 1e-6f);
    } else {
        sig0 = fmaxf(mx, 1e-6f);
    }
    float sig = sig0;
    switch (MODE) {
    case DTS_TM_LINEAR: sig = sig * P.param / P.peak; break;
    case DTS_TM_GAMMA:
        sig = sig > 0.05f ? pw(sig / P.peak, 1.f / P.param) : sig * pw(0.05f / P.peak, 1.f / P.param) / 0.05f;
        break;
    case DTS_TM_CLIP: sig = fminf(fmaxf(sig * P.param, 0.f), 1.f); break;
    case DTS_TM_REINHARD: sig = sig / (sig + P.param) * (P.peak + P.param) / P.peak; break;
    case DTS_TM_HABLE: break;                                 // folded into k below
    case DTS_TM_MOBIUS: sig = mobius(sig, P.param, P.peak); break;
    default: break;
    }
    float rr, gg, bb;
#if DTS_TM_OETF_POW
    (void)oetf;
    const float k = (MODE == DTS_TM_HABLE ? hable(sig0) * P.inv_hpeak : sig) * rcp(sig0);
    rr = oetf709(__builtin_fmaf(r, u, ol) * k);
    gg = oetf709(__builtin_fmaf(g, u, ol) * k);
    bb = oetf709(__builtin_fmaf(b, u, ol) * k);
#else
    // k = sig / sig0 x N.  hable: hable(x) = (x (Ax + CB) + DE) / (x (Ax + B) + DF) - E / F, and the
    // constant terms cancel exactly (DE - (E / F) DF = 0), so hable(x) / x = (A (1 - E/F) x +
    // B (C - E/F)) / (x (Ax + B) + DF): k = (hk1 sig0 + hk0) / den with N / hable(peak) folded
    // into hk1, hk0 (api.cpp tonemap_params) -- one reciprocal, no cancellation near 0
    float k;
    if (MODE == DTS_TM_HABLE) {
        const float den = __builtin_fmaf(sig0, __builtin_fmaf(sig0, 0.15f, 0.50f), 0.06f);
        k = __builtin_fmaf(sig0, P.hk1, P.hk0) * rcp(den);
    } else {
        k = sig * (N * rcp(sig0));
    }
    if (DESAT) {
        const float ku = u * k, ko = ol * k;
        rr = lut(oetf, __builtin_fmaf(r, ku, ko));
        gg = lut(oetf, __builtin_fmaf(g, ku, ko));
        bb = lut(oetf, __builtin_fmaf(b, ku, ko));
    } else {
        rr = lut(oetf, r * k);
        gg = lut(oetf, g * k);
        bb = lut(oetf, b * k);
    }
#endif
    // Y returned as 219 Y' + 16.5 (r=tv) or 255 Y' + 0.5 (r=pc): the quantiser's scale and
    // rounding half folded into the weights (api.cpp tonemap_params), so q8y is one truncation;
    // Cb' = (B' - Y') / (2 (1 - kb)) from that
    constexpr float sb = 1.f / (2.f * (1.f - kb7)), sr = 1.f / (2.f * (1.f - kr7));
    Y = __builtin_fmaf(P.qy[2], bb, __builtin_fmaf(P.qy[1], gg, __builtin_fmaf(P.qy[0], rr, P.qy[3])));
    C = make_float2(__builtin_fmaf(bb, sb, __builtin_fmaf(Y, P.qcb[0], P.qcb[1])),
                    __builtin_fmaf(rr, sr, __builtin_fmaf(Y, P.qcr[0], P.qcr[1])));
}

// Y' = kr R' + kg G' + kb B' with R', G', B' in [0, 1] (the OETF table's values, or oetf709's):
// pixel<> returns 219 Y' + 16.5 in [16.5, 235.5] or 255 Y' + 0.5 in [0.5, 255.5], so the
// quantiser is a truncation, no clip
__device__ __forceinline__ uint32_t q8y(float Y) { return (uint32_t)Y; }
// Cb', Cr' in [-1/2, 1/2]: 224 C + 128.5 in [16.5, 240.5]; 255 C + 128.5 reaches 256 at C = 1/2
__device__ __forceinline__ int q8c(const TonemapParams &P, float C)
{
    return (int)__builtin_fminf(__builtin_fmaf(P.qc, C, 128.5f), 255.f);
}

} // namespace

constexpr int kTmCRows = 8;                  // chroma rows per tile (16 luma rows)
constexpr int kTmTiles = 8;                  // tiles per workgroup, walked top to bottom (one table load)
constexpr int kTmLH = 2 * kTmCRows + 2;      // luma rows of a tile + ring: 16 + 2
constexpr int kTmLP = 130;                   // output-chroma row pitch (16-B rows): columns x0 - 1 .. x0 + 127 at 1 .. 129
constexpr int kTmCW = 66, kTmCH = kTmCRows + 2;        // chroma samples staged: 64 + 2 columns, 8 + 2 rows

// LDS: tables 16.4 KB + staged chroma 5.3 KB + output chroma 18.7 KB = 40.4 KB (four
// workgroups per CU; 32.2 KB, five, with DTS_TM_OETF_POW).  Tiles whose 128 x 16 luma block lies inside the picture (all
// but the bottom / right edge tiles) take the block path: one 2 x 2 luma block per
// thread, its chroma interpolated from the 3 x 2 staged samples it shares, two 4-byte
// luma loads, 16-byte (Cb, Cr) x 2 LDS stores; edge tiles and the one-pixel ring take
// the per-pixel path with the clamps.  The top ring row of tile t > 0 is the previous
// tile's last luma row, carried in LDS rather than recomputed.
template <int MODE, bool DESAT>
__global__ void __launch_bounds__(256) k_tonemap(const TonemapParams P)
{
    constexpr int kTabN = kTmPqN + (DTS_TM_OETF_POW ? 0 : kTmLutN + 1);   // PQ, then OETF
    constexpr int kRow = 129;                       // ring row: columns x0 - 1 .. x0 + 127
    constexpr int kCin = kTmCH * kTmCW;             // staged chroma samples per tile (660: 3 per thread)
    __shared__ float2 tl[kTabN];
    __shared__ float2 cin[kTmCH][kTmCW];            // (Cb', Cr') centred, 4:2:0
    __shared__ __attribute__((aligned(16))) float2 cc[kTmLH][kTmLP];   // output (Cb, Cr) at full resolution
    const int t = threadIdx.x, f = blockIdx.z;
    const int cw = P.w >> 1, ch = P.h >> 1;
    const int cx0 = blockIdx.x * 64;
    const int x0 = 2 * cx0;
    const uint64_t sf = (uint64_t)f * P.src.fstride, df = (uint64_t)f * P.dst.fstride;
    const uint64_t sy0 = P.src.data[0] + sf, sc0 = P.src.data[1] + sf;
    const int lp = P.src.pitch[0], cp = P.src.pitch[1];
    const bool a4 = ((P.src.data[0] + sf) & 3) == 0 && (P.src.pitch[0] & 3) == 0;
    for (int i = t; i < kTabN; i += 256) tl[i] = P.lut[i];
    // a thread's staged chroma samples (rows / columns fixed over the tiles) and block positions
    int cr[3], cxo[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int i = t + 256 * k, r = i / kTmCW, c = i - r * kTmCW;
        cr[k] = r;
        cxo[k] = 4 * min(max(cx0 - 1 + c, 0), cw - 1);
    }
    const int byl0 = t >> 6, bxl = t & 63;          // block items t and t + 256: rows byl0, byl0 + 4
    // ring item t of a tile: (lx, ly) of the ring -- rows y0 - 1 (first tile only) and y0 + 16,
    // columns x0 - 1 .. x0 + 127, and column x0 - 1 of the 16 rows between
    auto ring_at = [&](int i, int top, int &lx, int &ly) {
        if (i < top) {
            ly = 0;
            lx = i;
        } else if (i < top + kRow) {
            ly = kTmLH - 1;
            lx = i - top;
        } else {
            ly = 1 + (i - top - kRow);
            lx = 0;
        }
    };
    auto luma_at = [&](int xr, int yr) -> float {
        const int x = min(max(xr, 0), P.w - 1), y = min(max(yr, 0), P.h - 1);
        return (float)(gld<uint16_t>(sy0 + (uint64_t)y * lp + 2 * x) >> 6);
    };
    // loads of tile `tile` into registers: its staged chroma, its block path luma, its ring item t
    uint32_t ncin[3] = {0, 0, 0}, nl[4] = {0, 0, 0, 0};
    float nring = 0.f;
    auto fetch = [&](int tile) {
        const int cy0 = (blockIdx.y * kTmTiles + tile) * kTmCRows, y0 = 2 * cy0;
#pragma unroll
        for (int k = 0; k < 3; ++k)
            if (k < 2 || t + 512 < kCin)
                ncin[k] = gld<uint32_t>(sc0 + (uint64_t)min(max(cy0 - 1 + cr[k], 0), ch - 1) * cp + cxo[k]);
        if (a4 && x0 + 128 <= P.w && y0 + 16 <= P.h) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                const uint64_t ys = sy0 + (uint64_t)(y0 + 2 * (byl0 + 4 * kb)) * lp + 4 * (x0 / 2 + bxl);
                nl[2 * kb] = gld<uint32_t>(ys);
                nl[2 * kb + 1] = gld<uint32_t>(ys + lp);
            }
        }
        const int top = tile ? 0 : kRow;
        if (t < top + kRow + 2 * kTmCRows) {
            int lx, ly;
            ring_at(t, top, lx, ly);
            nring = luma_at(x0 - 1 + lx, y0 - 1 + ly);
        }
    };
    fetch(0);
    for (int tile = 0; tile < kTmTiles; ++tile) {
    const int cy0 = (blockIdx.y * kTmTiles + tile) * kTmCRows, y0 = 2 * cy0;
    if (cy0 >= ch) break;
    const bool blk = a4 && x0 + 128 <= P.w && y0 + 16 <= P.h;
    uint32_t l[4], vc[3];
    float yring = nring;
#pragma unroll
    for (int k = 0; k < 4; ++k) l[k] = nl[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) vc[k] = ncin[k];
    if (tile) __syncthreads();                      // the previous tile's chroma pass is done with cin / cc
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (k < 2 || t + 512 < kCin)
            (&cin[0][0])[t + 256 * k] = make_float2((float)((int)((vc[k] & 0xffffu) >> 6) - 512) * (1.f / 896.f),
                                                     (float)((int)(vc[k] >> 22) - 512) * (1.f / 896.f));
    if (tile)                                       // top ring row = the previous tile's luma row y0 - 1
        for (int i = t; i < kTmLP; i += 256) cc[0][i] = cc[kTmLH - 2][i];
    __syncthreads();
    // the next tile's loads fly during this tile's conversion
    if (tile + 1 < kTmTiles && cy0 + kTmCRows < ch) fetch(tile + 1);
    // one luma pixel (clamped into the picture): zimg bilinear up (chroma location left:
    // columns j, j + 1 at weights 1 - fx, fx; rows k, k2 at 3/4, 1/4) + the conversion
    auto pixc = [&](int xr, int yr, float y10, float &Yv, float2 &C) {
        const int x = min(max(xr, 0), P.w - 1), y = min(max(yr, 0), P.h - 1);
        const int ky = y >> 1, k = min(ky, ch - 1), k2 = min(max((y & 1) ? ky + 1 : ky - 1, 0), ch - 1);
        const int j = x >> 1, j1 = min(min(j + 1, cw - 1), cx0 + 64);   // (x even: j1 unused, fx = 0)
        const int lj = j - (cx0 - 1), lj1 = j1 - (cx0 - 1), lk = k - (cy0 - 1), lk2 = k2 - (cy0 - 1);
        const float fx = (x & 1) ? 0.5f : 0.f;
        const float2 a0 = cin[lk][lj], a1 = cin[lk][lj1], b0 = cin[lk2][lj], b1 = cin[lk2][lj1];
        const float2 c = make_float2(0.75f * (a0.x + fx * (a1.x - a0.x)) + 0.25f * (b0.x + fx * (b1.x - b0.x)),
                                     0.75f * (a0.y + fx * (a1.y - a0.y)) + 0.25f * (b0.y + fx * (b1.y - b0.y)));
        pixel<MODE, DESAT>(P, tl, y10, c, Yv, C);
    };
    if (blk) {
        // block path: the 2 x 2 luma block of chroma sample (cx0 + bxl, cy0 + byl); staged
        // rows byl .. byl + 2 = chroma rows by - 1 .. by + 1, columns bxl + 1, bxl + 2 = bx, bx + 1
#if DTS_TM_UNROLL
#pragma unroll
#endif
        for (int kb = 0; kb < 64 * kTmCRows / 256; ++kb) {
            const int byl = byl0 + 4 * kb;
            const float2 m0 = cin[byl][bxl + 1], m1 = cin[byl][bxl + 2];
            const float2 a0 = cin[byl + 1][bxl + 1], a1 = cin[byl + 1][bxl + 2];
            const float2 p0 = cin[byl + 2][bxl + 1], p1 = cin[byl + 2][bxl + 2];
            const float2 ah = make_float2(a0.x + 0.5f * (a1.x - a0.x), a0.y + 0.5f * (a1.y - a0.y));
            const float2 mh = make_float2(m0.x + 0.5f * (m1.x - m0.x), m0.y + 0.5f * (m1.y - m0.y));
            const float2 ph = make_float2(p0.x + 0.5f * (p1.x - p0.x), p0.y + 0.5f * (p1.y - p0.y));
            const float2 c[4] = {make_float2(0.75f * a0.x + 0.25f * m0.x, 0.75f * a0.y + 0.25f * m0.y),
                                 make_float2(0.75f * ah.x + 0.25f * mh.x, 0.75f * ah.y + 0.25f * mh.y),
                                 make_float2(0.75f * a0.x + 0.25f * p0.x, 0.75f * a0.y + 0.25f * p0.y),
                                 make_float2(0.75f * ah.x + 0.25f * ph.x, 0.75f * ah.y + 0.25f * ph.y)};
            const int xa = x0 + 2 * bxl, ya = y0 + 2 * byl;
            const uint32_t l0 = l[2 * kb], l1 = l[2 * kb + 1];
            const float y10[4] = {(float)__builtin_amdgcn_ubfe(l0, 6, 10), (float)(l0 >> 22),
                                  (float)__builtin_amdgcn_ubfe(l1, 6, 10), (float)(l1 >> 22)};
            float Yv[4];
            float2 C[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) pixel<MODE, DESAT>(P, tl, y10[q], c[q], Yv[q], C[q]);
#pragma unroll
            for (int r = 0; r < 2; ++r)
                *reinterpret_cast<float4 *>(&cc[1 + 2 * byl + r][2 + 2 * bxl]) =
                    make_float4(C[2 * r].x, C[2 * r].y, C[2 * r + 1].x, C[2 * r + 1].y);
            const uint64_t yd = P.dst.data[0] + df + (uint64_t)ya * P.dst.pitch[0] + xa;
            gst<uint16_t>(yd, (uint16_t)(q8y(Yv[0]) | (q8y(Yv[1]) << 8)));
            gst<uint16_t>(yd + P.dst.pitch[0], (uint16_t)(q8y(Yv[2]) | (q8y(Yv[3]) << 8)));
        }
    } else {
        // per-pixel path (edge tiles): out-of-picture blocks keep the clamped values the
        // 2:1 filter of the last chroma row / column reads
        for (int i = t; i < 64 * kTmCRows; i += 256) {
            const int byl = i >> 6, bx = i & 63;
            float Yv[4];
            float2 C[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int xr = x0 + 2 * bx + (q & 1), yr = y0 + 2 * byl + (q >> 1);
                pixc(xr, yr, luma_at(xr, yr), Yv[q], C[q]);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) cc[1 + 2 * byl + (q >> 1)][2 + 2 * bx + (q & 1)] = C[q];
            const int xa = x0 + 2 * bx, ya = y0 + 2 * byl;
            if (xa < P.w && ya < P.h) {                     // w, h even: the whole block is inside
                const uint64_t yd = P.dst.data[0] + df + (uint64_t)ya * P.dst.pitch[0] + xa;
                gst<uint16_t>(yd, (uint16_t)(q8y(Yv[0]) | (q8y(Yv[1]) << 8)));
                gst<uint16_t>(yd + P.dst.pitch[0], (uint16_t)(q8y(Yv[2]) | (q8y(Yv[3]) << 8)));
            }
        }
    }
    // ... and the ring the 2:1 filter reads (chroma only), in the same phase: item t with its
    // luma fetched a tile ahead; the first tile's 274 items leave 18 for a second round
    if (!(DTS_TM_ABLATE & 1)) {
        const int top = tile ? 0 : kRow, nr = top + kRow + 2 * kTmCRows;
        for (int i = t; i < nr; i += 256) {
            int lx, ly;
            ring_at(i, top, lx, ly);
            float Yv;
            float2 C;
            pixc(x0 - 1 + lx, y0 - 1 + ly, i == t ? yring : luma_at(x0 - 1 + lx, y0 - 1 + ly), Yv, C);
            cc[ly][1 + lx] = C;
        }
    }
    __syncthreads();
    // chroma 2:1 (location left): columns 2 bx - 1 .. 2 bx + 1 (indices 2 rx + 1 .. 2 rx + 3),
    // rows 2 by - 1 .. 2 by + 2 (ring row 0 = y0 - 1)
    constexpr float wy[4] = {0.125f, 0.375f, 0.375f, 0.125f};
    for (int i = t; i < ((DTS_TM_ABLATE & 2) ? 0 : 64 * kTmCRows); i += 256) {
        const int ry = i >> 6, rx = i & 63;
        const int bx = cx0 + rx, by = cy0 + ry;
        if (bx >= cw || by >= ch) continue;
        float sb = 0.f, sr = 0.f;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const float2 l = cc[2 * ry + a][2 * rx + 1];
            const float4 mr = *reinterpret_cast<const float4 *>(&cc[2 * ry + a][2 * rx + 2]);
            sb += wy[a] * (0.25f * l.x + 0.5f * mr.x + 0.25f * mr.z);
            sr += wy[a] * (0.25f * l.y + 0.5f * mr.y + 0.25f * mr.w);
        }
        const int u = q8c(P, sb), v = q8c(P, sr);
        if (P.dst_fmt == DTS_FMT_NV12) {
            gst<uint16_t>(P.dst.data[1] + df + (uint64_t)by * P.dst.pitch[1] + 2 * bx, (uint16_t)(u | (v << 8)));
        } else {
            gst<uint8_t>(P.dst.data[1] + df + (uint64_t)by * P.dst.pitch[1] + bx, (uint8_t)u);
            gst<uint8_t>(P.dst.data[2] + df + (uint64_t)by * P.dst.pitch[2] + bx, (uint8_t)v);
        }
    }
    }
}

// ---------------------------------------------------------------------------------------
// k_tonemap_w (round 5, the default): the same conversion as a column walk.  A wave owns 63
// chroma columns of one vertical chunk of the picture (lane 0 overlaps the strip to its left)
// and walks it top to bottom, one chroma row (a 2 x 2 luma block per lane) per step:
//  * the chroma a step interpolates (rows s - 1, s, s + 1 of columns cx and cx + 1) comes from
//    registers: rows s - 1 and s carried, row s + 1 loaded a step ahead with the block's luma;
//  * the 2:1 chroma filter of output row s - 1 reads full-resolution rows 2s - 3 .. 2s (three
//    carried in registers, the fourth this step's top row) at columns 2cx - 1 .. 2cx + 1, the
//    left one from lane - 1 (DPP wave_shr: every value is shifted once, when it is made);
//  * no LDS but the two transfer tables, no barrier after they are loaded, no ring: the
//    one-pixel ring of the tiled kernel (14 % more conversions) becomes lane 0's block (1/64)
//    and one extra block row per chunk edge.
// The arithmetic per pixel is pixel<> and the chroma / 2:1 expressions of k_tonemap above,
// term for term, so both kernels give the same bytes.
// chunk height and workgroup size (round-5 A/B on cfg3, tools/r05_tmab.sh: chunks of 34 / 68 / 135
// rows 79.5 k / 79.5 k / 78.7 k fps, 4-wave workgroups 79.1 k, column cx + 1 through DPP instead of
// a second load 78.4 k)
#ifndef DTS_TW_ROWS
#define DTS_TW_ROWS 68
#endif
#ifndef DTS_TW_WAVES
#define DTS_TW_WAVES 8
#endif
constexpr int kTwCols = 63;                      // output chroma columns per wave
constexpr int kTwRows = DTS_TW_ROWS;             // chroma rows per chunk (1080p: 8 chunks)
constexpr int kTwWaves = DTS_TW_WAVES;           // waves per workgroup (one table load)

__device__ __forceinline__ float shr1(float x)   // lane l gets lane l - 1's value (lane 0: 0)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x138, 0xf, 0xf, false));
}

__device__ __forceinline__ float2 cdec(uint32_t v)   // one p010 (Cb, Cr) pair, centred
{
    return make_float2((float)((int)((v & 0xffffu) >> 6) - 512) * (1.f / 896.f), (float)((int)(v >> 22) - 512) * (1.f / 896.f));
}

// a plane of this frame as a buffer resource (wave-uniform base and size): the row offsets of a
// step are scalar (soffset) and each lane's column offset is fixed for the walk (voffset), so no
// vector address arithmetic is left in the loop
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(uint64_t base, int64_t bytes)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)base);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(base >> 32));
    const int n = __builtin_amdgcn_readfirstlane((int)min(bytes, (int64_t)0x7fffffff));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

template <int MODE, bool DESAT>
__global__ void __launch_bounds__(64 * kTwWaves) k_tonemap_w(const TonemapParams P, int nstrips, int nchunks)
{
    constexpr int kTabN = kTmPqN + (DTS_TM_OETF_POW ? 0 : kTmLutN + 1);   // PQ, then OETF
    __shared__ float2 tl[kTabN];
    for (int i = threadIdx.x; i < kTabN; i += 64 * kTwWaves) tl[i] = P.lut[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int item = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * kTwWaves + (threadIdx.x >> 6)));
    if (item >= nstrips * nchunks) return;
    const int strip = item % nstrips, chunk = item / nstrips, f = blockIdx.z;
    const int cw = P.w >> 1, ch = P.h >> 1;
    const int r0 = chunk * kTwRows, r1 = min(r0 + kTwRows, ch);
    const int cx = strip * kTwCols + lane - 1;                // lane 0: the left neighbour's last column
    const bool out_col = lane > 0 && cx < cw;
    // the block's two luma columns 2 cx, 2 cx + 1, clamped into the picture as pixc clamps them:
    // lane 0 of the first strip (cx = -1) converts column 0 twice (chroma column 0, fx 0); lanes
    // past the picture (last strip) read its last block and store nothing
    const int cxc = min(max(cx, 0), cw - 1);
    const int xL = 2 * cxc;
    const float fx = cx < 0 ? 0.f : 0.5f;                    // the right column's weight of chroma column cx + 1
    const int jA = cxc, jB = min(cxc + 1, cw - 1);
    const bool lsplit = cx >= 0;                             // two luma samples (else column 0 twice)
    const uint64_t sf = (uint64_t)f * P.src.fstride, df = (uint64_t)f * P.dst.fstride;
    const int lp = (int)P.src.pitch[0], cp = (int)P.src.pitch[1];
    const __amdgpu_buffer_rsrc_t rY = plane_rsrc(P.src.data[0] + sf, (int64_t)lp * P.h);
    const __amdgpu_buffer_rsrc_t rC = plane_rsrc(P.src.data[1] + sf, (int64_t)cp * ch);
    const int dp0 = (int)P.dst.pitch[0], dp1 = (int)P.dst.pitch[1], dp2 = (int)P.dst.pitch[2];
    const bool nv12 = P.dst_fmt == DTS_FMT_NV12;
    const __amdgpu_buffer_rsrc_t wY = plane_rsrc(P.dst.data[0] + df, (int64_t)dp0 * P.h);
    const __amdgpu_buffer_rsrc_t wU = plane_rsrc(P.dst.data[1] + df, (int64_t)dp1 * ch);
    const __amdgpu_buffer_rsrc_t wV = plane_rsrc(P.dst.data[nv12 ? 1 : 2] + df, (int64_t)(nv12 ? dp1 : dp2) * ch);
    const int oA = 4 * jA, oB = 4 * jB, oL = 2 * xL;        // this lane's byte in a chroma / luma row
    auto crow = [&](int r, uint32_t &a, uint32_t &b) {     // chroma row r (clamped), columns jA, jB
        const int so = min(max(r, 0), ch - 1) * cp;
        a = __builtin_amdgcn_raw_buffer_load_b32(rC, oA, so, 0);
        b = __builtin_amdgcn_raw_buffer_load_b32(rC, oB, so, 0);
    };
    auto lrow = [&](int y) -> uint32_t { return __builtin_amdgcn_raw_buffer_load_b32(rY, oL, y * lp, 0); };
    const int s0 = r0 > 0 ? r0 - 1 : 0, s1 = r1 < ch ? r1 : ch - 1;
    // chroma input rows s - 1 (m) and s (a) carried decoded and interpolated to column cx + 1/2
    // (the h values), row s + 1 (p) and the block's luma loaded raw a step ahead
    uint32_t pA, pB, l0, l1;
    float2 m0, mh, a0, ah;
    {
        uint32_t xA, xB;
        crow(s0 - 1, xA, xB);
        const float2 u0 = cdec(xA), u1 = cdec(xB);
        m0 = u0;
        mh = make_float2(u0.x + fx * (u1.x - u0.x), u0.y + fx * (u1.y - u0.y));
        crow(s0, xA, xB);
        const float2 v0 = cdec(xA), v1 = cdec(xB);
        a0 = v0;
        ah = make_float2(v0.x + fx * (v1.x - v0.x), v0.y + fx * (v1.y - v0.y));
    }
    crow(s0 + 1, pA, pB);
    l0 = lrow(2 * s0);
    l1 = lrow(2 * s0 + 1);
    // carried output chroma of full-resolution rows 2s - 3 (b2), 2s - 2 (t1), 2s - 1 (b1), each
    // already as the 2:1 filter's horizontal sum 1/4 (2cx - 1) + 1/2 (2cx) + 1/4 (2cx + 1)
    float2 b2, t1, b1;
    constexpr float wy[4] = {0.125f, 0.375f, 0.375f, 0.125f};
    auto hsum = [&](float2 l, float2 m, float2 r) {
        return make_float2(0.25f * l.x + 0.5f * m.x + 0.25f * r.x, 0.25f * l.y + 0.5f * m.y + 0.25f * r.y);
    };
    auto emit = [&](int by, float2 a, float2 b, float2 c, float2 d) {
        if (by < r0 || by >= r1) return;
        const float2 h[4] = {a, b, c, d};
        float sb = 0.f, sr = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            sb += wy[k] * h[k].x;
            sr += wy[k] * h[k].y;
        }
        const int u = q8c(P, sb), v = q8c(P, sr);
        if (!out_col) return;
        if (nv12) {
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(u | (v << 8)), wU, 2 * cx, by * dp1, 0);
        } else {
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)u, wU, cx, by * dp1, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, wV, cx, by * dp2, 0);
        }
    };
    for (int s = s0; s <= s1; ++s) {
        const float2 p0 = cdec(pA), p1 = cdec(pB);
        const float2 ph = make_float2(p0.x + fx * (p1.x - p0.x), p0.y + fx * (p1.y - p0.y));
        const uint32_t q0 = l0, q1 = l1;
        // the next step's loads fly during this step's conversion
        if (s < s1) {
            crow(s + 2, pA, pB);
            l0 = lrow(2 * s + 2);
            l1 = lrow(2 * s + 3);
        }
        const float2 c[4] = {make_float2(0.75f * a0.x + 0.25f * m0.x, 0.75f * a0.y + 0.25f * m0.y),
                             make_float2(0.75f * ah.x + 0.25f * mh.x, 0.75f * ah.y + 0.25f * mh.y),
                             make_float2(0.75f * a0.x + 0.25f * p0.x, 0.75f * a0.y + 0.25f * p0.y),
                             make_float2(0.75f * ah.x + 0.25f * ph.x, 0.75f * ah.y + 0.25f * ph.y)};
        m0 = a0;
        mh = ah;
        a0 = p0;
        ah = ph;
        const float y0 = (float)__builtin_amdgcn_ubfe(q0, 6, 10), y2 = (float)__builtin_amdgcn_ubfe(q1, 6, 10);
        const float y10[4] = {y0, lsplit ? (float)(q0 >> 22) : y0, y2, lsplit ? (float)(q1 >> 22) : y2};
        float Yv[4];
        float2 C[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) pixel<MODE, DESAT>(P, tl, y10[q], c[q], Yv[q], C[q]);
        if (s >= r0 && s < r1 && out_col) {
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(q8y(Yv[0]) | (q8y(Yv[1]) << 8)), wY, 2 * cx, 2 * s * dp0, 0);
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(q8y(Yv[2]) | (q8y(Yv[3]) << 8)), wY, 2 * cx,
                                                  (2 * s + 1) * dp0, 0);
        }
        // this step's rows as horizontal sums, column 2cx - 1 from lane - 1 (all lanes active here)
        const float2 ht = hsum(make_float2(shr1(C[1].x), shr1(C[1].y)), C[0], C[1]);
        const float2 hb = hsum(make_float2(shr1(C[3].x), shr1(C[3].y)), C[2], C[3]);
        if (s == 0) {                                         // row -1 clamps to row 0
            b2 = ht;
        } else if (s > s0) {
            emit(s - 1, b2, t1, b1, ht);
            b2 = b1;
        }
        t1 = ht;
        b1 = hb;
    }
    if (r1 == ch)                                             // row h clamps to row h - 1
        emit(ch - 1, b2, t1, b1, b1);
}

hipError_t launch_tonemap_w(const TonemapParams &p, hipStream_t s)
{
    const int cw = p.w / 2, ch = p.h / 2;
    const int nstrips = (cw + kTwCols - 1) / kTwCols, nchunks = (ch + kTwRows - 1) / kTwRows;
    const dim3 grid((unsigned)((nstrips * nchunks + kTwWaves - 1) / kTwWaves), 1, (unsigned)p.nframes);
    const bool ds = p.desat > 0.f;
#define DTS_TM_CASE(m)                                                                                               \
    case m:                                                                                                          \
        if (ds) hipLaunchKernelGGL((k_tonemap_w<m, true>), grid, dim3(64 * kTwWaves), 0, s, p, nstrips, nchunks);   \
        else hipLaunchKernelGGL((k_tonemap_w<m, false>), grid, dim3(64 * kTwWaves), 0, s, p, nstrips, nchunks);     \
        break;
    switch (p.mode) {
    DTS_TM_CASE(DTS_TM_NONE)
    DTS_TM_CASE(DTS_TM_LINEAR)
    DTS_TM_CASE(DTS_TM_GAMMA)
    DTS_TM_CASE(DTS_TM_CLIP)
    DTS_TM_CASE(DTS_TM_REINHARD)
    DTS_TM_CASE(DTS_TM_HABLE)
    DTS_TM_CASE(DTS_TM_MOBIUS)
    default: return hipErrorInvalidValue;
    }
#undef DTS_TM_CASE
    return hipGetLastError();
}

hipError_t launch_tonemap(const TonemapParams &p, hipStream_t s)
{
    const int rows = kTmCRows * kTmTiles;
    const dim3 grid((unsigned)((p.w / 2 + 63) / 64), (unsigned)((p.h / 2 + rows - 1) / rows), (unsigned)p.nframes);
    const bool ds = p.desat > 0.f;
#define DTS_TM_CASE(m)                                                                                               \
    case m:                                                                                                          \
        if (ds) hipLaunchKernelGGL((k_tonemap<m, true>), grid, dim3(256), 0, s, p);                                 \
        else hipLaunchKernelGGL((k_tonemap<m, false>), grid, dim3(256), 0, s, p);                                   \
        break;
    switch (p.mode) {
    DTS_TM_CASE(DTS_TM_NONE)
    DTS_TM_CASE(DTS_TM_LINEAR)
    DTS_TM_CASE(DTS_TM_GAMMA)
    DTS_TM_CASE(DTS_TM_CLIP)
    DTS_TM_CASE(DTS_TM_REINHARD)
    DTS_TM_CASE(DTS_TM_HABLE)
    DTS_TM_CASE(DTS_TM_MOBIUS)
    default: return hipErrorInvalidValue;
    }
#undef DTS_TM_CASE
    return hipGetLastError();
}

} // namespace dts
