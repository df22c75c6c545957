// hdr.hip -- k_tonemap: HDR10 -> SDR bt709 8-bit 4:2:0 at the output size
// (BASELINE config 3), the stage a reference ffmpeg
// worker gets from
//   zscale=t=linear:npl=N,format=gbrpf32le,zscale=p=bt709,
//   tonemap=<mode>:param=P:desat=D:peak=K,zscale=t=bt709:m=bt709:r=tv,format=yuv420p
// after the libswscale scale (which the ladder kernel runs bit-exactly into a
// p010 intermediate).  Float path: the output must match the double-precision
// restatement (oracle/vf_tonemap_ref.c) within +-1 LSB.
//
// One lane = one 2x2 luma block and its chroma sample: two dword luma loads
// (row pair), one dword U16V16 load, 4 pixel conversions, 2 x u16 luma stores
// and the chroma mean.  Lanes of a wave take consecutive blocks, so every
// load and store of the wave is one contiguous run; a workgroup walks 16 block
// rows of a 64-block column strip.  The two transfer curves (PQ EOTF, 6 pow
// per pixel, and the BT.709 OETF, 3 pow per pixel) are 1024-interval tables
// (built in double on the host, 2 x (kTmLutN + 1) floats) staged in LDS once per
// workgroup and linearly interpolated: measured against the exact curves,
// 2e-4 of the 8-bit outputs move by one LSB, inside the +-1 LSB
// tolerance, and the kernel no longer waits on the transcendental unit.
#include "dts_internal.h"

namespace dts {

namespace {

__device__ __forceinline__ float pw(float x, float y)
{
    // x >= 0; v_log_f32 / v_exp_f32 (base 2); log2(0) = -inf -> 0
    return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
}

// table t[0..kTmLutN] of (value, slope to the next entry) of a curve on [0, 1],
// linearly interpolated: clamp (v_med3), scale, truncate / fract, one 8-byte LDS read, fma
__device__ __forceinline__ float lut(const float2 *t, float v)
{
    const float x = __builtin_amdgcn_fmed3f(v, 0.f, 1.f) * (float)kTmLutN;
    const float2 e = t[(int)x];
    return __builtin_fmaf(__builtin_amdgcn_fractf(x), e.y, e.x);   // x >= 0: fract(x) = x - (int)x exactly
}

__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }

__device__ __forceinline__ float hable(float in)
{
    const float a = 0.15f, b = 0.50f, c = 0.10f, d = 0.20f, e = 0.02f, f = 0.30f;
    return (in * (in * a + b * c) + d * e) * rcp(in * (in * a + b) + d * f) - e / f;
}

__device__ __forceinline__ float mobius(float in, float j, float peak)
{
    if (in <= j) return in;
    const float a = -j * j * (peak - 1.f) / (j * j - 2.f * j + peak);
    const float b = (j * j - 2.f * j * peak + peak) / fmaxf(peak - 1.f, 1e-6f);
    return (b * b + 2.f * b * j + j * j) / (b - a) * (in + a) / (in + b);
}

__device__ __forceinline__ int q8(float v)
{
    // floor(v + 0.5) clipped to [0, 255]: after the clip the value is >= 0, so truncation is the floor
    return (int)__builtin_amdgcn_fmed3f(v + 0.5f, 0.f, 255.f);
}

// One pixel: 10-bit Y, chroma (Cb', Cr' already centred) -> bt709 Y' / Cb' / Cr'
__device__ __forceinline__ void pixel(const TonemapParams &P, const float2 *tl, int y10, float cb, float cr, float &Y,
                                      float &Cb, float &Cr)
{
    const float2 *pq = tl, *oetf = tl + kTmLutN + 1;          // pq already scaled by 10000 / npl
    constexpr float kr2 = 0.2627f, kb2 = 0.0593f, kg2 = 1.f - kr2 - kb2;
    constexpr float kr7 = 0.2126f, kb7 = 0.0722f, kg7 = 1.f - kr7 - kb7;
    const float yy = (float)(y10 - 64) * (1.f / 876.f);
    const float rp = yy + 2.f * (1.f - kr2) * cr, bp = yy + 2.f * (1.f - kb2) * cb;
    const float gp = (yy - kr2 * rp - kb2 * bp) * (1.f / kg2);
    const float r0 = lut(pq, rp), g0 = lut(pq, gp), b0 = lut(pq, bp);
    float r = P.m[0] * r0 + P.m[1] * g0 + P.m[2] * b0;
    float g = P.m[3] * r0 + P.m[4] * g0 + P.m[5] * b0;
    float b = P.m[6] * r0 + P.m[7] * g0 + P.m[8] * b0;
    // vf_tonemap.c tonemap()
    if (P.desat > 0.f) {
        const float luma = kr7 * r + kg7 * g + kb7 * b;
        const float ob = fmaxf(luma - P.desat, 1e-6f) / fmaxf(luma, 1e-6f);
        r = r * (1.f - ob) + luma * ob;
        g = g * (1.f - ob) + luma * ob;
        b = b * (1.f - ob) + luma * ob;
    }
    const float sig0 = fmaxf(fmaxf(fmaxf(r, g), b), 1e-6f);
    float sig = sig0;
    switch (P.mode) {                                            // uniform over the launch
    case DTS_TM_LINEAR: sig = sig * P.param / P.peak; break;
    case DTS_TM_GAMMA:
        sig = sig > 0.05f ? pw(sig / P.peak, 1.f / P.param) : sig * pw(0.05f / P.peak, 1.f / P.param) / 0.05f;
        break;
    case DTS_TM_CLIP: sig = fminf(fmaxf(sig * P.param, 0.f), 1.f); break;
    case DTS_TM_REINHARD: sig = sig / (sig + P.param) * (P.peak + P.param) / P.peak; break;
    case DTS_TM_HABLE: sig = hable(sig) * P.inv_hpeak; break;
    case DTS_TM_MOBIUS: sig = mobius(sig, P.param, P.peak); break;
    default: break;
    }
    const float k = sig * rcp(sig0);
    r = lut(oetf, r * k);
    g = lut(oetf, g * k);
    b = lut(oetf, b * k);
    Y = kr7 * r + kg7 * g + kb7 * b;
    Cb = (b - Y) * (1.f / (2.f * (1.f - kb7)));
    Cr = (r - Y) * (1.f / (2.f * (1.f - kr7)));
}

} // namespace

__global__ void __launch_bounds__(256) k_tonemap(const TonemapParams P)
{
    __shared__ float2 tl[2 * (kTmLutN + 1)];
    for (int i = threadIdx.x; i < 2 * (kTmLutN + 1); i += 256) tl[i] = P.lut[i];
    __syncthreads();
    const int bx = blockIdx.x * 64 + (threadIdx.x & 63);
    const int f = blockIdx.z;
    if (bx >= (P.w >> 1)) return;
    const uint64_t sf = (uint64_t)f * P.src.fstride, df = (uint64_t)f * P.dst.fstride;
    const int by_end = min((int)(blockIdx.y + 1) * kTmRows, P.h >> 1);
    for (int by = blockIdx.y * kTmRows + (threadIdx.x >> 6); by < by_end; by += 4) {
        const uint64_t ys = P.src.data[0] + sf + (uint64_t)(2 * by) * P.src.pitch[0] + 4 * bx;
        const uint32_t l0 = *reinterpret_cast<const uint32_t *>(ys);
        const uint32_t l1 = *reinterpret_cast<const uint32_t *>(ys + P.src.pitch[0]);
        const uint32_t c =
            *reinterpret_cast<const uint32_t *>(P.src.data[1] + sf + (uint64_t)by * P.src.pitch[1] + 4 * bx);
        const float cb = (float)((int)((c & 0xffffu) >> 6) - 512) * (1.f / 896.f);
        const float cr = (float)((int)(c >> 22) - 512) * (1.f / 896.f);
        float Y[4], Cb[4], Cr[4];
        pixel(P, tl, (int)((l0 & 0xffffu) >> 6), cb, cr, Y[0], Cb[0], Cr[0]);
        pixel(P, tl, (int)(l0 >> 22), cb, cr, Y[1], Cb[1], Cr[1]);
        pixel(P, tl, (int)((l1 & 0xffffu) >> 6), cb, cr, Y[2], Cb[2], Cr[2]);
        pixel(P, tl, (int)(l1 >> 22), cb, cr, Y[3], Cb[3], Cr[3]);
        const uint64_t yd = P.dst.data[0] + df + (uint64_t)(2 * by) * P.dst.pitch[0] + 2 * bx;
        *reinterpret_cast<uint16_t *>(yd) = (uint16_t)(q8(16.f + 219.f * Y[0]) | (q8(16.f + 219.f * Y[1]) << 8));
        *reinterpret_cast<uint16_t *>(yd + P.dst.pitch[0]) =
            (uint16_t)(q8(16.f + 219.f * Y[2]) | (q8(16.f + 219.f * Y[3]) << 8));
        const int u = q8(128.f + 224.f * ((Cb[0] + Cb[1] + Cb[2] + Cb[3]) * 0.25f));
        const int v = q8(128.f + 224.f * ((Cr[0] + Cr[1] + Cr[2] + Cr[3]) * 0.25f));
        if (P.dst_fmt == DTS_FMT_NV12) {
            *reinterpret_cast<uint16_t *>(P.dst.data[1] + df + (uint64_t)by * P.dst.pitch[1] + 2 * bx) =
                (uint16_t)(u | (v << 8));
        } else {
            *reinterpret_cast<uint8_t *>(P.dst.data[1] + df + (uint64_t)by * P.dst.pitch[1] + bx) = (uint8_t)u;
            *reinterpret_cast<uint8_t *>(P.dst.data[2] + df + (uint64_t)by * P.dst.pitch[2] + bx) = (uint8_t)v;
        }
    }
}

hipError_t launch_tonemap(const TonemapParams &p, hipStream_t s)
{
    const dim3 grid((unsigned)((p.w / 2 + 63) / 64), (unsigned)((p.h / 2 + kTmRows - 1) / kTmRows), (unsigned)p.nframes);
    hipLaunchKernelGGL(k_tonemap, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

} // namespace dts
