// qfuse.hip -- the two small launches that finish k_ladder7's fused vf_psnr / vf_ssim
// (ladder7.hip qrb7; FFmpeg 4.4 vf_psnr.c compute_images_mse, vf_ssim.c ssim_4x4xn /
// ssim_end1 / ssim_plane, restated in kernels.hip k_quality and oracle/vf_quality_ref.c):
//
//  * k_qfix7: the 8x8 windows (stride 4) whose two block columns belong to two neighbouring
//    units of a rendition plane -- the only windows no single walk sees.  A workgroup takes
//    one boundary and 63 window rows: each thread sums one pixel row of the two 4-pixel
//    block slices (output and reference, read from HBM), the window rows are added up from
//    LDS, scored with ssim_end1 and reduced in a fixed order;
//  * k_qfin7: per (frame, rendition) the units' QPart7 records and the boundary sums, summed
//    in a fixed order into the dts_qraw record vf_psnr / vf_ssim keep per frame.
#include <algorithm>

#include "dts_internal.h"

namespace dts {

namespace {

constexpr int kFixRows = 63;                 // window rows per k_qfix7 workgroup (64 block rows)

__device__ __forceinline__ float ssim_end1_q(int s1, int s2, int ss, int s12)
{
    const int c1 = (int)(.01 * .01 * 255 * 255 * 64 + .5);
    const int c2 = (int)(.03 * .03 * 255 * 255 * 64 * 63 + .5);
    const int vars = ss * 64 - s1 * s1 - s2 * s2;
    const int covar = s12 * 64 - s1 * s2;
    return (float)(2 * s1 * s2 + c1) * (float)(2 * covar + c2) *
           __builtin_amdgcn_rcpf((float)(s1 * s1 + s2 * s2 + c1) * (float)(vars + c2));
}

// 8 pixels of plane `pl` at pixel column x of row y (two dwords; nv12 chroma de-interleaved)
__device__ __forceinline__ void px8(const DevPlanes &d, int fmt, int pl, int64_t f, int y, int x, uint32_t (&o)[2])
{
    const bool il = fmt == DTS_FMT_NV12 && pl > 0;
    const int dp = il ? 1 : pl;
    const uint8_t *row = reinterpret_cast<const uint8_t *>(d.data[dp] + (uint64_t)(f * d.fstride) +
                                                           (uint64_t)((int64_t)y * d.pitch[dp]));
    if (!il) {
        o[0] = *reinterpret_cast<const uint32_t *>(row + x);
        o[1] = *reinterpret_cast<const uint32_t *>(row + x + 4);
    } else {
        const uint32_t sel = pl == 2 ? 0x07050301u : 0x06040200u;
        const uint32_t *w = reinterpret_cast<const uint32_t *>(row + 2 * x);
        o[0] = __builtin_amdgcn_perm(w[1], w[0], sel);
        o[1] = __builtin_amdgcn_perm(w[3], w[2], sel);
    }
}

} // namespace

__global__ void __launch_bounds__(256) k_qfix7(const QFinParams P)
{
    __shared__ uint32_t rs[8][256];          // per pixel row: s1, s2, ss, s12 of the left, right slice
    __shared__ double red[256];
    const int t = threadIdx.x, nsp = gridDim.x / max(P.nbound, 1);
    const int b = blockIdx.x / nsp, span = blockIdx.x - b * nsp, f = blockIdx.y;
    const int gbx = P.qbound[2 * b], ri = P.qbound[2 * b + 1];
    const QRend7 R = P.rend[ri];
    const int W4 = R.w >> 2, H4 = R.h >> 2, gy0 = span * kFixRows;
    double v = 0.0;
    if (gbx + 1 < W4 && gy0 + 1 < H4) {      // (uniform) any window of this workgroup
        const int y = 4 * gy0 + t;
        uint32_t s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (y < 4 * H4) {
            uint32_t a[2], c[2];
            px8(P.out[R.rung], P.fmt[R.rung], R.plane, f, y, 4 * gbx, a);
            px8(P.ref[R.rung], P.fmt[R.rung], R.plane, f, y, 4 * gbx, c);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                s[4 * h] = __builtin_amdgcn_udot4(a[h], 0x01010101u, 0u, false);
                s[4 * h + 1] = __builtin_amdgcn_udot4(c[h], 0x01010101u, 0u, false);
                s[4 * h + 2] = __builtin_amdgcn_udot4(c[h], c[h], __builtin_amdgcn_udot4(a[h], a[h], 0u, false), false);
                s[4 * h + 3] = __builtin_amdgcn_udot4(a[h], c[h], 0u, false);
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) rs[i][t] = s[i];
        __syncthreads();
        const int gy = gy0 + t;
        if (t < kFixRows && gy + 1 < H4) {
            int w[4] = {0, 0, 0, 0};
            for (int r = 4 * t; r < 4 * t + 8; ++r)
#pragma unroll
                for (int i = 0; i < 4; ++i) w[i] += (int)(rs[i][r] + rs[4 + i][r]);
            v = (double)ssim_end1_q(w[0], w[1], w[2], w[3]);
        }
    }
    red[t] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) red[t] += red[t + o];
        __syncthreads();
    }
    if (t == 0) P.fixp[(int64_t)f * P.nbound * nsp + blockIdx.x] = red[0];
}

// one workgroup per (frame, rendition): its planes' unit records and boundary sums
__global__ void __launch_bounds__(256) k_qfin7(const QFinParams P, int nsp)
{
    __shared__ unsigned long long re[256];
    __shared__ double rd[256];
    const int t = threadIdx.x, f = blockIdx.x, rung = blockIdx.y;
    dts_qraw q{};
    bool any = false;
    for (int e = 0; e < P.nrend; ++e) {
        const QRend7 R = P.rend[e];
        if (R.rung != rung) continue;
        any = true;
        const int k = R.plane == 2 ? 1 : 0;  // a chroma unit's U, V records
        unsigned long long se = 0;
        double ss = 0.0;
        for (int i = t; i < R.nu; i += 256) {
            const QPart7 &u = P.qpart[(int64_t)f * P.nunits + P.qunit[R.u0 + i]];
            se += u.sse[k];
            ss += u.ssim[k];
        }
        for (int i = t; i < R.nb * nsp; i += 256)
            ss += P.fixp[(int64_t)f * P.nbound * nsp + (int64_t)(R.b0 * nsp + i)];
        re[t] = se;
        rd[t] = ss;
        __syncthreads();
        for (int o = 128; o > 0; o >>= 1) {
            if (t < o) {
                re[t] += re[t + o];
                rd[t] += rd[t + o];
            }
            __syncthreads();
        }
        q.sse[R.plane] = re[0];
        q.ssim_sum[R.plane] = rd[0];
        __syncthreads();
    }
    if (t == 0 && any) P.out_q[(int64_t)rung * P.qstride + f] = q;
}

// k_qfix7 over nsp spans of kFixRows window rows per boundary, then k_qfin7
hipError_t launch_qfuse7(const QFinParams &p, int nrungs, int max_h4, hipStream_t s)
{
    const int nsp = std::max(1, (max_h4 - 1 + kFixRows - 1) / kFixRows);
    if (p.nbound > 0) {
        hipLaunchKernelGGL(k_qfix7, dim3((unsigned)(p.nbound * nsp), (unsigned)p.nframes), dim3(256), 0, s, p);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_qfin7, dim3((unsigned)p.nframes, (unsigned)nrungs), dim3(256), 0, s, p, nsp);
    return hipGetLastError();
}

int qfuse7_spans(int max_h4) { return std::max(1, (max_h4 - 1 + kFixRows - 1) / kFixRows); }

} // namespace dts
