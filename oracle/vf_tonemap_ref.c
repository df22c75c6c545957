/*
 * vf_tonemap_ref.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement, in double precision, of the HDR10 -> SDR bt709 stage of
 * BASELINE config 3.  A reference ffmpeg worker would
 * run, after the libswscale scale to the output size in p010:
 *
 *   zscale=t=linear:npl=NPL,format=gbrpf32le,zscale=p=bt709,
 *   tonemap=tonemap=MODE:param=P:desat=D:peak=K,
 *   zscale=t=bt709:m=bt709:r=tv,format=yuv420p
 *
 * zscale is zimg, which is third-party even to FFmpeg and absent here, so the
 * zimg steps are restated from the published standards they implement:
 *   - bt2020nc limited-range Y'CbCr -> R'G'B' (ITU-R BT.2020 Kr/Kb),
 *     chroma of each 2x2 luma block replicated (zimg filter_c=point);
 *   - SMPTE ST 2084 (PQ) EOTF, scaled so NPL cd/m^2 -> 1.0;
 *   - bt2020 -> bt709 primaries in linear light (3x3 from the xy primaries and
 *     D65 white);
 *   - libavfilter/vf_tonemap.c tonemap() / hable() / mobius() (FFmpeg 4.4),
 *     restated from memory, including its peak fallback (10.0 for linear
 *     input without HDR side data) and param defaults (init());
 *   - BT.709 OETF (zimg's rec_709_oetf constants), bt709 limited-range
 *     Y'CbCr, chroma = mean of the 2x2 block (zimg bilinear 2:1, centred).
 * Parity status: unpinned (no zimg/ffmpeg here); the GPU must match this
 * restatement within +-1 LSB (float vs double).
 */
#include <math.h>
#include <stdint.h>

#include "oracle.h"

/* vf_tonemap.c enum TonemapAlgorithm */
enum { TM_NONE, TM_LINEAR, TM_GAMMA, TM_CLIP, TM_REINHARD, TM_HABLE, TM_MOBIUS };

static double hable(double in)
{
    const double a = 0.15, b = 0.50, c = 0.10, d = 0.20, e = 0.02, f = 0.30;
    return (in * (in * a + b * c) + d * e) / (in * (in * a + b) + d * f) - e / f;
}

static double mobius(double in, double j, double peak)
{
    double a, b;
    if (in <= j) return in;
    a = -j * j * (peak - 1.0) / (j * j - 2.0 * j + peak);
    b = (j * j - 2.0 * j * peak + peak) / fmax(peak - 1.0, 1e-6);
    return (b * b + 2.0 * b * j + j * j) / (b - a) * (in + a) / (in + b);
}

/* vf_tonemap.c init(): per-mode param defaults (NaN = not set) */
double orc_tonemap_param(int mode, double param)
{
    switch (mode) {
    case TM_GAMMA: if (isnan(param)) param = 1.8; break;
    case TM_REINHARD: if (!isnan(param)) param = (1.0 - param) / param; break;
    case TM_MOBIUS: if (isnan(param)) param = 0.3; break;
    }
    if (isnan(param)) param = 1.0;
    return param;
}

/* RGB -> XYZ of a primaries set with D65 white (columns scaled so white -> Y=1) */
static void rgb2xyz(const double xy[3][2], double m[3][3])
{
    const double wx = 0.3127, wy = 0.3290;
    double P[3][3], inv[3][3], W[3], S[3], det;
    int i, j;
    for (i = 0; i < 3; i++) {
        P[0][i] = xy[i][0] / xy[i][1];
        P[1][i] = 1.0;
        P[2][i] = (1.0 - xy[i][0] - xy[i][1]) / xy[i][1];
    }
    W[0] = wx / wy; W[1] = 1.0; W[2] = (1.0 - wx - wy) / wy;
    det = P[0][0] * (P[1][1] * P[2][2] - P[1][2] * P[2][1]) - P[0][1] * (P[1][0] * P[2][2] - P[1][2] * P[2][0]) +
          P[0][2] * (P[1][0] * P[2][1] - P[1][1] * P[2][0]);
    inv[0][0] = (P[1][1] * P[2][2] - P[1][2] * P[2][1]) / det;
    inv[0][1] = (P[0][2] * P[2][1] - P[0][1] * P[2][2]) / det;
    inv[0][2] = (P[0][1] * P[1][2] - P[0][2] * P[1][1]) / det;
    inv[1][0] = (P[1][2] * P[2][0] - P[1][0] * P[2][2]) / det;
    inv[1][1] = (P[0][0] * P[2][2] - P[0][2] * P[2][0]) / det;
    inv[1][2] = (P[0][2] * P[1][0] - P[0][0] * P[1][2]) / det;
    inv[2][0] = (P[1][0] * P[2][1] - P[1][1] * P[2][0]) / det;
    inv[2][1] = (P[0][1] * P[2][0] - P[0][0] * P[2][1]) / det;
    inv[2][2] = (P[0][0] * P[1][1] - P[0][1] * P[1][0]) / det;
    for (i = 0; i < 3; i++) S[i] = inv[i][0] * W[0] + inv[i][1] * W[1] + inv[i][2] * W[2];
    for (i = 0; i < 3; i++)
        for (j = 0; j < 3; j++) m[i][j] = P[i][j] * S[j];
}

static void inv3(double a[3][3], double o[3][3])
{
    double det = a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) - a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
                 a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]);
    o[0][0] = (a[1][1] * a[2][2] - a[1][2] * a[2][1]) / det;
    o[0][1] = (a[0][2] * a[2][1] - a[0][1] * a[2][2]) / det;
    o[0][2] = (a[0][1] * a[1][2] - a[0][2] * a[1][1]) / det;
    o[1][0] = (a[1][2] * a[2][0] - a[1][0] * a[2][2]) / det;
    o[1][1] = (a[0][0] * a[2][2] - a[0][2] * a[2][0]) / det;
    o[1][2] = (a[0][2] * a[1][0] - a[0][0] * a[1][2]) / det;
    o[2][0] = (a[1][0] * a[2][1] - a[1][1] * a[2][0]) / det;
    o[2][1] = (a[0][1] * a[2][0] - a[0][0] * a[2][1]) / det;
    o[2][2] = (a[0][0] * a[1][1] - a[0][1] * a[1][0]) / det;
}

/* bt2020 -> bt709 linear-light primaries matrix */
void orc_bt2020_to_bt709(double m[3][3])
{
    static const double p2020[3][2] = {{0.708, 0.292}, {0.170, 0.797}, {0.131, 0.046}};
    static const double p709[3][2] = {{0.640, 0.330}, {0.300, 0.600}, {0.150, 0.060}};
    double a[3][3], b[3][3], bi[3][3];
    int i, j, k;
    rgb2xyz(p2020, a);
    rgb2xyz(p709, b);
    inv3(b, bi);
    for (i = 0; i < 3; i++)
        for (j = 0; j < 3; j++) {
            m[i][j] = 0;
            for (k = 0; k < 3; k++) m[i][j] += bi[i][k] * a[k][j];
        }
}

static double clamp01(double v) { return v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v); }

/* SMPTE ST 2084 EOTF: E' in [0,1] -> cd/m^2 / 10000 */
static double pq_eotf(double e)
{
    const double m1 = 2610.0 / 16384.0, m2 = 2523.0 / 4096.0 * 128.0;
    const double c1 = 3424.0 / 4096.0, c2 = 2413.0 / 4096.0 * 32.0, c3 = 2392.0 / 4096.0 * 32.0;
    double p = pow(e, 1.0 / m2);
    double n = p - c1;
    if (n < 0.0) n = 0.0;
    return pow(n / (c2 - c3 * p), 1.0 / m1);
}

static double rec709_oetf(double l)
{
    const double alpha = 1.09929682680944, beta = 0.018053968510807;
    return l < beta ? 4.5 * l : alpha * pow(l, 0.45) - (alpha - 1.0);
}

static int q8(double v)
{
    double r = floor(v + 0.5);
    return r < 0.0 ? 0 : (r > 255.0 ? 255 : (int)r);
}

static int rd16(const uint8_t *p) { return (p[0] | (p[1] << 8)) >> 6; }

int orc_hdr_to_sdr_frame(int w, int h, const uint8_t *const src[3], const int64_t src_pitch[3],
                         int dstFmt, uint8_t *const dst[3], const int64_t dst_pitch[3],
                         int mode, double param, double desat, double peak, double npl)
{
    const double kr2 = 0.2627, kb2 = 0.0593, kg2 = 1.0 - kr2 - kb2;
    const double kr7 = 0.2126, kb7 = 0.0722, kg7 = 1.0 - kr7 - kb7;
    double M[3][3], scale, hpeak;
    int bx, by;
    if (w < 2 || h < 2 || (w & 1) || (h & 1)) return -22;
    if (dstFmt != ORC_FMT_YUV420P && dstFmt != ORC_FMT_NV12) return -22;
    if (mode < TM_NONE || mode > TM_MOBIUS) return -22;
    orc_bt2020_to_bt709(M);
    if (npl <= 0.0) npl = 100.0;
    if (peak <= 0.0) peak = 10.0;
    param = orc_tonemap_param(mode, param);
    scale = 10000.0 / npl;
    hpeak = hable(peak);
    for (by = 0; by < h / 2; by++)
        for (bx = 0; bx < w / 2; bx++) {
            const uint8_t *c = src[1] + (int64_t)by * src_pitch[1] + 4 * bx;
            const double cb = (rd16(c) - 512) / 896.0, cr = (rd16(c + 2) - 512) / 896.0;
            double sb = 0.0, sr = 0.0;
            int d;
            for (d = 0; d < 4; d++) {
                const int x = 2 * bx + (d & 1), y = 2 * by + (d >> 1);
                const double yy = (rd16(src[0] + (int64_t)y * src_pitch[0] + 2 * x) - 64) / 876.0;
                double rp = yy + 2.0 * (1.0 - kr2) * cr, bp = yy + 2.0 * (1.0 - kb2) * cb;
                double gp = (yy - kr2 * rp - kb2 * bp) / kg2;
                double r0 = pq_eotf(clamp01(rp)) * scale, g0 = pq_eotf(clamp01(gp)) * scale,
                       b0 = pq_eotf(clamp01(bp)) * scale;
                double r = M[0][0] * r0 + M[0][1] * g0 + M[0][2] * b0;
                double g = M[1][0] * r0 + M[1][1] * g0 + M[1][2] * b0;
                double b = M[2][0] * r0 + M[2][1] * g0 + M[2][2] * b0;
                double sig, sig0, Y, Cb, Cr;
                /* vf_tonemap.c tonemap() */
                if (desat > 0.0) {
                    double luma = kr7 * r + kg7 * g + kb7 * b;
                    double ob = fmax(luma - desat, 1e-6) / fmax(luma, 1e-6);
                    r = r * (1.0 - ob) + luma * ob;
                    g = g * (1.0 - ob) + luma * ob;
                    b = b * (1.0 - ob) + luma * ob;
                }
                sig = fmax(fmax(fmax(r, g), b), 1e-6);
                sig0 = sig;
                switch (mode) {
                case TM_LINEAR: sig = sig * param / peak; break;
                case TM_GAMMA:
                    sig = sig > 0.05 ? pow(sig / peak, 1.0 / param) : sig * pow(0.05 / peak, 1.0 / param) / 0.05;
                    break;
                case TM_CLIP: sig = fmin(fmax(sig * param, 0.0), 1.0); break;
                case TM_REINHARD: sig = sig / (sig + param) * (peak + param) / peak; break;
                case TM_HABLE: sig = hable(sig) / hpeak; break;
                case TM_MOBIUS: sig = mobius(sig, param, peak); break;
                default: break;
                }
                r *= sig / sig0;
                g *= sig / sig0;
                b *= sig / sig0;
                r = rec709_oetf(clamp01(r));
                g = rec709_oetf(clamp01(g));
                b = rec709_oetf(clamp01(b));
                Y = kr7 * r + kg7 * g + kb7 * b;
                Cb = (b - Y) / (2.0 * (1.0 - kb7));
                Cr = (r - Y) / (2.0 * (1.0 - kr7));
                dst[0][(int64_t)y * dst_pitch[0] + x] = (uint8_t)q8(16.0 + 219.0 * Y);
                sb += Cb;
                sr += Cr;
            }
            if (dstFmt == ORC_FMT_NV12) {
                dst[1][(int64_t)by * dst_pitch[1] + 2 * bx] = (uint8_t)q8(128.0 + 224.0 * sb * 0.25);
                dst[1][(int64_t)by * dst_pitch[1] + 2 * bx + 1] = (uint8_t)q8(128.0 + 224.0 * sr * 0.25);
            } else {
                dst[1][(int64_t)by * dst_pitch[1] + bx] = (uint8_t)q8(128.0 + 224.0 * sb * 0.25);
                dst[2][(int64_t)by * dst_pitch[2] + bx] = (uint8_t)q8(128.0 + 224.0 * sr * 0.25);
            }
        }
    return 0;
}
