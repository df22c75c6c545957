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
 *   - the 4:2:0 chroma resampled as vf_zscale configures zimg by default
 *     (FFmpeg 4.4 vf_zscale.c: filter = filterc = "bilinear"; chroma location
 *     taken from the frame, "left" = MPEG-2 4:2:0 siting: horizontally
 *     co-sited with the even luma columns, vertically between the two luma
 *     rows): up to 4:4:4 before the matrix by the triangle filter of radius 1
 *     (odd luma columns = mean of the two chroma neighbours; luma rows take
 *     0.75 / 0.25 of the nearer / farther chroma row), and back to 4:2:0 after
 *     the output matrix by the same filter stretched 2:1 (horizontal taps
 *     1/4 1/2 1/4 centred on the even column, vertical 1/8 3/8 3/8 1/8 around
 *     the row pair); samples beyond the plane edge repeat the edge sample
 *     (for radius-1 bilinear taps, zimg's edge mirroring gives the same);
 *   - bt2020nc limited-range Y'CbCr -> R'G'B' (ITU-R BT.2020 Kr/Kb);
 *   - SMPTE ST 2084 (PQ) EOTF, scaled so NPL cd/m^2 -> 1.0;
 *   - bt2020 -> bt709 primaries in linear light (3x3 from the xy primaries and
 *     D65 white);
 *   - libavfilter/vf_tonemap.c tonemap() / hable() / mobius() (FFmpeg 4.4),
 *     restated from memory, including its peak fallback (10.0 for linear
 *     input without HDR side data) and param defaults (init());
 *   - BT.709 OETF (zimg's rec_709_oetf constants), bt709 limited-range
 *     Y'CbCr (chroma 2:1 as above), rounded to 8 bits (zscale dither=none).
 * Parity status: unpinned (no zimg/ffmpeg here); the GPU must match this
 * restatement within +-1 LSB (float vs double).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

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

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* zimg bilinear, chroma location left: the 4:2:0 chroma value (Cb' or Cr', centred,
 * c = 0 Cb / 1 Cr) at luma pixel (x, y) */
static double chroma_up(const uint8_t *plane, int64_t pitch, int cw, int ch, int c, int x, int y)
{
    const int j = x >> 1, j1 = clampi(j + 1, 0, cw - 1);
    const double fx = (x & 1) ? 0.5 : 0.0;
    const int k = clampi(y >> 1, 0, ch - 1), k2 = clampi((y & 1) ? (y >> 1) + 1 : (y >> 1) - 1, 0, ch - 1);
    double v[2];
    int i;
    for (i = 0; i < 2; i++) {
        const uint8_t *row = plane + (int64_t)(i ? k2 : k) * pitch + 2 * c;
        const double a = (rd16(row + 4 * j) - 512) / 896.0, b = (rd16(row + 4 * j1) - 512) / 896.0;
        v[i] = (1.0 - fx) * a + fx * b;
    }
    return 0.75 * v[0] + 0.25 * v[1];
}

int orc_hdr_to_sdr_frame(int w, int h, const uint8_t *const src[3], const int64_t src_pitch[3],
                         int dstFmt, uint8_t *const dst[3], const int64_t dst_pitch[3],
                         int mode, double param, double desat, double peak, double npl, int out_full)
{
    const double kr2 = 0.2627, kb2 = 0.0593, kg2 = 1.0 - kr2 - kb2;
    const double kr7 = 0.2126, kb7 = 0.0722, kg7 = 1.0 - kr7 - kb7;
    static const double wx[3] = {0.25, 0.5, 0.25}, wy[4] = {0.125, 0.375, 0.375, 0.125};
    /* zimg's integer quantisation of the last zscale (depth conversion, no dither): r=tv Y 219 Y' + 16,
     * C 224 C + 128; r=pc Y 255 Y', C 255 C + 128 */
    const double qy = out_full ? 255.0 : 219.0, qo = out_full ? 0.0 : 16.0, qc = out_full ? 255.0 : 224.0;
    double M[3][3], scale, hpeak, *cb4, *cr4;
    int x, y, bx, by;
    const int cw = w / 2, ch = h / 2;
    if (w < 2 || h < 2 || (w & 1) || (h & 1)) return -22;
    if (dstFmt != ORC_FMT_YUV420P && dstFmt != ORC_FMT_NV12) return -22;
    if (mode < TM_NONE || mode > TM_MOBIUS) return -22;
    cb4 = (double *)malloc(sizeof(double) * (size_t)w * h);
    cr4 = (double *)malloc(sizeof(double) * (size_t)w * h);
    if (!cb4 || !cr4) {
        free(cb4);
        free(cr4);
        return -12;
    }
    orc_bt2020_to_bt709(M);
    if (npl <= 0.0) npl = 100.0;
    if (peak <= 0.0) peak = 10.0;
    param = orc_tonemap_param(mode, param);
    scale = 10000.0 / npl;
    hpeak = hable(peak);
    for (y = 0; y < h; y++)
        for (x = 0; x < w; x++) {
            const double cb = chroma_up(src[1], src_pitch[1], cw, ch, 0, x, y);
            const double cr = chroma_up(src[1], src_pitch[1], cw, ch, 1, x, y);
            const double yy = (rd16(src[0] + (int64_t)y * src_pitch[0] + 2 * x) - 64) / 876.0;
            double rp = yy + 2.0 * (1.0 - kr2) * cr, bp = yy + 2.0 * (1.0 - kb2) * cb;
            double gp = (yy - kr2 * rp - kb2 * bp) / kg2;
            double r0 = pq_eotf(clamp01(rp)) * scale, g0 = pq_eotf(clamp01(gp)) * scale,
                   b0 = pq_eotf(clamp01(bp)) * scale;
            double r = M[0][0] * r0 + M[0][1] * g0 + M[0][2] * b0;
            double g = M[1][0] * r0 + M[1][1] * g0 + M[1][2] * b0;
            double b = M[2][0] * r0 + M[2][1] * g0 + M[2][2] * b0;
            double sig, sig0, Y;
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
            cb4[(size_t)y * w + x] = (b - Y) / (2.0 * (1.0 - kb7));
            cr4[(size_t)y * w + x] = (r - Y) / (2.0 * (1.0 - kr7));
            dst[0][(int64_t)y * dst_pitch[0] + x] = (uint8_t)q8(qo + qy * Y);
        }
    /* 4:4:4 -> 4:2:0, chroma location left: taps 1/4 1/2 1/4 around column 2 bx,
     * 1/8 3/8 3/8 1/8 over rows 2 by - 1 .. 2 by + 2, edge samples repeated */
    for (by = 0; by < ch; by++)
        for (bx = 0; bx < cw; bx++) {
            double sb = 0.0, sr = 0.0;
            int i, t;
            for (i = 0; i < 4; i++) {
                const int yy = clampi(2 * by - 1 + i, 0, h - 1);
                for (t = 0; t < 3; t++) {
                    const int xx = clampi(2 * bx - 1 + t, 0, w - 1);
                    sb += wy[i] * wx[t] * cb4[(size_t)yy * w + xx];
                    sr += wy[i] * wx[t] * cr4[(size_t)yy * w + xx];
                }
            }
            if (dstFmt == ORC_FMT_NV12) {
                dst[1][(int64_t)by * dst_pitch[1] + 2 * bx] = (uint8_t)q8(128.0 + qc * sb);
                dst[1][(int64_t)by * dst_pitch[1] + 2 * bx + 1] = (uint8_t)q8(128.0 + qc * sr);
            } else {
                dst[1][(int64_t)by * dst_pitch[1] + bx] = (uint8_t)q8(128.0 + qc * sb);
                dst[2][(int64_t)by * dst_pitch[2] + bx] = (uint8_t)q8(128.0 + qc * sr);
            }
        }
    free(cb4);
    free(cr4);
    return 0;
}
