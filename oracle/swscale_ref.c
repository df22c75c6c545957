/*
 * swscale_ref.c -- TEST INFRASTRUCTURE ONLY (see oracle.h header).
 *
 * Plain-C restatement of the FFmpeg 4.4 libswscale C path that a reference
 * ffmpeg worker executes for `scale=W:H:flags=<m>+accurate_rnd+bitexact`
 * (the worker would be spawned via the ffmpeg-static path resolved at
 * /root/reference/index.js:9; W/H come from Jobs.width/height,
 * database.js:73-74).  Every function names the [ext] FFmpeg 4.4 function it
 * restates.  FFmpeg is not present anywhere in this container, so the
 * restatement is from the published C source as recalled: parity unpinned.
 *
 * Items flagged "from memory, unverified" in SURVEY.md 8a:
 *   - ff_dither_8x8_128 values (below),
 *   - SWS_MAX_REDUCE_CUTOFF = 0.002,
 *   - x86 filterAlign (H 4, V 2 -> 1 when minFilterSize == 1).
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define FFABS(a) ((a) >= 0 ? (a) : (-(a)))
#define FFMIN(a, b) ((a) > (b) ? (b) : (a))
#define FFMAX(a, b) ((a) > (b) ? (a) : (b))
#define ROUNDED_DIV(a, b) (((a) >= 0 ? (a) + ((b) >> 1) : (a) - ((b) >> 1)) / (b))
#define SWS_MAX_REDUCE_CUTOFF 0.002
#define MAX_FILTER_SIZE 256
#define APCK_SIZE 16

/* libswscale/swscale.c ff_dither_8x8_128 (from memory, unverified) */
static const uint8_t dither_8x8_128[9][8] = {
    {  36, 68,  60, 92,  34, 66,  58, 90, },
    { 100,  4, 124, 28,  98,  2, 122, 26, },
    {  52, 84,  44, 76,  50, 82,  42, 74, },
    { 116, 20, 108, 12, 114, 18, 106, 10, },
    {  32, 64,  56, 88,  38, 70,  62, 94, },
    {  96,  0, 120, 24, 102,  6, 126, 30, },
    {  48, 80,  40, 72,  54, 86,  46, 78, },
    { 112, 16, 104,  8, 118, 22, 110, 14, },
    {  36, 68,  60, 92,  34, 66,  58, 90, },
};
static const uint8_t flat64[8] = { 64, 64, 64, 64, 64, 64, 64, 64 };

static int av_log2_u(unsigned v)
{
    int n = 0;
    if (!v) return 0;
    while (v >>= 1) n++;
    return n;
}

/* libswscale/utils.c get_local_pos() */
int orc_get_local_pos(int chr_subsample, int pos)
{
    if (pos == -1 || pos <= -513)
        pos = (128 << chr_subsample) - 128;
    pos += 128;
    return pos >> chr_subsample;
}

/* libswscale/utils.c initFilter() (FFmpeg 4.4), scaled-kernel branches for
 * bilinear / bicubic / lanczos / area / gauss / sinc / x plus the unscaled
 * and point branches; srcFilter/dstFilter are NULL (vf_scale passes none). */
int orc_init_filter(int16_t *coeff_out, int32_t *pos_out, int cap_taps,
                    int xInc, int srcW, int dstW, int filterAlign, int one,
                    int flags, const double param[2], int srcPos, int dstPos)
{
    int i, filterSize, filter2Size, minFilterSize;
    int64_t *filter = NULL, *filter2 = NULL;
    int32_t *filterPos = NULL;
    const int64_t fone = 1LL << (54 - FFMIN(av_log2_u(srcW / dstW), 8));
    int ret = -1;

    filterPos = (int32_t *)calloc((size_t)dstW + 3, sizeof(int32_t));
    if (!filterPos) return -12;

    if (FFABS(xInc - 0x10000) < 10 && srcPos == dstPos) { /* unscaled */
        filterSize = 1;
        filter = (int64_t *)calloc((size_t)dstW * filterSize, sizeof(int64_t));
        for (i = 0; i < dstW; i++) {
            filter[i * filterSize] = fone;
            filterPos[i] = i;
        }
    } else if (flags & ORC_SWS_POINT) {
        int64_t xDstInSrc;
        filterSize = 1;
        filter = (int64_t *)calloc((size_t)dstW * filterSize, sizeof(int64_t));
        xDstInSrc = ((dstPos * (int64_t)xInc) >> 8) - ((srcPos * 0x8000LL) >> 7);
        for (i = 0; i < dstW; i++) {
            int xx = (int)((xDstInSrc - (filterSize - 1) * 0x8000LL + (1 << 15)) >> 16);
            filterPos[i] = xx;
            filter[i] = fone;
            xDstInSrc += xInc;
        }
    } else if ((xInc <= (1 << 16) && (flags & ORC_SWS_AREA)) ||
               (flags & ORC_SWS_FAST_BILINEAR)) { /* bilinear upscale */
        int64_t xDstInSrc;
        filterSize = 2;
        filter = (int64_t *)calloc((size_t)dstW * filterSize, sizeof(int64_t));
        xDstInSrc = ((dstPos * (int64_t)xInc) >> 8) - ((srcPos * 0x8000LL) >> 7);
        for (i = 0; i < dstW; i++) {
            int xx = (int)((xDstInSrc - (filterSize - 1) * 0x8000LL + (1 << 15)) >> 16);
            int j;
            filterPos[i] = xx;
            for (j = 0; j < filterSize; j++) {
                int64_t c = fone - FFABS((int64_t)xx * (1 << 16) - xDstInSrc) * (fone >> 16);
                if (c < 0) c = 0;
                filter[i * filterSize + j] = c;
                xx++;
            }
            xDstInSrc += xInc;
        }
    } else {
        int64_t xDstInSrc;
        int sizeFactor;
        if (flags & ORC_SWS_BICUBIC)       sizeFactor = 4;
        else if (flags & ORC_SWS_X)        sizeFactor = 8;
        else if (flags & ORC_SWS_AREA)     sizeFactor = 1;
        else if (flags & ORC_SWS_GAUSS)    sizeFactor = 8;
        else if (flags & ORC_SWS_LANCZOS)
            sizeFactor = param[0] != ORC_SWS_PARAM_DEFAULT ? (int)ceil(2 * param[0]) : 6;
        else if (flags & ORC_SWS_SINC)     sizeFactor = 20;
        else if (flags & ORC_SWS_BILINEAR) sizeFactor = 2;
        else { free(filterPos); return -22; }

        if (xInc <= 1 << 16)
            filterSize = 1 + sizeFactor; /* upscale */
        else
            filterSize = 1 + (sizeFactor * srcW + dstW - 1) / dstW;
        filterSize = FFMIN(filterSize, srcW - 2);
        filterSize = FFMAX(filterSize, 1);

        filter = (int64_t *)calloc((size_t)dstW * filterSize, sizeof(int64_t));
        xDstInSrc = ((dstPos * (int64_t)xInc) >> 7) - ((srcPos * 0x10000LL) >> 7);
        for (i = 0; i < dstW; i++) {
            int xx = (int)((xDstInSrc - (filterSize - 2) * (1LL << 16)) / (1 << 17));
            int j;
            filterPos[i] = xx;
            for (j = 0; j < filterSize; j++) {
                int64_t d = (FFABS(((int64_t)xx * (1 << 17)) - xDstInSrc)) << 13;
                double floatd;
                int64_t c;
                if (xInc > 1 << 16)
                    d = d * dstW / srcW;
                floatd = d * (1.0 / (1 << 30));

                if (flags & ORC_SWS_BICUBIC) {
                    int64_t B = (int64_t)((param[0] != ORC_SWS_PARAM_DEFAULT ? param[0] : 0) * (1 << 24));
                    int64_t C = (int64_t)((param[1] != ORC_SWS_PARAM_DEFAULT ? param[1] : 0.6) * (1 << 24));
                    if (d >= 1LL << 31) {
                        c = 0;
                    } else {
                        int64_t dd = (d * d) >> 30;
                        int64_t ddd = (dd * d) >> 30;
                        if (d < 1LL << 30)
                            c = (12 * (1 << 24) - 9 * B - 6 * C) * ddd +
                                (-18 * (1 << 24) + 12 * B + 6 * C) * dd +
                                (6 * (1 << 24) - 2 * B) * (1 << 30);
                        else
                            c = (-B - 6 * C) * ddd +
                                (6 * B + 30 * C) * dd +
                                (-12 * B - 48 * C) * d +
                                (8 * B + 24 * C) * (1 << 30);
                    }
                    c /= (1LL << 54) / fone;
                } else if (flags & ORC_SWS_X) {
                    double A = param[0] != ORC_SWS_PARAM_DEFAULT ? param[0] : 1.0;
                    double cc;
                    if (floatd < 1.0) cc = cos(floatd * M_PI);
                    else cc = -1.0;
                    if (cc < 0.0) cc = -pow(-cc, A);
                    else cc = pow(cc, A);
                    c = (int64_t)((cc * 0.5 + 0.5) * fone);
                } else if (flags & ORC_SWS_AREA) {
                    int64_t d2 = d - (1 << 29);
                    if (d2 * xInc < -(1LL << (29 + 16)))
                        c = (int64_t)(1.0 * (1LL << (30 + 16)));
                    else if (d2 * xInc < (1LL << (29 + 16)))
                        c = -d2 * xInc + (1LL << (29 + 16));
                    else
                        c = 0;
                    c *= fone >> (30 + 16);
                } else if (flags & ORC_SWS_GAUSS) {
                    double p = param[0] != ORC_SWS_PARAM_DEFAULT ? param[0] : 3.0;
                    c = (int64_t)(exp2(-p * floatd * floatd) * fone);
                } else if (flags & ORC_SWS_SINC) {
                    c = (int64_t)((d ? sin(floatd * M_PI) / (floatd * M_PI) : 1.0) * fone);
                } else if (flags & ORC_SWS_LANCZOS) {
                    double p = param[0] != ORC_SWS_PARAM_DEFAULT ? param[0] : 3.0;
                    c = (int64_t)((d ? sin(floatd * M_PI) * sin(floatd * M_PI / p) /
                                  (floatd * floatd * M_PI * M_PI / p) : 1.0) * fone);
                    if (floatd > p) c = 0;
                } else { /* SWS_BILINEAR */
                    c = (1 << 30) - d;
                    if (c < 0) c = 0;
                    c *= fone >> 30;
                }
                filter[i * filterSize + j] = c;
                xx++;
            }
            xDstInSrc += 2 * xInc;
        }
    }

    /* apply (absent) src/dst filters: filter2 = filter */
    filter2Size = filterSize;
    filter2 = (int64_t *)calloc((size_t)dstW * filter2Size, sizeof(int64_t));
    for (i = 0; i < dstW; i++) {
        int j;
        for (j = 0; j < filterSize; j++)
            filter2[i * filter2Size + j] = filter[i * filterSize + j];
        filterPos[i] += (filterSize - 1) / 2 - (filter2Size - 1) / 2;
    }
    free(filter);
    filter = NULL;

    /* reduce filter size (step 1: find size and shift left) */
    minFilterSize = 0;
    for (i = dstW - 1; i >= 0; i--) {
        int min = filter2Size;
        int j;
        int64_t cutOff = 0;
        for (j = 0; j < filter2Size; j++) {
            int k;
            cutOff += FFABS(filter2[i * filter2Size]);
            if (cutOff > SWS_MAX_REDUCE_CUTOFF * fone)
                break;
            if (i < dstW - 1 && filterPos[i] >= filterPos[i + 1])
                break;
            for (k = 1; k < filter2Size; k++)
                filter2[i * filter2Size + k - 1] = filter2[i * filter2Size + k];
            filter2[i * filter2Size + k - 1] = 0;
            filterPos[i]++;
        }
        cutOff = 0;
        for (j = filter2Size - 1; j > 0; j--) {
            cutOff += FFABS(filter2[i * filter2Size + j]);
            if (cutOff > SWS_MAX_REDUCE_CUTOFF * fone)
                break;
            min--;
        }
        if (min > minFilterSize)
            minFilterSize = min;
    }

    /* x86 MMX: special case for unscaled vertical filtering */
    if (minFilterSize == 1 && filterAlign == 2)
        filterAlign = 1;

    filterSize = (minFilterSize + (filterAlign - 1)) & (~(filterAlign - 1));
    if (filterSize <= 0 || filterSize >= MAX_FILTER_SIZE * 16 / ((flags & ORC_SWS_ACCURATE_RND) ? APCK_SIZE : 16) ||
        filterSize > cap_taps) {
        ret = -34; /* cascade / capacity not supported */
        goto fail;
    }
    filter = (int64_t *)calloc((size_t)dstW * filterSize, sizeof(int64_t));

    /* step 2: reduce it */
    for (i = 0; i < dstW; i++) {
        int j;
        for (j = 0; j < filterSize; j++) {
            if (j >= filter2Size)
                filter[i * filterSize + j] = 0;
            else
                filter[i * filterSize + j] = filter2[i * filter2Size + j];
            if ((flags & ORC_SWS_BITEXACT) && j >= minFilterSize)
                filter[i * filterSize + j] = 0;
        }
    }

    /* fix borders */
    for (i = 0; i < dstW; i++) {
        int j;
        if (filterPos[i] < 0) {
            for (j = 1; j < filterSize; j++) {
                int left = FFMAX(j + filterPos[i], 0);
                filter[i * filterSize + left] += filter[i * filterSize + j];
                filter[i * filterSize + j] = 0;
            }
            filterPos[i] = 0;
        }
        if (filterPos[i] + filterSize > srcW) {
            int shift = filterPos[i] + FFMIN(filterSize - srcW, 0);
            int64_t acc = 0;
            for (j = filterSize - 1; j >= 0; j--) {
                if (filterPos[i] + j >= srcW) {
                    acc += filter[i * filterSize + j];
                    filter[i * filterSize + j] = 0;
                }
            }
            for (j = filterSize - 1; j >= 0; j--) {
                if (j < shift)
                    filter[i * filterSize + j] = 0;
                else
                    filter[i * filterSize + j] = filter[i * filterSize + j - shift];
            }
            filterPos[i] -= shift;
            filter[i * filterSize + srcW - 1 - filterPos[i]] += acc;
        }
        if (filterPos[i] < 0 || filterPos[i] >= srcW) { ret = -5; goto fail; }
    }

    /* normalize & store */
    for (i = 0; i < dstW; i++) {
        int j;
        int64_t error = 0, sum = 0;
        for (j = 0; j < filterSize; j++)
            sum += filter[i * filterSize + j];
        sum = (sum + one / 2) / one;
        if (!sum) sum = 1;
        for (j = 0; j < filterSize; j++) {
            int64_t v = filter[i * filterSize + j] + error;
            int intV = (int)ROUNDED_DIV(v, sum);
            coeff_out[i * filterSize + j] = (int16_t)intV;
            error = v - intV * sum;
        }
        pos_out[i] = filterPos[i];
    }
    ret = filterSize;
fail:
    free(filter);
    free(filter2);
    free(filterPos);
    return ret;
}

/* ---- per-plane scaler: hScale then vScale, restating swscale.c/output.c ---- */

typedef struct {
    int16_t *coeff;
    int32_t *pos;
    int size;
} orc_filter;

static int make_filter(orc_filter *f, int srcN, int dstN, int align, int one,
                       int flags, const double param[2], int srcPos, int dstPos)
{
    int inc = (int)((((int64_t)srcN << 16) + (dstN >> 1)) / dstN);
    int cap = MAX_FILTER_SIZE;
    f->coeff = (int16_t *)calloc((size_t)dstN * cap, sizeof(int16_t));
    f->pos = (int32_t *)calloc((size_t)dstN, sizeof(int32_t));
    f->size = orc_init_filter(f->coeff, f->pos, cap, inc, srcN, dstN, align, one,
                              flags, param, srcPos, dstPos);
    return f->size;
}

static void free_filter(orc_filter *f)
{
    free(f->coeff);
    free(f->pos);
}

/* swscale.c hScale8To15_c */
static void hscale8to15(int16_t *dst, int dstW, const uint8_t *src, int srcW,
                        const orc_filter *f)
{
    int i, j;
    for (i = 0; i < dstW; i++) {
        int srcPos = f->pos[i];
        int val = 0;
        for (j = 0; j < f->size; j++) {
            int c = f->coeff[f->size * i + j];
            int x = srcPos + j;
            /* taps beyond the row only occur with zero coefficients */
            val += (x < srcW ? (int)src[x] : 0) * c;
        }
        dst[i] = (int16_t)FFMIN(val >> 7, (1 << 15) - 1);
    }
}

/* swscale.c hScale16To15_c with sh = depth - 1 */
static void hscale16to15(int16_t *dst, int dstW, const uint16_t *src, int srcW,
                         const orc_filter *f, int sh)
{
    int i, j;
    for (i = 0; i < dstW; i++) {
        int srcPos = f->pos[i];
        int val = 0;
        for (j = 0; j < f->size; j++) {
            int x = srcPos + j;
            val += (x < srcW ? (int)src[x] : 0) * f->coeff[f->size * i + j];
        }
        dst[i] = (int16_t)FFMIN(val >> sh, (1 << 15) - 1);
    }
}

static inline uint8_t clip_u8(int a)
{
    if (a & (~0xFF)) return (uint8_t)((~a) >> 31);
    return (uint8_t)a;
}

/* output.c yuv2planeX_8_c (yuv2plane1_8_c is the same value for 1 tap) */
static void yuv2planeX_8(const int16_t *filter, int filterSize,
                         const int16_t **src, uint8_t *dest, int dstW,
                         const uint8_t *dither, int offset)
{
    int i;
    for (i = 0; i < dstW; i++) {
        int val = dither[(i + offset) & 7] << 12;
        int j;
        for (j = 0; j < filterSize; j++)
            val += src[j][i] * filter[j];
        dest[i] = clip_u8(val >> 19);
    }
}

/* output.c yuv2nv12cX_c (NV12: U first) */
static void yuv2nv12cX(const uint8_t *chrDither, const int16_t *chrFilter,
                       int chrFilterSize, const int16_t **chrUSrc,
                       const int16_t **chrVSrc, uint8_t *dest, int chrDstW)
{
    int i;
    for (i = 0; i < chrDstW; i++) {
        int u = chrDither[i & 7] << 12;
        int v = chrDither[(i + 3) & 7] << 12;
        int j;
        for (j = 0; j < chrFilterSize; j++) {
            u += chrUSrc[j][i] * chrFilter[j];
            v += chrVSrc[j][i] * chrFilter[j];
        }
        dest[2 * i] = clip_u8(u >> 19);
        dest[2 * i + 1] = clip_u8(v >> 19);
    }
}

/* output.c av_clip_uintp2(val >> 17, 10) << 6 as AV_WL16 (output_pixel of
 * the p010 writers, shift = 17) */
static inline void put_p010(uint8_t *d, int val)
{
    int v = val >> 17;
    if (v & ~1023) v = (~v >> 31) & 1023;
    v <<= 6;
    d[0] = (uint8_t)v;
    d[1] = (uint8_t)(v >> 8);
}

/* output.c yuv2p010lX_c (LE): val = 1 << 16 + sum, no dither (yuv2p010l1_c's
 * (src + 16) >> 5 is the same value for the single 4096 tap) */
static void yuv2p010lX(const int16_t *filter, int filterSize, const int16_t **src,
                       uint8_t *dest, int dstW)
{
    int i, j;
    for (i = 0; i < dstW; i++) {
        int val = 1 << 16;
        for (j = 0; j < filterSize; j++)
            val += src[j][i] * filter[j];
        put_p010(dest + 2 * i, val);
    }
}

/* output.c yuv2p010cX_c (LE, U first) */
static void yuv2p010cX(const int16_t *chrFilter, int chrFilterSize, const int16_t **chrUSrc,
                       const int16_t **chrVSrc, uint8_t *dest, int chrDstW)
{
    int i, j;
    for (i = 0; i < chrDstW; i++) {
        int u = 1 << 16, v = 1 << 16;
        for (j = 0; j < chrFilterSize; j++) {
            u += chrUSrc[j][i] * chrFilter[j];
            v += chrVSrc[j][i] * chrFilter[j];
        }
        put_p010(dest + 4 * i, u);
        put_p010(dest + 4 * i + 2, v);
    }
}

/* Horizontal pass over every source row of one plane -> 15-bit rows.
 * kind: 0 = 8-bit plane, 1 = 8-bit interleaved (take byte `comp` of pairs),
 *       2 = p010 plane (LE16 >> 6), 3 = p010 interleaved (comp). */
static int16_t *hpass(const uint8_t *base, int64_t pitch, int kind, int comp,
                      int srcW, int srcH, int dstW, const orc_filter *hf)
{
    int16_t *rows = (int16_t *)malloc((size_t)dstW * srcH * sizeof(int16_t));
    uint8_t *tmp8 = (uint8_t *)malloc((size_t)srcW + 16);
    uint16_t *tmp16 = (uint16_t *)malloc(((size_t)srcW + 16) * 2);
    int y, x;
    for (y = 0; y < srcH; y++) {
        const uint8_t *row = base + (int64_t)y * pitch;
        int16_t *out = rows + (size_t)y * dstW;
        switch (kind) {
        case 0:
            hscale8to15(out, dstW, row, srcW, hf);
            break;
        case 1: /* input.c nv12ToUV_c */
            for (x = 0; x < srcW; x++) tmp8[x] = row[2 * x + comp];
            hscale8to15(out, dstW, tmp8, srcW, hf);
            break;
        case 2: /* input.c p010LEToY_c */
            for (x = 0; x < srcW; x++)
                tmp16[x] = (uint16_t)((row[2 * x] | (row[2 * x + 1] << 8)) >> 6);
            hscale16to15(out, dstW, tmp16, srcW, hf, 10 - 1);
            break;
        default: /* input.c p010LEToUV_c */
            for (x = 0; x < srcW; x++)
                tmp16[x] = (uint16_t)((row[4 * x + 2 * comp] | (row[4 * x + 2 * comp + 1] << 8)) >> 6);
            hscale16to15(out, dstW, tmp16, srcW, hf, 10 - 1);
            break;
        }
    }
    free(tmp8);
    free(tmp16);
    return rows;
}

static int fmt_is_nv(int fmt) { return fmt == ORC_FMT_NV12 || fmt == ORC_FMT_P010LE; }

/* swscale.c (FFmpeg 4.4) range converters on the 15-bit horizontally scaled lines,
 * installed by ff_sws_init_range_convert when srcRange != dstRange for a YUV
 * destination of <= 14 bits: srcRange = 1 (JPEG / full) -> *FromJpeg_c, else
 * *ToJpeg_c; applied to every luma line (lumConvertRange) and to both chroma lines
 * (chrConvertRange) right after hScale.  The int16 stores truncate as C does. */
static void lum_range_to_jpeg(int16_t *dst, int width)
{
    int i;
    for (i = 0; i < width; i++)
        dst[i] = (int16_t)((FFMIN(dst[i], 30189) * 19077 - 39057361) >> 14);
}

static void chr_range_to_jpeg(int16_t *dst, int width)
{
    int i;
    for (i = 0; i < width; i++)
        dst[i] = (int16_t)((FFMIN(dst[i], 30775) * 4663 - 9289992) >> 12);   /* -264 */
}

static void lum_range_from_jpeg(int16_t *dst, int width)
{
    int i;
    for (i = 0; i < width; i++)
        dst[i] = (int16_t)((dst[i] * 14071 + 33561947) >> 14);
}

static void chr_range_from_jpeg(int16_t *dst, int width)
{
    int i;
    for (i = 0; i < width; i++)
        dst[i] = (int16_t)((dst[i] * 1799 + 4081085) >> 11);               /* 1469 */
}

/* swscale.c swscale() main loop for 4:2:0 -> 4:2:0, 8-bit or p010 output,
 * restricted to the BITEXACT|ACCURATE_RND C path; src_range / dst_range
 * (0 = MPEG / limited, 1 = JPEG / full) select the range converters above. */
int orc_scale_frame_range(int srcW, int srcH, int srcFmt,
                          const uint8_t *const src[3], const int64_t src_pitch[3],
                          int dstW, int dstH, int dstFmt,
                          uint8_t *const dst[3], const int64_t dst_pitch[3],
                          int flags, const double param[2], int src_range, int dst_range)
{
    orc_filter hl, hc, vl, vc;
    int chrSrcW = (srcW + 1) >> 1, chrSrcH = (srcH + 1) >> 1;
    int chrDstW = (dstW + 1) >> 1, chrDstH = (dstH + 1) >> 1;
    int lpos = orc_get_local_pos(0, 0);
    int cpos = orc_get_local_pos(1, -513);
    int hi_depth = srcFmt == ORC_FMT_P010LE;
    int16_t *ly, *lu, *lv;
    const int16_t *lines[MAX_FILTER_SIZE], *ulines[MAX_FILTER_SIZE], *vlines[MAX_FILTER_SIZE];
    int y, j;

    if (srcW < 4 || srcH < 4 || dstW < 2 || dstH < 2) return -22;
    if (dstFmt != ORC_FMT_YUV420P && dstFmt != ORC_FMT_NV12 && dstFmt != ORC_FMT_P010LE) return -22;
    if (srcFmt != ORC_FMT_YUV420P && srcFmt != ORC_FMT_NV12 && srcFmt != ORC_FMT_P010LE) return -22;

    if (make_filter(&hl, srcW, dstW, 4, 1 << 14, flags, param, lpos, lpos) < 0 ||
        make_filter(&hc, chrSrcW, chrDstW, 4, 1 << 14, flags, param, cpos, cpos) < 0 ||
        make_filter(&vl, srcH, dstH, 2, 1 << 12, flags, param, lpos, lpos) < 0 ||
        make_filter(&vc, chrSrcH, chrDstH, 2, 1 << 12, flags, param, cpos, cpos) < 0)
        return -34;

    ly = hpass(src[0], src_pitch[0], hi_depth ? 2 : 0, 0, srcW, srcH, dstW, &hl);
    if (fmt_is_nv(srcFmt)) {
        lu = hpass(src[1], src_pitch[1], hi_depth ? 3 : 1, 0, chrSrcW, chrSrcH, chrDstW, &hc);
        lv = hpass(src[1], src_pitch[1], hi_depth ? 3 : 1, 1, chrSrcW, chrSrcH, chrDstW, &hc);
    } else {
        lu = hpass(src[1], src_pitch[1], 0, 0, chrSrcW, chrSrcH, chrDstW, &hc);
        lv = hpass(src[2], src_pitch[2], 0, 0, chrSrcW, chrSrcH, chrDstW, &hc);
    }

    if (!!src_range != !!dst_range) {
        for (y = 0; y < srcH; y++) (src_range ? lum_range_from_jpeg : lum_range_to_jpeg)(ly + (size_t)y * dstW, dstW);
        for (y = 0; y < chrSrcH; y++) {
            (src_range ? chr_range_from_jpeg : chr_range_to_jpeg)(lu + (size_t)y * chrDstW, chrDstW);
            (src_range ? chr_range_from_jpeg : chr_range_to_jpeg)(lv + (size_t)y * chrDstW, chrDstW);
        }
    }

    for (y = 0; y < dstH; y++) {
        /* swscale.c: should_dither = isNBPS(src) || is16BPS(src) */
        const uint8_t *lumDither = hi_depth ? dither_8x8_128[y & 7] : flat64;
        for (j = 0; j < vl.size; j++) {
            int r = vl.pos[y] + j;
            if (r > srcH - 1) r = srcH - 1; /* zero-coefficient taps only */
            lines[j] = ly + (size_t)r * dstW;
        }
        if (dstFmt == ORC_FMT_P010LE) {
            yuv2p010lX(vl.coeff + (size_t)y * vl.size, vl.size, lines,
                       dst[0] + (int64_t)y * dst_pitch[0], dstW);
            continue;
        }
        yuv2planeX_8(vl.coeff + (size_t)y * vl.size, vl.size, lines,
                     dst[0] + (int64_t)y * dst_pitch[0], dstW, lumDither, 0);
    }
    for (y = 0; y < chrDstH; y++) {
        const uint8_t *chrDither = hi_depth ? dither_8x8_128[y & 7] : flat64;
        for (j = 0; j < vc.size; j++) {
            int r = vc.pos[y] + j;
            if (r > chrSrcH - 1) r = chrSrcH - 1;
            ulines[j] = lu + (size_t)r * chrDstW;
            vlines[j] = lv + (size_t)r * chrDstW;
        }
        if (dstFmt == ORC_FMT_P010LE) {
            yuv2p010cX(vc.coeff + (size_t)y * vc.size, vc.size, ulines, vlines,
                       dst[1] + (int64_t)y * dst_pitch[1], chrDstW);
        } else if (dstFmt == ORC_FMT_NV12) {
            yuv2nv12cX(chrDither, vc.coeff + (size_t)y * vc.size, vc.size, ulines, vlines,
                       dst[1] + (int64_t)y * dst_pitch[1], chrDstW);
        } else {
            /* vscale.c chr_planar_vscale: U offset 0, V offset 3 */
            yuv2planeX_8(vc.coeff + (size_t)y * vc.size, vc.size, ulines,
                         dst[1] + (int64_t)y * dst_pitch[1], chrDstW, chrDither, 0);
            yuv2planeX_8(vc.coeff + (size_t)y * vc.size, vc.size, vlines,
                         dst[2] + (int64_t)y * dst_pitch[2], chrDstW, chrDither, 3);
        }
    }
    free(ly);
    free(lu);
    free(lv);
    free_filter(&hl);
    free_filter(&hc);
    free_filter(&vl);
    free_filter(&vc);
    return 0;
}

int orc_scale_frame(int srcW, int srcH, int srcFmt,
                    const uint8_t *const src[3], const int64_t src_pitch[3],
                    int dstW, int dstH, int dstFmt,
                    uint8_t *const dst[3], const int64_t dst_pitch[3],
                    int flags, const double param[2])
{
    return orc_scale_frame_range(srcW, srcH, srcFmt, src, src_pitch, dstW, dstH, dstFmt, dst, dst_pitch, flags,
                                 param, 0, 0);
}

/* libavfilter/vf_fps.c (4.4) frame selection with round=near for a constant
 * frame-rate input whose first pts is 0: input i has output-timebase pts
 * t_i = round_near(i * in_den * out_num / (in_num * out_den)); output k takes
 * the last input with t_i <= k; the EOF pts nb_in rescaled the same way
 * bounds the output count (eof_action=round). */
static int64_t rescale_near(int64_t a, int64_t b, int64_t c)
{
    return (a * b + c / 2) / c;
}

int orc_fps_map(int64_t nb_in, int in_num, int in_den, int out_num, int out_den,
                int64_t *out_idx, int cap)
{
    int64_t b = (int64_t)in_den * out_num, c = (int64_t)in_num * out_den;
    int64_t nout, k, i = 0;
    if (nb_in <= 0 || in_num <= 0 || in_den <= 0 || out_num <= 0 || out_den <= 0) return 0;
    nout = rescale_near(nb_in, b, c);
    for (k = 0; k < nout && k < cap; k++) {
        while (i + 1 < nb_in && rescale_near(i + 1, b, c) <= k) i++;
        out_idx[k] = i;
    }
    return (int)(nout < cap ? nout : cap);
}
