/*
 * vf_quality_ref.c -- TEST INFRASTRUCTURE ONLY (see oracle.h header).
 *
 * Restatement of the FFmpeg 4.4 libavfilter quality filters a reference
 * ffmpeg worker would attach for the per-segment quality check
 * (`psnr` / `ssim` filters; BASELINE.json config 4).  [ext] functions:
 *   vf_psnr.c  sse_line_8bit, compute_images_mse, get_psnr, do_psnr
 *   vf_ssim.c  ssim_4x4xn_8bit, ssim_end1, ssim_endn_8bit, ssim_plane,
 *              do_ssim, ssim_db
 * Parity unpinned (FFmpeg absent; reference has no tests, package.json:7).
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>

/* vf_psnr.c sse_line_8bit + compute_images_mse (one plane) */
uint64_t orc_plane_sse8(const uint8_t *a, int64_t apitch, const uint8_t *b,
                        int64_t bpitch, int w, int h)
{
    uint64_t m = 0;
    int i, j;
    for (i = 0; i < h; i++) {
        unsigned m2 = 0;
        const uint8_t *ma = a + i * apitch, *mb = b + i * bpitch;
        for (j = 0; j < w; j++) {
            int d = ma[j] - mb[j];
            m2 += (unsigned)(d * d);
        }
        m += m2;
    }
    return m;
}

/* vf_ssim.c ssim_4x4xn_8bit */
static void ssim_4x4xn_8bit(const uint8_t *main, int64_t main_stride,
                            const uint8_t *ref, int64_t ref_stride,
                            int (*sums)[4], int width)
{
    int x, y, z;
    for (z = 0; z < width; z++) {
        uint32_t s1 = 0, s2 = 0, ss = 0, s12 = 0;
        for (y = 0; y < 4; y++) {
            for (x = 0; x < 4; x++) {
                int a = main[x + y * main_stride];
                int b = ref[x + y * ref_stride];
                s1 += a;
                s2 += b;
                ss += a * a;
                ss += b * b;
                s12 += a * b;
            }
        }
        sums[z][0] = (int)s1;
        sums[z][1] = (int)s2;
        sums[z][2] = (int)ss;
        sums[z][3] = (int)s12;
        main += 4;
        ref += 4;
    }
}

/* vf_ssim.c ssim_end1 (8-bit) */
static float ssim_end1(int s1, int s2, int ss, int s12)
{
    static const int ssim_c1 = (int)(.01 * .01 * 255 * 255 * 64 + .5);
    static const int ssim_c2 = (int)(.03 * .03 * 255 * 255 * 64 * 63 + .5);
    int fs1 = s1, fs2 = s2, fss = ss, fs12 = s12;
    int vars = fss * 64 - fs1 * fs1 - fs2 * fs2;
    int covar = fs12 * 64 - fs1 * fs2;
    return (float)(2 * fs1 * fs2 + ssim_c1) * (float)(2 * covar + ssim_c2) /
           ((float)(fs1 * fs1 + fs2 * fs2 + ssim_c1) * (float)(vars + ssim_c2));
}

/* vf_ssim.c ssim_endn_8bit */
static float ssim_endn_8bit(const int (*sum0)[4], const int (*sum1)[4], int width)
{
    float ssim = 0.0f;
    int i;
    for (i = 0; i < width; i++)
        ssim += ssim_end1(sum0[i][0] + sum0[i + 1][0] + sum1[i][0] + sum1[i + 1][0],
                          sum0[i][1] + sum0[i + 1][1] + sum1[i][1] + sum1[i + 1][1],
                          sum0[i][2] + sum0[i + 1][2] + sum1[i][2] + sum1[i + 1][2],
                          sum0[i][3] + sum0[i + 1][3] + sum1[i][3] + sum1[i + 1][3]);
    return ssim;
}

/* vf_ssim.c ssim_plane (8-bit; float accumulator as in FFmpeg 4.4) */
double orc_plane_ssim8(const uint8_t *main, int64_t main_stride, const uint8_t *ref,
                       int64_t ref_stride, int width, int height)
{
    int z = 0, y;
    float ssim = 0.0f;
    int (*temp)[4] = (int (*)[4])calloc((size_t)2 * ((width >> 2) + 3), sizeof(int[4]));
    int (*sum0)[4] = temp;
    int (*sum1)[4] = sum0 + (width >> 2) + 3;
    double r;

    width >>= 2;
    height >>= 2;
    for (y = 1; y < height; y++) {
        for (; z <= y; z++) {
            int (*t)[4] = sum0;
            sum0 = sum1;
            sum1 = t;
            ssim_4x4xn_8bit(&main[4 * z * main_stride], main_stride,
                            &ref[4 * z * ref_stride], ref_stride, sum0, width);
        }
        ssim += ssim_endn_8bit((const int (*)[4])sum0, (const int (*)[4])sum1, width - 1);
    }
    free(temp);
    r = ssim / ((height - 1) * (width - 1));
    return r;
}

/* vf_psnr.c get_psnr */
static double get_psnr(double mse, uint64_t nb_frames, int max)
{
    return 10.0 * log10((double)((unsigned)max * (unsigned)max) / (mse / nb_frames));
}

/* vf_ssim.c ssim_db */
static double ssim_db(double ssim, double weight)
{
    return 10.0 * log10(weight / (weight - ssim));
}

/* do_psnr + do_ssim for one yuv420p frame (planes 0..2, 8-bit) */
void orc_quality_frame420(int w, int h, const uint8_t *const a[3],
                          const int64_t apitch[3], const uint8_t *const b[3],
                          const int64_t bpitch[3], orc_qstat *q)
{
    int pw[3], ph[3], c;
    double sum = 0, mse = 0, ssimv = 0;
    pw[0] = w;
    ph[0] = h;
    pw[1] = pw[2] = (w + 1) >> 1;
    ph[1] = ph[2] = (h + 1) >> 1;
    for (c = 0; c < 3; c++) sum += (double)pw[c] * ph[c];
    for (c = 0; c < 3; c++) {
        double weight = (double)pw[c] * ph[c] / sum;
        q->sse[c] = orc_plane_sse8(a[c], apitch[c], b[c], bpitch[c], pw[c], ph[c]);
        q->mse[c] = q->sse[c] / (double)(pw[c] * ph[c]);
        q->psnr[c] = get_psnr(q->mse[c], 1, 255);
        mse += q->mse[c] * weight;
        q->ssim[c] = orc_plane_ssim8(a[c], apitch[c], b[c], bpitch[c], pw[c], ph[c]);
        ssimv += weight * q->ssim[c];
    }
    q->mse_avg = mse;
    q->psnr_avg = get_psnr(mse, 1, 255); /* average_max = 255 for 8-bit */
    q->ssim_all = ssimv;
    q->ssim_db = ssim_db(ssimv, 1.0);
}
