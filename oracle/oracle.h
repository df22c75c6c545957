/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the pixel path a
 * reference ffmpeg worker would run (FFmpeg 4.4 libswscale + libavfilter C
 * paths).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library, and only as the checker / CPU baseline.  The
 * product (libdts.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned".  The reference repository
 * (/root/reference: index.js, database.js) contains no pixel code and no
 * tests (package.json:7); its only hot-path touchpoint is the unused
 * ffmpeg-static 4.4.0 binary path (index.js:9, package-lock.json:384-397).
 * No ffmpeg binary, libswscale or FFmpeg source exists in this container, so
 * this restatement is written from the published FFmpeg 4.4 C code and is
 * pinned only by known-answer properties that hold for libswscale by
 * construction (tests/test_oracle.py).  See DESIGN.md "Oracle".
 */
#ifndef DTS_ORACLE_H
#define DTS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* libswscale flag values (swscale.h, FFmpeg 4.4) */
#define ORC_SWS_FAST_BILINEAR 0x1
#define ORC_SWS_BILINEAR      0x2
#define ORC_SWS_BICUBIC       0x4
#define ORC_SWS_X             0x8
#define ORC_SWS_POINT         0x10
#define ORC_SWS_AREA          0x20
#define ORC_SWS_BICUBLIN      0x40
#define ORC_SWS_GAUSS         0x80
#define ORC_SWS_SINC          0x100
#define ORC_SWS_LANCZOS       0x200
#define ORC_SWS_SPLINE        0x400
#define ORC_SWS_ACCURATE_RND  0x40000
#define ORC_SWS_BITEXACT      0x80000
#define ORC_SWS_PARAM_DEFAULT 123456

/* pixel formats handled by the oracle (values match include/dts.h) */
#define ORC_FMT_YUV420P 0
#define ORC_FMT_NV12    1
#define ORC_FMT_P010LE  2

/* libswscale/utils.c initFilter() restated.  Caller supplies output storage
 * of capacity `cap_taps` taps per output (coeff is dstW*cap_taps int16,
 * pos is dstW int32).  Returns the final filter size (>0) or <0 on error. */
int orc_init_filter(int16_t *coeff, int32_t *pos, int cap_taps,
                    int xInc, int srcW, int dstW, int filterAlign, int one,
                    int flags, const double param[2], int srcPos, int dstPos);

/* utils.c get_local_pos() */
int orc_get_local_pos(int chr_subsample, int pos);

/* One frame through the scaler: src/dst formats in {YUV420P, NV12, P010LE}
 * (p010 output: output.c yuv2p010lX_c / yuv2p010cX_c); planes addressed by data[3]/pitch[3] in bytes (for NV12 and
 * P010 plane 1 is the interleaved UV plane, plane 2 unused).
 * Returns 0 or <0 on unsupported parameters. */
int orc_scale_frame(int srcW, int srcH, int srcFmt,
                    const uint8_t *const src[3], const int64_t src_pitch[3],
                    int dstW, int dstH, int dstFmt,
                    uint8_t *const dst[3], const int64_t dst_pitch[3],
                    int flags, const double param[2]);

/* The same with libswscale's range conversion: src_range / dst_range 0 = MPEG
 * (limited), 1 = JPEG (full); different ranges run swscale.c's lum/chrRange
 * To/FromJpeg_c on the 15-bit horizontal output. */
int orc_scale_frame_range(int srcW, int srcH, int srcFmt,
                          const uint8_t *const src[3], const int64_t src_pitch[3],
                          int dstW, int dstH, int dstFmt,
                          uint8_t *const dst[3], const int64_t dst_pitch[3],
                          int flags, const double param[2], int src_range, int dst_range);

/* vf_psnr compute_images_mse for one 8-bit plane: returns the integer SSE. */
uint64_t orc_plane_sse8(const uint8_t *a, int64_t apitch, const uint8_t *b,
                        int64_t bpitch, int w, int h);

/* vf_ssim ssim_plane for one 8-bit plane (mean SSIM over the plane). */
double orc_plane_ssim8(const uint8_t *a, int64_t apitch, const uint8_t *b,
                       int64_t bpitch, int w, int h);

/* vf_psnr / vf_ssim frame records for a 4:2:0 8-bit frame (3 planes). */
typedef struct {
    uint64_t sse[3];
    double mse[3], mse_avg;
    double psnr[3], psnr_avg;
    double ssim[3], ssim_all, ssim_db;
} orc_qstat;
void orc_quality_frame420(int w, int h, const uint8_t *const a[3],
                          const int64_t apitch[3], const uint8_t *const b[3],
                          const int64_t bpitch[3], orc_qstat *q);

/* vf_fps: output frame k -> input frame index (round=near).  Writes up to
 * `cap` indices, returns the number of output frames. */
int orc_fps_map(int64_t nb_in, int in_num, int in_den, int out_num, int out_den,
                int64_t *out_idx, int cap);

/* HDR10 (p010, PQ, bt2020nc, limited) -> SDR bt709 8-bit 4:2:0 at the same
 * size (vf_tonemap_ref.c): zscale linearise + primaries + vf_tonemap MODE
 * (0 none, 1 linear, 2 gamma, 3 clip, 4 reinhard, 5 hable, 6 mobius) + zscale
 * bt709 out (out_full: r=pc, else r=tv).  param NaN = vf_tonemap default;
 * peak <= 0 -> 10; npl <= 0 -> 100.  w and h even.  Returns 0 or <0. */
int orc_hdr_to_sdr_frame(int w, int h, const uint8_t *const src[3], const int64_t src_pitch[3],
                         int dstFmt, uint8_t *const dst[3], const int64_t dst_pitch[3],
                         int mode, double param, double desat, double peak, double npl, int out_full);
double orc_tonemap_param(int mode, double param);

/* vf_yadif (vf_yadif_ref.c) on one 8-bit yuv420p frame: prev/cur/next planes
 * share pitch[]; mode 0..3 (send_frame, send_field, *_nospatial); tff = field
 * order; is_second = second field of send_field modes.  Returns 0 or <0. */
int orc_yadif_frame(int w, int h, const uint8_t *const prev[3], const uint8_t *const cur[3],
                    const uint8_t *const next[3], const int64_t pitch[3], uint8_t *const dst[3],
                    const int64_t dpitch[3], int mode, int tff, int is_second);
void orc_bt2020_to_bt709(double m[3][3]);

#ifdef __cplusplus
}
#endif
#endif
