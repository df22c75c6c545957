/*
 * dts.h -- C-ABI of the MI355X-native transcoding worker (libdts.so).
 *
 * Drop-in boundary for the reference's per-segment pixel path.  The reference
 * (BadAimWeeb/distributed-transcoding-server) would get this path by spawning
 * the ffmpeg binary whose path it resolves at index.js:9
 * (`require("ffmpeg-static")`, ffmpeg 4.4.0 per package-lock.json:384-397)
 * with a filtergraph built from the job row fields Jobs.width / height /
 * framerate (database.js:73-75) for the segment JobChunks.chunkOffset
 * (database.js:109).  The spawn/dispatch code itself is absent from the
 * reference (index.js:13 constructs socket.io with no handlers), so each entry
 * point below names the ffmpeg/libav* interface it replaces:
 *
 *   dts_graph_create   <- `-vf scale=W:H:flags=<m>+accurate_rnd+bitexact,
 *                          format=<fmt>` / `-filter_complex split=N...`
 *                          (vf_scale.c config_props -> sws_init_context)
 *   dts_graph_submit   <- the per-frame filter_frame() of that graph
 *   (+ _wait)             (vf_scale.c scale_frame -> sws_scale), plus the
 *                          optional `psnr`/`ssim` filters against a reference
 *   dts_quality_*      <- vf_psnr.c do_psnr / vf_ssim.c do_ssim
 *   dts_fps_map        <- vf_fps.c frame selection (round=near)
 *   dts_yadif_run_device <- `-vf yadif` (vf_yadif.c)
 *   dts_synth_*        <- `-f lavfi testsrc2` (synthetic source; testsrc2 itself
 *                          needs ffmpeg, so this is a deterministic stand-in)
 *
 * Conventions: every call returns 0 (DTS_OK) or a negative DTS_E_* code and
 * never throws or aborts across the ABI.  Plain pointers and sizes only.
 *
 * Environment: the library reads two settings.  DTS_HOST_THREADS = host threads that
 * pack / unpack frames on the host path (default: the hardware threads, at most 16).
 * DTS_LADDER = 5 / 4 / 3 keeps a graph off the default ladder kernel (k_ladder7) and on
 * a fallback (k_ladder5 / k_ladder4 / the v3 kernel) -- the fallbacks run frames whose
 * planes are not 16-byte aligned or geometries k_ladder7 does not plan; the parity tests
 * force them with it.  Nothing else is read (diagnostic A/B builds under tools/ read more).
 * One dts_ctx per GPU; a ctx and its graphs are single-threaded (the caller
 * serialises calls); distinct ctxs may be driven from different threads.
 */
#ifndef DTS_H
#define DTS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 7: dts_host_alloc / dts_host_free / dts_host_register / dts_host_unregister (pinned
 * host frames the host path DMAs straight from and into).
 * ABI 6: dts_output_spec gained quality / qref_method (rendition quality).  A binding
 * compiled against this header checks dts_abi_version() == DTS_ABI_VERSION and
 * dts_abi_struct_size() of every struct it lays out before any other call. */
#define DTS_ABI_VERSION 7
#define DTS_MAX_OUTPUTS 4

/* error codes (AVERROR-style negative ints) */
#define DTS_OK             0
#define DTS_E_INVAL      (-22)   /* bad argument / spec */
#define DTS_E_NOMEM      (-12)
#define DTS_E_RANGE      (-34)   /* filter too large for the GPU tables */
#define DTS_E_UNSUPPORTED (-95)  /* format / method combination not built */
#define DTS_E_BUSY       (-16)   /* submit while a previous submit is pending */
#define DTS_E_NODEV      (-19)   /* no HIP device */
#define DTS_E_HIP      (-1000)   /* HIP runtime error; see dts_ctx_last_hip_error */

/* pixel formats (yuv420p / nv12 / p010le as in libavutil/pixfmt.h) */
#define DTS_FMT_YUV420P 0
#define DTS_FMT_NV12    1
#define DTS_FMT_P010LE  2

/* scaling methods = libswscale SWS_* flag values (swscale.h) */
#define DTS_SCALE_BILINEAR 0x2
#define DTS_SCALE_BICUBIC  0x4
#define DTS_SCALE_X        0x8
#define DTS_SCALE_POINT    0x10
#define DTS_SCALE_AREA     0x20
#define DTS_SCALE_GAUSS    0x80
#define DTS_SCALE_SINC     0x100
#define DTS_SCALE_LANCZOS  0x200
#define DTS_PARAM_DEFAULT  123456.0 /* SWS_PARAM_DEFAULT */

/* HDR10 -> SDR tone mapping curves: vf_tonemap.c enum TonemapAlgorithm */
#define DTS_TM_NONE     0
#define DTS_TM_LINEAR   1
#define DTS_TM_GAMMA    2
#define DTS_TM_CLIP     3
#define DTS_TM_REINHARD 4
#define DTS_TM_HABLE    5
#define DTS_TM_MOBIUS   6

/* quality checks (vf_psnr / vf_ssim) */
#define DTS_Q_NONE 0
#define DTS_Q_PSNR 1
#define DTS_Q_SSIM 2
#define DTS_Q_BOTH 3

typedef struct dts_ctx dts_ctx;
typedef struct dts_graph dts_graph;

typedef struct dts_tonemap_spec {
    int32_t mode;       /* DTS_TM_* (vf_tonemap tonemap=) */
    int32_t pad_;
    double param;       /* vf_tonemap param; NaN = the curve's default (init()) */
    double desat;       /* vf_tonemap desat; <= 0 = off.  vf_tonemap's default is 2.0
                           (FFmpeg 4.4 tonemap_options): the bindings (N-API addon,
                           dtsffi, node/ladder.js) default to it */
    double peak;        /* vf_tonemap peak (units of npl); <= 0 = its fallback for
                           linear input without HDR side data: 10 */
    double npl;         /* zscale npl, cd/m^2 mapped to 1.0; <= 0 = 100 */
} dts_tonemap_spec;

typedef struct dts_output_spec {
    int32_t w, h;       /* output size (even for 4:2:0 not required) */
    int32_t fmt;        /* DTS_FMT_YUV420P, DTS_FMT_NV12 or DTS_FMT_P010LE
                           (output.c yuv2p010lX_c / yuv2p010cX_c) */
    int32_t method;     /* DTS_SCALE_*; always run as method|ACCURATE_RND|BITEXACT */
    double param[2];    /* sws param[0..1]; DTS_PARAM_DEFAULT for defaults */
    /* Rendition quality (ABI 6): `[rendition][reference]psnr` / `ssim` of this output
     * against a reference rendition of the same size and format that the graph makes
     * from the same source frames with qref_method (e.g. DTS_SCALE_LANCZOS), all on the
     * device -- the quality a CPU worker gets from a second scale branch of its
     * filtergraph.  DTS_Q_* (0 = off); 8-bit outputs, no HDR graph, and not together
     * with dts_graph_spec.quality (an external reference). */
    int32_t quality;
    int32_t qref_method;    /* DTS_SCALE_*, or DTS_QREF_EXTERNAL: the reference renditions come
                               with every dts_graph_run_device call (its qref then points to nout
                               batches; entries of outputs without quality are not read) */
} dts_output_spec;

#define DTS_QREF_EXTERNAL (-1)

typedef struct dts_graph_spec {
    int32_t src_w, src_h, src_fmt;      /* source segment frames */
    int32_t nout;                       /* 1..DTS_MAX_OUTPUTS renditions */
    dts_output_spec out[DTS_MAX_OUTPUTS];
    int32_t quality;                    /* DTS_Q_* */
    int32_t quality_out;                /* output index compared with qref */
    int32_t max_batch;                  /* frames per device launch; 0 = 32 */
    /* HDR10 -> SDR (BASELINE config 3): the source is p010 PQ bt2020nc
     * limited range; every output (8-bit yuv420p/nv12, even w/h) is scaled
     * bit-exactly to a p010 intermediate and then converted as by
     *   zscale=t=linear:npl=NPL,format=gbrpf32le,zscale=p=bt709,
     *   tonemap=MODE:param=P:desat=D:peak=K,zscale=t=bt709:m=bt709:r=R
     * (float path, +-1 LSB vs the double restatement); R = tv, or pc when
     * `range` names a JPEG output range (the source range must be MPEG). */
    int32_t hdr_to_sdr;                 /* 0 = off */
    dts_tonemap_spec tonemap;
    /* Deinterlace ahead of the ladder (`-vf yadif=MODE:PARITY,scale=...`, vf_yadif.c):
     * 8-bit yuv420p sources, frame-rate modes 0 (send_frame) and 2 (send_frame_nospatial).
     * With it on, every source batch carries one context frame on each side: src
     * holds nframes + 2 frames, outputs are made for src[1 .. nframes] (each with
     * prev = its predecessor, next = its successor in the batch); at the start / end
     * of a stream the caller repeats the first / last frame (yadif's clone).
     * Segments therefore overlap their neighbours by one frame each way. */
    int32_t deint;                      /* 0 = off, 1 = yadif */
    int32_t deint_mode;                 /* 0 or 2 */
    int32_t deint_tff;                  /* 1 = top field first, 0 = bottom */
    /* YUV range conversion (`scale=in_range=R:out_range=R`, libswscale srcRange /
     * dstRange): source range | output range << 4, each DTS_RANGE_*.  Different
     * ranges run swscale.c's lum/chrRangeToJpeg / FromJpeg on the 15-bit
     * horizontal output (every rendition takes the output range).  Supported for
     * 8-bit planar sources on the v7 ladder (plane widths multiples of 16); else
     * dts_graph_create returns DTS_E_UNSUPPORTED.  HDR graphs: no swscale step, the
     * output range is the final zscale's r= (above). */
    int32_t range;
} dts_graph_spec;

#define DTS_RANGE_MPEG 0                /* limited / tv (16..235, 16..240) */
#define DTS_RANGE_JPEG 1                /* full / pc (0..255) */

/* host frame: plane p at data[p] with row pitch pitch[p] bytes.
 * yuv420p: Y, U, V.  nv12 / p010le: Y, interleaved UV, (unused). */
typedef struct dts_frame {
    void *data[3];
    int64_t pitch[3];
} dts_frame;

/* device-resident batch: frame f plane p at data[p] + f * frame_stride.
 * Source pitches and plane bases must be multiples of 16 bytes, output
 * pitches multiples of 4. */
typedef struct dts_dev_frames {
    void *data[3];
    int64_t pitch[3];
    int64_t frame_stride;
} dts_dev_frames;

/* raw per-frame quality record as produced on the device and gathered
 * across GPUs (integer SSE exact; SSIM window sums in f64). */
typedef struct dts_qraw {
    uint64_t sse[3];
    double ssim_sum[3];
} dts_qraw;

/* finished per-frame statistics, same meaning as the lavfi.psnr.* /
 * lavfi.ssim.* frame metadata of vf_psnr.c / vf_ssim.c */
typedef struct dts_qstat {
    uint64_t sse[3];
    double mse[3], mse_avg;
    double psnr[3], psnr_avg;   /* +inf when mse == 0 */
    double ssim[3], ssim_all, ssim_db;
} dts_qstat;

typedef struct dts_graph_info {
    int64_t src_frame_bytes;            /* packed algorithmic bytes per source frame */
    int64_t out_frame_bytes[DTS_MAX_OUTPUTS];
    int64_t algo_bytes_per_frame;       /* read src once + write outputs (+ read qref) */
    int32_t njobs;                      /* workgroups per frame in the ladder launch */
    int32_t lds_bytes;                  /* dynamic LDS per workgroup */
    int32_t h_taps[DTS_MAX_OUTPUTS][2]; /* GPU H tap span (luma, chroma) per output */
    int32_t v_taps[DTS_MAX_OUTPUTS][2]; /* GPU V tap span (luma, chroma) per output */
    int32_t sws_h_size[DTS_MAX_OUTPUTS][2]; /* libswscale filter sizes (luma, chroma) */
    int32_t sws_v_size[DTS_MAX_OUTPUTS][2];
    int32_t ladder_v4_mask;             /* bit 2*output+kind: that plane kind runs on the v4
                                           ladder kernel (the rest on v3; DTS_LADDER=3 forces v3) */
    int32_t h_pairs4[DTS_MAX_OUTPUTS][2]; /* v4 H tap pairs per output (luma, chroma), 0 = v3 */
    int32_t ladder_v5;                  /* 1: the whole graph runs on the v5 ladder kernel (H on the
                                           matrix cores); 3: on the v7 kernel (H and V on the matrix
                                           cores, H outputs in registers, waves in workgroups that
                                           stage each source strip once; plane widths multiples of
                                           16; v5 / v4 for frames whose planes are not 16-byte
                                           aligned).  2 (the retired v6 kernel) is no longer
                                           produced.  DTS_LADDER=5 (or 6) / 4 / 3 force v5 / v4 / v3 */
    int32_t v5_strip_width[2];          /* v5 source columns per strip (luma, chroma) */
    int32_t v5_strips[2];               /* v5 strips per plane kind */
} dts_graph_info;

const char *dts_version(void);
const char *dts_strerror(int err);
/* The ABI the library was built with (its DTS_ABI_VERSION), and sizeof() of each struct
 * above as the library sees it (DTS_STRUCT_*; DTS_E_INVAL for an unknown id). */
int dts_abi_version(void);
int64_t dts_abi_struct_size(int which);
#define DTS_STRUCT_TONEMAP_SPEC 0
#define DTS_STRUCT_OUTPUT_SPEC  1
#define DTS_STRUCT_GRAPH_SPEC   2
#define DTS_STRUCT_FRAME        3
#define DTS_STRUCT_DEV_FRAMES   4
#define DTS_STRUCT_QRAW         5
#define DTS_STRUCT_QSTAT        6
#define DTS_STRUCT_GRAPH_INFO   7

int dts_device_count(int *count);
int dts_ctx_create(int device, dts_ctx **out);
void dts_ctx_destroy(dts_ctx *ctx);
int dts_ctx_last_hip_error(const dts_ctx *ctx);

int dts_graph_create(dts_ctx *ctx, const dts_graph_spec *spec, dts_graph **out);
void dts_graph_destroy(dts_graph *g);
int dts_graph_info_get(const dts_graph *g, dts_graph_info *info);
/* Plan only: validates spec and fills info (filter sizes, kernel choice,
 * work items) exactly as dts_graph_create would, without a device. */
int dts_graph_plan(const dts_graph_spec *spec, dts_graph_info *info);

/* Host-memory path (the Node worker's path).  dst holds nframes*nout frames,
 * frame-major (dst[f*nout + k]); src holds nframes (+ 2 with deint: see above).
 * qref/q may be NULL when quality is off.  With rendition quality (dts_output_spec
 * quality) q, if not NULL, holds nframes*nout statistics, frame-major like dst
 * (entries of outputs without quality are zeroed) and qref is not used.  A graph with
 * an output whose qref_method is DTS_QREF_EXTERNAL is refused (DTS_E_UNSUPPORTED):
 * external references come with dts_graph_run_device only.
 * The caller keeps every buffer alive until dts_graph_wait returns. */
int dts_graph_submit(dts_graph *g, const dts_frame *src, int nframes,
                     const dts_frame *dst, const dts_frame *qref, dts_qstat *q);
int dts_graph_wait(dts_graph *g);

/* Pinned host memory for the host path (ABI 7).  A chunk of dts_graph_submit whose source
 * (and qref) frames all lie in pinned memory the library knows is copied to the device by
 * DMA straight from the caller's planes, and a chunk whose output frames all do is copied
 * straight into them: no pass through the library's pinned rings (the host threads'
 * pack / unpack copies, which bound the pageable path).  Frames anywhere else take the
 * ring as before.  Direct frames need the device batch's row pitch (row bytes rounded up
 * to 16); consecutive frames laid out exactly as the device batch (planes rounded up to
 * 256 bytes, frames back to back) move as one DMA per run, the padding bytes between their
 * planes included (an output run overwrites them).  dts_host_alloc: page-locked memory
 * usable by every device (hipHostMalloc portable), released by dts_host_free.  dts_host_register: page-lock a
 * caller range (hipHostRegister portable) until dts_host_unregister; a range overlapping an
 * allocation or another registered range is refused (DTS_E_INVAL).  Replaces the
 * pageable frame buffers an ffmpeg worker's decoder / encoder hand around. */
int dts_host_alloc(size_t bytes, void **out);
void dts_host_free(void *p);
int dts_host_register(void *p, size_t bytes);
int dts_host_unregister(void *p);

/* Device-resident path: enqueue one batch on `stream` (a hipStream_t, NULL =
 * the ctx's stream).  dst[k] is the batch of output k.  When the graph has
 * quality on, qref is the reference batch for output quality_out and qraw
 * receives nframes device-side dts_qraw records (device pointer).  With rendition
 * quality qref is not used and qraw receives nframes*nout records, output-major
 * (record k*nframes + f; those of outputs without quality are left as they were). */
int dts_graph_run_device(dts_graph *g, const dts_dev_frames *src, int nframes,
                         const dts_dev_frames *dst, const dts_dev_frames *qref,
                         dts_qraw *qraw_dev, void *stream);

/* Standalone quality (vf_psnr + vf_ssim) on device-resident 8-bit 4:2:0
 * batches (fmt yuv420p or nv12 for both a and b). */
int dts_quality_run_device(dts_ctx *ctx, int w, int h, int fmt,
                           const dts_dev_frames *a, const dts_dev_frames *b,
                           int nframes, dts_qraw *qraw_dev, void *stream);
/* The same on host frames (a[i] vs b[i], i < nframes): uploads, runs and returns
 * the finished per-frame statistics in out[nframes].  Synchronous.  Used by the
 * Node worker for each rendition against its reference rendition. */
int dts_quality_run_host(dts_ctx *ctx, int w, int h, int fmt, const dts_frame *a, const dts_frame *b,
                         int nframes, dts_qstat *out);
/* vf_yadif (FFmpeg 4.4, 8-bit yuv420p) on a device-resident sequence of nseq
 * frames: outputs are made for frames first .. first+count-1, each with
 * prev = frame i-1 and next = frame i+1 clamped to the sequence (yadif's
 * clone of the first / last frame).  mode 0 send_frame, 1 send_field (2 outputs
 * per frame: first then second field), 2 / 3 the same without the spatial
 * interlacing check; tff 1 = top field first (yadif parity auto on progressive-
 * flagged input), 0 = bottom first.  dst holds count (x2 for field modes)
 * frames.  Replaces `-vf yadif=mode:parity` (vf_yadif.c filter_slice). */
int dts_yadif_run_device(dts_ctx *ctx, int w, int h, int mode, int tff, const dts_dev_frames *seq, int nseq,
                         int first, int count, const dts_dev_frames *dst, void *stream);

/* vf_psnr get_psnr / vf_ssim ssim_db finishing of raw records (host). */
int dts_qstat_finalize(int w, int h, const dts_qraw *raw, int n, dts_qstat *out);
/* A segment's quality record: the n device records at raw_dev summed into one
 * record at sum_dev (u64 SSE exact, f64 SSIM window sums in a fixed order), on
 * `stream`.  These are the running sums vf_psnr / vf_ssim keep over a stream;
 * records of several segments (gathered from several GPUs) add up the same way. */
int dts_qraw_sum_device(dts_ctx *ctx, const dts_qraw *raw_dev, int n, dts_qraw *sum_dev, void *stream);
/* End-of-stream averages of nframes frames from their summed record, as vf_psnr /
 * vf_ssim print them at uninit: psnr[c] / psnr_avg from the mean MSE (not the mean
 * dB), ssim[c] / ssim_all the mean SSIM.  Replaces reading the "PSNR y:.. average:"
 * and "SSIM Y:.. All:" lines from an ffmpeg worker's log. */
int dts_qstat_stream(int w, int h, const dts_qraw *sum, int64_t nframes, dts_qstat *out);

/* Synthetic deterministic source (testsrc2-like): pattern 0 = gradient +
 * moving bars + seeded noise (limited range), 1 = uniform random full range. */
int dts_synth_host(int w, int h, int fmt, int pattern, uint32_t seed,
                   int64_t frame_index, const dts_frame *dst);
int dts_synth_device(dts_ctx *ctx, int w, int h, int fmt, int pattern,
                     uint32_t seed, int64_t first_frame,
                     const dts_dev_frames *dst, int nframes, void *stream);

/* Layout helper: bytes per plane for a tightly packed frame (pitch = row bytes). */
int dts_frame_layout(int w, int h, int fmt, int64_t pitch[3], int64_t rows[3],
                     int64_t *packed_bytes);

/* Diagnostic: the libswscale filter (initFilter, SWS_BITEXACT|ACCURATE_RND,
 * x86 filterAlign) that a graph builds for one direction of one plane.
 * one = 1<<14 (horizontal) or 1<<12 (vertical); pos = get_local_pos() siting.
 * Writes dst_n*cap int16 taps (row stride = returned size) and dst_n
 * positions; returns the filter size (>0) or <0.  Needs no device. */
int dts_sws_filter(int src_n, int dst_n, int one, int align, int method,
                   const double param[2], int pos, int16_t *coeff, int32_t *filter_pos,
                   int cap);

/* vf_fps (round=near) frame index map for a constant-rate input starting at
 * pts 0.  Returns the output frame count (<= cap written) or <0. */
int64_t dts_fps_map(int64_t nb_in, int in_num, int in_den, int out_num,
                    int out_den, int64_t *out_idx, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* DTS_H */
