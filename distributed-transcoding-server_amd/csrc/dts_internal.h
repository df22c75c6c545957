// dts_internal.h -- shared between the host side of libdts (api.cpp,
// filters.cpp) and the HIP kernels (kernels.hip).  All code here is compiled
// by hipcc for gfx950 (device) and x86-64 (host).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/dts.h"

namespace dts {

// Diagnostic A/B knobs (DTS_L7_W, DTS_L7_SORT, DTS_ORDER ...): read from the environment only
// in the diagnostic builds of tools/ (-DDTS_DIAG_KNOBS).  The default libdts.so reads two
// documented settings and nothing else: DTS_HOST_THREADS (host-path packing threads) and
// DTS_LADDER (kernel selection for the fallback parity tests; include/dts.h).
inline const char *diag_env(const char *name)
{
#ifdef DTS_DIAG_KNOBS
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}


// ---------------------------------------------------------------------------
// Ladder (scale + format convert) launch geometry
// ---------------------------------------------------------------------------
constexpr int kThreads = 256;      // workgroup size (4 waves)
constexpr int kBlkRows = 8;        // source rows per pipeline step (4 row pairs)
constexpr int kLumaCols = 256;     // output columns per luma strip (1 per thread)
constexpr int kChromaCols = 128;   // output columns per chroma strip (U: t<128, V: t>=128)
constexpr int kMaxLoads = 4;       // uint4 staging loads per thread per step
constexpr int kMaxRungs = DTS_MAX_OUTPUTS;

// H tap-dword counts the ladder kernel has unrolled code for; the host pads a
// filter's packed window with zero taps up to the next one.
inline int ladder_nd_round(int nd)
{
    if (nd <= 8) return nd < 1 ? 1 : nd;
    if (nd <= 16) return (nd + 1) & ~1;
    return nd;              // > 16: rejected at graph creation
}

// source kinds: what the staging loads unpack
enum SrcKind : int { kSrcPlanar8 = 0, kSrcNV12 = 1, kSrcP010 = 2 };

struct DevPlanes {                  // one batch of frames in HBM
    uint64_t data[3];
    int64_t pitch[3];
    int64_t fstride;
};

struct RungKind {                   // GPU tables of one rung for luma (0) or chroma (1)
    int32_t dstW, dstH;
    int32_t nd;                     // H: coefficient dwords per output (u8: 4 taps, p010: 2 taps)
    int32_t nv;                     // V: row pairs per output row
    int32_t nblocks;                // source pipeline steps
    int32_t pad_;
    const int32_t *hpos;            // [dstW] first source sample of the GPU window
    const int32_t *hbias;           // [dstW] 128 * sum(coeff) (u8 path)
    const uint32_t *hch;            // [nd][dstW] u8: high i8x4 parts; p010: int16x2 pairs
    const uint32_t *hcl;            // [nd][dstW] u8: low i8x4 parts
    const int32_t *vpos;            // [dstH] even first source row of the GPU window
    const uint32_t *vcoef;          // [dstH][nv] int16x2 (even row low, odd row high)
    const int32_t *vlim;            // [nblocks] output rows finished after step b
};

struct Job {                        // one workgroup's work inside a frame
    int16_t rung, kind;             // kind 0 = luma, 1 = chroma (U and V)
    int32_t x0;                     // first output column of the strip
    int32_t ncols;                  // columns in this strip
    int32_t sx0;                    // first source sample staged (16-byte aligned in bytes)
    int32_t swb;                    // staged bytes per source row per plane (multiple of 16)
    int32_t nload;                  // uint4 staging loads per step (all planes, all rows)
};

struct LadderParams {
    DevPlanes src;
    DevPlanes dst[kMaxRungs];
    int32_t dst_fmt[kMaxRungs];
    int32_t srcW, srcH, chrW, chrH;
    int32_t src_kind;
    int32_t nrungs;
    int32_t njobs;
    int32_t ring_pairs;             // power of two
    int32_t stage_bytes;            // one stage buffer (all planes), bytes
    int32_t nframes;
    int32_t nitems;                 // nframes * njobs work items (frame-major, heavy jobs first)
    const Job *jobs;                // device [njobs]
    const RungKind *rk;             // device [nrungs][2]
    unsigned int *queue;            // device work counter (zeroed before the launch)
};

// ---------------------------------------------------------------------------
// v4 ladder (ladder4.hip): row-pair H from VGPRs, LDS ring, per-column V
// ---------------------------------------------------------------------------
constexpr int kRing4Cols = 64;      // output columns per strip (V: lane = column)
constexpr int kRing4Slots = 96;     // ring row pairs: one 64-pair step + up to 32 pairs of V reach
constexpr int kRing4Dw = kRing4Slots * (kRing4Cols + 1);        // ring dwords (odd column pitch)
constexpr int kH4CoefDw = 256;      // LDS tap pairs per wave group (outputs x N rounded up to 4)
constexpr int kV4CoefDw = 1152;     // LDS V tap pairs per step buffer (rows x NV rounded up to 4)
constexpr int kV4SlotMax = 144;     // output rows per step buffer
constexpr int kLds4Bytes = 4 * (kRing4Dw + 4 * kH4CoefDw + 2 * kV4CoefDw + 2 * kV4SlotMax);

struct HGroup4 {                    // one wave's share of a strip
    uint64_t mask;                  // bit q: an output's window starts at sample pair q
    int32_t lofs;                   // byte offset of the window in the source row (16-aligned, may be < 0)
    int16_t nload;                  // 16-byte loads per row (per plane)
    int16_t qend;                   // 1 + last start pair (0: no outputs)
    int32_t coef;                   // first tap-pair dword of the group in its H table
    int32_t col0;                   // ring column of the group's first output
};

struct Job4 {                       // one strip of one plane of one rendition
    int16_t rk;                     // rung * 2 + kind
    int16_t kind;                   // 0 = luma, 1 = chroma
    int16_t rung;
    int16_t plane;                  // chroma: 0 = U, 1 = V
    int32_t x0, ncols, group0;      // first output column, columns, first HGroup4
};

struct RungKind4 {
    int32_t N;                      // H tap pairs per output (kernel bucket)
    int32_t NV;                     // V row pairs per output row
    int32_t nsteps;                 // 128-row source steps
    int32_t pad_;
    const HGroup4 *groups;          // [strips][4]
    const uint32_t *hcoef;          // int16x2 tap pairs, round_up(N, 4) per output, group after group
    const int32_t *vslot;           // [dstH] ring slot of the first row pair
    const uint32_t *vcoef;          // [dstH][round_up(NV, 4)] int16x2
    const int32_t *vlim;            // [nsteps] output rows finished after step b
};

struct Ladder4Params {
    DevPlanes src;
    DevPlanes dst[kMaxRungs];
    int32_t dst_fmt[kMaxRungs];
    int32_t srcH, chrH, ring, src_kind, njobs, nitems, nframes;
    int32_t nq;                     // work queues (1, or 8 = one per XCD; frame f in queue f % nq)
    const Job4 *jobs;
    const RungKind4 *rk;
    unsigned int *queue;            // nq counters
};

hipError_t launch_ladder4(const Ladder4Params &p, int lds_bytes, int grid, hipStream_t s);
int ladder4_blocks_per_cu(int src_kind, int lds_bytes);

// ---------------------------------------------------------------------------
// v5 ladder (ladder5.hip): both FIR passes on the matrix cores
// (v_mfma_i32_16x16x64_i8), every rendition of a column strip from one staged
// copy of the source rows.
// ---------------------------------------------------------------------------
constexpr int kL5Rows = 16;         // source rows of one H row block (the H MFMA's M)
constexpr int kL5Blk = 2;           // H row blocks per step (one barrier per step)
constexpr int kL5StepRows = kL5Rows * kL5Blk;
constexpr int kL5Waves = 12;        // waves per workgroup (one workgroup per CU: 3 waves per SIMD)
constexpr int kL5Threads = 64 * kL5Waves;
constexpr int kL5Ent = 5;           // H entries (K blocks of 64 source columns) per wave
constexpr int kL5MaxRings = 2 * DTS_MAX_OUTPUTS;
constexpr int kL5Stages = 3;        // stage buffers (bundle s in buffer s % 3: two in flight behind the one H reads)
constexpr int kL5FragBufs = 2;      // V fragment buffers (V(b)'s in buffer b % 2, loaded the step before)
constexpr int kL5MaxDma = 15;       // LDS-DMA instructions per wave per step (1 KB each)
constexpr int kL5MaxVkb = 2;        // V K blocks (64 source rows) per row group
constexpr int kL5Bias = 128 << 14;  // 128 * sum(H taps): the (src ^ 0x80) offset of every H output
constexpr int kL5VBias = (128 << 12) + (64 << 12);   // 128 * sum(V taps) ((y & 255) ^ 0x80) + flat dither
// per-item rendition table in LDS (bytes 16..): per rendition 16 dwords {x0, nct, pitch[3] (32-bit),
// pad, plane base lo/hi x 3 (this frame)}
constexpr int kL5RungTab = 4 * 16 * DTS_MAX_OUTPUTS;

struct Ent5 {                       // 16, 8 or 4 H outputs over one K block of 64 source columns
    int32_t bfrag;                  // B fragment pair (hi 1 KB, lo 1 KB; 16 B per lane)
    int16_t soff;                   // byte offset of the K block in the staged row (multiple of 8)
    int16_t col0;                   // ring column of the entry's first output
    int8_t plane;                   // staged plane (chroma: 0 = U, 1 = V)
    int8_t ring;                    // ring of the entry's outputs
    int8_t flags;                   // 4: nv12 V (odd bytes of the staged row); 8 / 16: 8 / 4 outputs
    int8_t pad_;
};

struct Ring5 {                      // H outputs of one (rendition, plane): two column-major byte planes
    int32_t hi;                     // LDS byte offset: y >> 8 of (column c, source row r) at hi + c*CP + r % RR
    int32_t lo;                     // LDS byte offset of (y & 255) ^ 0x80
    int32_t CP;                     // column pitch, bytes (16 x odd: conflict-free V A reads)
    int32_t RR;                     // rows held, a multiple of 16
};

struct VEnt5 {                      // one V row group of one rendition, ready after its step (one s_load)
    int32_t rung;
    int32_t G;                      // output rows 16 G .. 16 G + rows - 1
    int32_t rows;                   // valid rows (<= 16)
    int32_t w0;                     // ring row of the first source row of its K blocks (w0 % RR, multiple of 8)
    int32_t nkb;                    // K blocks of 64 source rows
    int32_t foff;                   // byte offset of its first V fragment pair (taps >> 8, taps & 255 as
                                    // signed bytes) in its step's fragment area
    int32_t fmt;                    // the rendition's output format
    int32_t dstW;                   // columns of its output plane(s) of this kind
    Ring5 ring0;                    // its ring (chroma: U)
    int32_t hi1, lo1;               // chroma: the V plane's ring (same CP, RR)
    int32_t pad_[2];
};

struct Out5 {                       // one rendition's output of this plane kind
    int32_t fmt;                    // DTS_FMT_YUV420P / DTS_FMT_NV12
    int32_t dstW, dstH;
    int32_t pad_;
};

struct Strip5 {                     // one column strip of a plane kind
    int32_t L;                      // first staged sample column (multiple of 16)
    int32_t cpr;                    // 16-B chunks per staged row per load plane (odd)
    int32_t Pb;                     // staged row pitch = 16 cpr bytes (16 x odd: conflict-free A reads)
    int32_t PS;                     // load plane stride in a stage buffer (16 rows, rounded up to 1 KB)
    int32_t nsi;                    // source LDS-DMA instructions per step (load planes x PS / 1 KB)
    int32_t hextra;                 // waves 0 .. hextra - 1 hold one H entry more than the rest
    int32_t pad_[2];
    int32_t ent0[kL5Waves], nent[kL5Waves];   // each wave's H entries
    int32_t x0[DTS_MAX_OUTPUTS];    // first output column per rendition (multiple of 16)
    int32_t nct[DTS_MAX_OUTPUTS];   // 16-column tiles per rendition
};

struct Kind5 {                      // luma (1 plane) or chroma (U + V) of every rendition
    int32_t nplanes, nsteps, srcH;
    int32_t nlp;                    // load planes (planar chroma 2; luma, nv12 chroma 1: U V interleaved)
    int32_t stage;                  // byte offset of the kL5Stages stage buffers (source rows)
    int32_t SB;                     // stage buffer size (load planes)
    int32_t FA;                     // byte offset of the kL5FragBufs V fragment buffers (V(b): buffer b % 2)
    int32_t FB;                     // fragment buffer size
    int32_t nrings, nrungs, nstrips;
    Ring5 ring[kL5MaxRings];        // rendition r, plane p: ring[r * nplanes + p]
    Out5 out[DTS_MAX_OUTPUTS];
    const Strip5 *strips;
    const Ent5 *ents;
    const uint32_t *bfrag;          // H, then V fragment pairs (in step order), 512 dwords each
    uint32_t nbfrag;                // fragment pairs
    const VEnt5 *vsched;            // the V row groups of every step, step after step
    const int4 *vstep;              // [nsteps + 1]: {first group, end, first V fragment pair, its KB count}
};

struct Job5 {
    int32_t kind, strip;
};

struct Ladder5Params {
    DevPlanes src;
    DevPlanes dst[kMaxRungs];
    int32_t njobs, nframes, nq, pad_;
    const Job5 *jobs;
    const Kind5 *kinds;
    unsigned int *queue;
};

hipError_t launch_ladder5(const Ladder5Params &p, int src_kind, int lds_bytes, int grid, hipStream_t s);
int ladder5_blocks_per_cu(int src_kind, int lds_bytes);

// ---------------------------------------------------------------------------
// ladder work units (plan6.cpp, ladder7.hip): one wave per (frame, plane kind,
// rendition, column group), walking the plane top to bottom; the H outputs stay
// in VGPRs (the H MFMA's C layout is the V MFMA's A layout).
// ---------------------------------------------------------------------------
constexpr int kL6Gran = 16;         // source rows per granule (the H MFMA's M)
constexpr int kL6Stages = 4;        // V fragment slots: row blocks firing within this many granules
constexpr int kL6Variants = 8;      // (column tiles CT, planes NP, H K blocks, V K blocks)

// variant v: NP planes (luma 1; chroma 2: U and V), HKB K blocks of 64 source columns
// per H tile, VKB K blocks of 64 source rows (4 VKB granules held) per V row block, and
// CT 16-column tiles per plane: 4 MFMA tiles when HKB = VKB = 1, else 2
// (k_ladder7 only: + 8 = "narrow", the one-K-block variants with half the tiles;
// + 16 = 16-bit (p010) source samples: one column tile per plane, the H K blocks of 64
// samples read as two MFMA K blocks of raw little-endian bytes)
constexpr int kL7Variants = 32;
constexpr int l6_variant(int np, int hkb, int vkb, bool narrow = false)
{
    return (np == 2 ? 4 : 0) + 2 * (hkb - 1) + (vkb - 1) + (narrow && hkb == 1 && vkb == 1 ? 8 : 0);
}
constexpr int l6_np(int v) { return (v & 4) ? 2 : 1; }
constexpr int l6_hkb(int v) { return ((v >> 1) & 1) + 1; }
constexpr int l6_vkb(int v) { return (v & 1) + 1; }
constexpr int l6_ct(int v) { return (v & 16) ? 1 : ((v & 3) == 0 && !(v & 8) ? 4 : 2) / l6_np(v); }
// k_ladder7 variants whose A operands are two ds_read_b64 (K windows on 8-column
// boundaries allowed): one H K block, two V K blocks (luma 2 tiles, chroma 1 tile per plane)
constexpr bool l7_b64(int v) { return v == 1 || v == 5; }

struct Unit6 {                      // one wave's share of a frame
    int32_t variant;                // l6_variant(): the walk shape
    int32_t kind;                   // 0 luma, 1 chroma (U and V planes in one unit)
    int32_t rung;
    int32_t col0;                   // first output column (multiple of 16)
    int32_t ncols;                  // output columns this unit stores (<= 16 CT)
    int32_t ngran;                  // source granules (srcH / 16, rounded up)
    int32_t srcH, dstH;
    int32_t nrb;                    // row blocks (16 output rows) of the rendition
    int32_t fmt;                    // the rendition's output format
    uint32_t hfrag;                 // H fragment pair of tile c, K block kb: hfrag + c * HKB + kb
    uint32_t vfrag;                 // V fragment pair of row block j, K block kb: vfrag + j * VKB + kb
    int32_t fire;                   // the rendition's fire table: row block j runs after granule fire[j]
    int32_t dstW;
    int32_t x0[4];                  // first source column of each column tile's H K blocks (multiple of 4,
                                    // except a right-edge tile ending at the plane's last column)
    int32_t fs;                     // V fragment slots in LDS: most row blocks firing within kL6Stages granules
    int32_t vdedup;                 // 1: the rendition's V fragments are stored once per distinct fragment and
                                    // fire entry j carries its index in bits 10..15 (granule in bits 0..9)
};


// ---------------------------------------------------------------------------
// v7 ladder (ladder7.hip, plan6.cpp plan7_graph): the work-unit waves (Unit6 variants,
// same H -> V register pipeline), grouped into workgroups that cover one source
// column strip of one plane kind for every rendition.  Per granule the group
// stages the strip's 16 source rows into LDS once (LDS-DMA pieces dealt over its
// waves, one barrier per granule) and every wave reads its A operands from there:
// the source crosses L2 -> CU about once per frame instead of once per rendition
// and column tile.
// ---------------------------------------------------------------------------
constexpr int kL7Stages = 2;        // staging batches per group (in flight + being read)
constexpr int kL7Batch = 2;         // granules per staging batch (one barrier per batch; 1: cfg2 143k, 2: 154k fps)
constexpr int kL7MaxWaves = 16;     // waves per group (workgroup of <= 1024 threads)

struct Unit7 {                      // one wave of a group
    int32_t variant;                // as Unit6
    int32_t kind, rung, col0, ncols, ngran, srcH, dstH, nrb, fmt;
    uint32_t hfrag, vfrag;
    int32_t fire, dstW;
    int32_t xo[4];                  // byte offset of each tile's H K window in the staged strip (x0 - X0, multiple
                                    // of 16; of 8 in the l7_b64 variants)
    int32_t fs;                     // V fragment slots of the rendition in this group
    int32_t flds;                   // LDS offset of the rendition's fragment slots
    int32_t lead;                   // 1: this wave DMAs the rendition's V fragments for the group
    int32_t rc_sh;                  // range conversion of the 15-bit H output (0: none):
    int32_t rc_cap, rc_mul, rc_add; //   y = (min(y, cap) * mul + add) >> sh, as swscale.c's lum/chr
                                    //   RangeToJpeg_c / RangeFromJpeg_c (int16 store)
    int32_t vdedup;                 // as Unit6
};

struct Group7 {                     // one workgroup's strip of one frame
    int32_t kind;                   // 0 luma, 1 chroma (U and V)
    int32_t X0;                     // first staged source column (multiple of 16)
    int32_t npc;                    // staged pieces per plane and granule (64 columns each)
    int32_t nwaves;                 // units (the other waves of the workgroup only stage)
    int32_t u0;                     // first unit
    int32_t ngran, srcH;
    int32_t scr;                    // LDS offset of the per-wave store exchange (1 KB per wave)
    int32_t xown;                   // the next strip's X0 (plane width for the last): diagnostics only
    int32_t bpc;                    // staged bytes per source column: 1 (8-bit planes; chroma: U and V
                                    // planes), 2 (nv12 chroma: U V byte pairs; p010 luma), 4 (p010
                                    // chroma: U V 16-bit pairs); bpc npc pieces per plane and granule
    int32_t st0;                    // first staging wave: waves st0.. deal the source pieces (a group's spare
                                    // waves when it has fewer units than the workgroup has waves, else all)
};

struct Ladder7Params {
    DevPlanes src;
    DevPlanes dst[kMaxRungs];
    int32_t ngroups, nframes;
    int32_t sup;                    // (diagnostic order 3: octets per luma-then-chroma run)
    int32_t pad7_;
    int32_t order, nluma;           // dispatch order (1: each frame octet's luma groups first, then the
                                    // chroma groups; 0: plan order; 2: chroma first), the plan's
                                    // leading kind-0 (luma) groups
    const Group7 *groups;
    const Unit7 *units;
    const uint32_t *frag;           // as Ladder6Params
    const int32_t *fire;
};

hipError_t launch_ladder7(const Ladder7Params &p, int grid, int waves, int lds_bytes, bool range_conv, int hsplit,
                          int src_kind, hipStream_t s);   // src_kind: SrcKind
void ladder7_compiled(int *stages, int *batch);   // NS7 / PB7 of the linked k_ladder7

// ---------------------------------------------------------------------------
// Quality (vf_psnr + vf_ssim) launch geometry
// ---------------------------------------------------------------------------
constexpr int kQTileBX = 64;        // 4x4 blocks per tile, x (nv12 chroma: 32, the same bytes per row)
constexpr int kQTileBY = 16;        // 4x4 blocks per tile, y
#ifndef DTS_Q_WALK
#define DTS_Q_WALK 4
#endif
#ifndef DTS_Q_WALK_NV12
#define DTS_Q_WALK_NV12 DTS_Q_WALK
#endif
#ifndef DTS_Q_BAL
#define DTS_Q_BAL 1        // 0: walks of exactly kQWalk tiles (the last one short)
#endif
constexpr int kQWalk = DTS_Q_WALK;  // tiles per k_quality workgroup, walked top to bottom
constexpr int kQWalkNV12 = DTS_Q_WALK_NV12;   // the same for nv12 renditions

struct QualityParams {
    DevPlanes a, b;
    int32_t pw[3], ph[3];           // plane sizes
    int32_t tbx[3];                 // tile width in blocks (kQTileBX; nv12 chroma kQTileBX / 2)
    int32_t tiles_x[3], tiles_y[3]; // tiles_y: walks of `walk` tiles
    int32_t walk[3];                // tiles per walk, per plane (about kQWalk / kQWalkNV12: quality_enqueue)
    int32_t tile_base[4];           // prefix of tiles per plane
    int32_t interleaved;            // 1 = nv12 (plane 1 holds U,V interleaved)
    int32_t nframes;
    double *partial_ssim;           // [nframes][tiles]
    unsigned long long *partial_sse;// [nframes][tiles]
    dts_qraw *out;                  // [nframes]
};

// ---------------------------------------------------------------------------
// HDR10 -> SDR (hdr.hip)
// ---------------------------------------------------------------------------
constexpr int kTmLutN = 1024;      // intervals of the PQ EOTF / BT.709 OETF tables over [0, 1]
// The PQ table is indexed by x + kTmPqOff for every x the 10-bit codes can produce (R', G', B' x
// kTmLutN lie in [-1176, 2220]: hdr.hip pixel<>), flat outside [0, kTmLutN], so its lookup
// needs no clamp: kTmPqN entries
constexpr int kTmPqOff = 1280, kTmPqN = 3584;
#ifndef DTS_TM_ROWS
#define DTS_TM_ROWS 64
#endif
constexpr int kTmRows = DTS_TM_ROWS; // 2x2-block rows per k_tonemap workgroup
struct TonemapParams {
    DevPlanes src;                  // p010 at the output size (ladder intermediate)
    DevPlanes dst;                  // 8-bit yuv420p / nv12
    int32_t dst_fmt, w, h, nframes; // w, h even; nframes <= 65535
    int32_t mode;                   // DTS_TM_*
    float param, desat, peak, hpeak, inv_hpeak, scale;   // hpeak = hable(peak), scale = 10000 / npl
    float inv_hpeak_n;              // kTmLutN / hpeak (hable's normalisation folded into the OETF table scale)
    float hk1, hk0;                 // hable(x) / x = (A (1 - E/F) x + B (C - E/F)) / den, x kTmLutN / hpeak
    float qy[4];                    // output range (zscale r=tv / r=pc): Y = qy0 R' + qy1 G' + qy2 B' + qy3
    float qcb[2], qcr[2];           // Cb' = sb B' + qcb0 Y + qcb1 (Cr' likewise), Y as above
    float qc;                       // chroma scale: 224 C + 128.5 (tv) / 255 C + 128.5 (pc)
    float m[9];                     // bt2020 -> bt709 linear primaries, row-major
    const float2 *lut;              // device [2][kTmLutN + 1] (intercept, slope) chords in table units: PQ EOTF
                                    // x 10000 / npl, BT.709 OETF
};
hipError_t launch_tonemap(const TonemapParams &p, hipStream_t s);     // tiled (k_tonemap)
hipError_t launch_tonemap_w(const TonemapParams &p, hipStream_t s);   // column walk (k_tonemap_w)

// ---------------------------------------------------------------------------
// vf_yadif (deint.hip)
// ---------------------------------------------------------------------------
struct YadifParams {
    DevPlanes seq;                  // nseq yuv420p frames (fstride apart)
    DevPlanes dst;                  // output frames of this launch
    int32_t w, h, nseq, first;      // outputs come from frames first, first + 1, ...
    int32_t mode, tff;              // yadif mode 0..3, field order
    int32_t aligned;                // every plane base / pitch of seq and dst is a multiple of 4
};
hipError_t launch_yadif(const YadifParams &p, int nout, hipStream_t s);
// the temporal walk (k_yadif_t): outputs of frames first .. first + count - 1 (x2 for the
// field modes); every plane base / pitch of seq and dst 16-byte aligned (yadif_t_ok)
bool yadif_t_ok(const YadifParams &p);
hipError_t launch_yadif_t(const YadifParams &p, int count, hipStream_t s);

// ---------------------------------------------------------------------------
// Synthetic source (testsrc2-like), identical on host and device
// ---------------------------------------------------------------------------
__host__ __device__ inline uint32_t synth_hash(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__host__ __device__ inline uint32_t synth_noise(uint32_t seed, int x, int y, int64_t f, int comp)
{
    return synth_hash(seed ^ ((uint32_t)x * 0x9E3779B1u) ^ ((uint32_t)y * 0x85EBCA77u) ^
                      ((uint32_t)f * 0xC2B2AE3Du) ^ ((uint32_t)comp * 0x27D4EB2Fu));
}

__host__ __device__ inline int synth_clampi(int v, int lo, int hi)
{
    return v < lo ? lo : (v > hi ? hi : v);
}

// comp 0 = Y (plane size w x h), 1 = U, 2 = V (plane size cw x ch).
// Returns an 8-bit sample, or a 10-bit sample when ten_bit.
__host__ __device__ inline int synth_sample(int pattern, uint32_t seed, int x, int y, int64_t f,
                                            int comp, int pw, int ph, bool ten_bit)
{
    uint32_t n = synth_noise(seed, x, y, f, comp);
    if (pattern == 1)
        return ten_bit ? (int)(n & 1023u) : (int)(n & 255u);
    int fm = (int)(f % 4096);
    int span = pw + ph;
    int v;
    if (comp == 0) {
        int g = ((x + y + 2 * fm) % span) * 219 / span;
        int barw = pw / 16 > 0 ? pw / 16 : 1;
        int bar = (((x + 4 * fm) / barw) & 1) ? 24 : 0;
        int nz = (int)(n & 31u) - 16;
        v = 16 + g + bar + nz;
        v = synth_clampi(v, 16, 235);
    } else {
        int g = comp == 1 ? ((x + fm) % (pw > 0 ? pw : 1)) * 224 / (pw > 0 ? pw : 1)
                          : ((y + fm) % (ph > 0 ? ph : 1)) * 224 / (ph > 0 ? ph : 1);
        int nz = (int)(n & 7u) - 4;
        v = synth_clampi(16 + g + nz, 16, 240);
    }
    if (ten_bit) {
        int lo = comp == 0 ? 64 : 64, hi = comp == 0 ? 940 : 960;
        v = synth_clampi(v * 4 + (int)((n >> 8) & 3u), lo, hi);
    }
    return v;
}

// ordered dither libswscale ff_dither_8x8_128 (FFmpeg 4.4 swscale.c; values
// restated from memory)
#define DTS_DITHER_8X8_128                                              \
    {                                                                   \
        {36, 68, 60, 92, 34, 66, 58, 90}, {100, 4, 124, 28, 98, 2, 122, 26}, \
        {52, 84, 44, 76, 50, 82, 42, 74}, {116, 20, 108, 12, 114, 18, 106, 10}, \
        {32, 64, 56, 88, 38, 70, 62, 94}, {96, 0, 120, 24, 102, 6, 126, 30}, \
        {48, 80, 40, 72, 54, 86, 46, 78}, {112, 16, 104, 8, 118, 22, 110, 14}, \
    }

// kernels.hip entry points (host-side launchers)
hipError_t launch_ladder(const LadderParams &p, int ndmax, int lds_bytes, int grid, hipStream_t s);
int ladder_blocks_per_cu(int src_kind, int ndmax, int lds_bytes);   // occupancy for the persistent grid
hipError_t launch_quality(const QualityParams &p, int total_tiles, hipStream_t s);
hipError_t launch_qsum(const dts_qraw *raw, int n, dts_qraw *sum, hipStream_t s);
hipError_t launch_synth(int w, int h, int fmt, int pattern, uint32_t seed, int64_t first,
                        const DevPlanes &dst, int nframes, hipStream_t s);
int ladder_ndmax_for(int nd);       // template bucket for a required nd (0 = unsupported)

} // namespace dts
