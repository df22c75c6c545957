// api.cpp -- C-ABI of libdts (include/dts.h).
//
// Host side of the MI355X worker: builds libswscale-identical filter tables
// once per graph (vf_scale config_props -> sws_init_context equivalent), owns
// the device tables / batch buffers / pinned staging rings, and enqueues the
// ladder + quality kernels.  Replaces the ffmpeg child process the reference
// would spawn from the path resolved at /root/reference/index.js:9.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "dts_internal.h"
#include "filters.h"

using namespace dts;

#ifdef DTS_L5_STAMP
namespace dts { int ladder5_stamps(unsigned long long *out, bool reset); }
#endif
#ifdef DTS_L7_STAMP
namespace dts { int ladder7_stamps(unsigned long long *out, bool reset); }
#endif

// Quality partials (per-tile SSE / SSIM sums) of one k_quality -> k_qreduce
// pair.  `ev` marks the last launch that used the buffer: the next user waits
// on it, whatever stream it runs on, so two in-flight batches never share
// partials (the host path's two streams used to race on one).
struct QScratch {
    void *p = nullptr;
    size_t bytes = 0;
    hipEvent_t ev = nullptr;
    // the deinterlaced source frames of a graph with deint on (one batch), ordered the same way
    void *dp = nullptr;
    size_t dbytes = 0;
    hipEvent_t dev = nullptr;
    // the reference renditions of rendition quality (one batch of each), ordered the same way
    void *rp = nullptr;
    size_t rbytes = 0;
    hipEvent_t rev = nullptr;
};

struct dts_ctx {
    int device = 0;
    int last_hip = 0;
    hipStream_t stream[2] = {nullptr, nullptr};
    QScratch qs;                               // dts_quality_run_device
    // dts_quality_run_host: one batch of both frame sets + its records, kept across calls
    // (the worker scores every segment of every rendition: no allocation per call)
    uint8_t *hq = nullptr;
    size_t hq_bytes = 0;
    // graphs hold a reference: the context outlives every graph made on it,
    // whichever of dts_ctx_destroy / dts_graph_destroy runs first
    std::atomic<int> refs{1};
};

namespace {

constexpr int kSwsAccurateRnd = 0x40000;
constexpr int kQueueSlots = 64;
constexpr int kQueueWidth = 8;            // counters per slot: one per XCD for k_ladder4

// k_ladder4 work queues: one per XCD unless DTS_XCD=0 (diagnostic A/B builds)
int ladder4_queues()
{
    const char *f = diag_env("DTS_XCD");
    return (f && f[0] == '0') ? 1 : kQueueWidth;
}
constexpr int kSwsBitexact = 0x80000;

#define HIPCHK(ctx, expr)                                  \
    do {                                                   \
        hipError_t e_ = (expr);                            \
        if (e_ != hipSuccess) {                            \
            (ctx)->last_hip = (int)e_;                     \
            return DTS_E_HIP;                              \
        }                                                  \
    } while (0)

int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

bool fmt_in_ok(int f) { return f == DTS_FMT_YUV420P || f == DTS_FMT_NV12 || f == DTS_FMT_P010LE; }
bool fmt_out_ok(int f) { return f == DTS_FMT_YUV420P || f == DTS_FMT_NV12 || f == DTS_FMT_P010LE; }
bool fmt_8bit(int f) { return f == DTS_FMT_YUV420P || f == DTS_FMT_NV12; }   // quality / SDR outputs
bool method_ok(int m)
{
    switch (m) {
    case DTS_SCALE_BILINEAR: case DTS_SCALE_BICUBIC: case DTS_SCALE_X: case DTS_SCALE_POINT:
    case DTS_SCALE_AREA: case DTS_SCALE_GAUSS: case DTS_SCALE_SINC: case DTS_SCALE_LANCZOS:
        return true;
    default:
        return false;
    }
}

// plane geometry of a frame: row bytes and rows per plane (plane 2 unused for semi-planar)
void plane_geom(int w, int h, int fmt, int64_t rowb[3], int64_t rows[3])
{
    const int cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    rows[0] = h;
    rows[1] = ch;
    switch (fmt) {
    case DTS_FMT_YUV420P:
        rowb[0] = w; rowb[1] = cw; rowb[2] = cw; rows[2] = ch;
        break;
    case DTS_FMT_NV12:
        rowb[0] = w; rowb[1] = 2 * cw; rowb[2] = 0; rows[2] = 0;
        break;
    default: // P010LE
        rowb[0] = 2 * w; rowb[1] = 4 * cw; rowb[2] = 0; rows[2] = 0;
        break;
    }
}

// device-side layout we use for our own batch buffers
struct DevLayout {
    int64_t pitch[3] = {0, 0, 0}, off[3] = {0, 0, 0}, rows[3] = {0, 0, 0}, rowb[3] = {0, 0, 0};
    int64_t fstride = 0;
    // tight: pitches rounded to 16 B and planes to 256 B (the host path's batches: the
    // pinned rings hold the same image, so a batch crosses PCIe as one contiguous copy
    // with almost no padding); else pitches + 16 rounded to 256 B, planes to 4 KiB
    void init(int w, int h, int fmt, bool tight = false)
    {
        plane_geom(w, h, fmt, rowb, rows);
        int64_t o = 0;
        for (int p = 0; p < 3; ++p) {
            pitch[p] = rowb[p] ? (tight ? align_up(rowb[p], 16) : align_up(rowb[p] + 16, 256)) : 0;
            off[p] = o;
            o += align_up(pitch[p] * rows[p], tight ? 256 : 4096);
        }
        fstride = o;
    }
    DevPlanes planes(uint8_t *base) const
    {
        DevPlanes d{};
        for (int p = 0; p < 3; ++p) {
            d.data[p] = (uint64_t)(base + off[p]);
            d.pitch[p] = pitch[p] ? pitch[p] : pitch[1];
        }
        if (!rowb[2]) d.data[2] = d.data[1];
        d.fstride = fstride;
        return d;
    }
};

int64_t packed_bytes(int w, int h, int fmt)
{
    int64_t rowb[3], rows[3];
    plane_geom(w, h, fmt, rowb, rows);
    return rowb[0] * rows[0] + rowb[1] * rows[1] + rowb[2] * rows[2];
}

} // namespace

struct dts_graph {
    dts_ctx *ctx = nullptr;
    dts_graph_spec spec{};
    dts_graph_info info{};
    int src_kind = 0;
    int ndmax = 0;
    int ring_pairs = 16;
    int stage_bytes = 0;
    int lds_bytes = 0;
    std::vector<Job> jobs;
    std::vector<RungKind> rk;             // host copy with device pointers
    void *dev_tables = nullptr;           // all per-graph device tables
    Job *dev_jobs = nullptr;
    RungKind *dev_rk = nullptr;
    unsigned int *dev_queue = nullptr;    // kQueueSlots work counters (one per in-flight launch)
    unsigned int queue_next = 0;
    int grid_cap = 0;                     // resident workgroups of the persistent ladder grid
    // v4 ladder (ladder4.hip) for the (rendition, kind) pairs it fits; the rest run on v3
    uint32_t v4_mask = 0;                 // bit 2*rung+kind
    void *dev_tables4 = nullptr;
    Job4 *dev_jobs4 = nullptr;
    RungKind4 *dev_rk4 = nullptr;
    int njobs4 = 0, lds4 = 0, grid4 = 0;
    // v5 ladder (ladder5.hip): every plane kind of every rendition, when the graph fits it
    bool v5 = false;
    void *dev_tables5 = nullptr;
    Job5 *dev_jobs5 = nullptr;
    Kind5 *dev_kinds5 = nullptr;
    int njobs5 = 0, lds5 = 0, grid5 = 0;
    // v7 ladder (ladder7.hip): wave walks in strip groups; k_ladder5 (8-bit) / k_ladder4
    // (p010) run frames whose planes are not 16-byte aligned
    bool v7 = false;
    void *dev_tables7 = nullptr;
    const Group7 *dev_groups7 = nullptr;
    const Unit7 *dev_units7 = nullptr;
    const uint32_t *dev_frag7 = nullptr;
    const int32_t *dev_fire7 = nullptr;
    int ngroups7 = 0, nluma7 = 0, lds7 = 0, waves7 = 0, hsplit7 = 256;

    QScratch qs;                          // dts_graph_run_device's quality partials
    QScratch hqs[2];                      // the host path's, one per slot / stream
    bool host_ready = false;              // every host-path buffer of both slots allocated
    // host-path batch resources (2 slots)
    int batch = 32;
    DevLayout lay_src, lay_out[DTS_MAX_OUTPUTS], lay_q;
    uint8_t *dev_src[2] = {nullptr, nullptr}, *dev_out[2][DTS_MAX_OUTPUTS] = {}, *dev_q[2] = {nullptr, nullptr};
    dts_qraw *dev_qraw[2] = {nullptr, nullptr};
    uint8_t *pin_in[2] = {nullptr, nullptr}, *pin_out[2] = {nullptr, nullptr};
    dts_qraw *pin_qraw[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    hipEvent_t kdone[2] = {nullptr, nullptr};  // the slot's kernels are done (its D2H may start)
    hipEvent_t h2d_done[2] = {nullptr, nullptr};  // the slot's inputs have crossed (its ring may refill)
    hipStream_t d2h = nullptr;            // the host path's device -> host copies (both slots), so a
                                          // chunk's D2H runs beside the next chunk's H2D
    int64_t pin_in_bytes = 0, pin_out_bytes = 0;
    // pending host submit
    bool pending = false;
    const dts_frame *p_dst = nullptr;
    dts_qstat *p_q = nullptr;
    int p_chunk_first[2] = {-1, -1}, p_chunk_n[2] = {0, 0};
    uint32_t p_zout[2] = {0, 0};          // bit k: the slot's output k went straight into pinned caller frames
    // HDR10 -> SDR: per output a p010 intermediate of `batch` frames, double-buffered
    // (an event per buffer orders reuse across the host path's two streams)
    bool hdr = false;
    DevLayout lay_mid[DTS_MAX_OUTPUTS];
    uint8_t *hdr_mid[2][DTS_MAX_OUTPUTS] = {};
    hipEvent_t hdr_ev[2] = {nullptr, nullptr};   // k_tonemap done reading intermediate sl
    int hdr_chunk = 0;                    // frames per ladder -> tonemap chunk (the graph's batch)
    unsigned hdr_next = 0;
    TonemapParams tm{};
    float *dev_tm_lut = nullptr;          // the transfer-curve tables of tm (TonemapParams::lut)
    // rendition quality (dts_output_spec.quality): a graph of the reference renditions
    // (output j of ref = this graph's output rq_out[j], scaled with its qref_method)
    dts_graph *ref = nullptr;
    int nrq = 0;
    int rq_out[DTS_MAX_OUTPUTS] = {};
};

// ---------------------------------------------------------------------------
// graph construction
// ---------------------------------------------------------------------------
namespace {

// RGB -> XYZ of a set of xy primaries with D65 white (columns scaled so white has Y = 1)
void rgb_to_xyz(const double xy[3][2], double m[3][3])
{
    double P[3][3], Pi[3][3];
    for (int i = 0; i < 3; ++i) {
        P[0][i] = xy[i][0] / xy[i][1];
        P[1][i] = 1.0;
        P[2][i] = (1.0 - xy[i][0] - xy[i][1]) / xy[i][1];
    }
    auto inv = [](const double a[3][3], double o[3][3]) {
        const double det = a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) -
                           a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
                           a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {   // cofactor transpose
                const int r0 = (j + 1) % 3, r1 = (j + 2) % 3, c0 = (i + 1) % 3, c1 = (i + 2) % 3;
                o[i][j] = (a[r0][c0] * a[r1][c1] - a[r0][c1] * a[r1][c0]) / det;
            }
    };
    inv(P, Pi);
    const double W[3] = {0.3127 / 0.3290, 1.0, (1.0 - 0.3127 - 0.3290) / 0.3290};
    double S[3];
    for (int i = 0; i < 3; ++i) S[i] = Pi[i][0] * W[0] + Pi[i][1] * W[1] + Pi[i][2] * W[2];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) m[i][j] = P[i][j] * S[j];
}

// zscale=p=bt709 on bt2020 linear light: XYZ->709 x 2020->XYZ
void bt2020_to_bt709(float out[9])
{
    static const double p2020[3][2] = {{0.708, 0.292}, {0.170, 0.797}, {0.131, 0.046}};
    static const double p709[3][2] = {{0.640, 0.330}, {0.300, 0.600}, {0.150, 0.060}};
    double a[3][3], b[3][3];
    rgb_to_xyz(p2020, a);
    rgb_to_xyz(p709, b);
    const double det = b[0][0] * (b[1][1] * b[2][2] - b[1][2] * b[2][1]) -
                       b[0][1] * (b[1][0] * b[2][2] - b[1][2] * b[2][0]) +
                       b[0][2] * (b[1][0] * b[2][1] - b[1][1] * b[2][0]);
    double bi[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const int r0 = (j + 1) % 3, r1 = (j + 2) % 3, c0 = (i + 1) % 3, c1 = (i + 2) % 3;
            bi[i][j] = (b[r0][c0] * b[r1][c1] - b[r0][c1] * b[r1][c0]) / det;
        }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double v = 0;
            for (int k = 0; k < 3; ++k) v += bi[i][k] * a[k][j];
            out[3 * i + j] = (float)v;
        }
}

// vf_tonemap.c init() param defaults, peak fallback (ff_determine_signal_peak for
// linear input without side data: 10) and zscale npl
TonemapParams tonemap_params(const dts_tonemap_spec &t, bool full_range)
{
    TonemapParams p{};
    p.mode = t.mode;
    double param = t.param;
    switch (t.mode) {
    case DTS_TM_GAMMA: if (std::isnan(param)) param = 1.8; break;
    case DTS_TM_REINHARD: if (!std::isnan(param)) param = (1.0 - param) / param; break;
    case DTS_TM_MOBIUS: if (std::isnan(param)) param = 0.3; break;
    default: break;
    }
    if (std::isnan(param)) param = 1.0;
    const double peak = t.peak > 0 ? t.peak : 10.0, npl = t.npl > 0 ? t.npl : 100.0;
    auto hable = [](double x) {
        const double a = 0.15, b = 0.50, c = 0.10, d = 0.20, e = 0.02, f = 0.30;
        return (x * (x * a + b * c) + d * e) / (x * (x * a + b) + d * f) - e / f;
    };
    p.param = (float)param;
    p.desat = (float)t.desat;
    p.peak = (float)peak;
    p.hpeak = (float)hable((float)peak);
    p.inv_hpeak = 1.0f / p.hpeak;
    p.inv_hpeak_n = (float)kTmLutN / p.hpeak;
    // (hdr.hip pixel<>: the constant terms of hable(x) - hable's E / F cancel, DE = (E / F) DF)
    p.hk1 = (float)(0.15 * (1.0 - 0.02 / 0.30) * kTmLutN / (double)p.hpeak);
    p.hk0 = (float)(0.50 * (0.10 - 0.02 / 0.30) * kTmLutN / (double)p.hpeak);
    p.scale = (float)(10000.0 / npl);
    bt2020_to_bt709(p.m);
    // zimg's 8-bit quantisation of the final zscale (r=tv: Y 219 Y' + 16, C 224 C + 128; r=pc:
    // 255 Y', 255 C + 128), rounding half folded into the offset; computed in float exactly as
    // hdr.hip's pixel<> spells the products out
    const float kr7 = 0.2126f, kb7 = 0.0722f, kg7 = 1.f - kr7 - kb7;
    const float sb = 1.f / (2.f * (1.f - kb7)), sr = 1.f / (2.f * (1.f - kr7));
    const float qy = full_range ? 255.f : 219.f, qo = full_range ? 0.5f : 16.5f;
    p.qy[0] = qy * kr7;
    p.qy[1] = qy * kg7;
    p.qy[2] = qy * kb7;
    p.qy[3] = qo;
    p.qcb[0] = -sb / qy;
    p.qcb[1] = sb * qo / qy;
    p.qcr[0] = -sr / qy;
    p.qcr[1] = sr * qo / qy;
    p.qc = full_range ? 255.f : 224.f;
    return p;
}

// [0..N]: SMPTE ST 2084 EOTF x 10000 / npl (zscale t=linear:npl), [N+1..2N+1]: BT.709
// OETF (zimg rec_709_oetf), sampled in double at i / N on [0, 1]; each entry is
// (value, slope to the next entry), the last one (value, 0)
std::vector<float> tonemap_luts(const dts_tonemap_spec &t)
{
    const double m1 = 2610.0 / 16384.0, m2 = 2523.0 / 4096.0 * 128.0;
    const double c1 = 3424.0 / 4096.0, c2 = 2413.0 / 4096.0 * 32.0, c3 = 2392.0 / 4096.0 * 32.0;
    const double alpha = 1.09929682680944, beta = 0.018053968510807;
    const double scale = 10000.0 / (t.npl > 0 ? t.npl : 100.0);
    std::vector<float> v(2 * (kTmLutN + 1));
    for (int i = 0; i <= kTmLutN; ++i) {
        const double x = (double)i / kTmLutN;
        const double p = std::pow(x, 1.0 / m2);
        v[i] = (float)(std::pow(std::max(p - c1, 0.0) / (c2 - c3 * p), 1.0 / m1) * scale);
        v[kTmLutN + 1 + i] = (float)(x < beta ? 4.5 * x : alpha * std::pow(x, 0.45) - (alpha - 1.0));
    }
    // entry i: (intercept, slope) of the chord from i to i + 1 in table units, so that the
    // interpolation at x in [i, i + 1] is one fma, intercept + x slope (hdr.hip lut).  The PQ
    // table first, indexed by x + kTmPqOff over kTmPqN entries (flat at 0 below x = 0 and at
    // PQ(1) above x = kTmLutN: no clamp in the lookup), then the OETF table over [0, kTmLutN]
    std::vector<float> o(2 * (kTmPqN + kTmLutN + 1));
    for (int i = 0; i < kTmPqN; ++i) {
        const int j = i - kTmPqOff;                  // the chord over x in [j, j + 1]
        double sl = 0.0, y0 = 0.0;
        if (j >= kTmLutN) {
            y0 = v[kTmLutN];
        } else if (j >= 0) {
            y0 = v[j];
            sl = (double)v[j + 1] - (double)v[j];
        }
        o[2 * i] = (float)(y0 - (double)i * sl);     // in units of x + kTmPqOff
        o[2 * i + 1] = (float)sl;
    }
    for (int i = 0; i <= kTmLutN; ++i) {
        const float *t = v.data() + kTmLutN + 1;
        const double sl = i < kTmLutN ? (double)t[i + 1] - (double)t[i] : 0.0;
        o[2 * (kTmPqN + i)] = (float)((double)t[i] - i * sl);
        o[2 * (kTmPqN + i) + 1] = (float)sl;
    }
    return o;
}

struct KindTables {
    SwsFilter fh;                         // the libswscale H filter (v4 plans from it)
    HTable h;
    VTable v;
    std::vector<int32_t> vlim;
    int srcW, srcH, dstW, dstH;
    int sws_h, sws_v;
};

int build_kind(const dts_graph_spec &s, int k, int kind, KindTables &kt)
{
    const dts_output_spec &o = s.out[k];
    const int flags = o.method | kSwsAccurateRnd | kSwsBitexact;
    kt.srcW = kind ? (s.src_w + 1) >> 1 : s.src_w;
    kt.srcH = kind ? (s.src_h + 1) >> 1 : s.src_h;
    kt.dstW = kind ? (o.w + 1) >> 1 : o.w;
    kt.dstH = kind ? (o.h + 1) >> 1 : o.h;
    // utils.c get_local_pos: luma (0, 0); 4:2:0 chroma default -513 -> centred
    const int pos = kind ? sws_local_pos(1, -513) : sws_local_pos(0, 0);
    SwsFilter fh, fv;
    int e = sws_build_filter(kt.srcW, kt.dstW, 1 << 14, 4, flags, o.param, pos, pos, fh);
    if (e) return e;
    e = sws_build_filter(kt.srcH, kt.dstH, 1 << 12, 2, flags, o.param, pos, pos, fv);
    if (e) return e;
    kt.sws_h = fh.size;
    kt.sws_v = fv.size;
    e = s.src_fmt == DTS_FMT_P010LE ? pack_h_p010(fh, kt.dstW, kt.h) : pack_h_u8(fh, kt.dstW, kt.h);
    if (e) return e;
    kt.fh = std::move(fh);
    return pack_v(fv, kt.dstH, kt.v);
}

// strips of one (rung, kind): window of source samples each strip stages
void make_jobs(const KindTables &kt, int rung, int kind, bool p010, std::vector<Job> &jobs, int &max_stage)
{
    const int maxcols = kind ? kChromaCols : kLumaCols;
    const int nplanes = kind ? 2 : 1;
    const int bps = p010 ? 2 : 1;                    // staged bytes per sample
    const int tap_bytes = p010 ? 4 : 4;              // bytes per coefficient dword
    int cols = maxcols;
    for (;;) {
        bool fits = true;
        std::vector<Job> js;
        for (int x0 = 0; x0 < kt.dstW; x0 += cols) {
            const int n = std::min(cols, kt.dstW - x0);
            int lo = kt.h.pos[x0], hi = 0;
            for (int i = x0; i < x0 + n; ++i) {
                lo = std::min(lo, kt.h.pos[i]);
                hi = std::max(hi, kt.h.pos[i] * bps + kt.h.nd * tap_bytes);
            }
            const int sx0 = (lo * bps) / 16 * 16 / bps;  // 16-byte aligned start (samples)
            const int swb = (int)align_up(hi - sx0 * bps, 16);
            const int nload = kBlkRows * (swb / 16) * nplanes;
            if (nload > kMaxLoads * kThreads) {
                fits = false;
                break;
            }
            Job j{};
            j.rung = (int16_t)rung;
            j.kind = (int16_t)kind;
            j.x0 = x0;
            j.ncols = n;
            j.sx0 = sx0;
            j.swb = swb;
            j.nload = nload;
            js.push_back(j);
            max_stage = std::max(max_stage, nplanes * kBlkRows * swb);
        }
        if (fits || cols <= 8) {
            jobs.insert(jobs.end(), js.begin(), js.end());
            return;
        }
        cols /= 2;
    }
}

template <class T>
size_t push_blob(std::vector<uint8_t> &blob, const std::vector<T> &v)
{
    const size_t off = align_up((int64_t)blob.size(), 256);
    blob.resize(off + v.size() * sizeof(T));
    if (!v.empty()) std::memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

// ---- planning: everything graph_create decides on the host (dts_graph_plan
// runs it without a device) ----------------------------------------------
struct GraphPlan {
    int src_kind = 0, ndmax = 4, ring_pairs = 8, stage_bytes = 0, lds_bytes = 0, lds4 = 0;
    uint32_t v4_mask = 0;                 // bit 2*rung+kind: that (rendition, kind) runs on k_ladder4
    std::vector<KindTables> kts;
    std::vector<Plan4> p4;
    std::vector<Job> jobs;                // v3 strips (the kinds not on v4)
    std::vector<Job4> jobs4;              // v4 strips
    bool v5 = false;                      // the whole graph runs on k_ladder5
    Plan5Kind p5[2];                      // luma, chroma
    std::vector<Job5> jobs5;
    int lds5 = 0;
    bool v7 = false;                      // ... and on k_ladder7 where frames are 16-byte aligned
    Plan7 p7;
    dts_graph_info info{};
};

// a swscale range conversion in the ladder (scale=in_range:out_range); an HDR graph's output range
// is the tone-map kernel's quantisation instead (tonemap_params)
bool ladder_range_conv(const dts_graph_spec &s)
{
    return !s.hdr_to_sdr && (s.range & 1) != ((s.range >> 4) & 1);
}

int validate_spec(const dts_graph_spec &s)
{
    if (s.src_w < 4 || s.src_h < 4 || s.src_w > 16384 || s.src_h > 16384 || !fmt_in_ok(s.src_fmt)) return DTS_E_INVAL;
    if (s.nout < 1 || s.nout > DTS_MAX_OUTPUTS) return DTS_E_INVAL;
    for (int k = 0; k < s.nout; ++k) {
        const dts_output_spec &o = s.out[k];
        if (o.w < 2 || o.h < 2 || o.w > 16384 || o.h > 16384) return DTS_E_INVAL;
        if (!fmt_out_ok(o.fmt)) return DTS_E_UNSUPPORTED;
        if (!method_ok(o.method)) return DTS_E_UNSUPPORTED;
    }
    if (s.quality < 0 || s.quality > DTS_Q_BOTH) return DTS_E_INVAL;
    if ((s.range & ~0x11) != 0) return DTS_E_INVAL;              // DTS_RANGE_* in bits 0 and 4
    // range conversion: the ladder's (k_ladder7) 15-bit converters, every source format; an HDR
    // graph's ranges are zscale's: HDR10 sources are limited range, the output range is the final
    // zscale r=tv / r=pc quantisation in the tone-map kernel (ladder_range_conv: no swscale step)
    if (s.hdr_to_sdr && (s.range & 1)) return DTS_E_UNSUPPORTED;
    if (s.quality && (s.quality_out < 0 || s.quality_out >= s.nout)) return DTS_E_INVAL;
    for (int k = 0; k < s.nout; ++k) {                  // rendition quality (ABI 6)
        const dts_output_spec &o = s.out[k];
        if (o.quality < 0 || o.quality > DTS_Q_BOTH) return DTS_E_INVAL;
        if (!o.quality) continue;
        if (o.qref_method != DTS_QREF_EXTERNAL && !method_ok(o.qref_method)) return DTS_E_UNSUPPORTED;
        if (s.quality || s.hdr_to_sdr || !fmt_8bit(o.fmt)) return DTS_E_UNSUPPORTED;
    }
    if (s.quality && !fmt_8bit(s.out[s.quality_out].fmt)) return DTS_E_UNSUPPORTED;   // vf_psnr/vf_ssim: 8-bit
    if (s.deint) {                                        // yadif ahead of the ladder: 8-bit yuv420p, frame modes
        if (s.deint != 1 || s.src_fmt != DTS_FMT_YUV420P || s.hdr_to_sdr) return DTS_E_UNSUPPORTED;
        if ((s.deint_mode != 0 && s.deint_mode != 2) || s.src_w < 16) return DTS_E_UNSUPPORTED;
    }
    if (s.hdr_to_sdr) {
        if (s.src_fmt != DTS_FMT_P010LE) return DTS_E_INVAL;                        // HDR10 sources are p010
        if (s.tonemap.mode < DTS_TM_NONE || s.tonemap.mode > DTS_TM_MOBIUS) return DTS_E_INVAL;
        for (int k = 0; k < s.nout; ++k)
            if (!fmt_8bit(s.out[k].fmt) || (s.out[k].w & 1) || (s.out[k].h & 1)) return DTS_E_UNSUPPORTED;
    }
    return DTS_OK;
}

// DTS_LADDER=3 keeps every (rendition, kind) on the v3 kernel (A/B runs, tests)
bool v4_enabled()
{
    const char *f = std::getenv("DTS_LADDER");
    return !(f && f[0] == '3');
}

// DTS_LADDER=4 / 3 keep the graph off the v5 kernel (A/B runs, tests)
bool v5_enabled()
{
    const char *f = std::getenv("DTS_LADDER");
    return !(f && (f[0] == '3' || f[0] == '4'));
}

// DTS_LADDER=5 / 4 / 3 keep the graph off the v7 kernel (6: the retired k_ladder6, read as 5)
bool v7_enabled()
{
    const char *f = std::getenv("DTS_LADDER");
    return !(f && (f[0] == '3' || f[0] == '4' || f[0] == '5' || f[0] == '6'));
}

// waves per k_ladder7 group (diagnostic DTS_L7_W, 1..16; default 8: two groups of 8 waves per CU)
int l7_waves()
{
    const char *f = diag_env("DTS_L7_W");
    const int w = f ? std::atoi(f) : 8;
    return std::min(std::max(w, 1), kL7MaxWaves);
}

// Staging batches per k_ladder7 group and granules per batch: what the linked kernel was
// compiled with (ladder7.hip NS7 / PB7; diagnostic builds change them with -DDTS_L7_NS /
// -DDTS_L7_PAIR).  The planner sizes the stage buffers and the V fragment slots from these.
int l7_stages()
{
    int ns, pb;
    ladder7_compiled(&ns, &pb);
    return ns;
}

// granules per k_ladder7 staging batch (see l7_stages)
int l7_pb()
{
    int ns, pb;
    ladder7_compiled(&ns, &pb);
    return pb;
}

// k_ladder7 groups: one rendition per group (diagnostic DTS_L7_GROUP=r) or every rendition of a
// source strip (the default)
bool l7_by_rung()
{
    const char *f = diag_env("DTS_L7_GROUP");
    return f ? f[0] == 'r' : false;
}

// k_ladder7 one-K-block walks with half the tiles (diagnostic DTS_L7_NARROW=1)
bool l7_narrow()
{
    const char *f = diag_env("DTS_L7_NARROW");
    return f ? f[0] == '1' : false;
}

// k_ladder7's plan with its group width: 8 waves, two groups per CU, unless two such groups do
// not fit the CU's 160 KB of LDS (8K sources: cfg4 plans 90 KB per group).  Then a CU holds one
// group whatever its width, and a 10-wave group keeps more waves resident (round-5 cfg4 A/B,
// 300-frame launches: W 8 / 10 / 12 / 14 / 16 52.1 k / 54.4 k / 53.2 k / 53.5 k / 52.8 k fps).
// The diagnostic DTS_L7_W fixes the width.
bool plan7_sized(const Plan5In *ins, bool narrow, Plan7 &out)
{
    if (!plan7_graph(ins, l7_waves(), l7_stages(), l7_pb(), l7_by_rung(), narrow, out)) return false;
    if (diag_env("DTS_L7_W") || 2 * out.lds_bytes <= 160 * 1024) return true;
    Plan7 wide;
    if (plan7_graph(ins, 10, l7_stages(), l7_pb(), l7_by_rung(), narrow, wide) && wide.lds_bytes <= 160 * 1024)
        out = std::move(wide);
    return true;
}

// k_ladder5 for every (rendition, kind) of an 8-bit 4:2:0 source with 8-bit outputs,
// and k_ladder7 too where it fits
bool plan5_graph(const dts_graph_spec &s, GraphPlan &gp)
{
    if (!v5_enabled() || s.hdr_to_sdr) return false;
    if (s.src_fmt != DTS_FMT_YUV420P && s.src_fmt != DTS_FMT_NV12) return false;
    Plan5In ins[2];
    for (int kind = 0; kind < 2; ++kind) {
        Plan5In &in = ins[kind];
        in.chroma = kind == 1;
        in.nv12_chroma = kind == 1 && s.src_fmt == DTS_FMT_NV12;
        in.srcW = kind ? (s.src_w + 1) >> 1 : s.src_w;
        in.srcH = kind ? (s.src_h + 1) >> 1 : s.src_h;
        if (ladder_range_conv(s)) in.range_conv = (s.range & 1) ? 2 : 1;   // from / to JPEG
        for (int k = 0; k < s.nout; ++k) {
            const KindTables &kt = gp.kts[(size_t)k * 2 + kind];
            in.rungs.push_back(Plan5Rung{&kt.fh, &kt.v, kt.dstW, kt.dstH, s.out[k].fmt});
        }
        if (!plan5_kind(in, gp.p5[kind])) return false;
    }
    for (int kind = 0; kind < 2; ++kind)
        for (int st = 0; st < (int)gp.p5[kind].strips.size(); ++st) gp.jobs5.push_back(Job5{kind, st});
    // strips in source-column order (luma x of the strip start): a queue hands out
    // neighbouring strips back to back, so their shared halo columns hit L2
    auto srcx = [&](const Job5 &j) { return (j.kind ? 2 : 1) * gp.p5[j.kind].strips[j.strip].L; };
    std::stable_sort(gp.jobs5.begin(), gp.jobs5.end(), [&](const Job5 &a, const Job5 &b) { return srcx(a) < srcx(b); });
    gp.lds5 = std::max(gp.p5[0].lds_bytes, gp.p5[1].lds_bytes);
    gp.v5 = true;
    // k_ladder7 takes planar and nv12 sources (k_ladder5: the fallback for frames that are
    // not 16-byte aligned)
    gp.v7 = v7_enabled() && plan7_sized(ins, l7_narrow(), gp.p7);
    return true;
}

// p010 sources on k_ladder7 (its 16-bit walks: the H sums from the samples' raw bytes,
// p010 / 8-bit dithered renditions); k_ladder4 stays planned for frames whose planes are
// not 16-byte aligned
bool plan7_p010(const dts_graph_spec &s, GraphPlan &gp)
{
    if (!v7_enabled() || s.src_fmt != DTS_FMT_P010LE) return false;
    Plan5In ins[2];
    for (int kind = 0; kind < 2; ++kind) {
        Plan5In &in = ins[kind];
        in.chroma = kind == 1;
        in.nv12_chroma = kind == 1;
        in.p10 = true;
        if (ladder_range_conv(s)) in.range_conv = (s.range & 1) ? 2 : 1;   // from / to JPEG
        in.srcW = kind ? (s.src_w + 1) >> 1 : s.src_w;
        in.srcH = kind ? (s.src_h + 1) >> 1 : s.src_h;
        for (int k = 0; k < s.nout; ++k) {
            const KindTables &kt = gp.kts[(size_t)k * 2 + kind];
            // an HDR graph's ladder writes the p010 intermediates k_tonemap reads
            in.rungs.push_back(Plan5Rung{&kt.fh, &kt.v, kt.dstW, kt.dstH,
                                         s.hdr_to_sdr ? (int)DTS_FMT_P010LE : s.out[k].fmt});
        }
    }
    return plan7_sized(ins, false, gp.p7);
}

bool plan4_for(const dts_graph_spec &s, const KindTables &kt, int kind, Plan4 &pl)
{
    const bool p010 = s.src_fmt == DTS_FMT_P010LE, nv12 = s.src_fmt == DTS_FMT_NV12;
    int64_t rowb[3], rows[3];
    plane_geom(s.src_w, s.src_h, s.src_fmt, rowb, rows);
    // bytes per sample in the (maybe interleaved) source row and the sample pairs the kernel's
    // eight 16-B loads per row hold (ladder4.hip item4: CAP)
    const int bps = kind ? (p010 ? 4 : (nv12 ? 2 : 1)) : (p010 ? 2 : 1);
    const int cap = 64 / bps;
    return plan4_kind(kt.fh, kt.v, kt.srcH, kt.dstW, kt.dstH, bps, 8, cap, kRing4Cols, rowb[kind ? 1 : 0],
                      kRing4Slots, pl);
}

int make_plan(const dts_graph_spec &s, GraphPlan &gp)
{
    int e = validate_spec(s);
    if (e) return e;
    gp.src_kind = s.src_fmt == DTS_FMT_P010LE ? kSrcP010 : (s.src_fmt == DTS_FMT_NV12 ? kSrcNV12 : kSrcPlanar8);
    const bool p010 = s.src_fmt == DTS_FMT_P010LE;
    const bool use4 = v4_enabled();
    gp.kts.resize((size_t)s.nout * 2);
    gp.p4.resize(gp.kts.size());
    for (size_t i = 0; i < gp.kts.size(); ++i) {
        e = build_kind(s, (int)(i >> 1), (int)(i & 1), gp.kts[i]);
        if (e) return e;
    }
    const bool v5 = plan5_graph(s, gp);
    if (!v5) gp.v7 = plan7_p010(s, gp);
    // range conversion runs in k_ladder7's H epilogue only
    if (ladder_range_conv(s) && !gp.v7) return DTS_E_UNSUPPORTED;
    int ndmax_need = 1;
    for (int k = 0; k < s.nout; ++k)
        for (int kind = 0; kind < 2; ++kind) {
            const size_t i = (size_t)k * 2 + kind;
            KindTables &kt = gp.kts[i];
            if (v5) {
                gp.info.h_taps[k][kind] = kt.h.span;
                gp.info.v_taps[k][kind] = kt.v.span;
                gp.info.sws_h_size[k][kind] = kt.sws_h;
                gp.info.sws_v_size[k][kind] = kt.sws_v;
                continue;
            }
            if (use4 && plan4_for(s, kt, kind, gp.p4[i]))
                gp.v4_mask |= 1u << i;
            else
                ndmax_need = std::max(ndmax_need, kt.h.nd);
            gp.info.h_taps[k][kind] = kt.h.span;
            gp.info.v_taps[k][kind] = kt.v.span;
            gp.info.sws_h_size[k][kind] = kt.sws_h;
            gp.info.sws_v_size[k][kind] = kt.sws_v;
            gp.info.h_pairs4[k][kind] = (gp.v4_mask >> i) & 1 ? gp.p4[i].N : 0;
        }
    gp.ndmax = ladder_ndmax_for(ndmax_need);
    if (!gp.ndmax) return DTS_E_RANGE;
    const bool on3 = !v5 && gp.v4_mask != (1u << gp.kts.size()) - 1;
    if (on3) {
        // v3 ring: smallest power of two holding every V window of the kinds v3 runs
        int rp = 8;
        for (; rp <= 256; rp *= 2) {
            bool ok = true;
            for (size_t i = 0; i < gp.kts.size(); ++i)
                if (!((gp.v4_mask >> i) & 1))
                    ok = ok && plan_vlimits(gp.kts[i].v, gp.kts[i].srcH, gp.kts[i].dstH, rp, gp.kts[i].vlim);
            if (ok) break;
        }
        if (rp > 256) return DTS_E_RANGE;
        gp.ring_pairs = rp;
        int max_stage = 0;
        for (size_t i = 0; i < gp.kts.size(); ++i)
            if (!((gp.v4_mask >> i) & 1)) make_jobs(gp.kts[i], (int)(i >> 1), (int)(i & 1), p010, gp.jobs, max_stage);
        // heaviest strips first (H taps x columns x source rows)
        std::stable_sort(gp.jobs.begin(), gp.jobs.end(), [&](const Job &a, const Job &b) {
            const KindTables &ka = gp.kts[(size_t)a.rung * 2 + a.kind], &kb = gp.kts[(size_t)b.rung * 2 + b.kind];
            const int64_t ca = (int64_t)ka.h.nd * a.ncols * ka.srcH * (a.kind ? 2 : 1);
            const int64_t cb = (int64_t)kb.h.nd * b.ncols * kb.srcH * (b.kind ? 2 : 1);
            return ca > cb;
        });
        gp.stage_bytes = (int)align_up(max_stage, 16);
        gp.lds_bytes = 2 * gp.stage_bytes + gp.ring_pairs * kLumaCols * 4;
        if (gp.lds_bytes > 160 * 1024) return DTS_E_RANGE;
    }
    for (size_t i = 0; i < gp.kts.size() && !v5; ++i) {
        if (!((gp.v4_mask >> i) & 1)) continue;
        const Plan4 &pl = gp.p4[i];
        for (int st = 0; st < pl.nstrips; ++st)
            for (int plane = 0; plane < ((i & 1) ? 2 : 1); ++plane) {   // chroma: U and V items side by side
                Job4 j{};
                j.rk = (int16_t)i;
                j.kind = (int16_t)(i & 1);
                j.rung = (int16_t)(i >> 1);
                j.plane = (int16_t)plane;
                j.x0 = st * pl.C;
                j.ncols = std::min(pl.C, gp.kts[i].dstW - j.x0);
                j.group0 = st * 4;
                gp.jobs4.push_back(j);
            }
    }
    // Strips in source-column order: every rendition and plane of a column range
    // together, so the items a queue hands out back to back walk the same source rows
    // and re-read them from L2 (r01: +3 % over heaviest-first at 256 frames per launch).
    // A single rendition keeps heaviest-first (H tap pairs x columns x source rows),
    // which shortens the launch tail (cfg4: 26.1k vs 25.0k fps); diagnostic DTS_ORDER=h / c force one.
    auto cost4 = [&](const Job4 &j) {
        return (int64_t)(2 * gp.p4[j.rk].N + 8) * j.ncols * gp.kts[j.rk].srcH;
    };
    std::stable_sort(gp.jobs4.begin(), gp.jobs4.end(), [&](const Job4 &a, const Job4 &b) { return cost4(a) > cost4(b); });
    const char *order = diag_env("DTS_ORDER");
    const bool by_column = order ? order[0] == 'c' : s.nout > 1;   // one rendition: no source re-reads to share
    if (by_column) {
        auto srcx = [&](const Job4 &j) { return (double)(j.x0 + 0.5 * j.ncols) / gp.kts[j.rk].dstW; };
        std::stable_sort(gp.jobs4.begin(), gp.jobs4.end(),
                         [&](const Job4 &a, const Job4 &b) { return srcx(a) < srcx(b); });
    }
    if (gp.v4_mask) gp.lds4 = kLds4Bytes;

    dts_graph_info &in = gp.info;
    in.src_frame_bytes = packed_bytes(s.src_w, s.src_h, s.src_fmt);
    int64_t algo = in.src_frame_bytes;
    for (int k = 0; k < s.nout; ++k) {
        in.out_frame_bytes[k] = packed_bytes(s.out[k].w, s.out[k].h, s.out[k].fmt);
        algo += in.out_frame_bytes[k];
    }
    if (s.quality) algo += in.out_frame_bytes[s.quality_out];
    in.algo_bytes_per_frame = algo;
    in.njobs = gp.v7 ? (int)gp.p7.groups.size()
                     : (int)(gp.jobs.size() + gp.jobs4.size() + gp.jobs5.size());
    in.lds_bytes = gp.v7 ? gp.p7.lds_bytes : std::max(std::max(gp.lds_bytes, gp.lds4), gp.lds5);
    in.ladder_v4_mask = (int32_t)gp.v4_mask;
    in.ladder_v5 = gp.v7 ? 3 : (gp.v5 ? 1 : 0);
    for (int kind = 0; kind < 2; ++kind) {
        in.v5_strip_width[kind] = gp.v5 ? gp.p5[kind].strip_width : 0;
        in.v5_strips[kind] = gp.v5 ? (int32_t)gp.p5[kind].strips.size() : 0;
    }
    return DTS_OK;
}

} // namespace

extern "C" {

#define DTS_STR2(x) #x
#define DTS_STR(x) DTS_STR2(x)
const char *dts_version(void) { return "dts-mi355x 0.7 (gfx950; abi " DTS_STR(DTS_ABI_VERSION) ")"; }

int dts_abi_version(void) { return DTS_ABI_VERSION; }

int64_t dts_abi_struct_size(int which)
{
    switch (which) {
    case DTS_STRUCT_TONEMAP_SPEC: return (int64_t)sizeof(dts_tonemap_spec);
    case DTS_STRUCT_OUTPUT_SPEC: return (int64_t)sizeof(dts_output_spec);
    case DTS_STRUCT_GRAPH_SPEC: return (int64_t)sizeof(dts_graph_spec);
    case DTS_STRUCT_FRAME: return (int64_t)sizeof(dts_frame);
    case DTS_STRUCT_DEV_FRAMES: return (int64_t)sizeof(dts_dev_frames);
    case DTS_STRUCT_QRAW: return (int64_t)sizeof(dts_qraw);
    case DTS_STRUCT_QSTAT: return (int64_t)sizeof(dts_qstat);
    case DTS_STRUCT_GRAPH_INFO: return (int64_t)sizeof(dts_graph_info);
    default: return DTS_E_INVAL;
    }
}

const char *dts_strerror(int err)
{
    switch (err) {
    case DTS_OK: return "success";
    case DTS_E_INVAL: return "invalid argument";
    case DTS_E_NOMEM: return "out of memory";
    case DTS_E_RANGE: return "filter does not fit the GPU tables";
    case DTS_E_UNSUPPORTED: return "unsupported format or method";
    case DTS_E_BUSY: return "a submit is still pending";
    case DTS_E_NODEV: return "no HIP device";
    case DTS_E_HIP: return "HIP runtime error";
    default: return "unknown error";
    }
}

int dts_device_count(int *count)
{
    if (!count) return DTS_E_INVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return DTS_OK;
}

int dts_ctx_create(int device, dts_ctx **out)
{
    if (!out) return DTS_E_INVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return DTS_E_NODEV;
    if (device < 0 || device >= n) return DTS_E_INVAL;
    dts_ctx *c = new (std::nothrow) dts_ctx();
    if (!c) return DTS_E_NOMEM;
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream[0], hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream[1], hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return DTS_E_HIP;
    }
    *out = c;
    return DTS_OK;
}

static void qscratch_free(QScratch &q)
{
    if (q.ev) {
        hipEventSynchronize(q.ev);
        hipEventDestroy(q.ev);
    }
    if (q.dev) {
        hipEventSynchronize(q.dev);
        hipEventDestroy(q.dev);
    }
    if (q.rev) {
        hipEventSynchronize(q.rev);
        hipEventDestroy(q.rev);
    }
    if (q.p) hipFree(q.p);
    if (q.dp) hipFree(q.dp);
    if (q.rp) hipFree(q.rp);
    q = QScratch{};
}

static void ctx_release(dts_ctx *c)
{
    if (c->refs.fetch_sub(1) != 1) return;
    hipSetDevice(c->device);
    qscratch_free(c->qs);
    if (c->hq) hipFree(c->hq);
    for (auto &s : c->stream)
        if (s) hipStreamDestroy(s);
    delete c;
}

void dts_ctx_destroy(dts_ctx *c)
{
    if (c) ctx_release(c);
}

int dts_ctx_last_hip_error(const dts_ctx *c) { return c ? c->last_hip : 0; }

int dts_frame_layout(int w, int h, int fmt, int64_t pitch[3], int64_t rows[3], int64_t *packed)
{
    if (w <= 0 || h <= 0 || !fmt_in_ok(fmt) || !pitch || !rows) return DTS_E_INVAL;
    plane_geom(w, h, fmt, pitch, rows);
    if (packed) *packed = pitch[0] * rows[0] + pitch[1] * rows[1] + pitch[2] * rows[2];
    return DTS_OK;
}

void dts_graph_destroy(dts_graph *g);

// v3 tables (every kind; the v3 jobs cover the kinds not on v4) + its grid
static int upload_v3(dts_graph *g, std::vector<KindTables> &kts)
{
    dts_ctx *ctx = g->ctx;
    std::vector<uint8_t> blob;
    struct Offs { size_t hpos, hbias, hch, hcl, vpos, vcoef, vlim; };
    std::vector<Offs> offs(kts.size());
    for (size_t i = 0; i < kts.size(); ++i) {
        KindTables &kt = kts[i];
        offs[i].hpos = push_blob(blob, kt.h.pos);
        offs[i].hbias = push_blob(blob, kt.h.bias);
        offs[i].hch = push_blob(blob, kt.h.hi);
        offs[i].hcl = push_blob(blob, kt.h.lo);
        offs[i].vpos = push_blob(blob, kt.v.pos);
        offs[i].vcoef = push_blob(blob, kt.v.coef);
        offs[i].vlim = push_blob(blob, kt.vlim);
    }
    const size_t jobs_off = push_blob(blob, g->jobs);
    const size_t rk_off = align_up((int64_t)blob.size(), 256);
    blob.resize(rk_off + kts.size() * sizeof(RungKind));
    HIPCHK(ctx, hipMalloc(&g->dev_tables, blob.size()));
    uint8_t *base = static_cast<uint8_t *>(g->dev_tables);
    g->rk.resize(kts.size());
    for (size_t i = 0; i < kts.size(); ++i) {
        KindTables &kt = kts[i];
        RungKind &r = g->rk[i];
        r.dstW = kt.dstW;
        r.dstH = kt.dstH;
        r.nd = kt.h.nd;
        r.nv = kt.v.nv;
        r.nblocks = (int)kt.vlim.size();
        r.hpos = reinterpret_cast<const int32_t *>(base + offs[i].hpos);
        r.hbias = reinterpret_cast<const int32_t *>(base + offs[i].hbias);
        r.hch = reinterpret_cast<const uint32_t *>(base + offs[i].hch);
        r.hcl = reinterpret_cast<const uint32_t *>(base + offs[i].hcl);
        r.vpos = reinterpret_cast<const int32_t *>(base + offs[i].vpos);
        r.vcoef = reinterpret_cast<const uint32_t *>(base + offs[i].vcoef);
        r.vlim = reinterpret_cast<const int32_t *>(base + offs[i].vlim);
    }
    std::memcpy(blob.data() + rk_off, g->rk.data(), kts.size() * sizeof(RungKind));
    g->dev_jobs = reinterpret_cast<Job *>(base + jobs_off);
    g->dev_rk = reinterpret_cast<RungKind *>(base + rk_off);
    HIPCHK(ctx, hipMemcpy(g->dev_tables, blob.data(), blob.size(), hipMemcpyHostToDevice));
    if (!g->jobs.empty()) {      // persistent grid: resident workgroups per CU x CUs
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus < 1)
            cus = 256;
        const int bpc = ladder_blocks_per_cu(g->src_kind, g->ndmax, g->lds_bytes);
        if (bpc < 1) return DTS_E_RANGE;
        g->grid_cap = bpc * cus;
    }
    return DTS_OK;
}

// v4 tables of the kinds in v4_mask -> one device blob, plus its grid
static int upload_v4(dts_graph *g, const GraphPlan &gp)
{
    dts_ctx *ctx = g->ctx;
    const size_t nk = gp.p4.size();
    std::vector<uint8_t> blob;
    struct Offs { size_t groups = 0, hcoef = 0, vslot = 0, vcoef = 0, vlim = 0; };
    std::vector<Offs> offs(nk);
    for (size_t i = 0; i < nk; ++i) {
        if (!((gp.v4_mask >> i) & 1)) continue;
        const Plan4 &pl = gp.p4[i];
        offs[i].groups = push_blob(blob, pl.groups);
        offs[i].hcoef = push_blob(blob, pl.hcoef);
        blob.resize(blob.size() + 16 * sizeof(uint32_t), 0);  // k_ladder4 prefetches one output's taps past the last
        offs[i].vslot = push_blob(blob, pl.vslot);
        offs[i].vcoef = push_blob(blob, pl.vcoef);
        offs[i].vlim = push_blob(blob, pl.vlim);
    }
    const size_t jobs_off = push_blob(blob, gp.jobs4);
    const size_t rk_off = (size_t)align_up((int64_t)blob.size(), 256);
    blob.resize(rk_off + nk * sizeof(RungKind4));
    HIPCHK(ctx, hipMalloc(&g->dev_tables4, blob.size()));
    uint8_t *base = static_cast<uint8_t *>(g->dev_tables4);
    std::vector<RungKind4> rk(nk);
    for (size_t i = 0; i < nk; ++i) {
        if (!((gp.v4_mask >> i) & 1)) continue;
        const Plan4 &pl = gp.p4[i];
        RungKind4 &r = rk[i];
        r.N = pl.N;
        r.NV = pl.NV;
        r.nsteps = pl.nsteps;
        r.groups = reinterpret_cast<const HGroup4 *>(base + offs[i].groups);
        r.hcoef = reinterpret_cast<const uint32_t *>(base + offs[i].hcoef);
        r.vslot = reinterpret_cast<const int32_t *>(base + offs[i].vslot);
        r.vcoef = reinterpret_cast<const uint32_t *>(base + offs[i].vcoef);
        r.vlim = reinterpret_cast<const int32_t *>(base + offs[i].vlim);
    }
    std::memcpy(blob.data() + rk_off, rk.data(), nk * sizeof(RungKind4));
    HIPCHK(ctx, hipMemcpy(g->dev_tables4, blob.data(), blob.size(), hipMemcpyHostToDevice));
    g->dev_jobs4 = reinterpret_cast<Job4 *>(base + jobs_off);
    g->dev_rk4 = reinterpret_cast<RungKind4 *>(base + rk_off);
    g->njobs4 = (int)gp.jobs4.size();
    g->lds4 = gp.lds4;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus < 1)
        cus = 256;
    const int bpc = ladder4_blocks_per_cu(g->src_kind, g->lds4);
    if (bpc < 1) return DTS_E_RANGE;
    g->grid4 = bpc * cus;
    return DTS_OK;
}

// v5 tables -> one device blob (strips, entries, B fragments, V tables, Kind5 x 2, jobs), plus its grid
static int upload_v5(dts_graph *g, const GraphPlan &gp)
{
    dts_ctx *ctx = g->ctx;
    std::vector<uint8_t> blob;
    struct Offs {
        size_t strips = 0, ents = 0, bfrag = 0, vsched = 0, vstep = 0;
    } offs[2];
    for (int kind = 0; kind < 2; ++kind) {
        const Plan5Kind &pk = gp.p5[kind];
        offs[kind].strips = push_blob(blob, pk.strips);
        offs[kind].ents = push_blob(blob, pk.ents);
        offs[kind].bfrag = push_blob(blob, pk.bfrag);
        offs[kind].vsched = push_blob(blob, pk.vsched);
        offs[kind].vstep = push_blob(blob, pk.vstep);
    }
    const size_t jobs_off = push_blob(blob, gp.jobs5);
    const size_t k_off = (size_t)align_up((int64_t)blob.size(), 256);
    blob.resize(k_off + 2 * sizeof(Kind5));
    HIPCHK(ctx, hipMalloc(&g->dev_tables5, blob.size()));
    uint8_t *base = static_cast<uint8_t *>(g->dev_tables5);
    Kind5 kinds[2];
    std::memset(kinds, 0, sizeof kinds);
    for (int kind = 0; kind < 2; ++kind) {
        const Plan5Kind &pk = gp.p5[kind];
        Kind5 &k = kinds[kind];
        k.nplanes = pk.nplanes;
        k.nsteps = pk.nsteps;
        k.srcH = kind ? (g->spec.src_h + 1) >> 1 : g->spec.src_h;
        k.nlp = pk.nlp;
        k.stage = pk.stage;
        k.SB = pk.SB;
        k.FA = pk.FA;
        k.FB = pk.FB;
        k.nbfrag = (uint32_t)(pk.bfrag.size() / 512);
        k.nrings = pk.nrings;
        k.nrungs = g->spec.nout;
        k.nstrips = (int32_t)pk.strips.size();
        for (int i = 0; i < kL5MaxRings; ++i) k.ring[i] = pk.ring[i];
        for (int r = 0; r < DTS_MAX_OUTPUTS; ++r) k.out[r] = pk.out[r];
        k.vsched = reinterpret_cast<const VEnt5 *>(base + offs[kind].vsched);
        k.vstep = reinterpret_cast<const int4 *>(base + offs[kind].vstep);
        k.strips = reinterpret_cast<const Strip5 *>(base + offs[kind].strips);
        k.ents = reinterpret_cast<const Ent5 *>(base + offs[kind].ents);
        k.bfrag = reinterpret_cast<const uint32_t *>(base + offs[kind].bfrag);
    }
    std::memcpy(blob.data() + k_off, kinds, sizeof kinds);
    HIPCHK(ctx, hipMemcpy(g->dev_tables5, blob.data(), blob.size(), hipMemcpyHostToDevice));
    g->dev_jobs5 = reinterpret_cast<Job5 *>(base + jobs_off);
    g->dev_kinds5 = reinterpret_cast<Kind5 *>(base + k_off);
    g->njobs5 = (int)gp.jobs5.size();
    g->lds5 = gp.lds5;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus < 1)
        cus = 256;
    const int bpc = ladder5_blocks_per_cu(g->src_kind, g->lds5);
    if (bpc < 1) return DTS_E_RANGE;
    g->grid5 = bpc * cus;
    g->v5 = true;
    return DTS_OK;
}

// v7 tables -> one device blob (groups, units, fragment pairs, fire tables)
static int upload_v7(dts_graph *g, const GraphPlan &gp)
{
    dts_ctx *ctx = g->ctx;
    std::vector<uint8_t> blob;
    const size_t g_off = push_blob(blob, gp.p7.groups);
    const size_t u_off = push_blob(blob, gp.p7.units);
    const size_t f_off = push_blob(blob, gp.p7.frag);
    const size_t r_off = push_blob(blob, gp.p7.fire);
    HIPCHK(ctx, hipMalloc(&g->dev_tables7, blob.size()));
    HIPCHK(ctx, hipMemcpy(g->dev_tables7, blob.data(), blob.size(), hipMemcpyHostToDevice));
    const uint8_t *base = static_cast<const uint8_t *>(g->dev_tables7);
    g->dev_groups7 = reinterpret_cast<const Group7 *>(base + g_off);
    g->dev_units7 = reinterpret_cast<const Unit7 *>(base + u_off);
    g->dev_frag7 = reinterpret_cast<const uint32_t *>(base + f_off);
    g->dev_fire7 = reinterpret_cast<const int32_t *>(base + r_off);
    g->ngroups7 = (int)gp.p7.groups.size();
    g->nluma7 = 0;
    while (g->nluma7 < g->ngroups7 && gp.p7.groups[(size_t)g->nluma7].kind == 0) ++g->nluma7;
    g->lds7 = gp.p7.lds_bytes;
    g->waves7 = gp.p7.waves;
    g->hsplit7 = gp.p7.hsplit;
    g->v7 = true;
    return DTS_OK;
}

int dts_graph_create(dts_ctx *ctx, const dts_graph_spec *spec, dts_graph **out)
{
    if (!ctx || !spec || !out) return DTS_E_INVAL;
    *out = nullptr;
    dts_graph *g = nullptr;
    try {
        GraphPlan gp;
        int e = make_plan(*spec, gp);
        if (e) return e;
        const dts_graph_spec &s = *spec;
        g = new dts_graph();
        g->ctx = ctx;
        ctx->refs.fetch_add(1);
        g->spec = s;
        g->batch = s.max_batch > 0 ? std::min(s.max_batch, 65535) : 32;
        g->src_kind = gp.src_kind;
        g->ndmax = gp.ndmax;
        g->ring_pairs = gp.ring_pairs;
        g->stage_bytes = gp.stage_bytes;
        g->lds_bytes = gp.lds_bytes;
        g->jobs = gp.jobs;
        g->v4_mask = gp.v4_mask;
        g->info = gp.info;
        hipSetDevice(ctx->device);
        e = gp.v5 ? DTS_OK : upload_v3(g, gp.kts);
        if (!e && gp.v4_mask) e = upload_v4(g, gp);
        if (!e && gp.v5) e = upload_v5(g, gp);
        if (!e && gp.v7) e = upload_v7(g, gp);
        if (!e && hipMalloc(&g->dev_queue, kQueueSlots * kQueueWidth * sizeof(unsigned int)) != hipSuccess) {
            ctx->last_hip = (int)hipGetLastError();
            e = DTS_E_HIP;
        }
        if (e) {
            dts_graph_destroy(g);
            return e;
        }
        g->lay_src.init(s.src_w, s.src_h, s.src_fmt, true);
        for (int k = 0; k < s.nout; ++k) g->lay_out[k].init(s.out[k].w, s.out[k].h, s.out[k].fmt, true);
        if (s.hdr_to_sdr) {
            g->hdr = true;
            g->tm = tonemap_params(s.tonemap, (s.range >> 4) & 1);
            // chunks of `batch` frames: the ladder writes a chunk's p010 intermediates, k_tonemap
            // converts them on the same stream (measured in rounds 3 and 4: smaller chunks, which keep
            // the intermediates in the Infinity Cache, and the tonemap on a second stream beside the
            // next chunk's ladder are slower -- DESIGN.md §4 k_tonemap)
            e = DTS_OK;
            for (int k = 0; k < s.nout; ++k) g->lay_mid[k].init(s.out[k].w, s.out[k].h, DTS_FMT_P010LE);
            g->hdr_chunk = g->batch;
            for (int sl = 0; sl < 2 && !e; ++sl) {
                for (int k = 0; k < s.nout && !e; ++k)
                    if (hipMalloc(&g->hdr_mid[sl][k], (size_t)g->hdr_chunk * g->lay_mid[k].fstride) != hipSuccess)
                        e = DTS_E_NOMEM;
                if (!e && hipEventCreateWithFlags(&g->hdr_ev[sl], hipEventDisableTiming) != hipSuccess) e = DTS_E_HIP;
            }
            if (!e) {
                const std::vector<float> luts = tonemap_luts(s.tonemap);
                const size_t nb = luts.size() * sizeof(float);
                if (hipMalloc(&g->dev_tm_lut, nb) != hipSuccess ||
                    hipMemcpy(g->dev_tm_lut, luts.data(), nb, hipMemcpyHostToDevice) != hipSuccess)
                    e = DTS_E_HIP;
                g->tm.lut = reinterpret_cast<const float2 *>(g->dev_tm_lut);
            }
            if (e) {
                ctx->last_hip = (int)hipGetLastError();
                dts_graph_destroy(g);
                return e;
            }
        }
        if (s.quality) g->lay_q.init(s.out[s.quality_out].w, s.out[s.quality_out].h, s.out[s.quality_out].fmt, true);
        // rendition quality: the reference renditions are a graph of their own over the same
        // source (deinterlaced first when the graph deinterlaces: it runs on our yadif output)
        dts_graph_spec rs = s;
        rs.nout = 0;
        rs.quality = 0;
        rs.deint = 0;
        rs.max_batch = g->batch;
        for (int k = 0; k < s.nout; ++k)
            if (s.out[k].quality && s.out[k].qref_method != DTS_QREF_EXTERNAL) {
                dts_output_spec &o = rs.out[rs.nout];
                o = s.out[k];
                o.method = s.out[k].qref_method;
                o.param[0] = o.param[1] = DTS_PARAM_DEFAULT;
                o.quality = 0;
                g->rq_out[rs.nout++] = k;
            }
        if (rs.nout) {
            for (int k = rs.nout; k < DTS_MAX_OUTPUTS; ++k) rs.out[k] = dts_output_spec{};
            e = dts_graph_create(ctx, &rs, &g->ref);
            if (e) {
                dts_graph_destroy(g);
                return e;
            }
            g->nrq = rs.nout;
        }
        *out = g;
        return DTS_OK;
    } catch (const std::bad_alloc &) {
        if (g) dts_graph_destroy(g);
        return DTS_E_NOMEM;
    } catch (...) {
        if (g) dts_graph_destroy(g);
        return DTS_E_INVAL;
    }
}

int dts_graph_plan(const dts_graph_spec *spec, dts_graph_info *info)
{
    if (!spec || !info) return DTS_E_INVAL;
    try {
        GraphPlan gp;
        const int e = make_plan(*spec, gp);
        if (e) return e;
        *info = gp.info;
        return DTS_OK;
    } catch (const std::bad_alloc &) {
        return DTS_E_NOMEM;
    } catch (...) {
        return DTS_E_INVAL;
    }
}

static void free_host_path(dts_graph *g);

void dts_graph_destroy(dts_graph *g)
{
    if (!g) return;
    hipSetDevice(g->ctx->device);
    free_host_path(g);
    for (int sl = 0; sl < 2; ++sl) {
        if (g->hdr_ev[sl]) {
            hipEventSynchronize(g->hdr_ev[sl]);
            hipEventDestroy(g->hdr_ev[sl]);
        }
        for (int k = 0; k < DTS_MAX_OUTPUTS; ++k)
            if (g->hdr_mid[sl][k]) hipFree(g->hdr_mid[sl][k]);
    }
    if (g->dev_tm_lut) hipFree(g->dev_tm_lut);
    if (g->ref) dts_graph_destroy(g->ref);
    if (g->dev_tables) hipFree(g->dev_tables);
    if (g->dev_tables4) hipFree(g->dev_tables4);
    if (g->dev_tables5) hipFree(g->dev_tables5);
    if (g->dev_tables7) hipFree(g->dev_tables7);
    if (g->dev_queue) hipFree(g->dev_queue);
    qscratch_free(g->qs);
    for (auto &q : g->hqs) qscratch_free(q);
    dts_ctx *ctx = g->ctx;
    delete g;
    ctx_release(ctx);
}

int dts_graph_info_get(const dts_graph *g, dts_graph_info *info)
{
    if (!g || !info) return DTS_E_INVAL;
    *info = g->info;
    return DTS_OK;
}

// ---------------------------------------------------------------------------
// device-resident path
// ---------------------------------------------------------------------------
static bool planes_ok(const dts_dev_frames &f, int w, int h, int fmt, int align)
{
    int64_t rowb[3], rows[3];
    plane_geom(w, h, fmt, rowb, rows);
    for (int p = 0; p < 3; ++p) {
        if (!rowb[p]) continue;
        if (!f.data[p] || f.pitch[p] < rowb[p]) return false;
        if (((uintptr_t)f.data[p] % align) || (f.pitch[p] % align)) return false;
    }
    return (f.frame_stride % align) == 0;
}

static DevPlanes to_dev(const dts_dev_frames &f, int fmt)
{
    DevPlanes d{};
    for (int p = 0; p < 3; ++p) {
        d.data[p] = (uint64_t)f.data[p];
        d.pitch[p] = f.pitch[p];
    }
    if (fmt != DTS_FMT_YUV420P) {
        d.data[2] = d.data[1];
        d.pitch[2] = d.pitch[1];
    }
    d.fstride = f.frame_stride;
    return d;
}

static int ensure_qscratch(dts_ctx *ctx, QScratch &q, size_t bytes)
{
    if (!q.ev) HIPCHK(ctx, hipEventCreateWithFlags(&q.ev, hipEventDisableTiming));
    if (q.bytes >= bytes) return DTS_OK;
    if (q.p) {
        HIPCHK(ctx, hipEventSynchronize(q.ev));         // its last user is done
        hipFree(q.p);
        q.p = nullptr;
        q.bytes = 0;
    }
    HIPCHK(ctx, hipMalloc(&q.p, bytes));
    q.bytes = bytes;
    return DTS_OK;
}

// one of our batch buffers as caller-style device frames
static dts_dev_frames dev_frames(uint8_t *base, const DevLayout &lay)
{
    dts_dev_frames d{};
    for (int p = 0; p < 3; ++p) {
        d.data[p] = lay.rowb[p] ? base + lay.off[p] : nullptr;
        d.pitch[p] = lay.pitch[p];
    }
    d.frame_stride = lay.fstride;
    return d;
}

// the deinterlace buffer of a QScratch (same reuse rule as the quality partials)
static int ensure_dscratch(dts_ctx *ctx, QScratch &q, size_t bytes)
{
    if (!q.dev) HIPCHK(ctx, hipEventCreateWithFlags(&q.dev, hipEventDisableTiming));
    if (q.dbytes >= bytes) return DTS_OK;
    if (q.dp) {
        HIPCHK(ctx, hipEventSynchronize(q.dev));
        hipFree(q.dp);
        q.dp = nullptr;
        q.dbytes = 0;
    }
    HIPCHK(ctx, hipMalloc(&q.dp, bytes));
    q.dbytes = bytes;
    return DTS_OK;
}

// k_yadif over outputs first .. first+count-1 of a device sequence (vf_yadif.c filter_slice)
static int yadif_enqueue(dts_ctx *ctx, int w, int h, int mode, int tff, const dts_dev_frames &seq, int nseq, int first,
                         int count, const dts_dev_frames &dst, hipStream_t st)
{
    const int fields = (mode & 1) ? 2 : 1;
    YadifParams p{};
    p.seq = to_dev(seq, DTS_FMT_YUV420P);
    p.w = w;
    p.h = h;
    p.nseq = nseq;
    p.mode = mode;
    p.tff = tff ? 1 : 0;
    p.aligned = planes_ok(seq, w, h, DTS_FMT_YUV420P, 4) && planes_ok(dst, w, h, DTS_FMT_YUV420P, 4);
    p.first = first;
    p.dst = to_dev(dst, DTS_FMT_YUV420P);
    if (yadif_t_ok(p) && !diag_env("DTS_YADIF_V1")) {    // the temporal walk (16-byte aligned frames)
        HIPCHK(ctx, launch_yadif_t(p, count, st));
        return DTS_OK;
    }
    const int chunk = 32768;                              // outputs per launch (grid z)
    for (int j0 = 0; j0 < count; j0 += chunk) {
        const int n = std::min(chunk, count - j0);
        p.first = first + j0;
        p.dst = to_dev(dst, DTS_FMT_YUV420P);
        for (int pl = 0; pl < 3; ++pl) p.dst.data[pl] += (uint64_t)((int64_t)j0 * fields * dst.frame_stride);
        HIPCHK(ctx, launch_yadif(p, n * fields, st));
    }
    return DTS_OK;
}

static int quality_enqueue(dts_ctx *ctx, QScratch &qs, int w, int h, int fmt, const dts_dev_frames &a,
                           const dts_dev_frames &b, int n, dts_qraw *qraw, hipStream_t st)
{
    QualityParams q{};
    q.a = to_dev(a, fmt);
    q.b = to_dev(b, fmt);
    q.pw[0] = w;
    q.ph[0] = h;
    q.pw[1] = q.pw[2] = (w + 1) >> 1;
    q.ph[1] = q.ph[2] = (h + 1) >> 1;
    int total = 0;
    const int walk = fmt == DTS_FMT_NV12 ? kQWalkNV12 : kQWalk;
    for (int p = 0; p < 3; ++p) {
        q.tbx[p] = fmt == DTS_FMT_NV12 && p > 0 ? kQTileBX / 2 : kQTileBX;
        q.tiles_x[p] = (q.pw[p] + 4 * q.tbx[p] - 1) / (4 * q.tbx[p]);
        // walks of about `walk` tiles, as many as the plane's tile rows round to, evened out: a
        // last walk of a few rows would cost a workgroup's setup, apron row and reduction
        const int trows = (q.ph[p] + 4 * kQTileBY - 1) / (4 * kQTileBY);
        const int nw = DTS_Q_BAL ? std::max(1, (trows + walk / 2) / walk) : (trows + walk - 1) / walk;
        q.walk[p] = DTS_Q_BAL ? (trows + nw - 1) / nw : walk;
        q.tiles_y[p] = (trows + q.walk[p] - 1) / q.walk[p];
        q.tile_base[p] = total;
        total += q.tiles_x[p] * q.tiles_y[p];
    }
    q.tile_base[3] = total;
    q.interleaved = fmt == DTS_FMT_NV12;
    q.nframes = n;
    const size_t need = (size_t)n * total * (sizeof(double) + sizeof(unsigned long long));
    int e = ensure_qscratch(ctx, qs, need);
    if (e) return e;
    q.partial_ssim = static_cast<double *>(qs.p);
    q.partial_sse = reinterpret_cast<unsigned long long *>(static_cast<uint8_t *>(qs.p) +
                                                          (size_t)n * total * sizeof(double));
    q.out = qraw;
    HIPCHK(ctx, hipStreamWaitEvent(st, qs.ev, 0));         // the previous user of these partials
    HIPCHK(ctx, launch_quality(q, total, st));
    HIPCHK(ctx, hipEventRecord(qs.ev, st));
    return DTS_OK;
}

// k_ladder7 writes its outputs with 4-byte (and wider) row segments: every output plane
// base and pitch 4-byte aligned
static bool planes_aligned4(const DevPlanes &p)
{
    for (int pl = 0; pl < 3; ++pl)
        if ((p.data[pl] | (uint64_t)p.pitch[pl]) & 3u) return false;
    return (p.fstride & 3) == 0;
}

// k_ladder7 stages source rows with 16-byte LDS-DMA lanes: every plane base and pitch
// 16-byte aligned (else k_ladder5 / k_ladder4)
static bool planes_aligned7(const DevPlanes &p)
{
    for (int pl = 0; pl < 3; ++pl)
        if ((p.data[pl] | (uint64_t)p.pitch[pl]) & 15u) return false;
    return (p.fstride & 15) == 0;
}

// The ladder launches (v4 kinds, then v3 kinds) for nframes frames of src into dst[k]
// (format dst_fmt[k]); persistent grids over nframes x njobs items, items per launch < 2^30.
static int enqueue_ladder(dts_graph *g, const DevPlanes &src, const DevPlanes *dst, const int *dst_fmt, int nframes,
                          hipStream_t st)
{
    const dts_graph_spec &s = g->spec;
    dts_ctx *ctx = g->ctx;
    LadderParams p{};
    p.src = src;
    for (int k = 0; k < DTS_MAX_OUTPUTS; ++k) {
        const int kk = k < s.nout ? k : 0;
        p.dst[k] = dst[kk];
        p.dst_fmt[k] = dst_fmt[kk];
    }
    p.srcW = s.src_w;
    p.srcH = s.src_h;
    p.chrW = (s.src_w + 1) >> 1;
    p.chrH = (s.src_h + 1) >> 1;
    p.src_kind = g->src_kind;
    p.nrungs = s.nout;
    p.njobs = (int)g->jobs.size();
    p.ring_pairs = g->ring_pairs;
    p.stage_bytes = g->stage_bytes;
    p.jobs = g->dev_jobs;
    p.rk = g->dev_rk;
    const int njobs_max = std::max(1, std::max(std::max(p.njobs, g->njobs4), g->njobs5));
    const int max_frames = std::max(1, (1 << 30) / njobs_max);
    for (int f0 = 0; f0 < nframes; f0 += max_frames) {
        const int n = std::min(max_frames, nframes - f0);
        LadderParams pp = p;
        pp.nframes = n;
        pp.nitems = n * p.njobs;
        for (int pl = 0; pl < 3; ++pl) pp.src.data[pl] += (uint64_t)(f0 * src.fstride);
        for (int k = 0; k < DTS_MAX_OUTPUTS; ++k)
            for (int pl = 0; pl < 3; ++pl) pp.dst[k].data[pl] += (uint64_t)(f0 * pp.dst[k].fstride);
        bool aligned7 = g->v7 && planes_aligned7(pp.src);
        for (int k = 0; k < s.nout && aligned7; ++k) aligned7 = planes_aligned4(pp.dst[k]);
        if (!aligned7 && ladder_range_conv(s)) return DTS_E_UNSUPPORTED;   // range conversion: v7 only
        if (aligned7) {
            Ladder7Params q{};
            q.src = pp.src;
            for (int k = 0; k < kMaxRungs; ++k) q.dst[k] = pp.dst[k];
            q.ngroups = g->ngroups7;
            q.nframes = n;
            // the luma groups of every frame octet, then the chroma groups of every octet: one
            // switch of plane kind per launch (round-5 A/B, one box each: cfg2 171.6-172.5 k ->
            // 179.7-179.9 k fps, cfg1 +5 %, cfg4 +3 %, cfg5 +4 %, cfg3 +1 % against each octet's
            // groups in plan order); diagnostic DTS_L7_ORDER=0 / 2 / 3 for the plan order, chroma
            // first, luma-then-chroma runs of DTS_L7_SUP octets
            q.nluma = g->nluma7;
            q.order = g->nluma7 > 0 && g->nluma7 < g->ngroups7 ? 1 : 0;
            if (const char *o = diag_env("DTS_L7_ORDER")) q.order = q.order ? std::min(std::max(std::atoi(o), 0), 3) : 0;
            q.sup = 4;
            if (const char *o = diag_env("DTS_L7_SUP")) q.sup = std::max(1, std::atoi(o));
            q.groups = g->dev_groups7;
            q.units = g->dev_units7;
            q.frag = g->dev_frag7;
            q.fire = g->dev_fire7;
            const int64_t grid = (int64_t)8 * ((n + 7) / 8) * g->ngroups7;
            if (grid > INT32_MAX) return DTS_E_RANGE;
            HIPCHK(ctx, launch_ladder7(q, (int)grid, g->waves7, g->lds7, ladder_range_conv(s),
                                       g->hsplit7, g->src_kind, st));
            continue;
        }
        if (g->v5) {
            Ladder5Params q{};
            q.src = pp.src;
            for (int k = 0; k < kMaxRungs; ++k) q.dst[k] = pp.dst[k];
            q.njobs = g->njobs5;
            q.nframes = n;
            q.nq = n >= 64 ? ladder4_queues() : 1;
            q.jobs = g->dev_jobs5;
            q.kinds = g->dev_kinds5;
            q.queue = g->dev_queue + kQueueWidth * (g->queue_next++ % kQueueSlots);
            HIPCHK(ctx, hipMemsetAsync(q.queue, 0, kQueueWidth * sizeof(unsigned int), st));
            int grid = std::min(n * g->njobs5, g->grid5);
            grid = std::max(q.nq, (grid + q.nq - 1) / q.nq * q.nq);
            HIPCHK(ctx, launch_ladder5(q, g->src_kind, g->lds5, grid, st));
            continue;
        }
        if (g->njobs4) {
            Ladder4Params q{};
            q.src = pp.src;
            for (int k = 0; k < kMaxRungs; ++k) {
                q.dst[k] = pp.dst[k];
                q.dst_fmt[k] = pp.dst_fmt[k];
            }
            q.srcH = s.src_h;
            q.chrH = (s.src_h + 1) >> 1;
            q.ring = kRing4Slots;
            q.src_kind = g->src_kind;
            q.njobs = g->njobs4;
            q.nframes = n;
            q.nitems = n * g->njobs4;
            q.jobs = g->dev_jobs4;
            q.rk = g->dev_rk4;
            q.nq = n >= 64 ? ladder4_queues() : 1;               // small batches keep one queue (all XCDs busy)
            q.queue = g->dev_queue + kQueueWidth * (g->queue_next++ % kQueueSlots);
            HIPCHK(ctx, hipMemsetAsync(q.queue, 0, kQueueWidth * sizeof(unsigned int), st));
            // every queue needs workgroups: a multiple of nq, at least nq
            int grid = std::min(q.nitems, g->grid4);
            grid = std::max(q.nq, (grid + q.nq - 1) / q.nq * q.nq);
            HIPCHK(ctx, launch_ladder4(q, g->lds4, grid, st));
        }
        if (p.njobs) {
            pp.queue = g->dev_queue + kQueueWidth * (g->queue_next++ % kQueueSlots);
            HIPCHK(ctx, hipMemsetAsync(pp.queue, 0, sizeof(unsigned int), st));
            HIPCHK(ctx, launch_ladder(pp, g->ndmax, g->lds_bytes, std::min(pp.nitems, g->grid_cap), st));
        }
    }
    return DTS_OK;
}

// HDR10 -> SDR: per chunk of hdr_chunk frames, the bit-exact ladder into a p010
// intermediate (two, alternating: a chunk's ladder may run while the other buffer's tonemap
// of the host path's other stream still reads), then k_tonemap from it into the caller's
// output, both on the caller's stream.  (Round 4 measured the tonemaps on a stream of their
// own beside the next chunk's ladder, with and without room for them on the ladder's CUs:
// no gain -- DESIGN.md, k_tonemap.)
static int enqueue_hdr(dts_graph *g, const DevPlanes &src, const DevPlanes *dst, int nframes, hipStream_t st)
{
    const dts_graph_spec &s = g->spec;
    dts_ctx *ctx = g->ctx;
    for (int f0 = 0; f0 < nframes; f0 += g->hdr_chunk) {
        const int n = std::min(g->hdr_chunk, nframes - f0);
        const int sl = (int)(g->hdr_next++ & 1u);
        HIPCHK(ctx, hipStreamWaitEvent(st, g->hdr_ev[sl], 0));   // the buffer's previous tonemap is done
        DevPlanes sc = src, mid[DTS_MAX_OUTPUTS];
        int mid_fmt[DTS_MAX_OUTPUTS];
        for (int pl = 0; pl < 3; ++pl) sc.data[pl] += (uint64_t)(f0 * src.fstride);
        for (int k = 0; k < s.nout; ++k) {
            mid[k] = g->lay_mid[k].planes(g->hdr_mid[sl][k]);
            mid_fmt[k] = DTS_FMT_P010LE;
        }
        int e = enqueue_ladder(g, sc, mid, mid_fmt, n, st);
        if (e) return e;
        for (int k = 0; k < s.nout; ++k) {
            TonemapParams tp = g->tm;
            tp.src = mid[k];
            tp.dst = dst[k];
            for (int pl = 0; pl < 3; ++pl) tp.dst.data[pl] += (uint64_t)(f0 * dst[k].fstride);
            tp.dst_fmt = s.out[k].fmt;
            tp.w = s.out[k].w;
            tp.h = s.out[k].h;
            tp.nframes = n;
            // the column walk (k_tonemap_w); diagnostic DTS_TM_TILED=1: the round-4 tiled kernel
            HIPCHK(ctx, diag_env("DTS_TM_TILED") ? launch_tonemap(tp, st) : launch_tonemap_w(tp, st));
        }
        HIPCHK(ctx, hipEventRecord(g->hdr_ev[sl], st));
    }
    return DTS_OK;
}

// the reference-rendition buffer of a QScratch (same reuse rule as the quality partials)
static int ensure_rscratch(dts_ctx *ctx, QScratch &q, size_t bytes)
{
    if (!q.rev) HIPCHK(ctx, hipEventCreateWithFlags(&q.rev, hipEventDisableTiming));
    if (q.rbytes >= bytes) return DTS_OK;
    if (q.rp) {
        HIPCHK(ctx, hipEventSynchronize(q.rev));
        hipFree(q.rp);
        q.rp = nullptr;
        q.rbytes = 0;
    }
    HIPCHK(ctx, hipMalloc(&q.rp, bytes));
    q.rbytes = bytes;
    return DTS_OK;
}

// The ladder of frames c0 .. c0 + m - 1 of a call over ntot frames (src / dst already at
// frame c0) and its quality: graph quality (qref = the quality_out reference batch, records
// qraw[c0 + f]), rendition quality against references the graph makes (g->ref, into scratch)
// or that come with the call (DTS_QREF_EXTERNAL: qref = nout batches), records
// qraw[k * ntot + c0 + f].  m <= g->batch when the graph makes references.
static int ladder_quality(dts_graph *g, QScratch &qs, const DevPlanes &src, const DevPlanes *dst, const int *dfmt,
                          int c0, int m, int ntot, const dts_dev_frames *qref, dts_qraw *qraw, hipStream_t st)
{
    const dts_graph_spec &s = g->spec;
    dts_ctx *ctx = g->ctx;
    const bool gq = s.quality && qref && qraw;
    bool ext = false, rq = g->ref && qraw;
    for (int k = 0; k < s.nout; ++k) ext = ext || (s.out[k].quality && s.out[k].qref_method == DTS_QREF_EXTERNAL);
    ext = ext && qref && qraw;
    if (!gq && !ext && !rq) return g->hdr ? enqueue_hdr(g, src, dst, m, st) : enqueue_ladder(g, src, dst, dfmt, m, st);
    DevPlanes qr[kMaxRungs] = {};
    dts_qraw *out_q = qraw + c0;
    int64_t qstride = ntot;
    auto at_c0 = [&](const dts_dev_frames &d, int fmt) {
        DevPlanes r = to_dev(d, fmt);
        for (int pl = 0; pl < 3; ++pl)
            if (r.data[pl]) r.data[pl] += (uint64_t)((int64_t)c0 * d.frame_stride);
        return r;
    };
    if (gq) {
        qr[s.quality_out] = at_c0(*qref, s.out[s.quality_out].fmt);
        qstride = 0;
    }
    if (ext)
        for (int k = 0; k < s.nout; ++k)
            if (s.out[k].quality && s.out[k].qref_method == DTS_QREF_EXTERNAL) qr[k] = at_c0(qref[k], s.out[k].fmt);
    if (rq) {                                    // the reference renditions of these frames, into scratch
        dts_graph *r = g->ref;
        size_t off[DTS_MAX_OUTPUTS], total = 0;
        for (int j = 0; j < g->nrq; ++j) {
            off[j] = total;
            total += (size_t)g->batch * (size_t)r->lay_out[j].fstride;
        }
        int e = ensure_rscratch(ctx, qs, total);
        if (e) return e;
        HIPCHK(ctx, hipStreamWaitEvent(st, qs.rev, 0));        // the buffer's previous user
        DevPlanes rd[DTS_MAX_OUTPUTS];
        int rf[DTS_MAX_OUTPUTS];
        for (int j = 0; j < g->nrq; ++j) {
            rd[j] = r->lay_out[j].planes(static_cast<uint8_t *>(qs.rp) + off[j]);
            rf[j] = r->spec.out[j].fmt;
            qr[g->rq_out[j]] = rd[j];
        }
        e = enqueue_ladder(r, src, rd, rf, m, st);
        if (e) return e;
    }
    // the ladder, then k_quality per output with a reference (a separate pass: fused into
    // k_ladder7's V epilogue it measured 2.3x slower, DESIGN.md §4 k_quality)
    int e = g->hdr ? enqueue_hdr(g, src, dst, m, st) : enqueue_ladder(g, src, dst, dfmt, m, st);
    for (int k = 0; k < s.nout && !e; ++k) {
        if (!qr[k].data[0]) continue;
        const dts_output_spec &o = s.out[k];
        dts_dev_frames a{}, b{};
        for (int pl = 0; pl < 3; ++pl) {
            a.data[pl] = dst[k].data[pl] ? reinterpret_cast<void *>(dst[k].data[pl]) : nullptr;
            a.pitch[pl] = dst[k].pitch[pl];
            b.data[pl] = qr[k].data[pl] ? reinterpret_cast<void *>(qr[k].data[pl]) : nullptr;
            b.pitch[pl] = qr[k].pitch[pl];
        }
        a.frame_stride = dst[k].fstride;
        b.frame_stride = qr[k].fstride;
        e = quality_enqueue(ctx, qs, o.w, o.h, o.fmt, a, b, m, out_q + (int64_t)k * qstride, st);
    }
    if (!e && rq) HIPCHK(ctx, hipEventRecord(qs.rev, st));
    return e;
}

static int run_device(dts_graph *g, QScratch &qs, const dts_dev_frames *src, int nframes, const dts_dev_frames *dst,
                      const dts_dev_frames *qref, dts_qraw *qraw_dev, void *stream)
{
    if (!g || !src || !dst || nframes < 0) return DTS_E_INVAL;
    if (nframes == 0) return DTS_OK;
    const dts_graph_spec &s = g->spec;
    if (!planes_ok(*src, s.src_w, s.src_h, s.src_fmt, 16)) return DTS_E_INVAL;
    for (int k = 0; k < s.nout; ++k)
        if (!planes_ok(dst[k], s.out[k].w, s.out[k].h, s.out[k].fmt, 4)) return DTS_E_INVAL;
    if (s.src_fmt == DTS_FMT_YUV420P && src->pitch[1] != src->pitch[2]) return DTS_E_INVAL;
    if (s.quality && qref && qraw_dev &&
        !planes_ok(*qref, s.out[s.quality_out].w, s.out[s.quality_out].h, s.out[s.quality_out].fmt, 4))
        return DTS_E_INVAL;
    for (int k = 0; k < s.nout && qref && qraw_dev; ++k)       // external reference renditions
        if (s.out[k].quality && s.out[k].qref_method == DTS_QREF_EXTERNAL &&
            !planes_ok(qref[k], s.out[k].w, s.out[k].h, s.out[k].fmt, 4))
            return DTS_E_INVAL;
    dts_ctx *ctx = g->ctx;
    hipSetDevice(ctx->device);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream[0];

    DevPlanes ddst[DTS_MAX_OUTPUTS];
    int dfmt[DTS_MAX_OUTPUTS];
    for (int k = 0; k < s.nout; ++k) {
        ddst[k] = to_dev(dst[k], s.out[k].fmt);
        dfmt[k] = s.out[k].fmt;
    }
    auto dst_at = [&](int c0, DevPlanes *dd) {
        for (int k = 0; k < s.nout; ++k) {
            dd[k] = ddst[k];
            for (int pl = 0; pl < 3; ++pl) dd[k].data[pl] += (uint64_t)((int64_t)c0 * dst[k].frame_stride);
        }
    };
    const int B = g->batch;
    if (s.deint) {
        // yadif into a batch of deinterlaced frames, then the ladder (and quality) from it;
        // src holds nframes + 2 frames (one context frame each side)
        int e = ensure_dscratch(ctx, qs, (size_t)B * g->lay_src.fstride);
        if (e) return e;
        const dts_dev_frames dbuf = dev_frames(static_cast<uint8_t *>(qs.dp), g->lay_src);
        for (int c0 = 0; c0 < nframes; c0 += B) {
            const int m = std::min(B, nframes - c0);
            HIPCHK(ctx, hipStreamWaitEvent(st, qs.dev, 0));   // the buffer's previous user
            e = yadif_enqueue(ctx, s.src_w, s.src_h, s.deint_mode, s.deint_tff, *src, nframes + 2, 1 + c0, m, dbuf, st);
            if (e) return e;
            DevPlanes dd[DTS_MAX_OUTPUTS];
            dst_at(c0, dd);
            e = ladder_quality(g, qs, to_dev(dbuf, s.src_fmt), dd, dfmt, c0, m, nframes, qref, qraw_dev, st);
            if (e) return e;
            HIPCHK(ctx, hipEventRecord(qs.dev, st));
        }
        return DTS_OK;
    }
    const DevPlanes dsrc = to_dev(*src, s.src_fmt);
    // diagnostic DTS_Q_SUB=n (round-5 A/B, DESIGN.md §4 k_quality): with rendition quality, the
    // ladder and its quality passes per sub-batch of n frames, so the renditions may still sit in
    // the Infinity Cache when k_quality reads them back
    const char *qsub_env = diag_env("DTS_Q_SUB");
    const int qsub = qsub_env && qraw_dev && qref ? std::max(0, std::atoi(qsub_env)) : 0;
    if (!(g->ref && qraw_dev) && !qsub)          // no reference renditions to make: one call
        return ladder_quality(g, qs, dsrc, ddst, dfmt, 0, nframes, nframes, qref, qraw_dev, st);
    const int step = g->ref && qraw_dev ? (qsub ? std::min(qsub, B) : B) : qsub;
    for (int c0 = 0; c0 < nframes; c0 += step) { // reference renditions: one batch of scratch at a time
        const int m = std::min(step, nframes - c0);
        DevPlanes sc = dsrc, dd[DTS_MAX_OUTPUTS];
        for (int pl = 0; pl < 3; ++pl) sc.data[pl] += (uint64_t)((int64_t)c0 * src->frame_stride);
        dst_at(c0, dd);
        const int e = ladder_quality(g, qs, sc, dd, dfmt, c0, m, nframes, qref, qraw_dev, st);
        if (e) return e;
    }
    return DTS_OK;
}

int dts_graph_run_device(dts_graph *g, const dts_dev_frames *src, int nframes, const dts_dev_frames *dst,
                         const dts_dev_frames *qref, dts_qraw *qraw_dev, void *stream)
{
    if (!g) return DTS_E_INVAL;
    return run_device(g, g->qs, src, nframes, dst, qref, qraw_dev, stream);
}

int dts_quality_run_device(dts_ctx *ctx, int w, int h, int fmt, const dts_dev_frames *a, const dts_dev_frames *b,
                           int nframes, dts_qraw *qraw_dev, void *stream)
{
    if (!ctx || !a || !b || !qraw_dev || nframes < 0 || w < 1 || h < 1) return DTS_E_INVAL;
    if (!fmt_8bit(fmt)) return DTS_E_UNSUPPORTED;
    if (!planes_ok(*a, w, h, fmt, 4) || !planes_ok(*b, w, h, fmt, 4)) return DTS_E_INVAL;
    if (nframes == 0) return DTS_OK;
    hipSetDevice(ctx->device);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream[0];
    return quality_enqueue(ctx, ctx->qs, w, h, fmt, *a, *b, nframes, qraw_dev, st);
}

// Host frames -> device batches -> k_quality -> finished statistics (the Node worker's
// per-rendition vf_psnr / vf_ssim against a reference rendition).  Synchronous on the
// ctx's stream 0.  Frames go through in batches of kQHostBatch into a device buffer the
// ctx keeps (grown once, reused by every later call): a 600-frame 4K segment needs one
// batch of scratch, not 2 x 600 frames.
constexpr int kQHostBatch = 32;

int dts_quality_run_host(dts_ctx *ctx, int w, int h, int fmt, const dts_frame *a, const dts_frame *b, int nframes,
                         dts_qstat *out)
{
    if (!ctx || !a || !b || !out || nframes < 0 || w < 1 || h < 1) return DTS_E_INVAL;
    if (!fmt_8bit(fmt)) return DTS_E_UNSUPPORTED;
    if (nframes == 0) return DTS_OK;
    int64_t rowb[3], rows[3];
    plane_geom(w, h, fmt, rowb, rows);
    for (int f = 0; f < nframes; ++f)
        for (int p = 0; p < 3; ++p)
            if (rowb[p] && (!a[f].data[p] || !b[f].data[p] || a[f].pitch[p] < rowb[p] || b[f].pitch[p] < rowb[p]))
                return DTS_E_INVAL;
    hipSetDevice(ctx->device);
    DevLayout lay;
    lay.init(w, h, fmt);
    const size_t fb = (size_t)lay.fstride, nb = (size_t)std::min(nframes, kQHostBatch);
    const size_t qoff = align_up((int64_t)(2 * fb * nb), 256), need = qoff + nb * sizeof(dts_qraw);
    hipStream_t st = ctx->stream[0];
    if (ctx->hq_bytes < need) {
        HIPCHK(ctx, hipStreamSynchronize(st));
        if (ctx->hq) hipFree(ctx->hq);
        ctx->hq = nullptr;
        ctx->hq_bytes = 0;
        HIPCHK(ctx, hipMalloc(&ctx->hq, need));
        ctx->hq_bytes = need;
    }
    uint8_t *dev = ctx->hq;
    dts_qraw *qd = reinterpret_cast<dts_qraw *>(dev + qoff);
    std::vector<dts_qraw> qh((size_t)nframes);
    dts_dev_frames da{}, db{};
    for (int p = 0; p < 3; ++p) {
        const int pp = rowb[p] ? p : 1;
        da.data[p] = dev + lay.off[pp];
        db.data[p] = dev + nb * fb + lay.off[pp];
        da.pitch[p] = db.pitch[p] = lay.pitch[pp];
    }
    da.frame_stride = db.frame_stride = (int64_t)fb;
    for (int f0 = 0; f0 < nframes; f0 += (int)nb) {
        const int m = std::min((int)nb, nframes - f0);
        for (int i = 0; i < m; ++i)
            for (int p = 0; p < 3; ++p) {
                if (!rowb[p]) continue;
                const dts_frame &fa = a[f0 + i], &fbh = b[f0 + i];
                HIPCHK(ctx, hipMemcpy2DAsync(dev + i * fb + lay.off[p], (size_t)lay.pitch[p], fa.data[p],
                                             (size_t)fa.pitch[p], (size_t)rowb[p], (size_t)rows[p],
                                             hipMemcpyHostToDevice, st));
                HIPCHK(ctx, hipMemcpy2DAsync(dev + (nb + i) * fb + lay.off[p], (size_t)lay.pitch[p], fbh.data[p],
                                             (size_t)fbh.pitch[p], (size_t)rowb[p], (size_t)rows[p],
                                             hipMemcpyHostToDevice, st));
            }
        int e = quality_enqueue(ctx, ctx->qs, w, h, fmt, da, db, m, qd, st);
        if (e) return e;
        HIPCHK(ctx, hipMemcpyAsync(qh.data() + f0, qd, (size_t)m * sizeof(dts_qraw), hipMemcpyDeviceToHost, st));
        HIPCHK(ctx, hipStreamSynchronize(st));      // the batch buffer is reused by the next batch
    }
    return dts_qstat_finalize(w, h, qh.data(), nframes, out);
}

int dts_qraw_sum_device(dts_ctx *ctx, const dts_qraw *raw_dev, int n, dts_qraw *sum_dev, void *stream)
{
    if (!ctx || !raw_dev || !sum_dev || n < 0) return DTS_E_INVAL;
    hipSetDevice(ctx->device);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream[0];
    HIPCHK(ctx, launch_qsum(raw_dev, n, sum_dev, st));
    return DTS_OK;
}

int dts_qstat_stream(int w, int h, const dts_qraw *sum, int64_t nframes, dts_qstat *out)
{
    if (!sum || !out || nframes < 1 || w < 1 || h < 1) return DTS_E_INVAL;
    // vf_psnr uninit: psnr(mse_comp[c] / nb_frames), psnr(mse / nb_frames) with mse the
    // area-weighted per-frame average; vf_ssim uninit: ssim[c] / nb_frames and
    // ssim_total / nb_frames.  Plane sizes are fixed, so both are the per-frame
    // formulas (dts_qstat_finalize) on the summed record with every count x nframes.
    const int pw[3] = {w, (w + 1) >> 1, (w + 1) >> 1}, ph[3] = {h, (h + 1) >> 1, (h + 1) >> 1};
    double area = 0;
    for (int c = 0; c < 3; ++c) area += (double)pw[c] * ph[c];
    double mse = 0, ssim = 0;
    const double n = (double)nframes;
    for (int c = 0; c < 3; ++c) {
        const double wgt = (double)pw[c] * ph[c] / area;
        out->sse[c] = sum->sse[c];
        out->mse[c] = sum->sse[c] / ((double)((int64_t)pw[c] * ph[c]) * n);
        out->psnr[c] = 10.0 * std::log10(255.0 * 255.0 / out->mse[c]);
        mse += out->mse[c] * wgt;
        const int nw = ((pw[c] >> 2) - 1) * ((ph[c] >> 2) - 1);
        out->ssim[c] = sum->ssim_sum[c] / ((double)nw * n);
        ssim += wgt * out->ssim[c];
    }
    out->mse_avg = mse;
    out->psnr_avg = 10.0 * std::log10(255.0 * 255.0 / mse);
    out->ssim_all = ssim;
    out->ssim_db = 10.0 * std::log10(1.0 / (1.0 - ssim));
    return DTS_OK;
}

int dts_yadif_run_device(dts_ctx *ctx, int w, int h, int mode, int tff, const dts_dev_frames *seq, int nseq,
                         int first, int count, const dts_dev_frames *dst, void *stream)
{
    if (!ctx || !seq || !dst || w < 16 || h < 4 || mode < 0 || mode > 3 || nseq < 1 || first < 0 || count < 0 ||
        first + count > nseq)
        return DTS_E_INVAL;
    if (!planes_ok(*seq, w, h, DTS_FMT_YUV420P, 1) || !planes_ok(*dst, w, h, DTS_FMT_YUV420P, 1))
        return DTS_E_INVAL;
    if (count == 0) return DTS_OK;
    hipSetDevice(ctx->device);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream[0];
    return yadif_enqueue(ctx, w, h, mode, tff, *seq, nseq, first, count, *dst, st);
}

int dts_qstat_finalize(int w, int h, const dts_qraw *raw, int n, dts_qstat *out)
{
    if (!raw || !out || n < 0 || w < 1 || h < 1) return DTS_E_INVAL;
    int pw[3] = {w, (w + 1) >> 1, (w + 1) >> 1}, ph[3] = {h, (h + 1) >> 1, (h + 1) >> 1};
    double area = 0;
    for (int c = 0; c < 3; ++c) area += (double)pw[c] * ph[c];
    for (int i = 0; i < n; ++i) {
        dts_qstat &q = out[i];
        double mse = 0, ssim = 0;
        for (int c = 0; c < 3; ++c) {
            const double wgt = (double)pw[c] * ph[c] / area;
            q.sse[c] = raw[i].sse[c];
            q.mse[c] = raw[i].sse[c] / (double)((int64_t)pw[c] * ph[c]);
            q.psnr[c] = 10.0 * std::log10(255.0 * 255.0 / q.mse[c]);   // vf_psnr get_psnr
            mse += q.mse[c] * wgt;
            const int nw = ((pw[c] >> 2) - 1) * ((ph[c] >> 2) - 1);
            q.ssim[c] = raw[i].ssim_sum[c] / nw;   // vf_ssim ssim_plane (0/0 = NaN for planes < 8x8, as vf_ssim)
            ssim += wgt * q.ssim[c];
        }
        q.mse_avg = mse;
        q.psnr_avg = 10.0 * std::log10(255.0 * 255.0 / mse);
        q.ssim_all = ssim;
        q.ssim_db = 10.0 * std::log10(1.0 / (1.0 - ssim));                // vf_ssim ssim_db
    }
    return DTS_OK;
}

// ---------------------------------------------------------------------------
// host-memory path: pinned double-buffered staging over two HIP streams
// ---------------------------------------------------------------------------
static void free_host_path(dts_graph *g)
{
    for (int sl = 0; sl < 2; ++sl) {
        if (g->done[sl]) hipEventSynchronize(g->done[sl]);
        if (g->dev_src[sl]) hipFree(g->dev_src[sl]);
        for (int k = 0; k < DTS_MAX_OUTPUTS; ++k)
            if (g->dev_out[sl][k]) hipFree(g->dev_out[sl][k]);
        if (g->dev_q[sl]) hipFree(g->dev_q[sl]);
        if (g->dev_qraw[sl]) hipFree(g->dev_qraw[sl]);
        if (g->pin_in[sl]) hipHostFree(g->pin_in[sl]);
        if (g->pin_out[sl]) hipHostFree(g->pin_out[sl]);
        if (g->pin_qraw[sl]) hipHostFree(g->pin_qraw[sl]);
        if (g->done[sl]) hipEventDestroy(g->done[sl]);
        if (g->kdone[sl]) hipEventDestroy(g->kdone[sl]);
        if (g->h2d_done[sl]) hipEventDestroy(g->h2d_done[sl]);
        g->done[sl] = g->kdone[sl] = g->h2d_done[sl] = nullptr;
        g->dev_src[sl] = g->dev_q[sl] = nullptr;
        for (int k = 0; k < DTS_MAX_OUTPUTS; ++k) g->dev_out[sl][k] = nullptr;
        g->dev_qraw[sl] = g->pin_qraw[sl] = nullptr;
        g->pin_in[sl] = g->pin_out[sl] = nullptr;
        g->done[sl] = nullptr;
        g->p_chunk_first[sl] = -1;
    }
    if (g->d2h) hipStreamDestroy(g->d2h);
    g->d2h = nullptr;
    g->host_ready = false;
}

// Pinned host memory the library knows about: dts_host_alloc allocations and
// dts_host_register'ed ranges.  The host path DMAs straight from / into frames whose
// planes lie inside one of them (no pack / unpack through the pinned rings).
extern "C++" {
namespace {
struct PinnedSet {
    std::mutex m;
    std::map<uintptr_t, std::pair<size_t, bool>> r;   // base -> (bytes, registered rather than allocated)
};
PinnedSet &pinned_set()
{
    static PinnedSet *p = new PinnedSet;             // (never destroyed: frees may come at exit)
    return *p;
}
bool pinned_range(const void *ptr, size_t n)
{
    if (!ptr) return false;
    const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
    PinnedSet &ps = pinned_set();
    std::lock_guard<std::mutex> lk(ps.m);
    auto it = ps.r.upper_bound(a);
    if (it == ps.r.begin()) return false;
    --it;
    return a >= it->first && a + n <= it->first + it->second.first;
}
// frame f can move by plain DMA: every plane (layout lay: rows x row bytes) lies in pinned
// memory with the device layout's pitch, so each plane crosses as one contiguous copy.  (Pitched
// 2-D copies between host and device measured ~2 GB/s on the box -- 150 fps for cfg2 -- so frames
// with other pitches take the pinned ring.)
bool frame_direct(const dts_frame &f, const DevLayout &lay)
{
    for (int p = 0; p < 3; ++p) {
        if (!lay.rows[p]) continue;
        if (!f.data[p] || f.pitch[p] != lay.pitch[p]) return false;
        if (!pinned_range(f.data[p], (size_t)((lay.rows[p] - 1) * f.pitch[p] + lay.rowb[p]))) return false;
    }
    return true;
}
// bytes of one frame image in layout lay, from plane 0 to the last byte of the last plane
int64_t image_bytes(const DevLayout &lay)
{
    int64_t e = 0;
    for (int p = 0; p < 3; ++p)
        if (lay.rows[p]) e = std::max(e, lay.off[p] + (lay.rows[p] - 1) * lay.pitch[p] + lay.rowb[p]);
    return e;
}
// frame f's planes sit at base + lay.off[p] with the layout's pitches: the frame is the
// device frame's image byte for byte
bool same_image(const dts_frame &f, const DevLayout &lay, const uint8_t *base)
{
    for (int p = 0; p < 3; ++p)
        if (lay.rows[p] && (f.data[p] != base + lay.off[p] || f.pitch[p] != lay.pitch[p])) return false;
    return true;
}
// Frames fr[0], fr[step], .. (n of them) in pinned memory between a device batch's frames
// dev, dev + fstride, ..: runs of frames laid out exactly as the batch (one image after another,
// fstride apart: dtsffi.alloc_frames_pinned) cross as one DMA per run, every other frame as one
// DMA per plane (frame_direct).  (Per-plane copies of 1-4 MB each cost ~10 % of the link rate in
// per-copy overhead on the box: cfg2 3.2 k against 3.6 k fps through the pinned ring.)
hipError_t copy_frames_direct(uint8_t *dev, const DevLayout &lay, const dts_frame *fr, int64_t step, int n, bool h2d,
                              hipStream_t st)
{
    const int64_t img = image_bytes(lay);
    for (int f = 0; f < n;) {
        const uint8_t *b0 = static_cast<const uint8_t *>(fr[f * step].data[0]) - lay.off[0];
        int m = 0;
        while (f + m < n && same_image(fr[(f + m) * step], lay, b0 + (int64_t)m * lay.fstride)) ++m;
        while (m > 1 && !pinned_range(b0, (size_t)((m - 1) * lay.fstride + img))) m = 1;
        hipError_t e;
        if (m > 1) {
            const size_t nb = (size_t)((m - 1) * lay.fstride + img);
            uint8_t *d = dev + (int64_t)f * lay.fstride;
            e = h2d ? hipMemcpyAsync(d, b0, nb, hipMemcpyHostToDevice, st)
                    : hipMemcpyAsync(const_cast<uint8_t *>(b0), d, nb, hipMemcpyDeviceToHost, st);
            f += m;
        } else {
            const dts_frame &fm = fr[f * step];
            uint8_t *d = dev + (int64_t)f * lay.fstride;
            e = hipSuccess;
            for (int p = 0; p < 3 && e == hipSuccess; ++p) {
                if (!lay.rows[p]) continue;
                const size_t nb = (size_t)((lay.rows[p] - 1) * lay.pitch[p] + lay.rowb[p]);
                e = h2d ? hipMemcpyAsync(d + lay.off[p], fm.data[p], nb, hipMemcpyHostToDevice, st)
                        : hipMemcpyAsync(fm.data[p], d + lay.off[p], nb, hipMemcpyDeviceToHost, st);
            }
            ++f;
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
} // namespace
} // extern "C++"

static int alloc_host_path(dts_graph *g);

// Every buffer of both slots, or none (a failed allocation frees what was made,
// so a retried submit starts from scratch).
static int ensure_host_path(dts_graph *g)
{
    if (g->host_ready) return DTS_OK;
    const int e = alloc_host_path(g);
    if (e) {
        free_host_path(g);
        return e;
    }
    g->host_ready = true;
    return DTS_OK;
}

static int alloc_host_path(dts_graph *g)
{
    dts_ctx *ctx = g->ctx;
    const dts_graph_spec &s = g->spec;
    const int B = g->batch;
    const int cf = s.deint ? 2 : 0;                      // deint: one context frame each side
    // the pinned rings hold batches in the device layout (lay_*): one DMA per batch and plane set
    g->pin_in_bytes = (int64_t)(B + cf) * g->lay_src.fstride;
    if (s.quality) g->pin_in_bytes += (int64_t)B * g->lay_q.fstride;
    g->pin_out_bytes = 0;
    for (int k = 0; k < s.nout; ++k) g->pin_out_bytes += (int64_t)B * g->lay_out[k].fstride;
    for (int sl = 0; sl < 2; ++sl) {
        HIPCHK(ctx, hipMalloc(&g->dev_src[sl], (size_t)(B + cf) * g->lay_src.fstride));
        for (int k = 0; k < s.nout; ++k) HIPCHK(ctx, hipMalloc(&g->dev_out[sl][k], (size_t)B * g->lay_out[k].fstride));
        if (s.quality) {
            HIPCHK(ctx, hipMalloc(&g->dev_q[sl], (size_t)B * g->lay_q.fstride));
            HIPCHK(ctx, hipMalloc(&g->dev_qraw[sl], (size_t)B * sizeof(dts_qraw)));
            HIPCHK(ctx, hipHostMalloc(&g->pin_qraw[sl], (size_t)B * sizeof(dts_qraw), hipHostMallocDefault));
        }
        if (g->ref) {                                    // rendition quality: B x nout records per slot
            const size_t nb = (size_t)B * (size_t)s.nout * sizeof(dts_qraw);
            HIPCHK(ctx, hipMalloc(&g->dev_qraw[sl], nb));
            HIPCHK(ctx, hipMemset(g->dev_qraw[sl], 0, nb));
            HIPCHK(ctx, hipHostMalloc(&g->pin_qraw[sl], nb, hipHostMallocDefault));
        }
        HIPCHK(ctx, hipHostMalloc(&g->pin_in[sl], (size_t)g->pin_in_bytes, hipHostMallocDefault));
        HIPCHK(ctx, hipHostMalloc(&g->pin_out[sl], (size_t)g->pin_out_bytes, hipHostMallocDefault));
        HIPCHK(ctx, hipEventCreateWithFlags(&g->done[sl], hipEventDisableTiming));
        HIPCHK(ctx, hipEventCreateWithFlags(&g->kdone[sl], hipEventDisableTiming));
        HIPCHK(ctx, hipEventCreateWithFlags(&g->h2d_done[sl], hipEventDisableTiming));
    }
    HIPCHK(ctx, hipStreamCreateWithFlags(&g->d2h, hipStreamNonBlocking));
    return DTS_OK;
}

// Host threads that pack / unpack the caller's frames (DTS_HOST_THREADS, default: the
// hardware threads, at most 16).  The host path's bound is this copy, not PCIe: one
// thread moves ~8 GB/s, a 4K cfg2 frame is 17.5 MB in + out of the pinned rings.
static int host_threads()
{
    static const int n = [] {
        const char *e = std::getenv("DTS_HOST_THREADS");
        int v = e ? std::atoi(e) : (int)std::thread::hardware_concurrency();
        return std::min(std::max(v, 1), 16);
    }();
    return n;
}

// f(i) for i in [0, n) over up to host_threads() threads (the caller's among them)
extern "C++" template <class F>
static void parallel_for(int n, F f)
{
    const int nt = std::min(n, host_threads());
    if (nt <= 1) {
        for (int i = 0; i < n; ++i) f(i);
        return;
    }
    std::vector<std::thread> th;
    th.reserve((size_t)nt - 1);
    for (int t = 1; t < nt; ++t)
        th.emplace_back([&, t] {
            for (int i = t; i < n; i += nt) f(i);
        });
    for (int i = 0; i < n; i += nt) f(i);
    for (auto &x : th) x.join();
}

// rows of a caller frame into / out of one frame of a pinned batch in layout `lay`
static void pack_frame(uint8_t *dst, const dts_frame &f, const DevLayout &lay)
{
    for (int p = 0; p < 3; ++p)
        for (int64_t y = 0; y < lay.rows[p]; ++y)
            std::memcpy(dst + lay.off[p] + y * lay.pitch[p], static_cast<const uint8_t *>(f.data[p]) + y * f.pitch[p],
                        (size_t)lay.rowb[p]);
}

static void unpack_frame(const uint8_t *src, const dts_frame &f, const DevLayout &lay)
{
    for (int p = 0; p < 3; ++p)
        for (int64_t y = 0; y < lay.rows[p]; ++y)
            std::memcpy(static_cast<uint8_t *>(f.data[p]) + y * f.pitch[p], src + lay.off[p] + y * lay.pitch[p],
                        (size_t)lay.rowb[p]);
}

// a pinned batch <-> the device batch: the same image, one contiguous copy
static hipError_t copy_frames(uint8_t *dev, const DevLayout &lay, uint8_t *host, int n, bool h2d, hipStream_t st)
{
    const size_t nb = (size_t)n * (size_t)lay.fstride;
    return h2d ? hipMemcpyAsync(dev, host, nb, hipMemcpyHostToDevice, st)
               : hipMemcpyAsync(host, dev, nb, hipMemcpyDeviceToHost, st);
}

static int finish_slot(dts_graph *g, int sl)
{
    if (g->p_chunk_first[sl] < 0) return DTS_OK;
    dts_ctx *ctx = g->ctx;
    const dts_graph_spec &s = g->spec;
    HIPCHK(ctx, hipEventSynchronize(g->done[sl]));
    const int f0 = g->p_chunk_first[sl], n = g->p_chunk_n[sl];
    const uint8_t *hp0 = g->pin_out[sl];         // per output: a region of `batch` packed frames
    if (g->p_zout[sl] != (1u << s.nout) - 1) parallel_for(n * s.nout, [&](int i) {
        const int f = i / s.nout, k = i % s.nout;
        if ((g->p_zout[sl] >> k) & 1) return;                      // (went straight into the caller's frame)
        const uint8_t *hp = hp0;
        for (int kk = 0; kk < k; ++kk) hp += (int64_t)g->batch * g->lay_out[kk].fstride;
        unpack_frame(hp + (int64_t)f * g->lay_out[k].fstride, g->p_dst[(int64_t)(f0 + f) * s.nout + k], g->lay_out[k]);
    });
    if (s.quality && g->p_q) {
        const dts_output_spec &o = s.out[s.quality_out];
        dts_qstat_finalize(o.w, o.h, g->pin_qraw[sl], n, g->p_q + f0);
    }
    if (g->ref && g->p_q) {                    // records [k][n] -> q[(f0 + f) * nout + k]
        std::vector<dts_qstat> tmp((size_t)n);
        for (int k = 0; k < s.nout; ++k) {
            if (s.out[k].quality)
                dts_qstat_finalize(s.out[k].w, s.out[k].h, g->pin_qraw[sl] + (int64_t)k * n, n, tmp.data());
            for (int f = 0; f < n; ++f)
                g->p_q[(int64_t)(f0 + f) * s.nout + k] = s.out[k].quality ? tmp[(size_t)f] : dts_qstat{};
        }
    }
    g->p_chunk_first[sl] = -1;
    return DTS_OK;
}

int dts_graph_submit(dts_graph *g, const dts_frame *src, int nframes, const dts_frame *dst, const dts_frame *qref,
                     dts_qstat *q)
{
    if (!g || !src || !dst || nframes < 0) return DTS_E_INVAL;
    if (g->pending) return DTS_E_BUSY;
    const dts_graph_spec &s = g->spec;
    if (s.quality && !qref) return DTS_E_INVAL;
    // external reference renditions (DTS_QREF_EXTERNAL) come with dts_graph_run_device only:
    // the host path has no way to take nout reference batches, so it refuses the graph rather
    // than return records it never computed
    for (int k = 0; k < s.nout; ++k)
        if (s.out[k].quality && s.out[k].qref_method == DTS_QREF_EXTERNAL) return DTS_E_UNSUPPORTED;
    dts_ctx *ctx = g->ctx;
    hipSetDevice(ctx->device);
    try {
        int e = ensure_host_path(g);
        if (e) return e;
        g->pending = true;
        g->p_dst = dst;
        g->p_q = q;
        const int B = g->batch;
        int chunk = 0;
        for (int f0 = 0; f0 < nframes; f0 += B, ++chunk) {
            const int sl = chunk & 1;
            const int n = std::min(B, nframes - f0);
            // Slot reuse without a host stall before the inputs go out: the input ring only waits
            // for chunk c - 2's H2D (h2d_done), the slot's device inputs for its kernels (stream
            // order), its device outputs for its D2H (done, on the device), and chunk c - 2's
            // results are handed over (finish_slot) only before this chunk's D2H reuses the output
            // ring -- so chunk c's H2D is queued while c - 2's results are still crossing
            hipStream_t st = ctx->stream[sl];
            uint8_t *hp = g->pin_in[sl];
            const int cf = s.deint ? 2 : 0;              // deint: src[f0 .. f0 + n + 1] (context frames)
            // frames in pinned memory (dts_host_alloc / dts_host_register) go to the device by DMA
            // straight from the caller's planes; others are packed into the pinned ring first
            bool zin = true;
            for (int f = 0; f < n + cf && zin; ++f) zin = frame_direct(src[f0 + f], g->lay_src);
            for (int f = 0; f < n && zin && s.quality; ++f) zin = frame_direct(qref[f0 + f], g->lay_q);
            if (!zin) HIPCHK(ctx, hipEventSynchronize(g->h2d_done[sl]));   // the input ring refills
            if (zin) {
                HIPCHK(ctx, copy_frames_direct(static_cast<uint8_t *>(g->dev_src[sl]), g->lay_src, src + f0, 1, n + cf,
                                               true, st));
            } else {
                parallel_for(n + cf, [&](int f) {
                    pack_frame(hp + (int64_t)f * g->lay_src.fstride, src[f0 + f], g->lay_src);
                });
                HIPCHK(ctx, copy_frames(g->dev_src[sl], g->lay_src, hp, n + cf, true, st));
            }
            uint8_t *qhp = hp + (int64_t)(B + cf) * g->lay_src.fstride;
            if (s.quality && zin) {
                HIPCHK(ctx, copy_frames_direct(static_cast<uint8_t *>(g->dev_q[sl]), g->lay_q, qref + f0, 1, n, true, st));
            } else if (s.quality) {
                parallel_for(n, [&](int f) {
                    pack_frame(qhp + (int64_t)f * g->lay_q.fstride, qref[f0 + f], g->lay_q);
                });
                HIPCHK(ctx, copy_frames(g->dev_q[sl], g->lay_q, qhp, n, true, st));
            }
            HIPCHK(ctx, hipEventRecord(g->h2d_done[sl], st));
            HIPCHK(ctx, hipStreamWaitEvent(st, g->done[sl], 0));    // chunk c - 2's outputs have left
            dts_dev_frames dsrc = dev_frames(g->dev_src[sl], g->lay_src);
            dts_dev_frames ddst[DTS_MAX_OUTPUTS];
            for (int k = 0; k < s.nout; ++k) ddst[k] = dev_frames(g->dev_out[sl][k], g->lay_out[k]);
            dts_dev_frames dq = s.quality ? dev_frames(g->dev_q[sl], g->lay_q) : dts_dev_frames{};
            e = run_device(g, g->hqs[sl], &dsrc, n, ddst, s.quality ? &dq : nullptr,
                           (s.quality || g->ref) ? g->dev_qraw[sl] : nullptr, st);
            if (e) return e;
            // the results leave on the D2H stream once the slot's kernels are done, beside the next
            // chunks' H2D (the two directions of the link at once)
            HIPCHK(ctx, hipEventRecord(g->kdone[sl], st));
            HIPCHK(ctx, hipStreamWaitEvent(g->d2h, g->kdone[sl], 0));
            e = finish_slot(g, sl);              // chunk c - 2's results out of the output ring
            if (e) return e;
            st = g->d2h;
            // per output: straight into the caller's pinned frames, or through the pinned ring
            uint32_t zout = 0;
            uint8_t *op = g->pin_out[sl];
            for (int k = 0; k < s.nout; ++k) {
                bool z = true;
                for (int f = 0; f < n && z; ++f) z = frame_direct(dst[(int64_t)(f0 + f) * s.nout + k], g->lay_out[k]);
                if (z) {
                    zout |= 1u << k;
                    HIPCHK(ctx, copy_frames_direct(static_cast<uint8_t *>(g->dev_out[sl][k]), g->lay_out[k],
                                                   dst + (int64_t)f0 * s.nout + k, s.nout, n, false, st));
                } else {
                    HIPCHK(ctx, copy_frames(g->dev_out[sl][k], g->lay_out[k], op, n, false, st));
                }
                op += (int64_t)B * g->lay_out[k].fstride;
            }
            g->p_zout[sl] = zout;
            if (s.quality || g->ref)
                HIPCHK(ctx, hipMemcpyAsync(g->pin_qraw[sl], g->dev_qraw[sl],
                                           (size_t)n * (g->ref ? s.nout : 1) * sizeof(dts_qraw),
                                           hipMemcpyDeviceToHost, st));
            HIPCHK(ctx, hipEventRecord(g->done[sl], st));
            g->p_chunk_first[sl] = f0;
            g->p_chunk_n[sl] = n;
        }
        return DTS_OK;
    } catch (const std::bad_alloc &) {
        return DTS_E_NOMEM;
    }
}

int dts_graph_wait(dts_graph *g)
{
    if (!g) return DTS_E_INVAL;
    if (!g->pending) return DTS_OK;
    hipSetDevice(g->ctx->device);
    // finish the older slot first (chunk order does not matter for correctness)
    int e0 = finish_slot(g, 0), e1 = finish_slot(g, 1);
    g->pending = false;
    return e0 ? e0 : e1;
}

int dts_host_alloc(size_t bytes, void **out)
{
    if (!out || !bytes) return DTS_E_INVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return DTS_E_NODEV;
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess || !p) return DTS_E_NOMEM;
    try {
        PinnedSet &ps = pinned_set();
        std::lock_guard<std::mutex> lk(ps.m);
        ps.r[reinterpret_cast<uintptr_t>(p)] = {bytes, false};
    } catch (...) {
        hipHostFree(p);
        return DTS_E_NOMEM;
    }
    *out = p;
    return DTS_OK;
}

void dts_host_free(void *p)
{
    if (!p) return;
    PinnedSet &ps = pinned_set();
    {
        std::lock_guard<std::mutex> lk(ps.m);
        auto it = ps.r.find(reinterpret_cast<uintptr_t>(p));
        if (it == ps.r.end() || it->second.second) return;   // not ours (or a registered range)
        ps.r.erase(it);
    }
    hipHostFree(p);
}

int dts_host_register(void *p, size_t bytes)
{
    if (!p || !bytes) return DTS_E_INVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return DTS_E_NODEV;
    // a range overlapping one the set already holds (an allocation or another registration) is
    // refused: one record per byte keeps dts_host_free / pinned_range unambiguous
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    PinnedSet &ps = pinned_set();
    std::lock_guard<std::mutex> lk(ps.m);
    {
        auto it = ps.r.lower_bound(a);                  // first base >= a: must start at or past a + bytes
        if (it != ps.r.end() && it->first < a + bytes) return DTS_E_INVAL;
        if (it != ps.r.begin()) {                       // the base below a: must end at or before a
            --it;
            if (it->first + it->second.first > a) return DTS_E_INVAL;
        }
    }
    if (hipHostRegister(p, bytes, hipHostRegisterPortable) != hipSuccess) return DTS_E_HIP;
    try {
        ps.r[a] = {bytes, true};
    } catch (...) {
        hipHostUnregister(p);
        return DTS_E_NOMEM;
    }
    return DTS_OK;
}

int dts_host_unregister(void *p)
{
    if (!p) return DTS_E_INVAL;
    PinnedSet &ps = pinned_set();
    {
        std::lock_guard<std::mutex> lk(ps.m);
        auto it = ps.r.find(reinterpret_cast<uintptr_t>(p));
        if (it == ps.r.end() || !it->second.second) return DTS_E_INVAL;
        ps.r.erase(it);
    }
    return hipHostUnregister(p) == hipSuccess ? DTS_OK : DTS_E_HIP;
}

int dts_sws_filter(int src_n, int dst_n, int one, int align, int method, const double param[2], int pos,
                   int16_t *coeff, int32_t *filter_pos, int cap)
{
    if (src_n < 1 || dst_n < 1 || !coeff || !filter_pos || cap < 1 || !method_ok(method)) return DTS_E_INVAL;
    const double dflt[2] = {DTS_PARAM_DEFAULT, DTS_PARAM_DEFAULT};
    try {
        SwsFilter f;
        const int e = sws_build_filter(src_n, dst_n, one, align, method | kSwsAccurateRnd | kSwsBitexact,
                                       param ? param : dflt, pos, pos, f);
        if (e) return e;
        if (f.size > cap) return DTS_E_RANGE;
        for (int i = 0; i < dst_n; ++i) {
            filter_pos[i] = f.pos[i];
            for (int j = 0; j < f.size; ++j) coeff[(size_t)i * f.size + j] = f.coeff[(size_t)i * f.size + j];
        }
        return f.size;
    } catch (...) {
        return DTS_E_NOMEM;
    }
}

// ---------------------------------------------------------------------------
// synthetic source
// ---------------------------------------------------------------------------
int dts_synth_host(int w, int h, int fmt, int pattern, uint32_t seed, int64_t frame, const dts_frame *dst)
{
    if (w < 1 || h < 1 || !fmt_in_ok(fmt) || !dst || pattern < 0 || pattern > 1) return DTS_E_INVAL;
    const int cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    const bool ten = fmt == DTS_FMT_P010LE;
    for (int y = 0; y < h; ++y) {
        uint8_t *row = static_cast<uint8_t *>(dst->data[0]) + (int64_t)y * dst->pitch[0];
        for (int x = 0; x < w; ++x) {
            const int v = synth_sample(pattern, seed, x, y, frame, 0, w, h, ten);
            if (ten) {
                row[2 * x] = (uint8_t)(v << 6);
                row[2 * x + 1] = (uint8_t)((v << 6) >> 8);
            } else {
                row[x] = (uint8_t)v;
            }
        }
    }
    for (int y = 0; y < ch; ++y)
        for (int x = 0; x < cw; ++x) {
            const int u = synth_sample(pattern, seed, x, y, frame, 1, cw, ch, ten);
            const int v = synth_sample(pattern, seed, x, y, frame, 2, cw, ch, ten);
            if (fmt == DTS_FMT_YUV420P) {
                static_cast<uint8_t *>(dst->data[1])[(int64_t)y * dst->pitch[1] + x] = (uint8_t)u;
                static_cast<uint8_t *>(dst->data[2])[(int64_t)y * dst->pitch[2] + x] = (uint8_t)v;
            } else if (fmt == DTS_FMT_NV12) {
                uint8_t *row = static_cast<uint8_t *>(dst->data[1]) + (int64_t)y * dst->pitch[1];
                row[2 * x] = (uint8_t)u;
                row[2 * x + 1] = (uint8_t)v;
            } else {
                uint8_t *row = static_cast<uint8_t *>(dst->data[1]) + (int64_t)y * dst->pitch[1];
                row[4 * x] = (uint8_t)(u << 6);
                row[4 * x + 1] = (uint8_t)((u << 6) >> 8);
                row[4 * x + 2] = (uint8_t)(v << 6);
                row[4 * x + 3] = (uint8_t)((v << 6) >> 8);
            }
        }
    return DTS_OK;
}

int dts_synth_device(dts_ctx *ctx, int w, int h, int fmt, int pattern, uint32_t seed, int64_t first,
                     const dts_dev_frames *dst, int nframes, void *stream)
{
    if (!ctx || !dst || w < 1 || h < 1 || !fmt_in_ok(fmt) || nframes < 0 || pattern < 0 || pattern > 1)
        return DTS_E_INVAL;
    if (!planes_ok(*dst, w, h, fmt, 1)) return DTS_E_INVAL;
    if (!nframes) return DTS_OK;
    hipSetDevice(ctx->device);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream[0];
    HIPCHK(ctx, launch_synth(w, h, fmt, pattern, seed, first, to_dev(*dst, fmt), nframes, st));
    return DTS_OK;
}

#ifdef DTS_L5_STAMP
// diagnostic builds only (tools/build_stamp5.sh): per-phase cycle sums of k_ladder5
int dts_debug_ladder5_stamps(unsigned long long *out, int reset) { return dts::ladder5_stamps(out, reset != 0); }
#endif

#ifdef DTS_L7_STAMP
// diagnostic builds only (tools/build_stamp7.sh): per-variant, per-phase cycle sums of k_ladder7
extern "C" int dts_debug_ladder7_stamps(unsigned long long *out, int reset) { return dts::ladder7_stamps(out, reset != 0); }
#endif

// vf_fps.c (FFmpeg 4.4) frame selection, round=near, constant-rate input
// whose first pts is 0: t_i = round(i * in_den*out_num / (in_num*out_den)),
// output k repeats the last input with t_i <= k; EOF pts bounds the count.
int64_t dts_fps_map(int64_t nb_in, int in_num, int in_den, int out_num, int out_den, int64_t *out_idx, int64_t cap)
{
    if (nb_in < 0 || in_num <= 0 || in_den <= 0 || out_num <= 0 || out_den <= 0 || cap < 0) return DTS_E_INVAL;
    if (cap > 0 && !out_idx) return DTS_E_INVAL;
    const __int128 b = (__int128)in_den * out_num, c = (__int128)in_num * out_den;
    auto near = [&](int64_t a) { return (int64_t)(((__int128)a * b + c / 2) / c); };
    const int64_t nout = nb_in ? near(nb_in) : 0;
    int64_t i = 0;
    for (int64_t k = 0; k < nout && k < cap; ++k) {
        while (i + 1 < nb_in && near(i + 1) <= k) ++i;
        out_idx[k] = i;
    }
    return nout;
}

} // extern "C"
