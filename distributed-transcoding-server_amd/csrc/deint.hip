// deint.hip -- k_yadif: vf_yadif deinterlacing of
// 8-bit yuv420p frames resident in HBM, bit-exact with libavfilter/vf_yadif.c
// filter_line_c / filter_edges / filter_slice (FFmpeg 4.4; oracle/vf_yadif_ref.c).
//
// One workgroup = 1024 consecutive pixels of one row of one plane of one
// output frame; a thread computes 4 pixels.  Copied rows (the kept field) are
// dword copies.  An interpolated 4-pixel group loads dwords: rows y +- 1 of cur
// as 12-byte windows (x0-4 .. x0+7, for the x+-3 spatial search), rows y +- 1
// of prev and next and rows y, y +- 2 of the field pair prev2/next2 as one
// dword each -- 16 loads for 4 pixels instead of ~80 byte loads.  Edge groups
// and planes that are not 4-byte aligned take the per-byte path.  The rows are
// shared with the neighbouring rows' threads through L1/L2, so HBM sees each
// input frame about once per output.
#include "dts_internal.h"

namespace dts {

#ifndef DTS_YADIF_ROWS
#define DTS_YADIF_ROWS 16
#endif
constexpr int kYadifRows = DTS_YADIF_ROWS;     // output rows per workgroup tile
#ifndef DTS_YADIF_SLIDE
#define DTS_YADIF_SLIDE 1   // interior tiles: sliding row window (0: every row loads its whole neighbourhood)
#endif

namespace {

__device__ __forceinline__ int iabs(int a) { return a < 0 ? -a : a; }

// vf_yadif.c FILTER() for one pixel.  at(f, r, d) is the sample of frame f
// (0 cur, 1 prev, 2 next, 3 prev2, 4 next2) on row r (-1 = mrefs, 1 = prefs,
// 0 = this row, -2 / 2 = two rows away) at column offset d (-3 .. 3).
template <class At>
__device__ __forceinline__ int yadif_px(const At &at, int mode, bool not_edge)
{
    const int c = at(0, -1, 0), e = at(0, 1, 0);
    const int d = (at(3, 0, 0) + at(4, 0, 0)) >> 1;
    const int td0 = iabs(at(3, 0, 0) - at(4, 0, 0));
    const int td1 = (iabs(at(1, -1, 0) - c) + iabs(at(1, 1, 0) - e)) >> 1;
    const int td2 = (iabs(at(2, -1, 0) - c) + iabs(at(2, 1, 0) - e)) >> 1;
    int diff = max(max(td0 >> 1, td1), td2);
    int spatial_pred = (c + e) >> 1;
    if (not_edge) {                                        // filter_line_c / filter_edges is_not_edge
        int score = iabs(at(0, -1, -1) - at(0, 1, -1)) + iabs(c - e) + iabs(at(0, -1, 1) - at(0, 1, 1)) - 1;
#define YADIF_SCORE(jj) (iabs(at(0, -1, -1 + (jj)) - at(0, 1, -1 - (jj))) + \
                         iabs(at(0, -1, (jj)) - at(0, 1, -(jj))) +           \
                         iabs(at(0, -1, 1 + (jj)) - at(0, 1, 1 - (jj))))
        int s = YADIF_SCORE(-1);                           // CHECK(-1) CHECK(-2)
        if (s < score) {
            score = s;
            spatial_pred = (at(0, -1, -1) + at(0, 1, 1)) >> 1;
            s = YADIF_SCORE(-2);
            if (s < score) {
                score = s;
                spatial_pred = (at(0, -1, -2) + at(0, 1, 2)) >> 1;
            }
        }
        s = YADIF_SCORE(1);                                // CHECK(1) CHECK(2)
        if (s < score) {
            score = s;
            spatial_pred = (at(0, -1, 1) + at(0, 1, -1)) >> 1;
            s = YADIF_SCORE(2);
            if (s < score) spatial_pred = (at(0, -1, 2) + at(0, 1, -2)) >> 1;
        }
#undef YADIF_SCORE
    }
    if (!(mode & 2)) {
        const int b = (at(3, -2, 0) + at(4, -2, 0)) >> 1;
        const int f = (at(3, 2, 0) + at(4, 2, 0)) >> 1;
        const int mx = max(max(d - e, d - c), min(b - c, f - e));
        const int mn = min(min(d - e, d - c), max(b - c, f - e));
        diff = max(max(diff, mn), -mx);
    }
    if (spatial_pred > d + diff)
        spatial_pred = d + diff;
    else if (spatial_pred < d - diff)
        spatial_pred = d - diff;
    return spatial_pred;
}

// samples through pointers (edges, unaligned planes)
struct AtPtr {
    const uint8_t *fr[5];
    int64_t mrefs, prefs;
    __device__ __forceinline__ int operator()(int f, int r, int d) const
    {
        const int64_t o = r == -1 ? mrefs : r == 1 ? prefs : r == -2 ? 2 * mrefs : r == 2 ? 2 * prefs : 0;
        return fr[f][o + d];
    }
};

// samples of pixel x0 + i from dwords in registers: cur rows mrefs / prefs as
// 12-byte windows (x0 - 4 .. x0 + 7), the other rows as the centre dword
struct AtReg {
    uint32_t cm[3], cp[3];                 // cur row mrefs / prefs: dwords at x0 - 4, x0, x0 + 4
    uint32_t pm, pp, nm, np;               // prev / next rows mrefs / prefs
    uint32_t p2, n2, p2m, p2p, n2m, n2p;   // prev2 / next2 this row, 2 rows away
    int i;
    __device__ __forceinline__ static int byte(uint32_t v, int k) { return (int)((v >> (8 * k)) & 255u); }
    __device__ __forceinline__ int operator()(int f, int r, int d) const
    {
        if (f == 0) {
            const int k = 4 + i + d;       // 1 .. 10 for |d| <= 3
            const uint32_t *w = r < 0 ? cm : cp;
            return byte(w[k >> 2], k & 3);
        }
        if (f == 1) return byte(r < 0 ? pm : pp, i);
        if (f == 2) return byte(r < 0 ? nm : np, i);
        if (f == 3) return byte(r == 0 ? p2 : r < 0 ? p2m : p2p, i);
        return byte(r == 0 ? n2 : r < 0 ? n2m : n2p, i);
    }
};

// global (not flat) loads / stores: the pointers are built from integers, so the
// compiler cannot infer the address space itself
typedef __attribute__((address_space(1))) const uint32_t g_cu32;
typedef __attribute__((address_space(1))) uint32_t g_u32;
__device__ __forceinline__ uint32_t ld32(const uint8_t *p) { return *(g_cu32 *)(uintptr_t)p; }
__device__ __forceinline__ void st32(uint8_t *p, uint32_t v) { *(g_u32 *)(uintptr_t)p = v; }

} // namespace

// 4 consecutive pixels x0 .. x0+3 of row y of plane p of output frame o.
__device__ __forceinline__ void yadif_quad(const YadifParams &P, int p, int w, int h, int y, int x0, int o, int i,
                                           int ip, int in, int is_second)
{
    const int64_t pitch = P.seq.pitch[p];
    const uint64_t base = P.seq.data[p] + (uint64_t)y * pitch + x0;
    const uint8_t *cur = reinterpret_cast<const uint8_t *>(base + (uint64_t)i * P.seq.fstride);
    uint8_t *dst = reinterpret_cast<uint8_t *>(P.dst.data[p] + (uint64_t)o * P.dst.fstride +
                                               (uint64_t)y * P.dst.pitch[p] + x0);
    const int td_parity = P.tff ^ !is_second;
    const bool fast = P.aligned && x0 >= 4 && x0 + 8 <= w;
    if (!((y ^ td_parity) & 1)) {                          // the kept field: copy
        if (P.aligned && x0 + 4 <= w) {
            st32(dst, ld32(cur));
        } else {
            for (int k = 0; k < 4 && x0 + k < w; ++k) dst[k] = cur[k];
        }
        return;
    }
    const uint8_t *prev = reinterpret_cast<const uint8_t *>(base + (uint64_t)ip * P.seq.fstride);
    const uint8_t *next = reinterpret_cast<const uint8_t *>(base + (uint64_t)in * P.seq.fstride);
    const int mode = (y == 1 || y + 2 == h) ? 2 : P.mode;
    const int64_t prefs = y + 1 < h ? pitch : -pitch, mrefs = y ? -pitch : pitch;
    const int parity = td_parity ^ P.tff;
    const uint8_t *prev2 = parity ? prev : cur, *next2 = parity ? cur : next;
    if (fast) {
        AtReg a;
        a.cm[0] = ld32(cur + mrefs - 4);
        a.cm[1] = ld32(cur + mrefs);
        a.cm[2] = ld32(cur + mrefs + 4);
        a.cp[0] = ld32(cur + prefs - 4);
        a.cp[1] = ld32(cur + prefs);
        a.cp[2] = ld32(cur + prefs + 4);
        a.pm = ld32(prev + mrefs);
        a.pp = ld32(prev + prefs);
        a.nm = ld32(next + mrefs);
        a.np = ld32(next + prefs);
        a.p2 = ld32(prev2);
        a.n2 = ld32(next2);
        a.p2m = a.p2p = a.n2m = a.n2p = 0;
        if (!(mode & 2)) {
            a.p2m = ld32(prev2 + 2 * mrefs);
            a.p2p = ld32(prev2 + 2 * prefs);
            a.n2m = ld32(next2 + 2 * mrefs);
            a.n2p = ld32(next2 + 2 * prefs);
        }
        uint32_t out = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {                      // 4 <= x < w - 4: never an edge pixel
            a.i = k;
            out |= (uint32_t)yadif_px(a, mode, true) << (8 * k);
        }
        st32(dst, out);
        return;
    }
    for (int k = 0; k < 4 && x0 + k < w; ++k) {
        AtPtr a{{cur + k, prev + k, next + k, prev2 + k, next2 + k}, mrefs, prefs};
        const int x = x0 + k;
        dst[k] = (uint8_t)yadif_px(a, mode, x >= 3 && x < w - 3);
    }
}

// A lane's 4 columns over the rows [y0, y1) of a tile whose interpolated rows all
// lie in 2 <= y <= h - 3 (no reflected references, no forced mode 2): the rows an
// interpolated row reads slide down by two rows per step, so after the first one
// each step loads only the new rows -- cur / prev / next row y + 3 and prev2 /
// next2 row y + 4 (or y + 2) for the next step, issued before this row's
// arithmetic -- 7 dwords instead of 12 or 16, and the kept rows are stored from
// the window's cur rows (no load).
__device__ __forceinline__ void yadif_tile_slide(const YadifParams &P, int p, int y0, int y1, int x0, int o, int i,
                                                 int ip, int in, int is_second)
{
    const int64_t pitch = P.seq.pitch[p], dpitch = P.dst.pitch[p];
    const uint64_t col = P.seq.data[p] + x0;
    const uint8_t *cur = reinterpret_cast<const uint8_t *>(col + (uint64_t)i * P.seq.fstride);
    const uint8_t *prev = reinterpret_cast<const uint8_t *>(col + (uint64_t)ip * P.seq.fstride);
    const uint8_t *next = reinterpret_cast<const uint8_t *>(col + (uint64_t)in * P.seq.fstride);
    uint8_t *dst = reinterpret_cast<uint8_t *>(P.dst.data[p] + (uint64_t)o * P.dst.fstride + x0);
    const int td_parity = P.tff ^ !is_second;
    const int parity = td_parity ^ P.tff;
    const uint8_t *prev2 = parity ? prev : cur, *next2 = parity ? cur : next;
    const int mode = P.mode;
    const bool far = !(mode & 2);
    // interpolated rows y = ya, ya + 2, ...; the kept rows between them are the
    // window's cur rows (y - 1 / y + 1), stored from registers
    int y = y0 + (((y0 ^ td_parity) & 1) ? 0 : 1);
    AtReg a;
    a.p2m = a.p2p = a.n2m = a.n2p = 0;
    {
        const int64_t r = (int64_t)y * pitch;
        a.cm[0] = ld32(cur + r - pitch - 4);
        a.cm[1] = ld32(cur + r - pitch);
        a.cm[2] = ld32(cur + r - pitch + 4);
        a.cp[0] = ld32(cur + r + pitch - 4);
        a.cp[1] = ld32(cur + r + pitch);
        a.cp[2] = ld32(cur + r + pitch + 4);
        a.pm = ld32(prev + r - pitch);
        a.pp = ld32(prev + r + pitch);
        a.nm = ld32(next + r - pitch);
        a.np = ld32(next + r + pitch);
        a.p2 = ld32(prev2 + r);
        a.n2 = ld32(next2 + r);
        if (far) {
            a.p2m = ld32(prev2 + r - 2 * pitch);
            a.p2p = ld32(prev2 + r + 2 * pitch);
            a.n2m = ld32(next2 + r - 2 * pitch);
            a.n2p = ld32(next2 + r + 2 * pitch);
        }
    }
    if (y > y0) st32(dst + (int64_t)y0 * dpitch, a.cm[1]);
    for (; y < y1; y += 2) {
        // the next step's new rows are in flight while this row is computed
        const bool more = y + 2 < y1;
        uint32_t c0 = 0, c1 = 0, c2 = 0, pq = 0, nq = 0, p2q = 0, n2q = 0;
        if (more) {
            const int64_t r3 = (int64_t)(y + 3) * pitch, r4 = (int64_t)(far ? y + 4 : y + 2) * pitch;
            c0 = ld32(cur + r3 - 4);
            c1 = ld32(cur + r3);
            c2 = ld32(cur + r3 + 4);
            pq = ld32(prev + r3);
            nq = ld32(next + r3);
            p2q = ld32(prev2 + r4);
            n2q = ld32(next2 + r4);
        }
        uint32_t out = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {                      // 4 <= x < w - 4: never an edge pixel
            a.i = k;
            out |= (uint32_t)yadif_px(a, mode, true) << (8 * k);
        }
        st32(dst + (int64_t)y * dpitch, out);
        if (y + 1 < y1) st32(dst + (int64_t)(y + 1) * dpitch, a.cp[1]);
        if (more) {                                        // slide by two rows
            a.cm[0] = a.cp[0];
            a.cm[1] = a.cp[1];
            a.cm[2] = a.cp[2];
            a.cp[0] = c0;
            a.cp[1] = c1;
            a.cp[2] = c2;
            a.pm = a.pp;
            a.pp = pq;
            a.nm = a.np;
            a.np = nq;
            if (far) {
                a.p2m = a.p2;
                a.p2 = a.p2p;
                a.p2p = p2q;
                a.n2m = a.n2;
                a.n2 = a.n2p;
                a.n2p = n2q;
            } else {
                a.p2 = p2q;
                a.n2 = n2q;
            }
        }
    }
}

// One workgroup = a 1024-pixel x kYadifRows tile of one plane of one output
// frame, walked row by row: the 5-row neighbourhoods of consecutive rows
// overlap, so the tile's input rows come from HBM once and are re-read from
// L1/L2 of the same CU (a one-row workgroup spread its neighbours over all 8
// XCDs' L2s).  A thread computes 4 pixels per row.
__global__ void __launch_bounds__(256) k_yadif(const YadifParams P)
{
    const int fields = (P.mode & 1) ? 2 : 1;
    const int o = blockIdx.z;                              // output frame of this launch
    const int j = o / fields, is_second = o - j * fields;
    const int i = P.first + j;
    const int ip = i > 0 ? i - 1 : 0, in = i + 1 < P.nseq ? i + 1 : P.nseq - 1;
    const int cw = (P.w + 1) >> 1, ch = (P.h + 1) >> 1;
    const int nbl = (P.h + kYadifRows - 1) / kYadifRows, nbc = (ch + kYadifRows - 1) / kYadifRows;
    int rb = blockIdx.y, p = 0;
    if (rb >= nbl) {
        rb -= nbl;
        p = 1 + (rb >= nbc);
        if (p == 2) rb -= nbc;
    }
    const int w = p ? cw : P.w, h = p ? ch : P.h;
    const int x0 = 4 * (blockIdx.x * 256 + threadIdx.x);
    if (x0 >= w) return;
    const int y0 = rb * kYadifRows, y1 = min(h, y0 + kYadifRows);
#if DTS_YADIF_SLIDE
    if (P.aligned && x0 >= 4 && x0 + 8 <= w && y0 >= 2 && y1 <= h - 2) {
        yadif_tile_slide(P, p, y0, y1, x0, o, i, ip, in, is_second);
        return;
    }
#endif
    for (int y = y0; y < y1; ++y) yadif_quad(P, p, w, h, y, x0, o, i, ip, in, is_second);
}

// ---------------------------------------------------------------------------
// k_yadif_t: the temporal walk.  One workgroup = a kYtW x kYtH tile of one plane, walking
// kYtWalk consecutive input frames (every field output of each).  Output frame i reads
// frames i - 1, i, i + 1 (vf_yadif prev / cur / next), so the tile of frame i + 1 staged for
// output i is output i + 1's cur and output i + 2's prev: a ring of four LDS slots holds
// prev, cur, next and the frame in flight, and each step stages ONE new frame tile (its
// rows y0 - 2 .. y1 + 1 and 16 columns each side: every row and column filter_line reads,
// reflections at the plane's top / bottom included) by LDS-DMA, one step ahead of its use.
// HBM and L2 see each source frame about once per output instead of the 2.5 frames the
// per-output kernel above fetches.  A thread computes kYtNP (16) pixels of one interpolated
// row from LDS (cur rows y -+ 1 as 48-byte windows for the x -+ 3 spatial search) and copies
// 16 bytes of one kept row; the 3-byte window sums of the spatial search are v_sad_u8 of
// v_perm-aligned operands.  The spatial search runs first and the other frames' rows are read
// after it a dword at a time (round 5: 90 registers instead of 93).  Round-5 A/B:
// 8 pixels per thread in 1024-thread workgroups fits 64 registers, two workgroups per CU and
// 8 waves per SIMD, yet runs 69.0 k fps against 78.4 k here -- the window sharing of the
// spatial search is worth more than the occupancy.  Round 6: the spatial search two pixels per
// dword (yspatial_pk) and, by default, two interpolated rows of 8 pixels per thread sharing their
// common rows (DTS_YT_R2: yspatial_pk3 + ytemporal2).  Sources and outputs 16-byte
// aligned, w >= 16.
// ---------------------------------------------------------------------------
constexpr int kYtW = 512;                       // output columns per tile (32 lanes x 16)
constexpr int kYtH = 32;                        // output rows per tile (16 interpolated + 16 kept)
constexpr int kYtPitch = kYtW + 32;             // LDS row: 16 columns of halo each side
constexpr int kYtRows = kYtH + 4;               // rows y0 - 2 .. y0 + kYtH + 1
constexpr int kYtChunks = kYtPitch / 16;        // 16-byte chunks per LDS row (34)
constexpr int kYtSlot = kYtRows * kYtPitch;     // one frame tile (19,584 B)
constexpr int kYtPieces = (kYtRows * kYtChunks + 63) / 64;   // 1-KB LDS-DMA pieces per frame tile
#ifndef DTS_YT_NP
#define DTS_YT_NP 8
#endif
#ifndef DTS_YT_R2
#define DTS_YT_R2 (DTS_YT_NP == 8)
#endif
constexpr int kYtNP = DTS_YT_NP;                // pixels of an interpolated row per thread (8 or 16)
constexpr int kYtCB = kYtNP == 16 ? 16 : 8;     // cur-row bytes staged in registers left / right of them
// 1: a thread takes two interpolated rows y, y + 2 (and the kept rows beside them), which share
// the cur row y + 1, the prev / next rows y + 1 and the prev2 / next2 rows y, y + 2 (ytemporal2)
constexpr int kYtR2 = DTS_YT_R2;
constexpr int kYtThreads = (kYtW / kYtNP) * (kYtH / (2 << kYtR2));
static_assert(kYtNP == 8 || kYtNP == 16, "8 or 16 pixels per thread");
static_assert(!kYtR2 || kYtNP == 8, "two rows per thread: 8 pixels each");
#ifndef DTS_YT_WPE
#define DTS_YT_WPE (kYtNP == 8 && !DTS_YT_R2 ? 8 : 1)   // waves per SIMD the register budget is sized for
#endif
#ifndef DTS_YADIF_WALK
#define DTS_YADIF_WALK 16
#endif
constexpr int kYtWalk = DTS_YADIF_WALK;         // input frames per workgroup
#ifndef DTS_YT_SB
#define DTS_YT_SB 1                             // pixels (yspatial_pk: pixel pairs) of the spatial search between scheduling barriers
#endif
#ifndef DTS_YT_ABLATE
#define DTS_YT_ABLATE 0                         // diagnostic bits (wrong output): 1 no arithmetic
#endif

namespace {

// s_waitcnt vmcnt(min(n, 15)) for a run-time n >= 0
__device__ __forceinline__ void vm_wait_yt(int n)
{
#define DTS_WYT(k) \
    case k: __builtin_amdgcn_s_waitcnt((k) | (7 << 4) | (15 << 8)); break;
    switch (min(max(n, 0), 15)) {
        DTS_WYT(0) DTS_WYT(1) DTS_WYT(2) DTS_WYT(3) DTS_WYT(4) DTS_WYT(5) DTS_WYT(6) DTS_WYT(7)
        DTS_WYT(8) DTS_WYT(9) DTS_WYT(10) DTS_WYT(11) DTS_WYT(12) DTS_WYT(13) DTS_WYT(14)
    default: DTS_WYT(15)
    }
#undef DTS_WYT
}

__device__ __forceinline__ int byte_at(const uint32_t *a, int i) { return (int)((a[i >> 2] >> (8 * (i & 3))) & 255u); }

// bytes i, i + 1, i + 2 of a[] in the low three bytes of a dword (top byte 0)
__device__ __forceinline__ uint32_t win3(const uint32_t *a, int i)
{
    const uint32_t b = (uint32_t)(i & 3);
    const uint32_t sel = b | ((b + 1) << 8) | ((b + 2) << 16) | (0x0cu << 24);
    return __builtin_amdgcn_perm(a[(i >> 2) + 1], a[i >> 2], sel);
}


// vf_yadif.c filter_line_c / filter_edges for the 16 pixels x .. x + 15 of one interpolated
// row.  cm / cp: cur rows mrefs / prefs, bytes x - 16 .. x + 31 (pixel k at byte 16 + k);
// the rest bytes x .. x + 15: pm / pp prev rows mrefs / prefs, nm / np next, p2 / n2 prev2 /
// next2 on this row, p2m .. n2p prev2 / next2 two rows away (FAR: mode 0 / 1 away from the
// top and bottom rows).  ne: bit k set when pixel k is not an edge pixel (3 <= x + k < w - 3);
// edge pixels skip the spatial search (filter_edges).  In three parts:
// - the temporal bounds d -+ diff (everything but the spatial search) for two pixels per
//   dword, as packed 16-bit lanes (v_pk_* arithmetic: half the instructions of a pixel at a
//   time; no value leaves [-510, 510]);
// - the spatial search per pixel, without a branch, so the 3-byte windows are shared between
//   neighbouring pixels (window i of cm serves pixels i - 1 .. i + 3: 20 windows per row for
//   16 pixels instead of 80) and the candidate predictions stay sums until one halving; a
//   scheduling barrier per pixel keeps the live windows to the sliding ten.  Edge pixels'
//   windows read the staged halo (clamped columns) and are replaced afterwards;
// - the clamp, packed again.
typedef short i16x2y __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2y __attribute__((ext_vector_type(2)));
__device__ __forceinline__ i16x2y pair16(uint32_t d, int h)   // bytes 2h, 2h + 1 of d, zero-extended
{
    return __builtin_bit_cast(i16x2y, __builtin_amdgcn_perm(0u, d, h ? 0x0c030c02u : 0x0c010c00u));
}
__device__ __forceinline__ i16x2y absd16(i16x2y a, i16x2y b)
{
    return __builtin_elementwise_max(a, b) - __builtin_elementwise_min(a, b);
}
// byte b of lo and byte b of hi in bytes 0, 1 (bytes 2, 3 zero)
__device__ __forceinline__ uint32_t two8(uint32_t hi, uint32_t lo, int b)
{
    return __builtin_amdgcn_perm(hi, lo, (uint32_t)b | ((uint32_t)(4 + b) << 8) | 0x0c0c0000u);
}
// |x0 - y0| + |x1 - y1| for the pixels 2h, 2h + 1 of four rows' dwords, as a 16-bit pair:
// v_sad_u8 of (x0, x1) against (y0, y1) per pixel, the second pixel's by v_sad_hi_u8 into the
// high half (td1 / td2 of filter_line_c before their halving)
__device__ __forceinline__ i16x2y sad2x(uint32_t x0, uint32_t x1, uint32_t y0, uint32_t y1, int h)
{
    const uint32_t lo = __builtin_amdgcn_sad_u8(two8(x1, x0, 2 * h), two8(y1, y0, 2 * h), 0u);
    return __builtin_bit_cast(i16x2y, __builtin_amdgcn_sad_hi_u8(two8(x1, x0, 2 * h + 1), two8(y1, y0, 2 * h + 1), lo));
}

// the spatial search of NP pixels: pr[] = 2 x 16-bit predictions per dword
template <int NP>
__device__ __forceinline__ void yspatial(const uint32_t (&cm)[(2 * kYtCB + NP) / 4], const uint32_t (&cp)[(2 * kYtCB + NP) / 4],
                                         uint32_t ne, uint32_t (&pr)[NP / 2])
{
    constexpr int CB = kYtCB;                          // pixel k of cm / cp at byte CB + k
    // the 3-byte windows of cm / cp starting at byte CB - 3 + i (i = 0 .. NP + 3), made as the
    // walk reaches them and passed through an empty asm: what depends on a window cannot be
    // scheduled before it, so the sliding ten are all that is live
    uint32_t wm[NP + 4], wp[NP + 4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        wm[i] = win3(cm, CB - 3 + i);
        wp[i] = win3(cp, CB - 3 + i);
        asm volatile("" : "+v"(wm[i]), "+v"(wp[i]));
    }
    auto b8 = [](uint32_t w, int i) { return (int)((w >> (8 * i)) & 255u); };
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        // pixel X = CB + k: windows starting at X - 3 .. X + 1 = indices k .. k + 4
        wm[k + 4] = win3(cm, CB + 1 + k);
        wp[k + 4] = win3(cp, CB + 1 + k);
        asm volatile("" : "+v"(wm[k + 4]), "+v"(wp[k + 4]));
        const uint32_t m3 = wm[k], m2 = wm[k + 1], m1 = wm[k + 2], m0 = wm[k + 3], m_1 = wm[k + 4];
        const uint32_t p3 = wp[k], p2_ = wp[k + 1], p1 = wp[k + 2], p0 = wp[k + 3], p_1 = wp[k + 4];
        // CHECK(j): cm window at X + j - 1 against cp window at X - j - 1
        int score = (int)__builtin_amdgcn_sad_u8(m1, p1, 0u) - 1;
        const int sm1 = (int)__builtin_amdgcn_sad_u8(m2, p0, 0u);
        const int sm2 = (int)__builtin_amdgcn_sad_u8(m3, p_1, 0u);
        const int s1 = (int)__builtin_amdgcn_sad_u8(m0, p2_, 0u);
        const int s2 = (int)__builtin_amdgcn_sad_u8(m_1, p3, 0u);
        // 2 x the candidate predictions, bytes of the same windows: window X - 1 holds X - 1 .. X + 1
        int ps = b8(m1, 1) + b8(p1, 1);                   // cm[X] + cp[X]
        const bool b1 = sm1 < score;
        score = b1 ? sm1 : score;
        ps = b1 ? b8(m1, 0) + b8(p0, 1) : ps;             // cm[X - 1] + cp[X + 1]
        const bool bb2 = b1 & (sm2 < score);
        score = bb2 ? sm2 : score;
        ps = bb2 ? b8(m2, 0) + b8(p0, 2) : ps;            // cm[X - 2] + cp[X + 2]
        const bool b3 = s1 < score;
        score = b3 ? s1 : score;
        ps = b3 ? b8(m0, 1) + b8(p1, 0) : ps;             // cm[X + 1] + cp[X - 1]
        const bool b4 = b3 & (s2 < score);
        ps = b4 ? b8(m0, 2) + b8(p2_, 0) : ps;            // cm[X + 2] + cp[X - 2]
        const uint32_t pv = (uint32_t)ps >> 1;
        pr[k >> 1] = (k & 1) ? pr[k >> 1] | (pv << 16) : pv;
        if ((k + 1) % DTS_YT_SB == 0) __builtin_amdgcn_sched_barrier(0);
    }
    if (ne != (1u << NP) - 1) {                           // filter_edges: no spatial search
#pragma unroll
        for (int k = 0; k < NP; ++k)
            if (!((ne >> k) & 1u)) {
                const uint32_t pv = (uint32_t)(byte_at(cm, CB + k) + byte_at(cp, CB + k)) >> 1;
                pr[k >> 1] = (k & 1) ? (pr[k >> 1] & 0xffffu) | (pv << 16) : (pr[k >> 1] & 0xffff0000u) | pv;
            }
    }
}

#ifndef DTS_YT_PK
#define DTS_YT_PK 1     // the spatial search two pixels per dword (yspatial_pk); 0: per pixel (yspatial)
#endif

// The spatial search of NP pixels as 16-bit pairs (round 6): pixels 2p and 2p + 1 share every
// instruction after the sums of absolute differences.  v_sad_u8 makes pixel 2p's score and
// v_sad_hi_u8 adds pixel 2p + 1's in the high half, so the five scores of a pair arrive packed;
// the candidate predictions cm[X + j] + cp[X - j] are sums of byte pairs unpacked by v_perm
// (bytes i, i + 1 of a row as two 16-bit lanes: one unpacking serves the five j of neighbouring
// pairs); each CHECK(j) of filter_line_c is a packed subtract whose sign (>> 15) is the lane mask
// of `score < spatial_score`, nested checks AND their masks, and the updates are bit selects.
// Scores stay in [0, 766] (held as score + 1), their differences in 16 bits.  The result is the
// same bytes as yspatial's, which it replaces.
template <int NP>
__device__ __forceinline__ void yspatial_pk(const uint32_t (&cm)[(2 * kYtCB + NP) / 4], const uint32_t (&cp)[(2 * kYtCB + NP) / 4],
                                            uint32_t ne, uint32_t (&pr)[NP / 2])
{
    constexpr int CB = kYtCB;                          // pixel k of cm / cp at byte CB + k
    uint32_t wm[NP + 4], wp[NP + 4];                   // 3-byte windows starting at byte CB - 3 + i
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        wm[i] = win3(cm, CB - 3 + i);
        wp[i] = win3(cp, CB - 3 + i);
        asm volatile("" : "+v"(wm[i]), "+v"(wp[i]));
    }
    // bytes i, i + 1 of a row, zero-extended into two 16-bit lanes
    auto u2 = [](const uint32_t *a, int i) {
        const uint32_t b = (uint32_t)(i & 3);
        // (b <= 2: the bytes lie in one dword and the other operand is 0, as pair16 has it, so the
        // temporal part's unpacking of the same cur-row pairs is the same instruction)
        return __builtin_bit_cast(i16x2y, __builtin_amdgcn_perm(b <= 2 ? 0u : a[(i >> 2) + 1], a[i >> 2],
                                                                b | (0x0cu << 8) | ((b + 1) << 16) | (0x0cu << 24)));
    };
    // the lane masks pass through an empty asm: seen as sign splats, the compiler turns the bit
    // selects back into a compare and a select per 16-bit lane
    auto lt = [](i16x2y a, i16x2y b) {                // a < b per lane: 0xffff / 0
        uint32_t m = __builtin_bit_cast(uint32_t, (i16x2y)((a - b) >> 15));
        asm volatile("" : "+v"(m));
        return m;
    };
    auto sel = [](uint32_t m, i16x2y a, i16x2y b) {  // v_bfi_b32
        return __builtin_bit_cast(i16x2y, (__builtin_bit_cast(uint32_t, a) & m) | (__builtin_bit_cast(uint32_t, b) & ~m));
    };
#pragma unroll
    for (int q = 0; q < NP / 2; ++q) {
        const int k = 2 * q, X = CB + k;
#pragma unroll
        for (int i = 0; i < 2; ++i) {                  // the windows pixels k, k + 1 reach first
            wm[k + 4 + i] = win3(cm, X + 1 + i);
            wp[k + 4 + i] = win3(cp, X + 1 + i);
            asm volatile("" : "+v"(wm[k + 4 + i]), "+v"(wp[k + 4 + i]));
        }
        // pixel k + h: windows k + h .. k + h + 4 are X + h - 3 .. X + h + 1; CHECK(j) compares the cm
        // window at X + j - 1 with the cp window at X - j - 1
        // (pixel k, pixel k + 1) scores of one check, + acc per half: scores are held as score + 1,
        // so spatial_score's initial - 1 disappears and each candidate's + 1 rides in the
        // accumulator operand (0x00010001: no carry between the halves)
        auto sc = [&](int jm, int jp, uint32_t acc) {
            const uint32_t lo = __builtin_amdgcn_sad_u8(wm[k + jm], wp[k + jp], acc);
            return __builtin_bit_cast(i16x2y, __builtin_amdgcn_sad_hi_u8(wm[k + 1 + jm], wp[k + 1 + jp], lo));
        };
        i16x2y score = sc(2, 2, 0u);
        const i16x2y sm1 = sc(1, 3, 0x00010001u), sm2 = sc(0, 4, 0x00010001u), s1 = sc(3, 1, 0x00010001u),
                     s2 = sc(4, 0, 0x00010001u);
        // CHECK(-1) { CHECK(-2) }: when sm1 < score, the pair's outcome is the better of -1 and -2
        // (-2 only if strictly better), decided apart from score; the same for CHECK(1) { CHECK(2) }
        const i16x2y psl = sel(lt(sm2, sm1), u2(cm, X - 2) + u2(cp, X + 2), u2(cm, X - 1) + u2(cp, X + 1));
        const i16x2y psr = sel(lt(s2, s1), u2(cm, X + 2) + u2(cp, X - 2), u2(cm, X + 1) + u2(cp, X - 1));
        i16x2y ps = u2(cm, X) + u2(cp, X);
        const uint32_t ml = lt(sm1, score);
        score = sel(ml, __builtin_elementwise_min(sm1, sm2), score);
        ps = sel(ml, psl, ps);
        ps = sel(lt(s1, score), psr, ps);
        pr[q] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2y, ps) >> 1);   // v_pk_lshrrev_b16
        if ((q + 1) % DTS_YT_SB == 0) __builtin_amdgcn_sched_barrier(0);
    }
    if (ne != (1u << NP) - 1) {                           // filter_edges: no spatial search
#pragma unroll
        for (int k = 0; k < NP; ++k)
            if (!((ne >> k) & 1u)) {
                const uint32_t pv = (uint32_t)(byte_at(cm, CB + k) + byte_at(cp, CB + k)) >> 1;
                pr[k >> 1] = (k & 1) ? (pr[k >> 1] & 0xffffu) | (pv << 16) : (pr[k >> 1] & 0xffff0000u) | pv;
            }
    }
}

// yspatial_pk for two interpolated rows y, y + 2 (cur rows c0 = y - 1, c1 = y + 1, c2 = y + 3):
// row y + 1's windows and byte pairs serve both (its cp and the other's cm)
template <int NP>
__device__ __forceinline__ void yspatial_pk3(const uint32_t (&c0)[(2 * kYtCB + NP) / 4], const uint32_t (&c1)[(2 * kYtCB + NP) / 4],
                                             const uint32_t (&c2)[(2 * kYtCB + NP) / 4], uint32_t ne, uint32_t (&pa)[NP / 2],
                                             uint32_t (&pb)[NP / 2])
{
    constexpr int CB = kYtCB;
    uint32_t w0[NP + 4], w1[NP + 4], w2[NP + 4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        w0[i] = win3(c0, CB - 3 + i);
        w1[i] = win3(c1, CB - 3 + i);
        w2[i] = win3(c2, CB - 3 + i);
        asm volatile("" : "+v"(w0[i]), "+v"(w1[i]), "+v"(w2[i]));
    }
    auto u2 = [](const uint32_t *a, int i) {
        const uint32_t b = (uint32_t)(i & 3);
        // (b <= 2: the bytes lie in one dword and the other operand is 0, as pair16 has it, so the
        // temporal part's unpacking of the same cur-row pairs is the same instruction)
        return __builtin_bit_cast(i16x2y, __builtin_amdgcn_perm(b <= 2 ? 0u : a[(i >> 2) + 1], a[i >> 2],
                                                                b | (0x0cu << 8) | ((b + 1) << 16) | (0x0cu << 24)));
    };
    auto lt = [](i16x2y a, i16x2y b) {
        uint32_t m = __builtin_bit_cast(uint32_t, (i16x2y)((a - b) >> 15));
        asm volatile("" : "+v"(m));
        return m;
    };
    auto sel = [](uint32_t m, i16x2y a, i16x2y b) {
        return __builtin_bit_cast(i16x2y, (__builtin_bit_cast(uint32_t, a) & m) | (__builtin_bit_cast(uint32_t, b) & ~m));
    };
#pragma unroll
    for (int q = 0; q < NP / 2; ++q) {
        const int k = 2 * q, X = CB + k;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            w0[k + 4 + i] = win3(c0, X + 1 + i);
            w1[k + 4 + i] = win3(c1, X + 1 + i);
            w2[k + 4 + i] = win3(c2, X + 1 + i);
            asm volatile("" : "+v"(w0[k + 4 + i]), "+v"(w1[k + 4 + i]), "+v"(w2[k + 4 + i]));
        }
        // one row's pair of pixels: cm windows / bytes wm, cm; cp windows / bytes wp, cp
        auto one = [&](const uint32_t *wm, const uint32_t *wp, const uint32_t *cm, const uint32_t *cp) {
            // scores held as score + 1: spatial_score's initial - 1 disappears and the candidates'
            // + 1 rides in the sums' accumulator operand (0x00010001: no carry between the halves)
            auto sc = [&](int jm, int jp, uint32_t acc) {
                const uint32_t lo = __builtin_amdgcn_sad_u8(wm[k + jm], wp[k + jp], acc);
                return __builtin_bit_cast(i16x2y, __builtin_amdgcn_sad_hi_u8(wm[k + 1 + jm], wp[k + 1 + jp], lo));
            };
            i16x2y score = sc(2, 2, 0u);
            const i16x2y sm1 = sc(1, 3, 0x00010001u), sm2 = sc(0, 4, 0x00010001u), s1 = sc(3, 1, 0x00010001u),
                         s2 = sc(4, 0, 0x00010001u);
            // CHECK(-1) { CHECK(-2) } and CHECK(1) { CHECK(2) } as in yspatial_pk
            const i16x2y psl = sel(lt(sm2, sm1), u2(cm, X - 2) + u2(cp, X + 2), u2(cm, X - 1) + u2(cp, X + 1));
            const i16x2y psr = sel(lt(s2, s1), u2(cm, X + 2) + u2(cp, X - 2), u2(cm, X + 1) + u2(cp, X - 1));
            i16x2y ps = u2(cm, X) + u2(cp, X);
            const uint32_t ml = lt(sm1, score);
            score = sel(ml, __builtin_elementwise_min(sm1, sm2), score);
            ps = sel(ml, psl, ps);
            ps = sel(lt(s1, score), psr, ps);
            return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2y, ps) >> 1);   // v_pk_lshrrev_b16
        };
        pa[q] = one(w0, w1, c0, c1);
        pb[q] = one(w1, w2, c1, c2);
        if ((q + 1) % DTS_YT_SB == 0) __builtin_amdgcn_sched_barrier(0);
    }
    if (ne != (1u << NP) - 1) {                           // filter_edges: no spatial search
#pragma unroll
        for (int k = 0; k < NP; ++k)
            if (!((ne >> k) & 1u)) {
                const uint32_t va = (uint32_t)(byte_at(c0, CB + k) + byte_at(c1, CB + k)) >> 1;
                const uint32_t vb = (uint32_t)(byte_at(c1, CB + k) + byte_at(c2, CB + k)) >> 1;
                pa[k >> 1] = (k & 1) ? (pa[k >> 1] & 0xffffu) | (va << 16) : (pa[k >> 1] & 0xffff0000u) | va;
                pb[k >> 1] = (k & 1) ? (pb[k >> 1] & 0xffffu) | (vb << 16) : (pb[k >> 1] & 0xffff0000u) | vb;
            }
    }
}

// the temporal bounds d -+ diff of NP pixels (two per dword as packed 16-bit lanes: v_pk_*
// arithmetic, no value leaves [-510, 510]) and the reference's two-sided clamp of the
// spatial predictions pr[] (diff >= 0: a median), packed back to bytes.  ld(r, q) reads dword
// q of row r: 0 / 1 prev mrefs / prefs, 2 / 3 next, 4 / 5 prev2 / next2 on this row, 6 .. 9
// prev2 / next2 two rows away (FAR) -- loaded per dword, so one dword of each is live at a time
template <int NP, bool FAR, class LD>
__device__ __forceinline__ void ytemporal(const uint32_t (&cm)[(2 * kYtCB + NP) / 4], const uint32_t (&cp)[(2 * kYtCB + NP) / 4],
                                          LD ld, const uint32_t (&pr)[NP / 2], uint32_t (&out)[NP / 4])
{
    constexpr int CQ = kYtCB / 4;
#pragma unroll
    for (int q = 0; q < NP / 4; ++q) {
        const uint32_t pm = ld(0, q), pp = ld(1, q), nm = ld(2, q), np = ld(3, q), p2 = ld(4, q), n2 = ld(5, q);
        const uint32_t p2m = FAR ? ld(6, q) : 0u, p2p = FAR ? ld(7, q) : 0u, n2m = FAR ? ld(8, q) : 0u,
                       n2p = FAR ? ld(9, q) : 0u;
        i16x2y r[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const i16x2y c = pair16(cm[CQ + q], h), e = pair16(cp[CQ + q], h);
            const i16x2y a2 = pair16(p2, h), b2 = pair16(n2, h);
            const i16x2y d = (a2 + b2) >> 1;
            // max(td0 >> 1, td1, td2) with td1, td2 the halved sums: all non-negative, so the three
            // halvings are one, after the max
            const i16x2y td0 = absd16(a2, b2);
            const i16x2y s1 = sad2x(pm, pp, cm[CQ + q], cp[CQ + q], h), s2 = sad2x(nm, np, cm[CQ + q], cp[CQ + q], h);
            i16x2y diff = __builtin_elementwise_max(__builtin_elementwise_max(td0, s1), s2) >> 1;
            if (FAR) {
                const i16x2y b = (pair16(p2m, h) + pair16(n2m, h)) >> 1;
                const i16x2y f = (pair16(p2p, h) + pair16(n2p, h)) >> 1;
                const i16x2y de = d - e, dc = d - c, bc = b - c, fe = f - e;
                const i16x2y mx = __builtin_elementwise_max(__builtin_elementwise_max(de, dc), __builtin_elementwise_min(bc, fe));
                const i16x2y mn = __builtin_elementwise_min(__builtin_elementwise_min(de, dc), __builtin_elementwise_max(bc, fe));
                diff = __builtin_elementwise_max(__builtin_elementwise_max(diff, mn), -mx);
            }
            r[h] = __builtin_elementwise_min(__builtin_elementwise_max(__builtin_bit_cast(i16x2y, pr[2 * q + h]), d - diff), d + diff);
        }
        out[q] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, r[1]), __builtin_bit_cast(uint32_t, r[0]), 0x06040200u);
    }
}

// ytemporal for two interpolated rows a = y and b = y + 2 (both interior: rows y - 2 .. y + 4 in
// the tile, the same FAR), sharing what row y + 1 and the frames' rows y, y + 2 give both: b's c
// is a's e, b's prev / next mrefs rows are a's prefs rows (so |pp - e| and |np - e| are computed
// once), b's d is a's f and a's d is b's b.  ld(r, q): 0 .. 9 as ytemporal's rows for a, then
// 10 / 11 prev / next row y + 3, 12 / 13 prev2 / next2 row y + 4
template <int NP, bool FAR, class LD>
__device__ __forceinline__ void ytemporal2(const uint32_t (&c0)[(2 * kYtCB + NP) / 4], const uint32_t (&c1)[(2 * kYtCB + NP) / 4],
                                           const uint32_t (&c2)[(2 * kYtCB + NP) / 4], LD ld, const uint32_t (&pra)[NP / 2],
                                           const uint32_t (&prb)[NP / 2], uint32_t (&oa)[NP / 4], uint32_t (&ob)[NP / 4])
{
    constexpr int CQ = kYtCB / 4;
#pragma unroll
    for (int q = 0; q < NP / 4; ++q) {
        const uint32_t pm = ld(0, q), pp = ld(1, q), nm = ld(2, q), np = ld(3, q), p2 = ld(4, q), n2 = ld(5, q);
        const uint32_t p2b = ld(7, q), n2b = ld(9, q), ppb = ld(10, q), npb = ld(11, q);
        const uint32_t p2m = FAR ? ld(6, q) : 0u, n2m = FAR ? ld(8, q) : 0u, p2pb = FAR ? ld(12, q) : 0u,
                       n2pb = FAR ? ld(13, q) : 0u;
        i16x2y ra[2], rb[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const i16x2y ca = pair16(c0[CQ + q], h), e = pair16(c1[CQ + q], h), eb = pair16(c2[CQ + q], h);
            const i16x2y A = pair16(p2, h), B = pair16(n2, h), Ab = pair16(p2b, h), Bb = pair16(n2b, h);
            const i16x2y da = (A + B) >> 1, db = (Ab + Bb) >> 1;
            // td1 / td2 of both rows as sums of absolute byte differences (the (c, e) byte pairs
            // of a row shared by its two sums)
            // (the halvings of td0, td1, td2 as one after their max: all non-negative)
            const i16x2y t1a = sad2x(pm, pp, c0[CQ + q], c1[CQ + q], h), t1b = sad2x(pp, ppb, c1[CQ + q], c2[CQ + q], h);
            const i16x2y t2a = sad2x(nm, np, c0[CQ + q], c1[CQ + q], h), t2b = sad2x(np, npb, c1[CQ + q], c2[CQ + q], h);
            i16x2y da_ = __builtin_elementwise_max(__builtin_elementwise_max(absd16(A, B), t1a), t2a) >> 1;
            i16x2y db_ = __builtin_elementwise_max(__builtin_elementwise_max(absd16(Ab, Bb), t1b), t2b) >> 1;
            if (FAR) {
                const i16x2y ba = (pair16(p2m, h) + pair16(n2m, h)) >> 1, fb = (pair16(p2pb, h) + pair16(n2pb, h)) >> 1;
                {   // row a: b = ba, f = db, c = ca, e = e
                    const i16x2y de = da - e, dc = da - ca, bc = ba - ca, fe = db - e;
                    const i16x2y mx = __builtin_elementwise_max(__builtin_elementwise_max(de, dc), __builtin_elementwise_min(bc, fe));
                    const i16x2y mn = __builtin_elementwise_min(__builtin_elementwise_min(de, dc), __builtin_elementwise_max(bc, fe));
                    da_ = __builtin_elementwise_max(__builtin_elementwise_max(da_, mn), -mx);
                }
                {   // row b: b = da, f = fb, c = e, e = eb
                    const i16x2y de = db - eb, dc = db - e, bc = da - e, fe = fb - eb;
                    const i16x2y mx = __builtin_elementwise_max(__builtin_elementwise_max(de, dc), __builtin_elementwise_min(bc, fe));
                    const i16x2y mn = __builtin_elementwise_min(__builtin_elementwise_min(de, dc), __builtin_elementwise_max(bc, fe));
                    db_ = __builtin_elementwise_max(__builtin_elementwise_max(db_, mn), -mx);
                }
            }
            ra[h] = __builtin_elementwise_min(__builtin_elementwise_max(__builtin_bit_cast(i16x2y, pra[2 * q + h]), da - da_), da + da_);
            rb[h] = __builtin_elementwise_min(__builtin_elementwise_max(__builtin_bit_cast(i16x2y, prb[2 * q + h]), db - db_), db + db_);
        }
        oa[q] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, ra[1]), __builtin_bit_cast(uint32_t, ra[0]), 0x06040200u);
        ob[q] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, rb[1]), __builtin_bit_cast(uint32_t, rb[0]), 0x06040200u);
    }
}

typedef unsigned int u32x4y __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4y g_u32x4y;
typedef __attribute__((address_space(1))) uint8_t g_u8y;
typedef unsigned int u32x2y __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) u32x2y g_u32x2y;
// NP bytes of an LDS row into NP / 4 dwords (one ds_read_b128 or b64)
template <int NP> __device__ __forceinline__ void ldsn(const uint8_t *p, uint32_t *o)
{
    if (NP == 16) {
        const u32x4y v = *reinterpret_cast<const u32x4y *>(p);
        o[0] = v.x, o[1] = v.y, o[2] = v.z, o[3] = v.w;
    } else {
        const u32x2y v = *reinterpret_cast<const u32x2y *>(p);
        o[0] = v.x, o[1] = v.y;
    }
}
// NP bytes to a plane row (room: bytes left in the row)
template <int NP> __device__ __forceinline__ void putn(uint64_t dst, const uint32_t *w, int room)
{
    if (room >= NP) {
        if (NP == 16)
            *(g_u32x4y *)(uintptr_t)dst = (u32x4y){w[0], w[1], w[2], w[3]};
        else
            *(g_u32x2y *)(uintptr_t)dst = (u32x2y){w[0], w[1]};
    } else {
        for (int i = 0; i < room; ++i) ((g_u8y *)(uintptr_t)dst)[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
}

} // namespace

__global__ void __launch_bounds__(kYtThreads, DTS_YT_WPE) k_yadif_t(const YadifParams P, int tiles_l, int tiles_c, int txl, int txc,
                                                        int count)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t yl[];
    // tile of this workgroup: the tiles of one XCD (b mod 8) are consecutive in raster order,
    // so neighbouring tiles' halo rows / columns meet in the same L2
    const int ntiles = tiles_l + 2 * tiles_c, per = (ntiles + 7) >> 3;
    const int b = (int)blockIdx.x, tix = (b & 7) * per + (b >> 3);
    if (tix >= ntiles) return;
    int p = 0, tl = tix, tx_n = txl;
    if (tl >= tiles_l) {
        tl -= tiles_l;
        p = 1 + (tl >= tiles_c);
        if (p == 2) tl -= tiles_c;
        tx_n = txc;
    }
    const int w = p ? (P.w + 1) >> 1 : P.w, h = p ? (P.h + 1) >> 1 : P.h;
    const int x0 = (tl % tx_n) * kYtW, y0 = (tl / tx_n) * kYtH;
    const int fields = (P.mode & 1) ? 2 : 1;
    const int j0 = (int)blockIdx.y * kYtWalk, j1 = min(count, j0 + kYtWalk);   // outputs' input frames, relative
    const int t = (int)threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t pitch = P.seq.pitch[p];
    const uint64_t sbase = P.seq.data[p];
    const int wr16 = (w + 15) & ~15;
    // one frame tile (sequence frame clamped to [0, nseq)) into LDS slot s: this wave's pieces
    auto stage = [&](int pos, int s) {
        const int f = min(max(P.first + pos, 0), P.nseq - 1);
        const uint64_t fb = sbase + (uint64_t)f * (uint64_t)P.seq.fstride;
        for (int k = wave; k < kYtPieces; k += kYtThreads / 64) {
            const int q = k * 64 + lane;
            if (q < kYtRows * kYtChunks) {
                const int r = q / kYtChunks, ch = q - r * kYtChunks;
                const int yy = min(max(y0 - 2 + r, 0), h - 1);
                const int xx = min(max(x0 - 16 + 16 * ch, 0), wr16 - 16);
                __builtin_amdgcn_global_load_lds((const void *)(uintptr_t)(fb + (uint64_t)((int64_t)yy * pitch) + (uint64_t)xx),
                                                 (__attribute__((address_space(3))) void *)(yl + s * kYtSlot + 1024 * k),
                                                 16, 0, 0);
            }
        }
    };
    // every output row of this tile is whole and every 16-byte segment inside the plane: the
    // stores are exactly two wave-instructions per step (else their count is not tracked)
    const bool whole = x0 + kYtW <= w && y0 + kYtH <= h;
    stage(j0 - 1, 0);
    stage(j0, 1);
    stage(j0 + 1, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int nst = 0;                               // this wave's stores of the previous step (when counted)
    constexpr int NP = kYtNP, NQ = NP / 4, CW = (2 * kYtCB + NP) / 4;
    // NP columns of one interpolated and one kept row (8 pixels: one row pair per wave, its row
    // arithmetic scalar)
    const int ci = t % (kYtW / NP), ri = kYtW / NP == 64 ? __builtin_amdgcn_readfirstlane(t / 64) : t / (kYtW / NP);
    constexpr int RR = 1 << kYtR2;             // interpolated rows per thread
    const int x = x0 + NP * ci;
    const uint64_t obase0 = P.dst.data[p] + (uint64_t)x;
    for (int j = j0; j < j1; ++j) {
        const int s = j - j0;
        // frame j + 1's pieces (issued a step ago, before that step's stores) have landed in
        // every wave; past the barrier every wave is also done with step j - 1, so frame
        // j - 2's slot takes frame j + 2 -- one barrier per step
        vm_wait_yt(nst);
        __syncthreads();
        if (j + 2 <= j1) stage(j + 2, (s + 3) & 3);
        const uint8_t *sl_p = yl + ((s + 0) & 3) * kYtSlot, *sl_c = yl + ((s + 1) & 3) * kYtSlot,
                      *sl_n = yl + ((s + 2) & 3) * kYtSlot;
        nst = 0;
        for (int is2 = 0; is2 < fields; ++is2) {
            const int td_parity = P.tff ^ !is2, parity = td_parity ^ P.tff;
            const int o = j * fields + is2;
            const uint64_t obase = obase0 + (uint64_t)o * (uint64_t)P.dst.fstride;
            const int64_t dp = P.dst.pitch[p];
            const int off = ((y0 ^ td_parity) & 1) ? 0 : 1;     // y0 + off: the tile's first interpolated row
            // kept rows: copies of cur
#pragma unroll
            for (int rr = 0; rr < RR; ++rr) {
                const int y = y0 + 2 * RR * ri + 2 * rr + (1 - off);
                if (y < h && x < w) {
                    uint32_t v[NQ];
                    ldsn<NP>(sl_c + (y - y0 + 2) * kYtPitch + NP * ci + 16, v);
                    putn<NP>(obase + (uint64_t)((int64_t)y * dp), v, w - x);
                }
            }
            const int ya = y0 + 2 * RR * ri + off;
            auto rowp = [&](const uint8_t *sl, int yy) { return sl + (yy - y0 + 2) * kYtPitch + NP * ci + 16; };
            // two interior rows (rows ya - 2 .. ya + 4 in the plane: no clamped mrefs / prefs, and
            // both FAR unless the mode skips the spatial interlacing check)
            const bool pair2 = kYtR2 && ya >= 2 && ya + 4 < h;
            if (kYtR2 && pair2) {
                if (x < w) {
                    const bool far = !(P.mode & 2);
                    const uint8_t *prv = sl_p, *cur = sl_c, *nxt = sl_n;
                    const uint8_t *pv2 = parity ? prv : cur, *nx2 = parity ? cur : nxt;
                    uint32_t c0[CW], c1[CW], c2[CW];
#pragma unroll
                    for (int h3 = 0; h3 < 3; ++h3) {
                        ldsn<NP>(rowp(cur, ya - 1) - kYtCB + NP * h3, c0 + NQ * h3);
                        ldsn<NP>(rowp(cur, ya + 1) - kYtCB + NP * h3, c1 + NQ * h3);
                        ldsn<NP>(rowp(cur, ya + 3) - kYtCB + NP * h3, c2 + NQ * h3);
                    }
                    uint32_t ne = 0;
#pragma unroll
                    for (int k = 0; k < NP; ++k) ne |= (x + k >= 3 && x + k < w - 3) ? 1u << k : 0u;
                    uint32_t pa[NP / 2], pb[NP / 2], ra[NQ], rb[NQ];
                    yspatial_pk3<NP>(c0, c1, c2, ne, pa, pb);
                    __builtin_amdgcn_sched_barrier(0);
                    const uint8_t *rows[14] = {rowp(prv, ya - 1), rowp(prv, ya + 1), rowp(nxt, ya - 1), rowp(nxt, ya + 1),
                                               rowp(pv2, ya), rowp(nx2, ya), rowp(pv2, ya - 2), rowp(pv2, ya + 2),
                                               rowp(nx2, ya - 2), rowp(nx2, ya + 2), rowp(prv, ya + 3), rowp(nxt, ya + 3),
                                               rowp(pv2, ya + 4), rowp(nx2, ya + 4)};
                    auto ld = [&](int r, int q) { return *reinterpret_cast<const uint32_t *>(rows[r] + 4 * q); };
                    if (far)
                        ytemporal2<NP, true>(c0, c1, c2, ld, pa, pb, ra, rb);
                    else
                        ytemporal2<NP, false>(c0, c1, c2, ld, pa, pb, ra, rb);
                    putn<NP>(obase + (uint64_t)((int64_t)ya * dp), ra, w - x);
                    putn<NP>(obase + (uint64_t)((int64_t)(ya + 2) * dp), rb, w - x);
                }
                nst += 2 * RR;
                continue;
            }
#pragma unroll 1
            for (int rr = 0; rr < RR; ++rr) {
            const int y = ya + 2 * rr;
            if (y < h && x < w) {
                const int rm = y ? y - 1 : y + 1, rp = y + 1 < h ? y + 1 : y - 1;
                const bool far = !((P.mode & 2) || y == 1 || y + 2 == h);
                const uint8_t *prv = sl_p, *cur = sl_c, *nxt = sl_n;
                const uint8_t *pv2 = parity ? prv : cur, *nx2 = parity ? cur : nxt;
                auto row = [&](const uint8_t *sl, int yy) { return sl + (yy - y0 + 2) * kYtPitch + NP * ci + 16; };
                uint32_t cm[CW], cp[CW];
#pragma unroll
                for (int h3 = 0; h3 < 3; ++h3) {       // cur rows: bytes x - CB .. x + NP + CB - 1
                    ldsn<NP>(row(cur, rm) - kYtCB + NP * h3, cm + NQ * h3);
                    ldsn<NP>(row(cur, rp) - kYtCB + NP * h3, cp + NQ * h3);
                }
                uint32_t ne = 0;
#pragma unroll
                for (int k = 0; k < NP; ++k) ne |= (x + k >= 3 && x + k < w - 3) ? 1u << k : 0u;
                // the spatial search first, then the other frames' rows (loaded past a scheduling
                // barrier, a dword at a time: the two phases' operands are not live at once)
                uint32_t pr[NP / 2], res[NQ];
                if (!(DTS_YT_ABLATE & 1)) {
                    if (DTS_YT_PK)
                        yspatial_pk<NP>(cm, cp, ne, pr);
                    else
                        yspatial<NP>(cm, cp, ne, pr);
                }
                __builtin_amdgcn_sched_barrier(0);
                const int rm2 = 2 * rm - y, rp2 = 2 * rp - y;   // 2 mrefs / 2 prefs
                const uint8_t *rows[10] = {row(prv, rm), row(prv, rp), row(nxt, rm), row(nxt, rp), row(pv2, y),
                                           row(nx2, y), row(pv2, rm2), row(pv2, rp2), row(nx2, rm2), row(nx2, rp2)};
                auto ld = [&](int r, int q) { return *reinterpret_cast<const uint32_t *>(rows[r] + 4 * q); };
                if (DTS_YT_ABLATE & 1) {               // diagnostic: no arithmetic (wrong output)
#pragma unroll
                    for (int q = 0; q < NQ; ++q) res[q] = cm[NQ + q] ^ cp[NQ + q] ^ ld(0, q) ^ ld(3, q) ^ ld(4, q) ^ ld(5, q);
                } else if (far) {
                    ytemporal<NP, true>(cm, cp, ld, pr, res);
                } else {
                    ytemporal<NP, false>(cm, cp, ld, pr, res);
                }
                putn<NP>(obase + (uint64_t)((int64_t)y * dp), res, w - x);
            }
            }
            nst += 2 * RR;
        }
        if (!whole) nst = 0;                   // (edge tiles: wait for their stores too)
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

bool yadif_t_ok(const YadifParams &p)
{
    for (int pl = 0; pl < 3; ++pl)
        if (((p.seq.data[pl] | (uint64_t)p.seq.pitch[pl]) & 15u) || ((p.dst.data[pl] | (uint64_t)p.dst.pitch[pl]) & 15u))
            return false;
    return ((p.seq.fstride | p.dst.fstride) & 15) == 0 && p.w >= 16 && p.h >= 4;
}

hipError_t launch_yadif_t(const YadifParams &p, int count, hipStream_t s)
{
    const int cw = (p.w + 1) >> 1, ch = (p.h + 1) >> 1;
    const int txl = (p.w + kYtW - 1) / kYtW, txc = (cw + kYtW - 1) / kYtW;
    const int tiles_l = txl * ((p.h + kYtH - 1) / kYtH), tiles_c = txc * ((ch + kYtH - 1) / kYtH);
    const int ntiles = tiles_l + 2 * tiles_c;
    // grid.y is one walk of kYtWalk frames; a longer sequence goes out in launches of at most
    // 65535 walks (the y-dimension limit), each starting kMax frames further into the sequence
    // and writing kMax * fields output frames further on
    constexpr int kMax = 65535 * kYtWalk;
    const int fields = (p.mode & 1) ? 2 : 1;
    for (int done = 0; done < count; done += kMax) {
        const int n = count - done < kMax ? count - done : kMax;
        YadifParams q = p;
        q.first += done;
        for (int pl = 0; pl < 3; ++pl) q.dst.data[pl] += (uint64_t)done * fields * (uint64_t)p.dst.fstride;
        const dim3 grid((unsigned)(8 * ((ntiles + 7) / 8)), (unsigned)((n + kYtWalk - 1) / kYtWalk));
        hipLaunchKernelGGL(k_yadif_t, grid, dim3(kYtThreads), 4 * kYtSlot, s, q, tiles_l, tiles_c, txl, txc, n);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_yadif(const YadifParams &p, int nout, hipStream_t s)
{
    const int ch = (p.h + 1) >> 1;
    const int nb = (p.h + kYadifRows - 1) / kYadifRows + 2 * ((ch + kYadifRows - 1) / kYadifRows);
    const dim3 grid((unsigned)((p.w + 1023) / 1024), (unsigned)nb, (unsigned)nout);
    hipLaunchKernelGGL(k_yadif, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

} // namespace dts
