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
// per-output kernel above fetches.  A thread computes 16 pixels of one interpolated row
// from LDS (cur rows y -+ 1 as 48-byte windows for the x -+ 3 spatial search) and copies 16
// bytes of one kept row; the 3-byte window sums of the spatial search are v_sad_u8 of
// v_perm-aligned operands.  Sources and outputs 16-byte aligned, w >= 16.
// ---------------------------------------------------------------------------
constexpr int kYtW = 512;                       // output columns per tile (32 lanes x 16)
constexpr int kYtH = 32;                        // output rows per tile (16 interpolated + 16 kept)
constexpr int kYtPitch = kYtW + 32;             // LDS row: 16 columns of halo each side
constexpr int kYtRows = kYtH + 4;               // rows y0 - 2 .. y0 + kYtH + 1
constexpr int kYtChunks = kYtPitch / 16;        // 16-byte chunks per LDS row (34)
constexpr int kYtSlot = kYtRows * kYtPitch;     // one frame tile (19,584 B)
constexpr int kYtPieces = (kYtRows * kYtChunks + 63) / 64;   // 1-KB LDS-DMA pieces per frame tile
constexpr int kYtThreads = 512;
#ifndef DTS_YADIF_WALK
#define DTS_YADIF_WALK 16
#endif
constexpr int kYtWalk = DTS_YADIF_WALK;         // input frames per workgroup

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

__device__ __forceinline__ int absd(int a, int b) { return (int)__builtin_amdgcn_sad_u8((uint32_t)a, (uint32_t)b, 0u); }

// vf_yadif.c filter_line_c / filter_edges for the 16 pixels x .. x + 15 of one interpolated
// row.  cm / cp: cur rows mrefs / prefs, bytes x - 16 .. x + 31 (pixel k at byte 16 + k);
// the rest bytes x .. x + 15: pm / pp prev rows mrefs / prefs, nm / np next, p2 / n2 prev2 /
// next2 on this row, p2m .. n2p prev2 / next2 two rows away (mode 0 only).  ne: bit k set
// when pixel k is not an edge pixel (3 <= x + k < w - 3).
template <bool FAR>
__device__ __forceinline__ void yadif16(const uint32_t (&cm)[12], const uint32_t (&cp)[12], const uint32_t (&pm)[4],
                                        const uint32_t (&pp)[4], const uint32_t (&nm)[4], const uint32_t (&np)[4],
                                        const uint32_t (&p2)[4], const uint32_t (&n2)[4], const uint32_t (&p2m)[4],
                                        const uint32_t (&p2p)[4], const uint32_t (&n2m)[4], const uint32_t (&n2p)[4],
                                        uint32_t ne, uint32_t (&out)[4])
{
#pragma unroll
    for (int q = 0; q < 4; ++q) out[q] = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int X = 16 + k;
        const int c = byte_at(cm, X), e = byte_at(cp, X);
        const int a2 = byte_at(p2, k), b2 = byte_at(n2, k);
        const int d = (a2 + b2) >> 1;
        const int td0 = absd(a2, b2);
        const int td1 = (absd(byte_at(pm, k), c) + absd(byte_at(pp, k), e)) >> 1;
        const int td2 = (absd(byte_at(nm, k), c) + absd(byte_at(np, k), e)) >> 1;
        int diff = max(max(td0 >> 1, td1), td2);
        int pred = (c + e) >> 1;
        if ((ne >> k) & 1u) {               // (a branch per pixel, uniform in interior tiles: computed
                                            // unconditionally the sixteen pixels' window sums share
                                            // values across pixels and need 241 VGPRs)
            // CHECK(j): the 3-byte windows cm[x + j - 1 ..] vs cp[x - j - 1 ..]
            int score = (int)__builtin_amdgcn_sad_u8(win3(cm, X - 1), win3(cp, X - 1), 0u) - 1;
            const int sm1 = (int)__builtin_amdgcn_sad_u8(win3(cm, X - 2), win3(cp, X), 0u);
            const int sm2 = (int)__builtin_amdgcn_sad_u8(win3(cm, X - 3), win3(cp, X + 1), 0u);
            const int s1 = (int)__builtin_amdgcn_sad_u8(win3(cm, X), win3(cp, X - 2), 0u);
            const int s2 = (int)__builtin_amdgcn_sad_u8(win3(cm, X + 1), win3(cp, X - 3), 0u);
            const bool b1 = sm1 < score;
            score = b1 ? sm1 : score;
            pred = b1 ? (byte_at(cm, X - 1) + byte_at(cp, X + 1)) >> 1 : pred;
            const bool bb2 = b1 && sm2 < score;
            score = bb2 ? sm2 : score;
            pred = bb2 ? (byte_at(cm, X - 2) + byte_at(cp, X + 2)) >> 1 : pred;
            const bool b3 = s1 < score;
            score = b3 ? s1 : score;
            pred = b3 ? (byte_at(cm, X + 1) + byte_at(cp, X - 1)) >> 1 : pred;
            const bool b4 = b3 && s2 < score;
            pred = b4 ? (byte_at(cm, X + 2) + byte_at(cp, X - 2)) >> 1 : pred;
        }
        if (FAR) {
            const int b = (byte_at(p2m, k) + byte_at(n2m, k)) >> 1;
            const int f = (byte_at(p2p, k) + byte_at(n2p, k)) >> 1;
            const int mx = max(max(d - e, d - c), min(b - c, f - e));
            const int mn = min(min(d - e, d - c), max(b - c, f - e));
            diff = max(max(diff, mn), -mx);
        }
        // diff >= 0, so the reference's two-sided clamp is a median
        pred = min(max(pred, d - diff), d + diff);
        out[k >> 2] |= (uint32_t)pred << (8 * (k & 3));
    }
}

typedef unsigned int u32x4y __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4y g_u32x4y;
typedef __attribute__((address_space(1))) uint8_t g_u8y;
__device__ __forceinline__ u32x4y lds16(const uint8_t *p) { return *reinterpret_cast<const u32x4y *>(p); }
__device__ __forceinline__ void put16(uint64_t dst, u32x4y v, int room)
{
    if (room >= 16) {
        *(g_u32x4y *)(uintptr_t)dst = v;
    } else {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (int i = 0; i < room; ++i) ((g_u8y *)(uintptr_t)dst)[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
}
__device__ __forceinline__ void unpack4(u32x4y v, uint32_t *o)
{
    o[0] = v.x;
    o[1] = v.y;
    o[2] = v.z;
    o[3] = v.w;
}

} // namespace

__global__ void __launch_bounds__(kYtThreads) k_yadif_t(const YadifParams P, int tiles_l, int tiles_c, int txl, int txc,
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
    int ops = 0;
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
            ++ops;
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
    const int ci = t & 31, ri = t >> 5;        // 16 columns of one interpolated and one kept row
    const int x = x0 + 16 * ci;
    const uint64_t obase0 = P.dst.data[p] + (uint64_t)x;
    for (int j = j0; j < j1; ++j) {
        const int s = j - j0;
        if (s) __syncthreads();                // every wave is done with frame j - 2's slot
        const int dma0 = ops;
        if (j + 2 <= j1) stage(j + 2, (s + 3) & 3);
        // frame j + 1's pieces: issued before the previous step's stores and these pieces
        vm_wait_yt(nst + (ops - dma0));
        __syncthreads();
        const uint8_t *sl_p = yl + ((s + 0) & 3) * kYtSlot, *sl_c = yl + ((s + 1) & 3) * kYtSlot,
                      *sl_n = yl + ((s + 2) & 3) * kYtSlot;
        nst = 0;
        for (int is2 = 0; is2 < fields; ++is2) {
            const int td_parity = P.tff ^ !is2, parity = td_parity ^ P.tff;
            const int o = j * fields + is2;
            const uint64_t obase = obase0 + (uint64_t)o * (uint64_t)P.dst.fstride;
            const int64_t dp = P.dst.pitch[p];
            const int off = ((y0 ^ td_parity) & 1) ? 0 : 1;     // y0 + off: the tile's first interpolated row
            // kept row: a copy of cur
            {
                const int y = y0 + 2 * ri + (1 - off);
                if (y < h && x < w) {
                    const u32x4y v = lds16(sl_c + (y - y0 + 2) * kYtPitch + 16 * ci + 16);
                    put16(obase + (uint64_t)((int64_t)y * dp), v, w - x);
                }
            }
            const int y = y0 + 2 * ri + off;
            if (y < h && x < w) {
                const int rm = y ? y - 1 : y + 1, rp = y + 1 < h ? y + 1 : y - 1;
                const bool far = !((P.mode & 2) || y == 1 || y + 2 == h);
                const uint8_t *prv = sl_p, *cur = sl_c, *nxt = sl_n;
                const uint8_t *pv2 = parity ? prv : cur, *nx2 = parity ? cur : nxt;
                auto row = [&](const uint8_t *sl, int yy) { return sl + (yy - y0 + 2) * kYtPitch + 16 * ci + 16; };
                uint32_t cm[12], cp[12], pm[4], pp[4], nm[4], np[4], p2[4], n2[4], p2m[4], p2p[4], n2m[4], n2p[4];
#pragma unroll
                for (int h3 = 0; h3 < 3; ++h3) {
                    unpack4(lds16(row(cur, rm) - 16 + 16 * h3), cm + 4 * h3);
                    unpack4(lds16(row(cur, rp) - 16 + 16 * h3), cp + 4 * h3);
                }
                unpack4(lds16(row(prv, rm)), pm);
                unpack4(lds16(row(prv, rp)), pp);
                unpack4(lds16(row(nxt, rm)), nm);
                unpack4(lds16(row(nxt, rp)), np);
                unpack4(lds16(row(pv2, y)), p2);
                unpack4(lds16(row(nx2, y)), n2);
                uint32_t ne = 0;
#pragma unroll
                for (int k = 0; k < 16; ++k) ne |= (x + k >= 3 && x + k < w - 3) ? 1u << k : 0u;
                uint32_t res[4];
                if (far) {
                    const int rm2 = 2 * rm - y, rp2 = 2 * rp - y;   // 2 mrefs / 2 prefs
                    unpack4(lds16(row(pv2, rm2)), p2m);
                    unpack4(lds16(row(pv2, rp2)), p2p);
                    unpack4(lds16(row(nx2, rm2)), n2m);
                    unpack4(lds16(row(nx2, rp2)), n2p);
                    yadif16<true>(cm, cp, pm, pp, nm, np, p2, n2, p2m, p2p, n2m, n2p, ne, res);
                } else {
                    yadif16<false>(cm, cp, pm, pp, nm, np, p2, n2, p2m, p2p, n2m, n2p, ne, res);
                }
                put16(obase + (uint64_t)((int64_t)y * dp), (u32x4y){res[0], res[1], res[2], res[3]}, w - x);
            }
            nst += 2;
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
    const dim3 grid((unsigned)(8 * ((ntiles + 7) / 8)), (unsigned)((count + kYtWalk - 1) / kYtWalk));
    hipLaunchKernelGGL(k_yadif_t, grid, dim3(kYtThreads), 4 * kYtSlot, s, p, tiles_l, tiles_c, txl, txc, count);
    return hipGetLastError();
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
