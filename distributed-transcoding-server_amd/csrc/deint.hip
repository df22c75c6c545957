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

hipError_t launch_yadif(const YadifParams &p, int nout, hipStream_t s)
{
    const int ch = (p.h + 1) >> 1;
    const int nb = (p.h + kYadifRows - 1) / kYadifRows + 2 * ((ch + kYadifRows - 1) / kYadifRows);
    const dim3 grid((unsigned)((p.w + 1023) / 1024), (unsigned)nb, (unsigned)nout);
    hipLaunchKernelGGL(k_yadif, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

} // namespace dts
