// deint.hip -- k_yadif: vf_yadif deinterlacing of
// 8-bit yuv420p frames resident in HBM, bit-exact with libavfilter/vf_yadif.c
// filter_line_c / filter_edges / filter_slice (FFmpeg 4.4; oracle/vf_yadif_ref.c).
//
// One workgroup = 256 consecutive pixels of one row of one plane of one output
// frame; a thread computes one pixel.  Copied rows (the kept field) are plain
// byte copies.  An interpolated pixel reads rows y +- 1 of cur (x-3 .. x+3),
// rows y +- 1 of prev and next, and rows y, y +- 2 of the field pair
// prev2/next2: ~12 rows of the three frames, all shared with the neighbouring
// threads and rows through L1/L2, so HBM sees each input frame about once per
// output.  HBM-bound integer work, no LDS staging needed at this size.
#include "dts_internal.h"

namespace dts {

namespace {

__device__ __forceinline__ int iabs(int a) { return a < 0 ? -a : a; }

} // namespace

__global__ void __launch_bounds__(256) k_yadif(const YadifParams P)
{
    const int fields = (P.mode & 1) ? 2 : 1;
    const int o = blockIdx.z;                              // output frame of this launch
    const int j = o / fields, is_second = o - j * fields;
    const int i = P.first + j;
    const int ip = i > 0 ? i - 1 : 0, in = i + 1 < P.nseq ? i + 1 : P.nseq - 1;
    const int cw = (P.w + 1) >> 1, ch = (P.h + 1) >> 1;
    int r = blockIdx.y, p = 0;
    if (r >= P.h) {
        r -= P.h;
        p = 1 + (r >= ch);
        if (p == 2) r -= ch;
    }
    const int w = p ? cw : P.w, h = p ? ch : P.h, y = r;
    const int x = blockIdx.x * 256 + threadIdx.x;
    if (x >= w) return;
    const int64_t pitch = P.seq.pitch[p];
    const uint64_t base = P.seq.data[p] + (uint64_t)y * pitch + x;
    const uint8_t *cur = reinterpret_cast<const uint8_t *>(base + (uint64_t)i * P.seq.fstride);
    uint8_t *dst = reinterpret_cast<uint8_t *>(P.dst.data[p] + (uint64_t)o * P.dst.fstride +
                                               (uint64_t)y * P.dst.pitch[p] + x);
    const int td_parity = P.tff ^ !is_second;
    if (!((y ^ td_parity) & 1)) {                          // the kept field: copy
        *dst = *cur;
        return;
    }
    const uint8_t *prev = reinterpret_cast<const uint8_t *>(base + (uint64_t)ip * P.seq.fstride);
    const uint8_t *next = reinterpret_cast<const uint8_t *>(base + (uint64_t)in * P.seq.fstride);
    const int mode = (y == 1 || y + 2 == h) ? 2 : P.mode;
    const int64_t prefs = y + 1 < h ? pitch : -pitch, mrefs = y ? -pitch : pitch;
    const int parity = td_parity ^ P.tff;
    const uint8_t *prev2 = parity ? prev : cur, *next2 = parity ? cur : next;

    const int c = cur[mrefs], e = cur[prefs];
    const int d = (prev2[0] + next2[0]) >> 1;
    const int td0 = iabs(prev2[0] - next2[0]);
    const int td1 = (iabs(prev[mrefs] - c) + iabs(prev[prefs] - e)) >> 1;
    const int td2 = (iabs(next[mrefs] - c) + iabs(next[prefs] - e)) >> 1;
    int diff = max(max(td0 >> 1, td1), td2);
    int spatial_pred = (c + e) >> 1;
    if (x >= 3 && x < w - 3) {                             // filter_line_c / filter_edges is_not_edge
        int score = iabs(cur[mrefs - 1] - cur[prefs - 1]) + iabs(c - e) + iabs(cur[mrefs + 1] - cur[prefs + 1]) - 1;
#define YADIF_SCORE(jj) (iabs(cur[mrefs - 1 + (jj)] - cur[prefs - 1 - (jj)]) + \
                         iabs(cur[mrefs + (jj)] - cur[prefs - (jj)]) +         \
                         iabs(cur[mrefs + 1 + (jj)] - cur[prefs + 1 - (jj)]))
        int s = YADIF_SCORE(-1);                           // CHECK(-1) CHECK(-2)
        if (s < score) {
            score = s;
            spatial_pred = (cur[mrefs - 1] + cur[prefs + 1]) >> 1;
            s = YADIF_SCORE(-2);
            if (s < score) {
                score = s;
                spatial_pred = (cur[mrefs - 2] + cur[prefs + 2]) >> 1;
            }
        }
        s = YADIF_SCORE(1);                                // CHECK(1) CHECK(2)
        if (s < score) {
            score = s;
            spatial_pred = (cur[mrefs + 1] + cur[prefs - 1]) >> 1;
            s = YADIF_SCORE(2);
            if (s < score) spatial_pred = (cur[mrefs + 2] + cur[prefs - 2]) >> 1;
        }
#undef YADIF_SCORE
    }
    if (!(mode & 2)) {
        const int b = (prev2[2 * mrefs] + next2[2 * mrefs]) >> 1;
        const int f = (prev2[2 * prefs] + next2[2 * prefs]) >> 1;
        const int mx = max(max(d - e, d - c), min(b - c, f - e));
        const int mn = min(min(d - e, d - c), max(b - c, f - e));
        diff = max(max(diff, mn), -mx);
    }
    if (spatial_pred > d + diff)
        spatial_pred = d + diff;
    else if (spatial_pred < d - diff)
        spatial_pred = d - diff;
    *dst = (uint8_t)spatial_pred;
}

hipError_t launch_yadif(const YadifParams &p, int nout, hipStream_t s)
{
    const int ch = (p.h + 1) >> 1;
    const dim3 grid((unsigned)((p.w + 255) / 256), (unsigned)(p.h + 2 * ch), (unsigned)nout);
    hipLaunchKernelGGL(k_yadif, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

} // namespace dts
