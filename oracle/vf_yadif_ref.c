/*
 * vf_yadif_ref.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of FFmpeg 4.4 libavfilter/vf_yadif.c (SURVEY.md §8a row
 * a10) for 8-bit planar frames:
 *   - filter_line_c / filter_edges: the FILTER macro with the nested CHECK()
 *     spatial search (is_not_edge for 3 <= x < w - 3, which is what the
 *     filter_line_c [3, w-7) + filter_edges [0,3) / [w-7,w-3) / [w-3,w) split
 *     amounts to for 8-bit data, MAX_ALIGN 8);
 *   - filter_slice: rows with (y ^ td->parity) & 1 are interpolated, the rest
 *     copied from cur; prefs/mrefs mirror at the bottom/top row; mode is
 *     forced to 2 (no b/f temporal check) for y == 1 and y + 2 == h;
 *   - return_frame / filter: td->parity = tff ^ !is_second, the line filter's
 *     parity argument is td->parity ^ tff (prev2/next2 choice);
 *   - sequence ends: the first frame's prev and the last frame's next are the
 *     frame itself (yadif clones cur / next at start and EOF).
 * Restated from memory (no FFmpeg source here); bit-exact target.
 */
#include <stdint.h>
#include <stdlib.h>

#include "oracle.h"

static inline int iabs(int a) { return a < 0 ? -a : a; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int imin(int a, int b) { return a < b ? a : b; }

static void filter_line(uint8_t *dst, const uint8_t *prev, const uint8_t *cur, const uint8_t *next, int w,
                        int prefs, int mrefs, int parity, int mode)
{
    const uint8_t *prev2 = parity ? prev : cur;
    const uint8_t *next2 = parity ? cur : next;
    int x;
    for (x = 0; x < w; x++) {
        int c = cur[x + mrefs];
        int d = (prev2[x] + next2[x]) >> 1;
        int e = cur[x + prefs];
        int td0 = iabs(prev2[x] - next2[x]);
        int td1 = (iabs(prev[x + mrefs] - c) + iabs(prev[x + prefs] - e)) >> 1;
        int td2 = (iabs(next[x + mrefs] - c) + iabs(next[x + prefs] - e)) >> 1;
        int diff = imax(imax(td0 >> 1, td1), td2);
        int spatial_pred = (c + e) >> 1;
        if (x >= 3 && x < w - 3) {
            int spatial_score = iabs(cur[x + mrefs - 1] - cur[x + prefs - 1]) + iabs(c - e) +
                                iabs(cur[x + mrefs + 1] - cur[x + prefs + 1]) - 1;
            int j, s;
#define YADIF_SCORE(j) (iabs(cur[x + mrefs - 1 + (j)] - cur[x + prefs - 1 - (j)]) + \
                        iabs(cur[x + mrefs + (j)] - cur[x + prefs - (j)]) +           \
                        iabs(cur[x + mrefs + 1 + (j)] - cur[x + prefs + 1 - (j)]))
            /* CHECK(-1) CHECK(-2): the second only when the first improved */
            for (j = -1; j >= -2; j--) {
                s = YADIF_SCORE(j);
                if (s >= spatial_score) break;
                spatial_score = s;
                spatial_pred = (cur[x + mrefs + j] + cur[x + prefs - j]) >> 1;
            }
            /* CHECK(1) CHECK(2) */
            for (j = 1; j <= 2; j++) {
                s = YADIF_SCORE(j);
                if (s >= spatial_score) break;
                spatial_score = s;
                spatial_pred = (cur[x + mrefs + j] + cur[x + prefs - j]) >> 1;
            }
#undef YADIF_SCORE
        }
        if (!(mode & 2)) {
            int b = (prev2[x + 2 * mrefs] + next2[x + 2 * mrefs]) >> 1;
            int f = (prev2[x + 2 * prefs] + next2[x + 2 * prefs]) >> 1;
            int mx = imax(imax(d - e, d - c), imin(b - c, f - e));
            int mn = imin(imin(d - e, d - c), imax(b - c, f - e));
            diff = imax(imax(diff, mn), -mx);
        }
        if (spatial_pred > d + diff)
            spatial_pred = d + diff;
        else if (spatial_pred < d - diff)
            spatial_pred = d - diff;
        dst[x] = (uint8_t)spatial_pred;
    }
}

/* filter_slice over one plane (w x h, pitch bytes) */
static void yadif_plane(uint8_t *dst, int64_t dpitch, const uint8_t *prev, const uint8_t *cur,
                        const uint8_t *next, int64_t pitch, int w, int h, int td_parity, int tff, int mode)
{
    int y, x;
    for (y = 0; y < h; y++) {
        uint8_t *d = dst + (int64_t)y * dpitch;
        const int64_t o = (int64_t)y * pitch;
        if ((y ^ td_parity) & 1) {
            const int m = (y == 1 || y + 2 == h) ? 2 : mode;
            const int prefs = y + 1 < h ? (int)pitch : -(int)pitch;
            const int mrefs = y ? -(int)pitch : (int)pitch;
            filter_line(d, prev + o, cur + o, next + o, w, prefs, mrefs, td_parity ^ tff, m);
        } else {
            for (x = 0; x < w; x++) d[x] = cur[o + x];
        }
    }
}

int orc_yadif_frame(int w, int h, const uint8_t *const prev[3], const uint8_t *const cur[3],
                    const uint8_t *const next[3], const int64_t pitch[3], uint8_t *const dst[3],
                    const int64_t dpitch[3], int mode, int tff, int is_second)
{
    int p;
    if (w < 16 || h < 4 || mode < 0 || mode > 3) return -22;
    for (p = 0; p < 3; p++) {
        const int pw = p ? (w + 1) >> 1 : w, ph = p ? (h + 1) >> 1 : h;
        yadif_plane(dst[p], dpitch[p], prev[p], cur[p], next[p], pitch[p], pw, ph, tff ^ !is_second, tff, mode);
    }
    return 0;
}
