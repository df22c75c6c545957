// plan6.cpp -- host planning of the ladder work units (ladder7.hip, dts_internal.h
// "ladder work units"): per frame, one work unit per (plane kind, rendition, group of
// 16-column tiles); per tile the H K blocks (64 source columns each) and their
// B fragments; per rendition the V row blocks (16 output rows), the granule
// after which each runs and its B fragments.  The taps are the libswscale
// ones (filters.cpp sws_build_filter = FFmpeg 4.4 utils.c initFilter and
// pack_v), re-laid for v_mfma_i32_16x16x64_i8; nothing here changes a tap.
//
// K order.  The MFMA multiplies lane (m, g)'s A byte j with lane (n, g)'s B
// byte j and sums over (g, j) (tools/probe_mfma_i8.hip), so any K labelling
// both operands share is exact:
//  * H: lane (row m, group g) loads 16 consecutive source bytes at x0 + 64 kb
//    + 16 g; B byte j of lane (output n, g) is the tap of column x0 + 64 kb +
//    16 g + j;
//  * V: the H C registers of 4 VKB granules are the A operand as they stand
//    (lane (column, g) holds rows 4g..4g+3 of each granule); K block kb's
//    dword d is ring slot 4 kb + d, which holds granule q - ((q - s) mod R)
//    when the block runs after granule q.  B byte 4d + i of lane (output row n,
//    g) is the tap of source row 16 granule + 4 g + i.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "filters.h"

namespace dts {

namespace {

void extent6(const SwsFilter &f, int i, int &a, int &z)
{
    a = 1 << 30;
    z = -1;
    for (int j = 0; j < f.size; ++j)
        if (f.coeff[(size_t)i * f.size + j]) {
            a = std::min(a, f.pos[i] + j);
            z = std::max(z, f.pos[i] + j);
        }
}

int htap6(const SwsFilter &f, int i, int src)
{
    const int j = src - f.pos[i];
    return (j >= 0 && j < f.size) ? f.coeff[(size_t)i * f.size + j] : 0;
}

int vtap6(const VTable &v, int y, int row)
{
    const int d = row - v.pos[y];
    if (d < 0 || d >= 2 * v.nv) return 0;
    const uint32_t w = v.coef[(size_t)y * v.nv + d / 2];
    return (int16_t)(d & 1 ? w >> 16 : w & 0xffff);
}

// The H fragment triple of a 16-bit source (k_ladder7, ladder7.hip walk7 P10): the A
// operand is 16 raw little-endian bytes of 8 samples per lane, hi byte hb = s >> 2 and lo
// byte lbm = (s & 3) << 6 once masked, both offset by 128.  With c = 256 chi + clo (signed
// bytes) the sum over the window is
//   sum(64 s c) = 65536 sum(hb' chi) + 256 (sum(hb' clo) + sum(lbm' chi)) + sum(lbm' clo) + K
// so three B operands, L = [clo, 0], M = [chi, clo], A = [0, 2 chi] over the (lo, hi) byte
// positions, give the three terms; false if a tap does not split (2 chi beyond a byte).
template <class F>
bool put6p(std::vector<uint32_t> &bf, uint32_t pair, F tapf)
{
    uint8_t *L = reinterpret_cast<uint8_t *>(bf.data() + (size_t)pair * 512);
    uint8_t *M = L + 1024, *A = L + 2048;
    for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 16; ++j) {
            const int c = tapf(lane, j / 2);          // sample j / 2 of the lane's 8
            const int lo = (int8_t)(c & 0xff), hi = (c - lo) >> 8;
            if (hi < -64 || hi > 63) return false;
            const bool odd = j & 1;                   // the hi byte of the sample
            L[lane * 16 + j] = (uint8_t)(odd ? 0 : lo);
            M[lane * 16 + j] = (uint8_t)(odd ? lo : hi);
            A[lane * 16 + j] = (uint8_t)(odd ? 2 * hi : 0);
        }
    return true;
}

// one fragment pair from tapf(lane, j) (j = byte of the lane's 16): c = 256 hi + lo,
// hi and lo signed bytes (split 256), or c = 128 hi + lo with lo in [0, 127] (split 128);
// false if a tap does not split
template <class F>
bool put6(std::vector<uint32_t> &bf, uint32_t frag, F tapf, int split = 256)
{
    uint8_t *hi = reinterpret_cast<uint8_t *>(bf.data() + (size_t)frag * 512);
    uint8_t *lo = hi + 1024;
    for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 16; ++j) {
            const int c = tapf(lane, j);
            const int l = split == 128 ? (c & 127) : (int8_t)(c & 0xff), h = split == 128 ? (c >> 7) : (c - l) >> 8;
            if (h < -128 || h > 127) return false;
            hi[lane * 16 + j] = (uint8_t)h;
            lo[lane * 16 + j] = (uint8_t)l;
        }
    return true;
}

struct Rend6 {                      // one (plane kind, rendition)
    int hkb = 0, vkb = 0;
    std::vector<int> x0;            // per 16-column tile
    std::vector<int> fire;          // per row block
};

// H K blocks and per-tile x0 (a multiple of align); false if a tile's taps span more
// than 2 K blocks
bool plan_h6(const SwsFilter &f, int srcW, int dstW, Rend6 &r, int align)
{
    const int ntiles = (dstW + 15) / 16;
    if (align > 4 && srcW % align) return false;          // (align 4: a right-edge tile may start unaligned)
    for (int hkb = 1; hkb <= 2; ++hkb) {
        if (srcW < 64 * hkb) return false;
        const int xmax = srcW - 64 * hkb;
        bool ok = true;
        r.x0.assign(ntiles, 0);
        for (int t = 0; t < ntiles && ok; ++t) {
            int a = 1 << 30, z = -1;
            for (int o = 16 * t; o < std::min(16 * t + 16, dstW); ++o) {
                int ai, zi;
                extent6(f, o, ai, zi);
                if (zi < 0) continue;
                a = std::min(a, ai);
                z = std::max(z, zi);
            }
            if (z < 0) continue;                           // all-zero taps (never for a normalised filter)
            const int x0 = std::min(a & ~(align - 1), xmax);
            r.x0[t] = x0;
            ok = z < x0 + 64 * hkb;
        }
        if (ok) {
            r.hkb = hkb;
            return true;
        }
    }
    return false;
}

// V: the granule after which each row block runs, and the ring depth
bool plan_v6(const VTable &v, int srcH, int dstH, Rend6 &r)
{
    const int ngran = (srcH + kL6Gran - 1) / kL6Gran;
    const int nrb = (dstH + 15) / 16;
    std::vector<int> a(nrb), z(nrb);
    for (int j = 0; j < nrb; ++j) {
        a[j] = 1 << 30;
        z[j] = -1;
        for (int y = 16 * j; y < std::min(16 * j + 16, dstH); ++y)
            for (int d = 0; d < 2 * v.nv; ++d)
                if (vtap6(v, y, v.pos[y] + d)) {
                    a[j] = std::min(a[j], v.pos[y] + d);
                    z[j] = std::max(z[j], v.pos[y] + d);
                }
        if (z[j] < 0 || z[j] >= srcH || a[j] < 0) return false;
    }
    r.fire.assign(nrb, 0);
    for (int j = 0; j < nrb; ++j) {
        r.fire[j] = std::min(z[j] / kL6Gran, ngran - 1);
        if (j && r.fire[j] < r.fire[j - 1]) return false;   // the kernel runs row blocks in order
    }
    for (int vkb = 1; vkb <= 2; ++vkb) {
        const int R = 4 * vkb;
        bool ok = true;
        for (int j = 0; j < nrb && ok; ++j) ok = a[j] >= kL6Gran * (r.fire[j] - R + 1);
        if (ok) {
            r.vkb = vkb;
            return true;
        }
    }
    return false;
}

} // namespace

bool plan6_graph(const Plan5In kinds[2], Plan6 &out, int align, bool sort, bool narrow, int fs_window, int hsplit)
{
    out = Plan6{};
    struct Cost { Unit6 u; int64_t cost; };
    std::vector<Cost> units;
    uint32_t nfrag = 0;
    struct Pending { int kind, rung; Rend6 r; uint32_t hfrag, vfrag; int fire; int ct; };
    std::vector<Pending> todo;
    for (int kind = 0; kind < 2; ++kind) {
        const Plan5In &in = kinds[kind];
        if ((in.nv12_chroma || in.p10) && align) return false;   // 4-column windows: planar 8-bit sources only
        if ((int)in.rungs.size() < 1 || (int)in.rungs.size() > DTS_MAX_OUTPUTS) return false;
        for (int k = 0; k < (int)in.rungs.size(); ++k) {
            const Plan5Rung &R = in.rungs[k];
            // p010 renditions: k_ladder7 from p010 sources (one column tile per plane)
            if (R.fmt != DTS_FMT_YUV420P && R.fmt != DTS_FMT_NV12 && (align || !in.p10 || R.fmt != DTS_FMT_P010LE))
                return false;
            const SwsFilter &f = *R.fh;
            for (int i = 0; i < R.dstW; ++i) {             // H bias = 128 * 16384
                int sum = 0;
                for (int j = 0; j < f.size; ++j) sum += f.coeff[(size_t)i * f.size + j];
                if (sum != 1 << 14) return false;
            }
            for (int y = 0; y < R.dstH; ++y) {             // V bias = 128 * 4096
                int sum = 0;
                for (int d = 0; d < 2 * R.v->nv; ++d) sum += vtap6(*R.v, y, R.v->pos[y] + d);
                if (sum != 1 << 12) return false;
            }
            Pending p;
            p.kind = kind;
            p.rung = k;
            const int np = in.chroma ? 2 : 1;
            if (align) {
                if (!plan_h6(f, in.srcW, R.dstW, p.r, align) || !plan_v6(*R.v, in.srcH, R.dstH, p.r)) return false;
            } else if (in.p10) {
                // 16-bit samples: windows on 8-sample (16-byte) boundaries, one 64-sample K block
                // (two raw-byte MFMA K blocks; wider windows keep the graph on k_ladder4: their
                // B operands and A reads would not fit the walk's 128 registers)
                if (!plan_h6(f, in.srcW, R.dstW, p.r, 8) || !plan_v6(*R.v, in.srcH, R.dstH, p.r)) return false;
                if (p.r.hkb != 1 || (in.chroma && p.r.vkb != 1)) return false;   // (chroma: one V K block too)
            } else {
                // k_ladder7: K windows on 16-column boundaries (one ds_read_b128 per A operand),
                // or on 8-column boundaries where that saves a K block and the variant reads
                // its A operands as two ds_read_b64 (l7_b64: the one-K-block, two-tile variants)
                Rend6 r8 = p.r;
                const bool ok16 = plan_h6(f, in.srcW, R.dstW, p.r, 16) && plan_v6(*R.v, in.srcH, R.dstH, p.r);
                const bool ok8 = plan_h6(f, in.srcW, R.dstW, r8, 8) && plan_v6(*R.v, in.srcH, R.dstH, r8);
                if (ok8 && l7_b64(l6_variant(np, r8.hkb, r8.vkb)) && (!ok16 || r8.hkb < p.r.hkb))
                    p.r = r8;
                else if (!ok16)
                    return false;
            }
            p.ct = l6_ct(l6_variant(np, p.r.hkb, p.r.vkb, narrow) | (in.p10 ? 16 : 0));
            const int ntiles = (R.dstW + 15) / 16;
            const int ntp = (ntiles + p.ct - 1) / p.ct * p.ct;  // tiles padded to whole units
            p.r.x0.resize(ntp, 0);
            p.hfrag = nfrag;
            // 16-bit sources: per tile 2 hkb raw K blocks, a fragment triple (2 pair slots) each
            nfrag += (uint32_t)(ntp * p.r.hkb * (in.p10 ? 4 : 1));
            p.vfrag = nfrag;
            nfrag += (uint32_t)(p.r.fire.size() * p.r.vkb);
            p.fire = (int)out.fire.size();
            out.fire.insert(out.fire.end(), p.r.fire.begin(), p.r.fire.end());
            todo.push_back(std::move(p));
        }
    }
    out.frag.assign((size_t)nfrag * 512, 0);
    for (const Pending &p : todo) {
        const Plan5In &in = kinds[p.kind];
        const Plan5Rung &R = in.rungs[p.rung];
        const SwsFilter &f = *R.fh;
        const VTable &v = *R.v;
        const int np = in.chroma ? 2 : 1;
        const int var = l6_variant(np, p.r.hkb, p.r.vkb, narrow) | (in.p10 ? 16 : 0);
        const int ntp = (int)p.r.x0.size();
        for (int t = 0; t < ntp && in.p10; ++t)
            for (int rkb = 0; rkb < 2 * p.r.hkb; ++rkb) {
                const int base = p.r.x0[t] + 32 * rkb;        // raw K block rkb: 32 samples
                if (!put6p(out.frag, p.hfrag + (uint32_t)(t * 2 * p.r.hkb + rkb) * 2u, [&](int lane, int js) {
                        const int o = 16 * t + (lane & 15);
                        return o < R.dstW ? htap6(f, o, base + 8 * (lane >> 4) + js) : 0;
                    }))
                    return false;
            }
        for (int t = 0; t < ntp && !in.p10; ++t)
            for (int kb = 0; kb < p.r.hkb; ++kb) {
                const int base = p.r.x0[t] + 64 * kb;
                if (!put6(out.frag, p.hfrag + (uint32_t)(t * p.r.hkb + kb), [&](int lane, int j) {
                        const int o = 16 * t + (lane & 15);
                        return o < R.dstW ? htap6(f, o, base + 16 * (lane >> 4) + j) : 0;
                    }, hsplit))
                    return false;
            }
        const int R4 = 4 * p.r.vkb;
        for (int jb = 0; jb < (int)p.r.fire.size(); ++jb) {
            const int q = p.r.fire[jb];
            std::vector<int> got(16, 0);
            for (int kb = 0; kb < p.r.vkb; ++kb) {
                if (!put6(out.frag, p.vfrag + (uint32_t)(jb * p.r.vkb + kb), [&](int lane, int jj) {
                        const int s = 4 * kb + jj / 4;
                        const int gran = q - ((q - s) % R4 + R4) % R4;
                        const int row = kL6Gran * gran + 4 * (lane >> 4) + (jj & 3);
                        const int y = 16 * jb + (lane & 15);
                        const int c = (gran >= 0 && row < in.srcH && y < R.dstH) ? vtap6(v, y, row) : 0;
                        got[lane & 15] += c;
                        return c;
                    }))
                    return false;
            }
            for (int n = 0; n < 16; ++n)                   // every tap of the block landed in a slot
                if (16 * jb + n < R.dstH && got[n] != 1 << 12) return false;
        }
        const int ngran = (in.srcH + kL6Gran - 1) / kL6Gran;
        const int nrb = (int)p.r.fire.size();
        // k_ladder7 reads a fire entry's granule from its low 10 bits (the fragment index of
        // a deduplicated rendition rides above them): a granule that does not fit keeps the
        // graph off v7 rather than corrupt its V schedule (validate_spec's 16384-row
        // cap gives at most 1024 granules today)
        for (int jb = 0; jb < nrb; ++jb)
            if (p.r.fire[jb] < 0 || p.r.fire[jb] >= 1024) return false;
        // V fragment slots: the fragments of the row blocks firing in granules q .. q + fs_window - 1
        // are in LDS together (each is DMA'd with the source of its fire granule)
        int fs = 1;
        for (int a = 0, z = 0; a < nrb; ++a) {
            while (z < nrb && p.r.fire[z] < p.r.fire[a] + fs_window) ++z;
            fs = std::max(fs, z - a);
        }
        // Distinct V fragments (round 5): row blocks whose fragments are byte-identical (the
        // filter repeats with the output phase: 4 / 10 / 18 distinct of 68 / 45 / 30 row blocks
        // for the 4K cfg2 luma renditions) share one copy, and the row block's fire entry carries
        // its index in bits 10..15.  A group's lead waves then DMA from a table of ~0.2 MB
        // instead of 1.1 MB, which stays in L2.  More than 64 distinct: stored per row block.
        int vdedup = 0;
        {
            const size_t fw = (size_t)p.r.vkb * 512;
            auto at = [&](int jb) { return out.frag.data() + (size_t)(p.vfrag + (uint32_t)(jb * p.r.vkb)) * 512; };
            std::vector<int> uniq, vid((size_t)nrb);
            for (int jb = 0; jb < nrb; ++jb) {
                int found = -1;
                for (int u = 0; u < (int)uniq.size() && found < 0; ++u)
                    if (!std::memcmp(at(jb), at(uniq[(size_t)u]), fw * 4)) found = u;
                if (found < 0) {
                    found = (int)uniq.size();
                    uniq.push_back(jb);
                }
                vid[(size_t)jb] = found;
            }
            bool ok = uniq.size() <= 64;
            for (int jb = 0; jb < nrb && ok; ++jb) ok = p.r.fire[jb] < 1024;
            if (ok) {
                for (int u = 0; u < (int)uniq.size(); ++u)     // compact: slot u <= its first row block
                    if (uniq[(size_t)u] != u) std::memmove(at(u), at(uniq[(size_t)u]), fw * 4);
                for (int jb = 0; jb < nrb; ++jb) out.fire[(size_t)p.fire + jb] |= vid[(size_t)jb] << 10;
                vdedup = 1;
            }
            if (diag_env("DTS_PLAN_DEBUG"))
                std::fprintf(stderr, "plan6 kind %d rung %d nrb %d vkb %d distinct V fragments %zu fs %d dedup %d\n",
                             p.kind, p.rung, nrb, p.r.vkb, uniq.size(), fs, vdedup);
        }
        for (int u = 0; u * p.ct < ntp; ++u) {
            Unit6 w{};
            w.variant = var;
            w.kind = p.kind;
            w.rung = p.rung;
            w.col0 = 16 * p.ct * u;
            w.ncols = std::min(16 * p.ct, R.dstW - w.col0);
            w.ngran = ngran;
            w.srcH = in.srcH;
            w.dstH = R.dstH;
            w.dstW = R.dstW;
            w.nrb = nrb;
            w.fmt = R.fmt;
            w.hfrag = p.hfrag + (uint32_t)(u * p.ct * p.r.hkb * (in.p10 ? 4 : 1));
            w.vfrag = p.vfrag;
            w.fire = p.fire;
            for (int c = 0; c < 4; ++c) w.x0[c] = c < p.ct ? p.r.x0[(size_t)u * p.ct + c] : 0;
            w.fs = fs;
            w.vdedup = vdedup;
            // MFMAs per unit: H ngran x tiles x HKB x 2, V row blocks x tiles x VKB x 4
            const int tiles = p.ct * np;
            const int64_t cost = (int64_t)ngran * tiles * p.r.hkb * 2 + (int64_t)nrb * tiles * p.r.vkb * 4;
            units.push_back({w, cost});
        }
    }
    // heaviest units first: the dispatcher starts them first, which shortens a frame's tail
    if (sort)
        std::stable_sort(units.begin(), units.end(), [](const Cost &a, const Cost &b) { return a.cost > b.cost; });
    for (const Cost &c : units) out.units.push_back(c.u);
    return !out.units.empty();
}

// v7: the v6 units with 16-column-aligned K windows, grouped per plane kind by source
// position into workgroups of at most wmax waves; each group stages the columns
// [X0, X0 + 64 npc) of its plane(s), which hold every K window of its waves.
bool plan7_graph(const Plan5In kinds[2], int wmax, int stages, int pb, bool by_rung, bool narrow, Plan7 &out)
{
    out = Plan7{};
    // stages of pb granules each; the V fragment slots hold the row blocks of pb (stages + 1)
    // granules (the batches in flight + the one-granule V deferral; ladder7.hip)
    if (wmax < 1 || wmax > kL7MaxWaves || stages < 2 || stages > 4 || pb < 1 || pb > 2) return false;
    Plan6 p6;
    // H taps split 128 (one shift in the H epilogue, walk7 HS = 128) where every tap fits
    // (|c| < 16384: not a 1:1 tap of exactly 1 << 14), else 256
    out.hsplit = 128;
    if (!plan6_graph(kinds, p6, 0, false, narrow, pb * (stages + 1), 128)) {
        out.hsplit = 256;
        if (!plan6_graph(kinds, p6, 0, false, narrow, pb * (stages + 1), 256)) return false;
    }
    if (const char *hs = diag_env("DTS_L7_HSPLIT"))       // diagnostic A/B: force the 256 split
        if (std::atoi(hs) == 256 && out.hsplit == 128) {
            out.hsplit = 256;
            if (!plan6_graph(kinds, p6, 0, false, narrow, pb * (stages + 1), 256)) return false;
        }
    out.frag = std::move(p6.frag);
    out.fire = std::move(p6.fire);
    const int wmax0 = wmax;
    for (int kind = 0; kind < 2; ++kind) {
        const int srcW = kinds[kind].srcW, np = kinds[kind].chroma ? 2 : 1;
        if (srcW % 16) return false;
        // p010 chroma stages 4 bytes per column: groups of half the waves keep two
        // workgroups' stages within one CU's LDS
        wmax = kinds[kind].p10 && kind ? std::max(1, wmax0 / 2) : wmax0;
        std::vector<Unit6> us;
        for (const Unit6 &u : p6.units)
            if (u.kind == kind) us.push_back(u);
        if (us.empty()) return false;
        // window start of a unit (its first tile's x0) orders the plane's units left to right;
        // by_rung: groups of one rendition each (their waves do the same work per granule)
        // (diagnostic DTS_L7_SORT: 1 = by window centre, 2 = by window end)
        const char *se = diag_env("DTS_L7_SORT");
        const int sort_key = se ? std::atoi(se) : 0;
        auto wkey = [&](const Unit6 &w) {
            if (!sort_key) return 2 * w.x0[0];
            const int hkb = l6_hkb(w.variant), ct = l6_ct(w.variant);
            int x1 = 0;
            for (int c = 0; c < ct; ++c)
                if (16 * c < w.ncols) x1 = std::max(x1, w.x0[c] + 64 * hkb);
            return sort_key == 1 ? w.x0[0] + x1 : 2 * x1;
        };
        std::stable_sort(us.begin(), us.end(), [&](const Unit6 &a, const Unit6 &b) {
            if (by_rung && a.rung != b.rung) return a.rung < b.rung;
            return wkey(a) < wkey(b);
        });
        // window extent [wa, wz) of every unit (the source columns its tiles' K windows cover)
        std::vector<int> wa(us.size()), wz(us.size());
        for (size_t i = 0; i < us.size(); ++i) {
            const Unit6 &w = us[i];
            const int hkb = l6_hkb(w.variant), ct = l6_ct(w.variant);
            wa[i] = 1 << 30;
            wz[i] = 0;
            for (int c = 0; c < ct; ++c)
                if (16 * c < w.ncols) {
                    wa[i] = std::min(wa[i], w.x0[c]);
                    wz[i] = std::max(wz[i], w.x0[c] + 64 * hkb);
                }
        }
        // runs of units grouped together: the whole plane kind, or one rendition
        std::vector<std::pair<int, int>> runs;
        const char *dpe = diag_env("DTS_L7_DP");
        const int dp_slack = dpe ? std::atoi(dpe) : 0;
        for (int a = 0, n = (int)us.size(); a < n;) {
            int z = a + 1;
            while (z < n && (!by_rung || us[z].rung == us[a].rung)) ++z;
            const int ng = (z - a + wmax - 1) / wmax;
            if (dp_slack > 0 && ng > 1) {
                // diagnostic (DTS_L7_DP=s): the same number of groups, sizes in [wmax - s, wmax],
                // boundaries chosen to minimise the staged pieces (sum of npc) by dynamic programming
                const int m = z - a, lo = std::max(1, wmax - dp_slack);
                const int inf = 1 << 29;
                std::vector<std::vector<int>> best(ng + 1, std::vector<int>(m + 1, inf)), from(ng + 1, std::vector<int>(m + 1, -1));
                best[0][0] = 0;
                for (int g = 1; g <= ng; ++g)
                    for (int e = 1; e <= m; ++e)
                        for (int sz = lo; sz <= std::min(wmax, e); ++sz) {
                            const int b0 = e - sz;
                            if (best[g - 1][b0] >= inf) continue;
                            int x0 = 1 << 30, x1 = 0;
                            for (int i = b0; i < e; ++i) {
                                x0 = std::min(x0, wa[a + i]);
                                x1 = std::max(x1, wz[a + i]);
                            }
                            const int cost = best[g - 1][b0] + (x1 - (x0 & ~15) + 63) / 64;
                            if (cost < best[g][e]) {
                                best[g][e] = cost;
                                from[g][e] = b0;
                            }
                        }
                if (best[ng][m] < inf) {
                    std::vector<int> sizes;
                    for (int g = ng, e = m; g > 0; e = from[g][e], --g) sizes.push_back(e - from[g][e]);
                    for (int gi = ng - 1; gi >= 0; --gi) runs.push_back({sizes[gi], 0});
                    a = z;
                    continue;
                }
            }
            for (int gi = 0; gi < ng; ++gi) runs.push_back({(z - a) / ng + (gi < (z - a) % ng ? 1 : 0), 0});
            a = z;
        }
        // Waves w and w + 4 of a workgroup share a SIMD (waves are dealt to the CU's four
        // SIMDs in turn).  Within each group the heaviest units (MFMAs per granule: the
        // 1080p walks) take waves 0..3 and the lightest 4..7, so no SIMD carries two heavy
        // walks of one group (the heavy waves set the group's pace at every barrier).
        const char *bal = diag_env("DTS_L7_BAL");
        if (!bal || std::atoi(bal) != 0)
            for (int gi = 0, u = 0; gi < (int)runs.size(); u += runs[gi].first, ++gi) {
                const int cnt = runs[gi].first;
                auto cost = [](const Unit6 &w) {
                    const int t = l6_ct(w.variant) * l6_np(w.variant);
                    return (int64_t)w.ngran * t * l6_hkb(w.variant) * 2 + (int64_t)w.nrb * t * l6_vkb(w.variant) * 4;
                };
                std::vector<Unit6> part(us.begin() + u, us.begin() + u + cnt);
                std::stable_sort(part.begin(), part.end(), [&](const Unit6 &a, const Unit6 &b) { return cost(a) > cost(b); });
                for (int i = 0; i < cnt; ++i) us[u + i] = part[i];
            }
        for (int gi = 0, u = 0; gi < (int)runs.size(); ++gi) {
            const int cnt = runs[gi].first;                 // groups as even as possible
            Group7 g{};
            g.kind = kind;
            g.nwaves = cnt;
            g.u0 = (int)out.units.size();
            g.ngran = us[u].ngran;
            g.srcH = us[u].srcH;
            int a = 1 << 30, z = 0;
            for (int i = u; i < u + cnt; ++i) {
                const Unit6 &w = us[i];
                const int hkb = l6_hkb(w.variant), ct = l6_ct(w.variant);
                for (int c = 0; c < ct; ++c)
                    if (16 * c < w.ncols) {                // tiles past the unit's columns have no taps
                        a = std::min(a, w.x0[c]);
                        z = std::max(z, w.x0[c] + 64 * hkb);
                    }
            }
            a &= ~15;                                      // (8-aligned windows of the b64 variants)
            g.npc = (z - a + 63) / 64;
            g.X0 = std::min(a, srcW - 64 * g.npc);
            if (g.X0 < 0 || g.X0 % 16) return false;
            // per rendition: the first wave of the group DMAs its V fragments; slots in LDS
            const int bpc = kinds[kind].p10 ? (np == 2 ? 4 : 2) : (kinds[kind].nv12_chroma ? 2 : 1);
            int lds = stages * pb * (bpc == 1 ? np : 1) * bpc * g.npc * 1024;
            int flds[DTS_MAX_OUTPUTS], lead[DTS_MAX_OUTPUTS];
            for (int r = 0; r < DTS_MAX_OUTPUTS; ++r) flds[r] = lead[r] = -1;
            for (int i = u; i < u + cnt; ++i) {
                const Unit6 &w = us[i];
                Unit7 v{};
                v.variant = w.variant;
                v.kind = w.kind;
                v.rung = w.rung;
                v.col0 = w.col0;
                v.ncols = w.ncols;
                v.ngran = w.ngran;
                v.srcH = w.srcH;
                v.dstH = w.dstH;
                v.nrb = w.nrb;
                v.fmt = w.fmt;
                v.hfrag = w.hfrag;
                v.vfrag = w.vfrag;
                v.fire = w.fire;
                v.dstW = w.dstW;
                const int ct = l6_ct(w.variant);
                for (int c = 0; c < 4; ++c)
                    v.xo[c] = (c < ct && 16 * c < w.ncols) ? w.x0[c] - g.X0 : w.x0[0] - g.X0;
                v.fs = w.fs;
                v.vdedup = w.vdedup;
                // swscale.c (FFmpeg 4.4) range converters (oracle/swscale_ref.c restates them)
                static const int32_t rc[2][2][4] = {
                    {{14, 30189, 19077, -39057361}, {14, 32767, 14071, 33561947}},   // luma: To, From
                    {{12, 30775, 4663, -9289992}, {11, 32767, 1799, 4081085}}};     // chroma: To, From
                if (kinds[kind].range_conv) {
                    const int32_t *c = rc[kind][kinds[kind].range_conv - 1];
                    v.rc_sh = c[0];
                    v.rc_cap = c[1];
                    v.rc_mul = c[2];
                    v.rc_add = c[3];
                }
                if (lead[w.rung] < 0) {
                    lead[w.rung] = i;
                    flds[w.rung] = lds;
                    lds += w.fs * l6_vkb(w.variant) * 2048;
                    v.lead = 1;
                }
                v.flds = flds[w.rung];
                if (w.ngran != g.ngran) return false;
                out.units.push_back(v);
            }
            g.scr = lds;
            g.bpc = bpc;
            out.groups.push_back(g);
            u += cnt;
        }
    }
    for (size_t i = 0; i < out.groups.size(); ++i) {       // (ladder7.hip DTS_L7_ABLATE & 4)
        Group7 &g = out.groups[i];
        const bool last = i + 1 == out.groups.size() || out.groups[i + 1].kind != g.kind;
        g.xown = last ? kinds[g.kind].srcW : std::max(out.groups[i + 1].X0, g.X0 + 64);
    }
    if (diag_env("DTS_PLAN_DEBUG"))                     // diagnostic: staged columns per plane kind
        for (const Group7 &g : out.groups)
            std::fprintf(stderr, "plan7 group kind %d X0 %d npc %d waves %d scr %d\n", g.kind, g.X0, g.npc, g.nwaves, g.scr);
    // the widest group sets the workgroup size; every group's LDS fits that many waves
    for (const Group7 &g : out.groups) out.waves = std::max(out.waves, g.nwaves);
    // the staging waves: a group's spare waves, else all of its waves
    for (Group7 &g : out.groups) {
        g.st0 = g.nwaves < out.waves ? g.nwaves : 0;
        out.lds_bytes = std::max(out.lds_bytes, g.scr + out.waves * 1024);
    }
    return out.lds_bytes <= 160 * 1024;
}

} // namespace dts
