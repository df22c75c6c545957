// plan5.cpp -- host planning of the v5 ladder (ladder5.hip, dts_internal.h
// "v5 ladder"): column strips, H tiles and V row groups on the matrix cores,
// the H-output rings and the per-step V schedule.  The taps are the
// libswscale ones (filters.cpp sws_build_filter = FFmpeg 4.4 utils.c
// initFilter), re-laid for v_mfma_i32_16x16x64_i8; nothing here changes a tap.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "filters.h"

namespace dts {

namespace {

// first / last nonzero tap (source column) of H output i
void extent(const SwsFilter &f, int i, int &a, int &z)
{
    a = f.pos[i];
    z = f.pos[i];
    bool any = false;
    for (int j = 0; j < f.size; ++j)
        if (f.coeff[(size_t)i * f.size + j]) {
            if (!any) a = f.pos[i] + j;
            z = f.pos[i] + j;
            any = true;
        }
}

int htap(const SwsFilter &f, int i, int src)
{
    const int j = src - f.pos[i];
    return (j >= 0 && j < f.size) ? f.coeff[(size_t)i * f.size + j] : 0;
}

// V tap of output row y on source row `row` (the packed pairs of filters.cpp pack_v)
int vtap(const VTable &v, int y, int row)
{
    const int d = row - v.pos[y];
    if (d < 0 || d >= 2 * v.nv) return 0;
    const uint32_t w = v.coef[(size_t)y * v.nv + d / 2];
    return (int16_t)(d & 1 ? w >> 16 : w & 0xffff);
}

struct Tile {                       // 16 H outputs of one rendition (one V column tile)
    int split;                      // H entries: 1, 2 or 4 (16 / split outputs each, one K block of
                                    // 64 source columns per entry)
    int base[4];                    // first staged column of each entry's K block (multiple of 8)
    int centre;                     // strip assignment key
    int frag;                       // first B fragment pair (split of them)
};

int round_up(int v, int a) { return (v + a - 1) / a * a; }

// 16 x odd >= v (column / row pitches whose 4-dword lane groups hit distinct banks)
int pitch16odd(int v)
{
    int p = round_up(std::max(v, 16), 16);
    if ((p / 16) % 2 == 0) p += 16;
    return p;
}

// K order inside one lane's 16 A/B bytes (ladder5.hip reads A this way):
// bytes 0-7 = K block rows/columns 8g..8g+7, bytes 8-15 = 32+8g..32+8g+7 (g = lane >> 4)
int kcol_of(int lane, int j)
{
    const int g = lane >> 4;
    return j < 8 ? 8 * g + j : 32 + 8 * g + (j - 8);
}

// one fragment pair: tap(lane, k) split as 256 hi + lo (signed bytes); false if out of range
template <class F>
bool put_frag(std::vector<uint32_t> &bf, int frag, F tapf)
{
    uint8_t *hi = reinterpret_cast<uint8_t *>(bf.data() + (size_t)frag * 512);
    uint8_t *lo = hi + 1024;
    for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 16; ++j) {
            const int c = tapf(lane, kcol_of(lane, j));
            const int l = (int8_t)(c & 0xff), h = (c - l) >> 8;
            if (h < -128 || h > 127) return false;
            hi[lane * 16 + j] = (uint8_t)h;
            lo[lane * 16 + j] = (uint8_t)l;
        }
    return true;
}

} // namespace

bool plan5_kind(const Plan5In &in, Plan5Kind &out)
{
    out = Plan5Kind{};
    const int nr = (int)in.rungs.size();
    if (nr < 1 || nr > DTS_MAX_OUTPUTS) return false;
    const int nplanes = in.chroma ? 2 : 1;
    const int nsteps = (in.srcH + kL5StepRows - 1) / kL5StepRows;
    // ---- H tiles per rendition ---------------------------------------------
    std::vector<std::vector<Tile>> tiles(nr);
    int nfrag = 0;
    for (int r = 0; r < nr; ++r) {
        const Plan5Rung &R = in.rungs[r];
        const SwsFilter &f = *R.fh;
        if (R.fmt != DTS_FMT_YUV420P && R.fmt != DTS_FMT_NV12) return false;   // 8-bit outputs only
        for (int i = 0; i < R.dstW; ++i) {                                      // bias = 128 * 16384
            int sum = 0;
            for (int j = 0; j < f.size; ++j) sum += f.coeff[(size_t)i * f.size + j];
            if (sum != 1 << 14) return false;
        }
        for (int t0 = 0; t0 < R.dstW; t0 += 16) {
            // split the 16 outputs until every part's taps fit one 64-column K block
            Tile t{};
            int A = 1 << 30, Z = -1;
            for (t.split = 1; t.split <= 4; t.split *= 2) {
                const int no = 16 / t.split;
                bool fits = true;
                for (int s = 0; s < t.split; ++s) {
                    int a = 1 << 30, z = -1;
                    for (int i = t0 + s * no; i < std::min(t0 + (s + 1) * no, R.dstW); ++i) {
                        int ai, zi;
                        extent(f, i, ai, zi);
                        a = std::min(a, ai);
                        z = std::max(z, zi);
                    }
                    if (z < 0) a = z = A < (1 << 30) ? A : 0;      // a part past the plane's right edge
                    t.base[s] = a & ~7;
                    fits = fits && z - t.base[s] < 64;
                    A = std::min(A, a);
                    Z = std::max(Z, z);
                }
                if (fits) break;
            }
            if (t.split > 4) return false;
            t.centre = (A + Z) / 2;
            t.frag = nfrag;
            nfrag += t.split;
            tiles[r].push_back(t);
        }
    }
    // ---- V row groups per rendition: window, K blocks, ready step, fragments ----
    struct Group { int rows, w0, nkb, step, frag; };
    std::vector<std::vector<Group>> groups(nr);
    std::vector<int> RR(nr, 32);
    for (int r = 0; r < nr; ++r) {
        const VTable &v = *in.rungs[r].v;
        const int dstH = in.rungs[r].dstH;
        for (int y = 0; y < dstH; ++y) {                                       // bias = 128 * 4096
            int sum = 0;
            for (int d = 0; d < 2 * v.nv; ++d) sum += vtap(v, y, v.pos[y] + d);
            if (sum != 1 << 12) return false;
        }
        for (int G = 0; 16 * G < dstH; ++G) {
            Group g{};
            g.rows = std::min(16, dstH - 16 * G);
            int a = 1 << 30, z = -1;
            for (int y = 16 * G; y < 16 * G + g.rows; ++y)
                for (int d = 0; d < 2 * v.nv; ++d)
                    if (vtap(v, y, v.pos[y] + d)) {
                        a = std::min(a, v.pos[y] + d);
                        z = std::max(z, v.pos[y] + d);
                    }
            if (z < 0) return false;
            g.w0 = a & ~7;
            g.nkb = (z - g.w0) / 64 + 1;
            if (g.nkb > kL5MaxVkb) return false;
            g.step = std::min(z / kL5StepRows, nsteps - 1);  // ready: after H(step)
            g.frag = -1;
            groups[r].push_back(g);
        }
    }
    // ---- V schedule: groups run at their ready step or up to kMaxDefer steps later, so
    // that no step runs more than `cap` K blocks (the fragment buffers are sized by the
    // busiest step; a later step costs its ring 16 more rows: measured, the rings cost
    // more LDS than the fragment buffers save, so kMaxDefer = 0) --------------------
    constexpr int kMaxDefer = 0;
    {
        struct QG { int r, G, ready; };
        std::vector<QG> order;
        int maxkb = 1;
        for (int r = 0; r < nr; ++r)
            for (int G = 0; G < (int)groups[r].size(); ++G) {
                order.push_back({r, G, groups[r][G].step});
                maxkb = std::max(maxkb, groups[r][G].nkb);
            }
        std::stable_sort(order.begin(), order.end(), [](const QG &a, const QG &b) { return a.ready < b.ready; });
        for (int cap = maxkb;; ++cap) {
            bool ok = true;
            size_t q = 0;
            std::vector<int> when(order.size(), -1);
            for (int b = 0; b < nsteps && ok; ++b) {
                int used = 0;
                for (size_t k = q; k < order.size() && order[k].ready <= b; ++k) {
                    if (when[k] >= 0) continue;
                    const int nkb = groups[order[k].r][order[k].G].nkb;
                    if (used + nkb > cap && b < nsteps - 1) {
                        if (b - order[k].ready >= kMaxDefer) ok = false;   // too late: raise the cap
                        continue;
                    }
                    when[k] = b;
                    used += nkb;
                }
                while (q < order.size() && when[q] >= 0) ++q;
            }
            if (!ok) continue;
            for (size_t k = 0; k < order.size(); ++k) groups[order[k].r][order[k].G].step = when[k];
            break;
        }
    }
    for (int r = 0; r < nr; ++r) {
        // V(step) reads rows [w0, z] while H(step + 1) writes [16 (step + 1), 16 (step + 2));
        // the V A reads of a group cover w0 + [0, 64 nkb): with RR >= 64 nkb one
        // conditional subtract wraps them (ladder5.hip vtile2)
        for (const Group &g : groups[r]) {
            RR[r] = std::max(RR[r], round_up(kL5StepRows * (g.step + 2) - g.w0, 16));
            RR[r] = std::max(RR[r], kL5StepRows);
            RR[r] = std::max(RR[r], 64 * g.nkb);
        }
        if (RR[r] > 4096) return false;
    }
    // V fragments in step order: the groups of one step are one contiguous run, which
    // the kernel copies into a fragment buffer by LDS-DMA the step before they run
    std::vector<int> vf0(nsteps + 1, 0), vkb(nsteps + 1, 0);
    int FM = 0;                                            // most V K blocks of any step
    for (int b = 0; b < nsteps; ++b) {
        vf0[b] = nfrag;
        for (int r = 0; r < nr; ++r)
            for (Group &g : groups[r])
                if (g.step == b) {
                    g.frag = nfrag;
                    nfrag += g.nkb;
                }
        vkb[b] = nfrag - vf0[b];
        FM = std::max(FM, vkb[b]);
    }
    vf0[nsteps] = nfrag;
    // ---- fragments: H (B = taps of 16 outputs over 64 source columns), V (B = taps of
    // 16 output rows over 64 source rows)
    out.bfrag.assign((size_t)nfrag * 512, 0);
    for (int r = 0; r < nr; ++r) {
        const SwsFilter &f = *in.rungs[r].fh;
        const int dstW = in.rungs[r].dstW;
        for (size_t ti = 0; ti < tiles[r].size(); ++ti) {
            const Tile &t = tiles[r][ti];
            const int no = 16 / t.split;
            for (int s = 0; s < t.split; ++s) {
                const bool ok = put_frag(out.bfrag, t.frag + s, [&](int lane, int k) {
                    const int o = (int)ti * 16 + s * no + (lane & 15);
                    return (lane & 15) < no && o < dstW ? htap(f, o, t.base[s] + k) : 0;
                });
                if (!ok) return false;
            }
        }
        const VTable &v = *in.rungs[r].v;
        const int dstH = in.rungs[r].dstH;
        for (size_t G = 0; G < groups[r].size(); ++G) {
            const Group &g = groups[r][G];
            for (int kb = 0; kb < g.nkb; ++kb) {
                const bool ok = put_frag(out.bfrag, g.frag + kb, [&](int lane, int k) {
                    const int y = (int)G * 16 + (lane & 15);
                    return y < dstH ? vtap(v, y, g.w0 + 64 * kb + k) : 0;
                });
                if (!ok) return false;
            }
        }
    }
    // ---- per-step V schedule (ring fields filled in once the rings are laid out) --
    std::vector<int> voff(nsteps + 1, 0);
    for (int b = 0; b < nsteps; ++b) {
        voff[b] = (int)out.vsched.size();
        for (int r = 0; r < nr; ++r)
            for (size_t G = 0; G < groups[r].size(); ++G) {
                const Group &g = groups[r][G];
                if (g.step != b) continue;
                VEnt5 e{};
                e.rung = r;
                e.G = (int)G;
                e.rows = g.rows;
                e.w0 = g.w0 % RR[r];                  // ring row of the window start
                e.nkb = g.nkb;
                e.foff = (g.frag - vf0[b]) * 2048;
                e.fmt = in.rungs[r].fmt;
                e.dstW = in.rungs[r].dstW;
                out.vsched.push_back(e);
            }
    }
    voff[nsteps] = (int)out.vsched.size();
    out.vstep.assign((size_t)4 * (nsteps + 1), 0);
    for (int b = 0; b <= nsteps; ++b) {
        const int e0 = voff[b], e1 = b < nsteps ? voff[b + 1] : e0;
        out.vstep[4 * b] = e0;
        out.vstep[4 * b + 1] = e1;
        out.vstep[4 * b + 2] = vf0[b];
        out.vstep[4 * b + 3] = 2 * vkb[b];                  // 1 KB DMA units (hi, lo per K block)
    }
    const int nlp = in.chroma && !in.nv12_chroma ? 2 : 1;  // load planes
    // ---- strips ---------------------------------------------------------------
    const int bps = in.nv12_chroma ? 2 : 1;
    for (int SW = round_up(std::min(in.srcW, 1024), 16); SW >= 64; SW -= 16) {
        Plan5Kind pk;
        pk.nplanes = nplanes;
        pk.nsteps = nsteps;
        const int nstrips = (in.srcW + SW - 1) / SW;
        std::vector<std::vector<int>> t0(nstrips, std::vector<int>(nr, 0)), t1 = t0;
        for (int r = 0; r < nr; ++r) {
            const auto &T = tiles[r];
            size_t ti = 0;
            for (int s = 0; s < nstrips; ++s) {
                t0[s][r] = (int)ti;
                while (ti < T.size() && (T[ti].centre < (s + 1) * SW || s == nstrips - 1)) ++ti;
                t1[s][r] = (int)ti;
            }
        }
        bool ok = true;
        int PSmax = 1024;
        std::vector<int> pcols(nr, 16);
        for (int s = 0; s < nstrips && ok; ++s) {
            Strip5 st{};
            int L = 1 << 30, E = 0;
            for (int r = 0; r < nr; ++r)
                for (int ti = t0[s][r]; ti < t1[s][r]; ++ti)
                    for (int k = 0; k < tiles[r][ti].split; ++k) {
                        L = std::min(L, tiles[r][ti].base[k]);
                        E = std::max(E, tiles[r][ti].base[k] + 64);
                    }
            if (L == 1 << 30) {
                L = 0;
                E = 16;
            }
            L &= ~15;
            const int W = round_up(E - L, 16);
            st.L = L;
            st.cpr = W * bps / 16;
            st.cpr += 1 - (st.cpr & 1);                    // odd: 16 x odd row pitch
            st.Pb = 16 * st.cpr;
            st.PS = round_up(kL5StepRows * st.Pb, 1024);   // one DMA instruction never spans two planes
            st.nsi = nlp * st.PS / 1024;
            PSmax = std::max(PSmax, st.PS);
            // source DMA instructions per step, dealt over the waves
            if ((st.nsi + kL5Waves - 1) / kL5Waves > kL5MaxDma) {
                ok = false;
                break;
            }
            // H entries: tiles (both planes for chroma) to the least loaded wave, K blocks together
            struct TE { int r, ti, plane; };
            std::vector<TE> list;
            for (int r = 0; r < nr; ++r)
                for (int ti = t0[s][r]; ti < t1[s][r]; ++ti)
                    for (int p = 0; p < nplanes; ++p) list.push_back({r, ti, p});
            std::vector<std::vector<Ent5>> wl(kL5Waves);
            int wnext = 0;
            for (const TE &e : list) {
                const Tile &t = tiles[e.r][e.ti];
                for (int k = 0; k < t.split; ++k) {          // entries dealt round robin
                    const int w = wnext;
                    wnext = (wnext + 1) % kL5Waves;
                    if ((int)wl[w].size() >= kL5Ent) {
                        ok = false;
                        break;
                    }
                    Ent5 en{};
                    en.bfrag = t.frag + k;
                    en.soff = (int16_t)((t.base[k] - L) * bps);   // byte offset in the staged row
                    en.col0 = (int16_t)(16 * (e.ti - t0[s][e.r]) + k * (16 / t.split));
                    en.plane = (int8_t)e.plane;
                    en.ring = (int8_t)(e.r * nplanes + e.plane);
                    en.flags = (int8_t)((in.nv12_chroma && e.plane ? 4 : 0) | (t.split == 1 ? 0 : t.split == 2 ? 8 : 16));
                    wl[w].push_back(en);
                }
                if (!ok) break;
            }
            if (!ok) break;
            st.hextra = wnext;                             // entries were dealt round robin from wave 0
            for (int w = 0; w < kL5Waves; ++w) {
                st.ent0[w] = (int)pk.ents.size();
                st.nent[w] = (int)wl[w].size();
                pk.ents.insert(pk.ents.end(), wl[w].begin(), wl[w].end());
            }
            for (int r = 0; r < nr; ++r) {
                st.x0[r] = 16 * t0[s][r];
                st.nct[r] = t1[s][r] - t0[s][r];
                pcols[r] = std::max(pcols[r], 16 * st.nct[r]);
            }
            pk.strips.push_back(st);
        }
        if (!ok) continue;
        // stage buffers: the load planes (16 rows each), then the V fragment area
        int lds = 16 + kL5RungTab;                         // the dequeue slot, the per-item rendition table
        pk.nlp = nlp;
        pk.stage = lds;
        pk.SB = nlp * PSmax;
        lds += kL5Stages * pk.SB;
        pk.FA = lds;                                       // fragment buffers (V(b) in buffer b % kL5FragBufs)
        pk.FB = 2048 * std::max(FM, 1);
        lds += kL5FragBufs * pk.FB;
        // rings: (rendition, plane), two column-major byte planes each
        pk.nrings = nr * nplanes;
        for (int r = 0; r < nr; ++r)
            for (int p = 0; p < nplanes; ++p) {
                Ring5 &g = pk.ring[r * nplanes + p];
                g.RR = RR[r];
                g.CP = pitch16odd(RR[r]);
                g.hi = lds;
                lds += pcols[r] * g.CP;
                g.lo = lds;
                lds += pcols[r] * g.CP;
            }
        if (lds > in.lds_cap) continue;
        for (int r = 0; r < nr; ++r) {
            pk.out[r].fmt = in.rungs[r].fmt;
            pk.out[r].dstW = in.rungs[r].dstW;
            pk.out[r].dstH = in.rungs[r].dstH;
        }
        pk.lds_bytes = lds;
        pk.bfrag = std::move(out.bfrag);
        pk.vsched = std::move(out.vsched);
        pk.vstep = std::move(out.vstep);
        for (VEnt5 &e : pk.vsched) {
            e.ring0 = pk.ring[e.rung * nplanes];
            e.hi1 = nplanes == 2 ? pk.ring[e.rung * 2 + 1].hi : e.ring0.hi;
            e.lo1 = nplanes == 2 ? pk.ring[e.rung * 2 + 1].lo : e.ring0.lo;
        }
        pk.strip_width = SW;
        out = std::move(pk);
        return true;
    }
    return false;
}

} // namespace dts
