// plan5.cpp -- host planning of the v5 ladder (ladder5.hip, dts_internal.h
// "v5 ladder"): column strips, H tiles on the matrix cores, V rings and the
// per-step V row lists.  The tables are the libswscale ones (filters.cpp
// sws_build_filter = FFmpeg 4.4 utils.c initFilter), re-laid for
// v_mfma_i32_16x16x64_i8; nothing here changes a tap.
#include <algorithm>
#include <cstring>

#include "filters.h"

namespace dts {

namespace {

// first / last nonzero tap (source column) of output i
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

int tap(const SwsFilter &f, int i, int src)
{
    const int j = src - f.pos[i];
    return (j >= 0 && j < f.size) ? f.coeff[(size_t)i * f.size + j] : 0;
}

struct Tile {                       // 16 outputs of one rendition
    int base;                       // first staged column of its K blocks (multiple of 8)
    int nkb;                        // K blocks of 64 columns
    int centre;                     // strip assignment key
    int frag;                       // first B fragment pair
};

int round_up(int v, int a) { return (v + a - 1) / a * a; }

} // namespace

// K order inside one lane's 16 A/B bytes (must match ladder5.hip a_frag):
// bytes 0-7 = K block columns 8g..8g+7, bytes 8-15 = 32+8g..32+8g+7 (g = lane >> 4)
static inline int kcol_of(int lane, int j)
{
    const int g = lane >> 4;
    return j < 8 ? 8 * g + j : 32 + 8 * g + (j - 8);
}

bool plan5_kind(const Plan5In &in, Plan5Kind &out)
{
    out = Plan5Kind{};
    const int nr = (int)in.rungs.size();
    if (nr < 1 || nr > DTS_MAX_OUTPUTS) return false;
    const int nplanes = in.chroma ? 2 : 1;
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
            int a = 1 << 30, z = -1;
            for (int i = t0; i < std::min(t0 + 16, R.dstW); ++i) {
                int ai, zi;
                extent(f, i, ai, zi);
                a = std::min(a, ai);
                z = std::max(z, zi);
            }
            Tile t;
            t.base = a & ~7;
            t.nkb = (z - t.base) / 64 + 1;
            if (t.nkb > 4) return false;
            t.centre = (a + z) / 2;
            t.frag = nfrag;
            nfrag += t.nkb;
            tiles[r].push_back(t);
        }
    }
    // ---- B fragments: per K block a hi and a lo 1 KB fragment ----------------
    out.bfrag.assign((size_t)nfrag * 2 * 256, 0);
    for (int r = 0; r < nr; ++r) {
        const SwsFilter &f = *in.rungs[r].fh;
        const int dstW = in.rungs[r].dstW;
        for (size_t ti = 0; ti < tiles[r].size(); ++ti) {
            const Tile &t = tiles[r][ti];
            for (int kb = 0; kb < t.nkb; ++kb) {
                uint8_t *hi = reinterpret_cast<uint8_t *>(out.bfrag.data() + (size_t)(t.frag + kb) * 2 * 256);
                uint8_t *lo = hi + 1024;
                for (int lane = 0; lane < 64; ++lane)
                    for (int j = 0; j < 16; ++j) {
                        const int o = (int)ti * 16 + (lane & 15);
                        const int c = o < dstW ? tap(f, o, t.base + 64 * kb + kcol_of(lane, j)) : 0;
                        const int l = (int8_t)(c & 0xff), h = (c - l) >> 8;
                        if (h < -128 || h > 127) return false;
                        hi[lane * 16 + j] = (uint8_t)h;
                        lo[lane * 16 + j] = (uint8_t)l;
                    }
            }
        }
    }
    // ---- V: per rendition, ring slots and the rows each 16-row step completes --
    const int nsteps = (in.srcH + kL5Rows - 1) / kL5Rows;
    const int pairs_total = (in.srcH + 1) / 2;
    std::vector<int> Rslots(nr), np4(nr), rows_max(nr, 0);
    std::vector<std::vector<int32_t>> vlim(nr);
    for (int r = 0; r < nr; ++r) {
        const VTable &v = *in.rungs[r].v;
        const int dstH = in.rungs[r].dstH;
        np4[r] = (v.nv + 3) & ~3;
        if (np4[r] > 32) return false;
        vlim[r].assign(nsteps, 0);
        int y = 0, need = 16;
        for (int b = 0; b < nsteps; ++b) {
            const int done = std::min(8 * (b + 1), pairs_total), y0 = y;
            int pmin = 1 << 30;
            while (y < dstH && std::min(v.pos[y] / 2 + v.nv, pairs_total) <= done) {
                pmin = std::min(pmin, v.pos[y] / 2);
                ++y;
            }
            vlim[r][b] = y;
            rows_max[r] = std::max(rows_max[r], y - y0);
            // V(b) reads pairs [pmin, done) while H(b + 1) writes [8(b + 1), 8(b + 2))
            if (y > y0) need = std::max(need, 8 * (b + 2) - pmin);
        }
        if (y != dstH) return false;
        Rslots[r] = round_up(need, 8);
        if (Rslots[r] > 256) return false;
    }
    // one ring size for the kind (the kernel keeps one slot counter per step)
    int Ru = 8, Mu = 0;
    for (int r = 0; r < nr; ++r) {
        Ru = std::max(Ru, Rslots[r]);
        Mu = std::max(Mu, in.rungs[r].v->nv - 1);
    }
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
        int Wmax = 16;
        std::vector<int> pcols(nr, 16);
        for (int s = 0; s < nstrips && ok; ++s) {
            Strip5 st{};
            int L = 1 << 30, E = 0;
            for (int r = 0; r < nr; ++r)
                for (int ti = t0[s][r]; ti < t1[s][r]; ++ti) {
                    L = std::min(L, tiles[r][ti].base);
                    E = std::max(E, tiles[r][ti].base + 64 * tiles[r][ti].nkb);
                }
            if (L == 1 << 30) {
                L = 0;
                E = 16;
            }
            L &= ~15;
            const int W = round_up(E - L, 16);
            Wmax = std::max(Wmax, W);
            st.L = L;
            st.cpr = W * bps / 16;
            st.nchunk = in.nv12_chroma ? kL5Rows * st.cpr : nplanes * kL5Rows * st.cpr;
            if (st.nchunk > kL5MaxLoads * 256) {
                ok = false;
                break;
            }
            // H entries: tiles (both planes for chroma) to the least loaded wave, K blocks together
            struct TE { int r, ti, plane; };
            std::vector<TE> list;
            for (int r = 0; r < nr; ++r)
                for (int ti = t0[s][r]; ti < t1[s][r]; ++ti)
                    for (int p = 0; p < nplanes; ++p) list.push_back({r, ti, p});
            std::stable_sort(list.begin(), list.end(), [&](const TE &a, const TE &b) {
                return tiles[a.r][a.ti].nkb > tiles[b.r][b.ti].nkb;
            });
            std::vector<std::vector<Ent5>> wl(4);
            for (const TE &e : list) {
                const Tile &t = tiles[e.r][e.ti];
                int w = 0;
                for (int k = 1; k < 4; ++k)
                    if (wl[k].size() < wl[w].size()) w = k;
                if ((int)wl[w].size() + t.nkb > kL5Ent) {
                    ok = false;
                    break;
                }
                for (int kb = 0; kb < t.nkb; ++kb) {
                    Ent5 en{};
                    en.bfrag = t.frag + kb;
                    en.soff = (int16_t)(t.base + 64 * kb - L);
                    en.col0 = (int16_t)(16 * (e.ti - t0[s][e.r]));
                    en.plane = (int8_t)e.plane;
                    en.ring = (int8_t)(e.r * nplanes + e.plane);
                    en.flags = (int8_t)((kb == 0 ? 1 : 0) | (kb == t.nkb - 1 ? 2 : 0));
                    wl[w].push_back(en);
                }
            }
            if (!ok) break;
            for (int w = 0; w < 4; ++w) {
                st.ent0[w] = (int)pk.ents.size();
                st.nent[w] = (int)wl[w].size();
                pk.ents.insert(pk.ents.end(), wl[w].begin(), wl[w].end());
            }
            for (int r = 0; r < nr; ++r) {
                st.x0[r] = 16 * t0[s][r];
                pcols[r] = std::max(pcols[r], 16 * (t1[s][r] - t0[s][r]));
            }
            pk.strips.push_back(st);
        }
        if (!ok) continue;
        // staged row pitch: 16 x odd bytes >= every strip's width (A reads conflict-free)
        int P = round_up(Wmax, 16);
        if ((P / 16) % 2 == 0) P += 16;
        pk.P = P;
        int lds = 4;                                       // dwords 0-3: the dequeue slot
        pk.stage = lds;
        lds += 2 * nplanes * kL5Rows * P / 4;
        // rings: (rendition, plane), quad-major, slots allocated = 1 mod 8
        pk.nrings = nr * nplanes;
        for (int r = 0; r < nr; ++r)
            for (int p = 0; p < nplanes; ++p) {
                Ring5 &g = pk.ring[r * nplanes + p];
                int alloc = std::max(Ru + np4[r] - 1, Ru + round_up(std::max(Mu, 1), 8));
                while (alloc % 8 != 1) ++alloc;
                g.qstride = 4 * alloc;
                g.lds = lds;
                lds += (pcols[r] / 4) * g.qstride;
            }
        // V units and their per-step staging
        pk.nunits = 0;
        for (int r = 0; r < nr; ++r) {
            auto add = [&](int mode, int plane, int ring0, int ring1, int cols) {
                Unit5 &u = pk.unit[pk.nunits++];
                u.rung = r;
                u.mode = mode;
                u.plane = plane;
                u.ring0 = ring0;
                u.ring1 = ring1;
                u.np4 = np4[r];
                u.dstW = cols;
                u.vco_dw = std::max(rows_max[r], 1) * (4 + np4[r]);
                u.vco = lds;
                lds += 2 * u.vco_dw;
            };
            const int W = in.rungs[r].dstW;
            if (!in.chroma)
                add(0, 0, r, r, W);
            else if (in.rungs[r].fmt == DTS_FMT_NV12)
                add(1, 1, 2 * r, 2 * r + 1, W);
            else {
                add(0, 1, 2 * r, 2 * r, W);
                add(0, 2, 2 * r + 1, 2 * r + 1, W);
            }
        }
        for (size_t s = 0; s < pk.strips.size(); ++s) {
            Strip5 &st = pk.strips[s];
            for (int u = 0; u < pk.nunits; ++u) {
                const Unit5 &U = pk.unit[u];
                const int cols = std::max(0, std::min(16 * t1[s][U.rung], U.dstW) - 16 * t0[s][U.rung]);
                st.quads[u] = U.mode == 1 ? (cols + 1) / 2 : (cols + 3) / 4;
            }
        }
        pk.lds_dw = lds;
        if (lds * 4 > in.lds_cap) continue;
        // V tables
        pk.vslot.resize(nr);
        pk.vcoef.resize(nr);
        pk.vlim = vlim;
        for (int r = 0; r < nr; ++r) {
            const VTable &v = *in.rungs[r].v;
            const int dstH = in.rungs[r].dstH;
            pk.vslot[r].resize(dstH);
            pk.vcoef[r].assign((size_t)dstH * np4[r], 0);
            for (int y = 0; y < dstH; ++y) {
                pk.vslot[r][y] = (v.pos[y] / 2) % Ru;
                for (int t = 0; t < v.nv; ++t) pk.vcoef[r][(size_t)y * np4[r] + t] = v.coef[(size_t)y * v.nv + t];
            }
        }
        pk.bfrag = std::move(out.bfrag);
        pk.strip_width = SW;
        pk.R = Ru;
        pk.M = Mu;
        out = std::move(pk);
        return true;
    }
    return false;
}

} // namespace dts
