// filters.cpp -- see filters.h.  Filter math follows FFmpeg 4.4
// libswscale/utils.c initFilter() (the [ext] function the reference's ffmpeg
// worker runs for `scale`, index.js:9 / database.js:73-74); packing is ours.
#include "filters.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "dts_internal.h"

namespace dts {

namespace {

constexpr double kReduceCutoff = 0.002;   // SWS_MAX_REDUCE_CUTOFF
constexpr int kMaxFilterSize = 256;       // SWS_MAX_FILTER_SIZE
constexpr double kParamDefault = DTS_PARAM_DEFAULT;

int ilog2(unsigned v)
{
    int n = 0;
    while (v > 1) {
        v >>= 1;
        ++n;
    }
    return n;
}

int64_t iabs64(int64_t v) { return v < 0 ? -v : v; }

int64_t rounded_div(int64_t a, int64_t b)
{
    return (a >= 0 ? a + (b >> 1) : a - (b >> 1)) / b;
}

// Raw (un-normalised) tap weight of one scaled-kernel method for distance d
// (2^-30 source pixels, already rescaled for downscaling).
int64_t kernel_weight(int flags, const double param[2], int64_t d, int64_t fone, int xInc)
{
    const double fd = d * (1.0 / (1 << 30));
    if (flags & DTS_SCALE_BICUBIC) {
        const int64_t B = (int64_t)((param[0] != kParamDefault ? param[0] : 0) * (1 << 24));
        const int64_t C = (int64_t)((param[1] != kParamDefault ? param[1] : 0.6) * (1 << 24));
        int64_t w;
        if (d >= 1LL << 31) {
            w = 0;
        } else {
            const int64_t d2 = (d * d) >> 30;
            const int64_t d3 = (d2 * d) >> 30;
            if (d < 1LL << 30)
                w = (12 * (1 << 24) - 9 * B - 6 * C) * d3 + (-18 * (1 << 24) + 12 * B + 6 * C) * d2 +
                    (6 * (1 << 24) - 2 * B) * (1 << 30);
            else
                w = (-B - 6 * C) * d3 + (6 * B + 30 * C) * d2 + (-12 * B - 48 * C) * d +
                    (8 * B + 24 * C) * (1 << 30);
        }
        return w / ((1LL << 54) / fone);
    }
    if (flags & DTS_SCALE_X) {
        const double A = param[0] != kParamDefault ? param[0] : 1.0;
        double c = fd < 1.0 ? std::cos(fd * M_PI) : -1.0;
        c = c < 0.0 ? -std::pow(-c, A) : std::pow(c, A);
        return (int64_t)((c * 0.5 + 0.5) * fone);
    }
    if (flags & DTS_SCALE_AREA) {
        const int64_t d2 = d - (1 << 29);
        int64_t w;
        if (d2 * xInc < -(1LL << (29 + 16)))
            w = (int64_t)(1.0 * (1LL << (30 + 16)));
        else if (d2 * xInc < (1LL << (29 + 16)))
            w = -d2 * xInc + (1LL << (29 + 16));
        else
            w = 0;
        return w * (fone >> (30 + 16));
    }
    if (flags & DTS_SCALE_GAUSS) {
        const double p = param[0] != kParamDefault ? param[0] : 3.0;
        return (int64_t)(std::exp2(-p * fd * fd) * fone);
    }
    if (flags & DTS_SCALE_SINC)
        return (int64_t)((d ? std::sin(fd * M_PI) / (fd * M_PI) : 1.0) * fone);
    if (flags & DTS_SCALE_LANCZOS) {
        const double p = param[0] != kParamDefault ? param[0] : 3.0;
        int64_t w = (int64_t)((d ? std::sin(fd * M_PI) * std::sin(fd * M_PI / p) / (fd * fd * M_PI * M_PI / p)
                                 : 1.0) * fone);
        return fd > p ? 0 : w;
    }
    // bilinear
    int64_t w = (1 << 30) - d;
    if (w < 0) w = 0;
    return w * (fone >> 30);
}

int size_factor(int flags, const double param[2])
{
    if (flags & DTS_SCALE_BICUBIC) return 4;
    if (flags & DTS_SCALE_X) return 8;
    if (flags & DTS_SCALE_AREA) return 1;
    if (flags & DTS_SCALE_GAUSS) return 8;
    if (flags & DTS_SCALE_LANCZOS) return param[0] != kParamDefault ? (int)std::ceil(2 * param[0]) : 6;
    if (flags & DTS_SCALE_SINC) return 20;
    if (flags & DTS_SCALE_BILINEAR) return 2;
    return -1;
}

} // namespace

int sws_local_pos(int chr_subsample, int pos)
{
    if (pos == -1 || pos <= -513) pos = (128 << chr_subsample) - 128;
    return (pos + 128) >> chr_subsample;
}

int sws_build_filter(int srcN, int dstN, int one, int align, int flags,
                     const double param[2], int srcPos, int dstPos, SwsFilter &out)
{
    if (srcN < 1 || dstN < 1) return DTS_E_INVAL;
    const int xInc = (int)((((int64_t)srcN << 16) + (dstN >> 1)) / dstN);
    const int64_t fone = 1LL << (54 - std::min(ilog2((unsigned)(srcN / dstN)), 8));

    // ---- stage 1: raw int64 kernel per output ----------------------------
    int fsize;
    std::vector<int64_t> raw;
    std::vector<int32_t> fpos(dstN);
    if (std::abs(xInc - 0x10000) < 10 && srcPos == dstPos) {          // unscaled
        fsize = 1;
        raw.assign(dstN, fone);
        for (int i = 0; i < dstN; ++i) fpos[i] = i;
    } else if (flags & DTS_SCALE_POINT) {
        fsize = 1;
        raw.assign(dstN, fone);
        int64_t x = ((dstPos * (int64_t)xInc) >> 8) - ((srcPos * 0x8000LL) >> 7);
        for (int i = 0; i < dstN; ++i, x += xInc) fpos[i] = (int)((x + (1 << 15)) >> 16);
    } else if (xInc <= (1 << 16) && (flags & DTS_SCALE_AREA)) {       // area upscale = linear
        fsize = 2;
        raw.assign((size_t)dstN * 2, 0);
        int64_t x = ((dstPos * (int64_t)xInc) >> 8) - ((srcPos * 0x8000LL) >> 7);
        for (int i = 0; i < dstN; ++i, x += xInc) {
            int xx = (int)((x - 0x8000LL + (1 << 15)) >> 16);
            fpos[i] = xx;
            for (int j = 0; j < 2; ++j, ++xx) {
                int64_t w = fone - iabs64((int64_t)xx * (1 << 16) - x) * (fone >> 16);
                raw[(size_t)i * 2 + j] = w < 0 ? 0 : w;
            }
        }
    } else {
        const int sf = size_factor(flags, param);
        if (sf <= 0) return DTS_E_UNSUPPORTED;
        fsize = xInc <= (1 << 16) ? 1 + sf : 1 + (sf * srcN + dstN - 1) / dstN;
        fsize = std::max(std::min(fsize, srcN - 2), 1);
        raw.assign((size_t)dstN * fsize, 0);
        int64_t x = ((dstPos * (int64_t)xInc) >> 7) - ((srcPos * 0x10000LL) >> 7);
        for (int i = 0; i < dstN; ++i, x += 2 * (int64_t)xInc) {
            int xx = (int)((x - (fsize - 2) * (1LL << 16)) / (1 << 17));
            fpos[i] = xx;
            for (int j = 0; j < fsize; ++j, ++xx) {
                int64_t d = iabs64((int64_t)xx * (1 << 17) - x) << 13;
                if (xInc > 1 << 16) d = d * dstN / srcN;
                raw[(size_t)i * fsize + j] = kernel_weight(flags, param, d, fone, xInc);
            }
        }
    }

    // ---- stage 2: trim near-zero taps (left by shifting, right by counting)
    int minSize = 0;
    for (int i = dstN - 1; i >= 0; --i) {
        int64_t *f = &raw[(size_t)i * fsize];
        int64_t cut = 0;
        for (int j = 0; j < fsize; ++j) {
            cut += iabs64(f[0]);
            if (cut > kReduceCutoff * fone) break;
            if (i < dstN - 1 && fpos[i] >= fpos[i + 1]) break;   // keep filterPos monotonic
            std::copy(f + 1, f + fsize, f);
            f[fsize - 1] = 0;
            fpos[i]++;
        }
        int keep = fsize;
        cut = 0;
        for (int j = fsize - 1; j > 0; --j) {
            cut += iabs64(f[j]);
            if (cut > kReduceCutoff * fone) break;
            --keep;
        }
        minSize = std::max(minSize, keep);
    }

    // ---- stage 3: align (x86 MMX rules) and BITEXACT zeroing --------------
    if (minSize == 1 && align == 2) align = 1;
    const int size = (minSize + (align - 1)) & ~(align - 1);
    if (size <= 0 || size >= kMaxFilterSize) return DTS_E_RANGE;
    std::vector<int64_t> filt((size_t)dstN * size, 0);
    for (int i = 0; i < dstN; ++i)
        for (int j = 0; j < size && j < fsize && j < minSize; ++j)   // BITEXACT: taps >= minSize are 0
            filt[(size_t)i * size + j] = raw[(size_t)i * fsize + j];

    // ---- stage 4: fold taps outside [0, srcN) onto the edge samples ------
    for (int i = 0; i < dstN; ++i) {
        int64_t *f = &filt[(size_t)i * size];
        if (fpos[i] < 0) {
            for (int j = 1; j < size; ++j) {
                const int left = std::max(j + fpos[i], 0);
                f[left] += f[j];
                f[j] = 0;
            }
            fpos[i] = 0;
        }
        if (fpos[i] + size > srcN) {
            const int shift = fpos[i] + std::min(size - srcN, 0);
            int64_t acc = 0;
            for (int j = size - 1; j >= 0; --j)
                if (fpos[i] + j >= srcN) {
                    acc += f[j];
                    f[j] = 0;
                }
            for (int j = size - 1; j >= 0; --j) f[j] = j < shift ? 0 : f[j - shift];
            fpos[i] -= shift;
            f[srcN - 1 - fpos[i]] += acc;
        }
        if (fpos[i] < 0 || fpos[i] >= srcN) return DTS_E_RANGE;
    }

    // ---- stage 5: normalise to `one` with error diffusion ----------------
    out.size = size;
    out.coeff.assign((size_t)dstN * size, 0);
    out.pos = fpos;
    for (int i = 0; i < dstN; ++i) {
        const int64_t *f = &filt[(size_t)i * size];
        int64_t sum = 0;
        for (int j = 0; j < size; ++j) sum += f[j];
        sum = (sum + one / 2) / one;
        if (!sum) sum = 1;
        int64_t err = 0;
        for (int j = 0; j < size; ++j) {
            const int64_t v = f[j] + err;
            const int q = (int)rounded_div(v, sum);
            out.coeff[(size_t)i * size + j] = (int16_t)q;
            err = v - (int64_t)q * sum;
        }
    }
    return DTS_OK;
}

namespace {
// first/last nonzero tap of output i (both 0 for an all-zero row)
void nonzero_extent(const SwsFilter &f, int i, int &j0, int &j1)
{
    j0 = 0;
    j1 = 0;
    bool any = false;
    for (int j = 0; j < f.size; ++j)
        if (f.coeff[(size_t)i * f.size + j]) {
            if (!any) j0 = j;
            j1 = j;
            any = true;
        }
}

int tap_at(const SwsFilter &f, int i, int src)
{
    const int j = src - f.pos[i];
    return (j >= 0 && j < f.size) ? f.coeff[(size_t)i * f.size + j] : 0;
}
} // namespace

int pack_h_u8(const SwsFilter &f, int n, HTable &out)
{
    int span = 1;
    std::vector<int32_t> start(n);
    for (int i = 0; i < n; ++i) {
        int j0, j1;
        nonzero_extent(f, i, j0, j1);
        start[i] = (f.pos[i] + j0) & ~3;
        span = std::max(span, f.pos[i] + j1 - start[i] + 1);
    }
    const int nd = ladder_nd_round((span + 3) / 4);
    out.nd = nd;
    out.span = span;
    out.pos = start;
    out.bias.assign(n, 0);
    out.hi.assign((size_t)nd * n, 0);
    out.lo.assign((size_t)nd * n, 0);
    for (int i = 0; i < n; ++i) {
        int sum = 0;
        for (int d = 0; d < nd; ++d) {
            uint32_t hw = 0, lw = 0;
            for (int b = 0; b < 4; ++b) {
                const int c = tap_at(f, i, start[i] + 4 * d + b);
                const int lo = (int8_t)(c & 0xff);
                const int hi = (c - lo) >> 8;
                if (hi < -128 || hi > 127) return DTS_E_RANGE;
                sum += c;
                hw |= (uint32_t)(uint8_t)hi << (8 * b);
                lw |= (uint32_t)(uint8_t)lo << (8 * b);
            }
            out.hi[(size_t)d * n + i] = hw;
            out.lo[(size_t)d * n + i] = lw;
        }
        out.bias[i] = 128 * sum;
    }
    return DTS_OK;
}

int pack_h_p010(const SwsFilter &f, int n, HTable &out)
{
    int span = 1;
    std::vector<int32_t> start(n);
    for (int i = 0; i < n; ++i) {
        int j0, j1;
        nonzero_extent(f, i, j0, j1);
        start[i] = (f.pos[i] + j0) & ~1;
        span = std::max(span, f.pos[i] + j1 - start[i] + 1);
    }
    const int nd = ladder_nd_round((span + 1) / 2);
    out.nd = nd;
    out.span = span;
    out.pos = start;
    out.bias.assign(n, 0);
    out.hi.assign((size_t)nd * n, 0);
    out.lo.assign((size_t)nd * n, 0);
    for (int i = 0; i < n; ++i)
        for (int d = 0; d < nd; ++d) {
            const int c0 = tap_at(f, i, start[i] + 2 * d);
            const int c1 = tap_at(f, i, start[i] + 2 * d + 1);
            out.hi[(size_t)d * n + i] = (uint32_t)(uint16_t)(int16_t)c0 | ((uint32_t)(uint16_t)(int16_t)c1 << 16);
        }
    return DTS_OK;
}

int pack_v(const SwsFilter &f, int n, VTable &out)
{
    int span = 1;
    std::vector<int32_t> start(n);
    for (int i = 0; i < n; ++i) {
        int j0, j1;
        nonzero_extent(f, i, j0, j1);
        start[i] = (f.pos[i] + j0) & ~1;
        span = std::max(span, f.pos[i] + j1 - start[i] + 1);
    }
    const int nv = (span + 1) / 2;
    out.nv = nv;
    out.span = span;
    out.pos = start;
    out.coef.assign((size_t)n * nv, 0);
    for (int i = 0; i < n; ++i)
        for (int d = 0; d < nv; ++d) {
            const int c0 = tap_at(f, i, start[i] + 2 * d);
            const int c1 = tap_at(f, i, start[i] + 2 * d + 1);
            out.coef[(size_t)i * nv + d] = (uint32_t)(uint16_t)(int16_t)c0 | ((uint32_t)(uint16_t)(int16_t)c1 << 16);
        }
    return DTS_OK;
}

namespace {
const int kN4[] = {2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 14, 16};   // ladder4.hip hdispatch cases

// pair positions the unrolled H code of ladder4.hip handles (its qmax4)
int qmax4(int n, int cap) { return std::min(std::min(4 * n + 8, cap - n + 1), 64); }

struct Group4Ctx {
    const SwsFilter &fh;
    const std::vector<int> &a, &z;   // first / last nonzero source sample per output
    int bps, nlmax, cap, N;
    int64_t row_bytes;
};

// Fits outputs [i0, i1) into one wave group: a 16-B aligned window whose
// sample pairs hold every output's taps, one output per start pair (earlier
// starts for outputs whose first taps coincide, e.g. at the left edge where
// initFilter folds taps onto sample 0; the window may begin left of the row,
// those chunks read as zero).  Fills h and p (start pair per output).
bool fit_group(const Group4Ctx &c, int i0, int i1, HGroup4 &h, std::vector<int> &p)
{
    const int64_t L = ((int64_t)c.a[i0] * c.bps) & ~(int64_t)15;
    for (int64_t pad = 0; pad <= 32; pad += 16) {
        const int64_t lofs = L - pad;
        const int X0 = (int)(lofs / c.bps);
        bool ok = true;
        for (int i = i1 - 1; i >= i0 && ok; --i) {
            if (c.a[i] < X0) {
                ok = false;
                break;
            }
            int pi = (c.a[i] - X0) >> 1;
            if (i + 1 < i1) pi = std::min(pi, p[i + 1] - 1);
            if (pi < 0 || ((c.z[i] - X0) >> 1) - pi + 1 > c.N) ok = false;
            p[i] = pi;
        }
        if (!ok) continue;
        const int last = p[i1 - 1];
        const int pairs = last + c.N;
        if (last + 1 > qmax4(c.N, c.cap) || pairs > c.cap) continue;
        if ((i1 - i0) * ((c.N + 3) & ~3) > kH4CoefDw) continue;          // the group's taps in LDS
        int64_t nload = ((int64_t)pairs * 2 * c.bps + 15) / 16;
        nload = std::min(nload, (c.row_bytes - lofs + 15) / 16);
        if (nload > c.nlmax || nload < 1) continue;
        h.lofs = (int32_t)lofs;
        h.nload = (int16_t)nload;
        h.qend = (int16_t)(last + 1);
        h.mask = 0;
        for (int i = i0; i < i1; ++i) h.mask |= 1ull << p[i];
        return true;
    }
    return false;
}

uint32_t pack_pair(int c0, int c1)
{
    return (uint32_t)(uint16_t)(int16_t)c0 | ((uint32_t)(uint16_t)(int16_t)c1 << 16);
}
} // namespace

bool plan4_kind(const SwsFilter &fh, const VTable &v, int srcH, int dstW, int dstH, int bps, int nlmax, int cap,
                int maxcols, int64_t row_bytes, int ring, Plan4 &out)
{
    if (v.nv < 1 || v.nv > 16 || v.nv > ring - 64 || dstW < 1 || dstH < 1) return false;
    if ((int64_t)dstW * bps > row_bytes) return false;      // horizontal upscale: v3
    std::vector<int> a(dstW), z(dstW), p(dstW);
    int nmin = 1;
    for (int i = 0; i < dstW; ++i) {
        int j0, j1;
        nonzero_extent(fh, i, j0, j1);
        a[i] = fh.pos[i] + j0;
        z[i] = fh.pos[i] + j1;
        nmin = std::max(nmin, (z[i] - (a[i] & ~1)) / 2 + 1);
    }
    // V: ring slots and the output rows each 64-pair step completes
    Plan4 base;
    base.NV = v.nv;
    const int pairs_total = (srcH + 1) / 2;
    base.nsteps = (pairs_total + 63) / 64;
    const int nvp = (v.nv + 3) & ~3;                          // LDS rows are 16-B aligned
    base.vslot.resize(dstH);
    for (int y = 0; y < dstH; ++y) base.vslot[y] = (v.pos[y] / 2) % ring;
    base.vcoef.assign((size_t)dstH * nvp, 0);
    for (int y = 0; y < dstH; ++y)
        for (int t = 0; t < v.nv; ++t) base.vcoef[(size_t)y * nvp + t] = v.coef[(size_t)y * v.nv + t];
    base.vlim.assign(base.nsteps, 0);
    {
        int y = 0;
        for (int b = 0; b < base.nsteps; ++b) {
            const int done = std::min(64 * (b + 1), pairs_total), y0 = y;
            while (y < dstH && std::min(v.pos[y] / 2 + v.nv, pairs_total) <= done) {
                if (v.pos[y] / 2 < 64 * (b + 1) - ring) return false;   // window left the ring
                ++y;
            }
            // the step's V taps and slots are staged in LDS
            if (y - y0 > kV4SlotMax || (y - y0) * nvp > kV4CoefDw) return false;
            base.vlim[b] = y;
        }
        if (y != dstH) return false;
    }
    // H: smallest tap-pair bucket, then the widest strip whose columns fit four wave groups
    for (int N : kN4) {
        if (N < nmin) continue;
        // outputs whose starts crowd into the same pair (ratios < 2, upscaling) are pushed to
        // earlier pairs at the price of wider windows; past 2 wasted tap pairs v3 is cheaper
        if (N > nmin + 2) break;
        const Group4Ctx c{fh, a, z, bps, nlmax, cap, N, row_bytes};
        for (int C = maxcols; C >= maxcols / 2; C -= 8) {   // narrower strips idle too many V lanes
            Plan4 pl = base;
            pl.N = N;
            pl.C = C;
            pl.nstrips = (dstW + C - 1) / C;
            bool ok = true;
            for (int s = 0; s < pl.nstrips && ok; ++s) {
                const int x0 = s * C, x1 = std::min(x0 + C, dstW);
                int i = x0;
                for (int g = 0; g < 4; ++g) {
                    HGroup4 h{};
                    h.col0 = i - x0;
                    h.coef = (int32_t)pl.hcoef.size();
                    const int rem = x1 - i;
                    if (rem > 0) {
                        int k = (rem + (3 - g)) / (4 - g);
                        while (k > 0 && !fit_group(c, i, i + k, h, p)) --k;
                        if (k == 0) {
                            ok = false;
                            break;
                        }
                        const int X0 = (int)(h.lofs / bps);
                        for (int o = i; o < i + k; ++o)
                            for (int t = 0; t < ((N + 3) & ~3); ++t) {    // rows of 16 B in LDS
                                const int x = X0 + 2 * (p[o] + t);
                                pl.hcoef.push_back(t < N ? pack_pair(tap_at(fh, o, x), tap_at(fh, o, x + 1)) : 0u);
                            }
                        i += k;
                    }
                    pl.groups.push_back(h);
                }
                if (i < x1) ok = false;
            }
            if (!ok) continue;
            out = std::move(pl);
            return true;
        }
    }
    return false;
}

bool plan_vlimits(const VTable &v, int srcH, int dstH, int ring_pairs, std::vector<int32_t> &vlim)
{
    const int srcHe = (srcH + 1) & ~1;
    const int nblocks = (srcHe + kBlkRows - 1) / kBlkRows;
    vlim.assign(nblocks, 0);
    int y = 0;
    for (int b = 0; b < nblocks; ++b) {
        const int done = std::min((b + 1) * kBlkRows, srcHe);
        while (y < dstH && std::min(v.pos[y] + 2 * v.nv, srcHe) <= done) {
            // the ring holds row pairs [done/2 - ring_pairs, done/2)
            if (v.pos[y] / 2 < done / 2 - ring_pairs) return false;
            ++y;
        }
        vlim[b] = y;
    }
    return y == dstH;
}

} // namespace dts
