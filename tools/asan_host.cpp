// asan_host.cpp -- host-only C-ABI calls under AddressSanitizer / UBSan (no GPU needed):
// dts_graph_plan over a grid of graph specs (sizes down to 2x2 and up to 8K, every source /
// output format, scale method, quality, tonemap, deinterlace and range combination the ABI
// accepts or refuses), dts_sws_filter, dts_fps_map, dts_frame_layout, dts_synth_host and the
// quality-record finishers.  Built and run by tools/asan_host.sh against a library whose host
// objects carry -fsanitize=address,undefined (the device code is the ordinary build).
// Exit status 0 = every call returned and the sanitizers stayed quiet.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../include/dts.h"

static int g_calls = 0, g_ok = 0;

static void plan(int sw, int sh, int sfmt, const std::vector<dts_output_spec> &outs, int batch, int quality,
                 const dts_tonemap_spec *tm, int deint, int range)
{
    dts_graph_spec s;
    std::memset(&s, 0, sizeof s);
    s.src_w = sw;
    s.src_h = sh;
    s.src_fmt = sfmt;
    s.nout = (int)outs.size();
    for (size_t k = 0; k < outs.size() && k < DTS_MAX_OUTPUTS; ++k) s.out[k] = outs[k];
    s.max_batch = batch;
    s.quality = quality;
    if (tm) {
        s.tonemap = *tm;
        s.hdr_to_sdr = 1;
    }
    s.deint = deint != 0;
    s.deint_mode = deint == 2 ? 2 : 0;
    s.deint_tff = 1;
    s.range = range;
    dts_graph_info info;
    std::memset(&info, 0, sizeof info);
    const int e = dts_graph_plan(&s, &info);
    ++g_calls;
    if (e == DTS_OK) ++g_ok;
}

int main()
{
    std::printf("%s\n", dts_version());
    const int fmts[3] = {DTS_FMT_YUV420P, DTS_FMT_NV12, DTS_FMT_P010LE};
    const int methods[] = {DTS_SCALE_BILINEAR, DTS_SCALE_BICUBIC, DTS_SCALE_LANCZOS, DTS_SCALE_POINT,
                           DTS_SCALE_AREA, DTS_SCALE_GAUSS, DTS_SCALE_SINC};
    const int sizes[][2] = {{2, 2},     {4, 2},     {16, 6},     {66, 34},   {130, 71},  {640, 360},
                            {854, 480}, {1280, 720}, {1920, 1080}, {3840, 2160}, {7680, 4320}};
    dts_tonemap_spec tm;
    std::memset(&tm, 0, sizeof tm);
    tm.mode = DTS_TM_HABLE;
    tm.param = __builtin_nan("");
    tm.desat = 2.0;
    tm.npl = 100.0;
    for (auto &sz : sizes)
        for (int sf : fmts)
            for (auto &dz : sizes) {
                if (dz[0] > 2 * sz[0] + 64 || dz[1] > 2 * sz[1] + 64) continue;   // keep the grid to ladders
                for (int of : fmts)
                    for (int m : methods) {
                        dts_output_spec o;
                        std::memset(&o, 0, sizeof o);
                        o.w = dz[0];
                        o.h = dz[1];
                        o.fmt = of;
                        o.method = m;
                        o.param[0] = o.param[1] = DTS_PARAM_DEFAULT;
                        plan(sz[0], sz[1], sf, {o}, 4, DTS_Q_NONE, nullptr, 0, 0);
                        if (m == DTS_SCALE_BICUBIC) {
                            plan(sz[0], sz[1], sf, {o}, 64, DTS_Q_BOTH, nullptr, 0, 0);
                            plan(sz[0], sz[1], sf, {o, o, o}, 16, DTS_Q_NONE, nullptr, 2, 0);
                            plan(sz[0], sz[1], sf, {o}, 8, DTS_Q_NONE, nullptr, 0, DTS_RANGE_JPEG);
                            plan(sz[0], sz[1], sf, {o}, 8, DTS_Q_NONE, &tm, 0, 0);
                            dts_output_spec q = o;
                            q.quality = DTS_Q_BOTH;
                            q.qref_method = DTS_QREF_EXTERNAL;
                            plan(sz[0], sz[1], sf, {q, o}, 8, DTS_Q_NONE, nullptr, 0, 0);
                        }
                    }
            }
    // the cfg2 ladder and a full DTS_MAX_OUTPUTS ladder
    {
        std::vector<dts_output_spec> L;
        const int ws[][2] = {{1920, 1080}, {1280, 720}, {854, 480}, {640, 360}, {426, 240}, {256, 144}, {3840, 2160}, {2560, 1440}};
        for (int k = 0; k < DTS_MAX_OUTPUTS && k < 8; ++k) {
            dts_output_spec o;
            std::memset(&o, 0, sizeof o);
            o.w = ws[k][0];
            o.h = ws[k][1];
            o.fmt = DTS_FMT_NV12;
            o.method = DTS_SCALE_BICUBIC;
            o.param[0] = o.param[1] = DTS_PARAM_DEFAULT;
            L.push_back(o);
            plan(3840, 2160, DTS_FMT_YUV420P, L, 512, DTS_Q_NONE, nullptr, 0, 0);
        }
    }
    // refusals: zero / negative sizes, too many outputs, bad formats
    plan(0, 0, DTS_FMT_YUV420P, {}, 1, 0, nullptr, 0, 0);
    plan(-4, 8, 99, {}, 0, 0, nullptr, 0, 0);
    // filters, fps maps, layouts, synthetic frames, quality finishers
    const int cap = 512;
    std::vector<int16_t> coeff((size_t)4320 * cap);
    std::vector<int32_t> pos(4320);
    const double prm[2] = {DTS_PARAM_DEFAULT, DTS_PARAM_DEFAULT};
    for (int sn : {1, 2, 3, 17, 720, 1080, 2160, 4320})
        for (int dn : {1, 2, 5, 240, 480, 1080, 4320})
            for (int m : methods) {
                dts_sws_filter(sn, dn, 1 << 14, 1, m, prm, 0, coeff.data(), pos.data(), cap);
                dts_sws_filter(sn, dn, 1 << 12, 1, m, prm, 128, coeff.data(), pos.data(), cap);
                ++g_calls;
            }
    std::vector<int64_t> map(4096);
    for (int64_t n : {0, 1, 7, 600, 4000}) {
        dts_fps_map(n, 60000, 1001, 30, 1, map.data(), (int64_t)map.size());
        dts_fps_map(n, 25, 1, 60, 1, map.data(), (int64_t)map.size());
        g_calls += 2;
    }
    for (auto &sz : sizes)
        for (int f : fmts) {
            int64_t pitch[3], rows[3], fbytes = 0;
            dts_frame_layout(sz[0], sz[1], f, pitch, rows, &fbytes);
            if (sz[0] * sz[1] <= 1920 * 1080 && fbytes > 0) {
                std::vector<uint8_t> buf((size_t)fbytes);
                dts_frame fr;
                std::memset(&fr, 0, sizeof fr);
                uint8_t *p = buf.data();
                for (int pl = 0; pl < 3; ++pl) {
                    if (!rows[pl]) continue;
                    fr.data[pl] = p;
                    fr.pitch[pl] = pitch[pl];
                    p += pitch[pl] * rows[pl];
                }
                dts_synth_host(sz[0], sz[1], f, 0, 0x5EEDu, 3, &fr);
            }
            g_calls += 2;
        }
    std::vector<dts_qraw> raw(5);
    std::memset(raw.data(), 0, raw.size() * sizeof(dts_qraw));
    for (int i = 0; i < 5; ++i)
        for (int c = 0; c < 3; ++c) {
            raw[i].sse[c] = (uint64_t)(i * 1000 + c);
            raw[i].ssim_sum[c] = 10.0 * i + c;
        }
    std::vector<dts_qstat> st(5);
    dts_qstat_finalize(1920, 1080, raw.data(), 5, st.data());
    dts_qstat one;
    dts_qstat_stream(1920, 1080, &raw[0], 5, &one);
    dts_qstat_finalize(2, 2, raw.data(), 1, st.data());
    g_calls += 3;
    std::printf("asan_host: %d calls, %d graph plans accepted\n", g_calls, g_ok);
    return 0;
}
