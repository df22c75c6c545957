"""GPU parity: the HIP ladder (scale + format convert) vs the CPU oracle.

Bit-exact for every method (the GPU consumes the same integer tables the
libswscale C path builds; the oracle restates that path).  Calls go through
the C-ABI (libdts.so).  Oracle parity vs libswscale itself is unpinned: see
DESIGN.md "Oracle".
"""
import numpy as np
import pytest

import dtsffi as D
import orc
from _util import first_diff, oracle_frame, planes_equal, random_frame

pytestmark = pytest.mark.gpu

BIC, BIL, LAN = D.SCALE_BICUBIC, D.SCALE_BILINEAR, D.SCALE_LANCZOS


KERNELS = ["v7", "v5", "v4", "v3"]


@pytest.fixture(autouse=True)
def _default_kernel(monkeypatch):
    """Every case runs on the library's own kernel choice: k_ladder7 wherever the graph fits
    it and the planes are 16-byte aligned; k_ladder5 for 8-bit sources it does not plan (the
    odd sizes below: plane widths not multiples of 16), k_ladder4 / the v3 kernel for such
    p010 sources.  The fallbacks on geometries k_ladder7 would take are forced (DTS_LADDER)
    only in the `ladder_kernel` tests."""
    monkeypatch.delenv("DTS_LADDER", raising=False)


@pytest.fixture(params=KERNELS)
def ladder_kernel(request, monkeypatch):
    """The default choice (v7), DTS_LADDER=5 (v5 where it fits), DTS_LADDER=4 (v4 where the
    geometry fits it, else v3) and DTS_LADDER=3 (v3 for every plane)."""
    if request.param == "v7":
        monkeypatch.delenv("DTS_LADDER", raising=False)
    else:
        monkeypatch.setenv("DTS_LADDER", request.param[1])
    return request.param


def run_and_check(ctx, sw, sh, sfmt, outs, frames):
    g = D.Graph(ctx, D.make_spec(sw, sh, sfmt, outs))
    got, _ = g.run_host(frames)
    for f, src in enumerate(frames):
        for k, o in enumerate(outs):
            want = oracle_frame(src, sw, sh, sfmt, o[0], o[1], o[2], o[3], o[4] if len(o) > 4 else
                                (D.PARAM_DEFAULT, D.PARAM_DEFAULT))
            assert planes_equal(got[f][k], want), f"frame {f} out {k} {o}: {first_diff(got[f][k], want)}"
    g.close()


@pytest.mark.parametrize("method", [BIC, BIL, LAN])
def test_ladder_small(ctx, method):
    """4K-ladder shape at 1/10 scale: 384x216 -> 192x108 / 128x72 / 86x48 nv12."""
    frames = [D.synth_host(384, 216, D.FMT_YUV420P, 0, 0x5EED, f) for f in range(3)]
    outs = [(192, 108, D.FMT_NV12, method), (128, 72, D.FMT_NV12, method), (86, 48, D.FMT_NV12, method)]
    run_and_check(ctx, 384, 216, D.FMT_YUV420P, outs, frames)


@pytest.mark.parametrize("sw,sh,dw,dh", [(37, 23, 19, 11), (64, 36, 32, 18), (100, 60, 150, 90),
                                         (333, 211, 97, 55), (640, 360, 1280, 720), (1000, 8, 300, 5),
                                         (17, 300, 40, 41)])
@pytest.mark.parametrize("method", [BIC, BIL, LAN, D.SCALE_POINT, D.SCALE_AREA, D.SCALE_GAUSS])
def test_odd_sizes_random(ctx, sw, sh, dw, dh, method):
    rng = np.random.default_rng(sw * 1000 + dh + method)
    frames = [random_frame(sw, sh, D.FMT_YUV420P, rng) for _ in range(2)]
    run_and_check(ctx, sw, sh, D.FMT_YUV420P, [(dw, dh, D.FMT_YUV420P, method), (dw, dh, D.FMT_NV12, method)],
                  frames)


@pytest.mark.parametrize("sfmt", [D.FMT_NV12, D.FMT_P010LE])
@pytest.mark.parametrize("method", [BIC, LAN, BIL])
def test_semiplanar_sources(ctx, sfmt, method):
    rng = np.random.default_rng(7 + sfmt)
    frames = [random_frame(258, 146, sfmt, rng), D.synth_host(258, 146, sfmt, 0, 3, 5)]
    run_and_check(ctx, 258, 146, sfmt, [(130, 74, D.FMT_NV12, method), (97, 51, D.FMT_YUV420P, method),
                                        (258, 146, D.FMT_YUV420P, method)], frames)


def test_same_size_identity(ctx):
    """1:1 luma is the identity, yuv420p -> nv12 is a lossless interleave."""
    rng = np.random.default_rng(1)
    src = random_frame(130, 66, D.FMT_YUV420P, rng)
    g = D.Graph(ctx, D.make_spec(130, 66, D.FMT_YUV420P, [(130, 66, D.FMT_NV12, BIC)]))
    (out,), _ = g.run_host([src])
    out = out[0]
    assert np.array_equal(out[0], src[0])
    assert np.array_equal(out[1][:, 0::2], src[1]) and np.array_equal(out[1][:, 1::2], src[2])


def test_params_bicubic_b_c(ctx):
    frames = [D.synth_host(200, 120, D.FMT_YUV420P, 1, 11, 0)]
    run_and_check(ctx, 200, 120, D.FMT_YUV420P, [(90, 50, D.FMT_NV12, BIC, (1 / 3, 1 / 3)),
                                                 (90, 50, D.FMT_NV12, LAN, (2.0, D.PARAM_DEFAULT))], frames)


def test_ladder_4k_one_frame(ctx, ladder_kernel):
    """BASELINE config 2 geometry at full size, one frame, bit-exact."""
    frames = [D.synth_host(3840, 2160, D.FMT_YUV420P, 0, 0x5EED, 0)]
    outs = [(1920, 1080, D.FMT_NV12, BIC), (1280, 720, D.FMT_NV12, BIC), (854, 480, D.FMT_NV12, BIC)]
    g = D.Graph(ctx, D.make_spec(3840, 2160, D.FMT_YUV420P, outs))
    assert g.info.ladder_v5 == {"v7": 3, "v5": 1}.get(ladder_kernel, 0)
    assert g.info.ladder_v4_mask == (0x3f if ladder_kernel == "v4" else 0)
    g.close()
    run_and_check(ctx, 3840, 2160, D.FMT_YUV420P, outs, frames)


@pytest.mark.parametrize("sfmt", [D.FMT_YUV420P, D.FMT_NV12, D.FMT_P010LE])
@pytest.mark.parametrize("method", [BIC, LAN, BIL, D.SCALE_GAUSS])
def test_downscales_every_source(ctx, sfmt, method):
    """Downscale ratios 1.5 .. 5 from every source format, odd output sizes (the
    v4 kernel's domain: strips, wave groups, left-edge folded taps, ring wrap)."""
    rng = np.random.default_rng(11 + sfmt + method)
    frames = [random_frame(520, 300, sfmt, rng), D.synth_host(520, 300, sfmt, 0, 5, 2)]
    run_and_check(ctx, 520, 300, sfmt, [(346, 200, D.FMT_NV12, method), (260, 150, D.FMT_YUV420P, method),
                                        (171, 97, D.FMT_NV12, method), (104, 60, D.FMT_NV12, method)], frames)


def test_p010_4k_to_1080p(ctx):
    """BASELINE config 3 geometry (scale/convert part): 4K p010 -> 1080p yuv420p with ordered dither."""
    frames = [D.synth_host(3840, 2160, D.FMT_P010LE, 0, 0x5EED, 0)]
    run_and_check(ctx, 3840, 2160, D.FMT_P010LE, [(1920, 1080, D.FMT_YUV420P, BIC)], frames)


def test_many_frames_batches(ctx):
    """More frames than one batch; both pinned slots cycle."""
    frames = [D.synth_host(160, 90, D.FMT_YUV420P, 0, 9, f) for f in range(11)]
    g = D.Graph(ctx, D.make_spec(160, 90, D.FMT_YUV420P, [(80, 46, D.FMT_NV12, BIC)], max_batch=4))
    got, _ = g.run_host(frames)
    for f, src in enumerate(frames):
        want = oracle_frame(src, 160, 90, D.FMT_YUV420P, 80, 46, D.FMT_NV12, BIC)
        assert planes_equal(got[f][0], want), first_diff(got[f][0], want)


@pytest.mark.parametrize("n,w,h", [(5, 640, 360), (77, 192, 108)])
def test_device_path_matches_host_path(ctx, n, w, h):
    """dts_graph_run_device on torch-allocated HBM == the oracle.  77 frames
    (>= 64) exercise the per-XCD work queues (frame f in queue f % 8)."""
    import torch
    outs = [(w // 2, h // 2, D.FMT_NV12, BIC), ((w // 3 + 3) // 4 * 4, h // 3, D.FMT_NV12, BIC)]
    g = D.Graph(ctx, D.make_spec(w, h, D.FMT_YUV420P, outs))
    src = torch.empty((n, h * w + 2 * ((w + 1) // 2) * ((h + 1) // 2) + 64), dtype=torch.uint8, device="cuda")
    fstride = src.stride(0)
    assert fstride % 16 == 0
    base = src.data_ptr()
    cw, ch = (w + 1) // 2, (h + 1) // 2
    sf = D.DevFrames()
    sf.data[0], sf.data[1], sf.data[2] = base, base + h * w, base + h * w + cw * ch
    sf.pitch[0], sf.pitch[1], sf.pitch[2] = w, cw, cw
    sf.frame_stride = fstride
    # plane offsets and pitches are multiples of 16 for these geometries
    ctx.synth_device(w, h, D.FMT_YUV420P, 0, 42, 0, sf, n, torch.cuda.current_stream().cuda_stream)
    dsts, bufs = [], []
    for (ow, oh, of, _m) in outs:
        size = ow * oh + 2 * ((ow + 1) // 2) * ((oh + 1) // 2)
        b = torch.empty((n, size + 60), dtype=torch.uint8, device="cuda")
        d = D.DevFrames()
        d.data[0], d.data[1], d.data[2] = b.data_ptr(), b.data_ptr() + ow * oh, 0
        d.pitch[0], d.pitch[1], d.pitch[2] = ow, 2 * ((ow + 1) // 2), 0
        d.frame_stride = b.stride(0)
        dsts.append(d)
        bufs.append(b)
    g.run_device(sf, n, dsts, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for f in range(n):
        host_src = D.synth_host(w, h, D.FMT_YUV420P, 0, 42, f)
        got_src = src[f].cpu().numpy()
        assert np.array_equal(got_src[:h * w].reshape(h, w), host_src[0]), "device synth != host synth"
        for k, (ow, oh, of, m) in enumerate(outs):
            raw = bufs[k][f].cpu().numpy()
            y = raw[:ow * oh].reshape(oh, ow)
            uv = raw[ow * oh: ow * oh + 2 * ((ow + 1) // 2) * ((oh + 1) // 2)].reshape((oh + 1) // 2, -1)
            want = oracle_frame(host_src, w, h, D.FMT_YUV420P, ow, oh, of, m)
            assert planes_equal([y, uv, None], want), first_diff([y, uv, None], want)


@pytest.mark.parametrize("pad", [0, 4, 1])
def test_device_path_plane_alignment(ctx, pad):
    """dts_graph_run_device takes source planes on 16-byte boundaries (k_ladder7 stages
    rows with 16-byte LDS-DMA lanes; include/dts.h): pitches padded by 0 run bit-exact,
    pitches padded by 4 or 1 are refused with DTS_E_INVAL before any launch."""
    import torch
    n, w, h = 3, 320, 180
    outs = [(160, 90, D.FMT_NV12, BIC), (104, 60, D.FMT_YUV420P, BIC)]
    g = D.Graph(ctx, D.make_spec(w, h, D.FMT_YUV420P, outs))
    cw, ch = (w + 1) // 2, (h + 1) // 2
    pl, pc = w + pad, cw + pad
    size = pl * h + 2 * pc * ch
    src = torch.zeros((n, (size + 64 + 15) // 16 * 16), dtype=torch.uint8, device="cuda")
    host = [D.synth_host(w, h, D.FMT_YUV420P, 0, 7, f) for f in range(n)]
    for f in range(n):
        buf = np.zeros(src.shape[1], np.uint8)
        for p_, (off, pitch, rows) in enumerate([(0, pl, h), (pl * h, pc, ch), (pl * h + pc * ch, pc, ch)]):
            plane = host[f][p_]
            for y in range(rows):
                buf[off + y * pitch: off + y * pitch + plane.shape[1]] = plane[y]
        src[f].copy_(torch.from_numpy(buf))
    base = src.data_ptr()
    sf = D.DevFrames()
    sf.data[0], sf.data[1], sf.data[2] = base, base + pl * h, base + pl * h + pc * ch
    sf.pitch[0], sf.pitch[1], sf.pitch[2] = pl, pc, pc
    sf.frame_stride = src.stride(0)
    dsts, bufs = [], []
    for (ow, oh, of, _m) in outs:
        ocw, och = (ow + 1) // 2, (oh + 1) // 2
        b = torch.zeros((n, ow * oh + 2 * ocw * och + 64), dtype=torch.uint8, device="cuda")
        d = D.DevFrames()
        d.data[0], d.data[1] = b.data_ptr(), b.data_ptr() + ow * oh
        d.data[2] = 0 if of == D.FMT_NV12 else b.data_ptr() + ow * oh + ocw * och
        d.pitch[0], d.pitch[1], d.pitch[2] = ow, 2 * ocw if of == D.FMT_NV12 else ocw, 0 if of == D.FMT_NV12 else ocw
        d.frame_stride = b.stride(0)
        dsts.append(d)
        bufs.append(b)
    if pad:
        with pytest.raises(D.DtsError):
            g.run_device(sf, n, dsts, stream=torch.cuda.current_stream().cuda_stream)
        return
    g.run_device(sf, n, dsts, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for f in range(n):
        for k, (ow, oh, of, m) in enumerate(outs):
            raw = bufs[k][f].cpu().numpy()
            ocw, och = (ow + 1) // 2, (oh + 1) // 2
            y = raw[:ow * oh].reshape(oh, ow)
            if of == D.FMT_NV12:
                got = [y, raw[ow * oh: ow * oh + 2 * ocw * och].reshape(och, 2 * ocw), None]
            else:
                got = [y, raw[ow * oh: ow * oh + ocw * och].reshape(och, ocw),
                       raw[ow * oh + ocw * och: ow * oh + 2 * ocw * och].reshape(och, ocw)]
            want = oracle_frame(host[f], w, h, D.FMT_YUV420P, ow, oh, of, m)
            assert planes_equal(got, want), f"pad {pad} frame {f} out {k}: {first_diff(got, want)}"


V7_GEOMS = [
    (128, 18, [(64, 9), (128, 18)]),                  # one granule row (chroma: 9 rows), 1:1 rendition
    (256, 48, [(400, 90), (128, 24)]),                # upscale (several row blocks per granule) + 2:1
    (1024, 16, [(512, 8), (341, 5)]),                 # a single source granule
    (256, 1000, [(64, 900), (128, 250)]),             # tall: mild vertical, 4:1 / 2:1 horizontal
    (4096, 64, [(1024, 16), (2730, 40)]),             # wide: many groups, 1.5:1
    (640, 480, [(640, 480), (320, 240), (214, 160)]),  # 1:1 + ladder
]


@pytest.mark.parametrize("sw,sh,outs", V7_GEOMS)
@pytest.mark.parametrize("method", [BIC, LAN, BIL, D.SCALE_AREA])
def test_v7_geometries(ctx, sw, sh, outs, method):
    """Plane widths that are multiples of 16 (k_ladder7's domain): single-granule
    planes, upscales, tall / wide planes, 1:1 renditions; nv12 and yuv420p outputs,
    bit-exact vs the oracle."""
    rng = np.random.default_rng(sw + 7 * sh + method)
    frames = [random_frame(sw, sh, D.FMT_YUV420P, rng), D.synth_host(sw, sh, D.FMT_YUV420P, 0, 5, 3)]
    run_and_check(ctx, sw, sh, D.FMT_YUV420P,
                  [(w, h, D.FMT_NV12 if k % 2 == 0 else D.FMT_YUV420P, method) for k, (w, h) in enumerate(outs)],
                  frames)


@pytest.mark.parametrize("kernel", ["v7", "v5"])
@pytest.mark.parametrize("src_range,dst_range", [(0, 1), (1, 0)])
@pytest.mark.parametrize("method", [BIC, LAN, BIL])
@pytest.mark.parametrize("sfmt", [D.FMT_YUV420P, D.FMT_NV12, D.FMT_P010LE])
def test_range_conversion(ctx, monkeypatch, kernel, src_range, dst_range, method, sfmt):
    """`scale=in_range:out_range`: swscale.c's lum/chrRange{To,From}Jpeg_c on the
    15-bit H output, in k_ladder7's H epilogue, bit-exact vs the oracle (random and
    full-swing frames, nv12 and yuv420p renditions; planar, nv12 and p010 sources -- nv12
    chroma de-interleaved in the A reads; p010 sources (round 5) through the same 15-bit
    converters, since every rendition has dstBpc <= 14).  Other kernels refuse it."""
    sw, sh = 384, 216
    outs = [(192, 108, D.FMT_NV12, method), (128, 72, D.FMT_YUV420P, method), (384, 216, D.FMT_NV12, method)]
    if sfmt == D.FMT_P010LE:                  # renditions k_ladder7's p010 walks plan (else k_ladder4: refused)
        outs = [(192, 108, D.FMT_NV12, method), (160, 90, D.FMT_YUV420P, method), (256, 144, D.FMT_P010LE, method)]
    spec = D.make_spec(sw, sh, sfmt, outs, src_range=src_range, dst_range=dst_range)
    if kernel != "v7":
        monkeypatch.setenv("DTS_LADDER", kernel[1])
        with pytest.raises(D.DtsError):
            D.Graph(ctx, spec)
        return
    rng = np.random.default_rng(17 + src_range + method)
    swing = [np.where((np.arange(sw)[None, :] // 3) % 2 == 0, 255, 0).astype(np.uint8).repeat(sh, 0),
             np.full((sh // 2, sw // 2), 255, np.uint8), np.zeros((sh // 2, sw // 2), np.uint8)]
    frames = [random_frame(sw, sh, D.FMT_YUV420P, rng), D.synth_host(sw, sh, D.FMT_YUV420P, 0, 3, 1), swing]
    if sfmt == D.FMT_NV12:                    # the same pictures, chroma interleaved
        frames = [[f[0], np.ascontiguousarray(np.stack([f[1], f[2]], -1).reshape(f[1].shape[0], -1)), None]
                  for f in frames]
    if sfmt == D.FMT_P010LE:                  # the same pictures as 10-bit codes (x 4, and random low bits)
        def p010(f):
            w16 = lambda a: (a.astype(np.uint16) << 8) | rng.integers(0, 256, a.shape, dtype=np.uint16)
            uv = np.stack([w16(f[1]), w16(f[2])], -1).reshape(f[1].shape[0], -1)
            return [w16(f[0]).view(np.uint8), np.ascontiguousarray(uv).view(np.uint8), None]
        frames = [p010(f) for f in frames]
    g = D.Graph(ctx, spec)
    got, _ = g.run_host(frames)
    for f, src in enumerate(frames):
        for k, (w, h, fmt, m) in enumerate(outs):
            want = orc.scale_frame(src, sw, sh, sfmt, w, h, fmt, m, src_range=src_range, dst_range=dst_range)
            assert planes_equal(got[f][k], want), f"frame {f} out {k}: {first_diff(got[f][k], want)}"
    g.close()


@pytest.mark.parametrize("method", [BIC, LAN, D.SCALE_GAUSS])
def test_clip_stress(ctx, method):
    """Patterns that drive the 15-bit horizontal clip (FFMIN(val >> 7, 32767)) and the
    u8 output clip at both ends: bright samples on the positive lobes, black on the
    negative ones, plus single-pixel spikes."""
    w, h = 256, 64
    y = np.zeros((h, w), np.uint8)
    y[:, 1::4] = 255
    y[:, 2::4] = 255
    y[::7, ::5] = 255
    y[3::9] = 0
    u = np.full(((h + 1) // 2, (w + 1) // 2), 255, np.uint8)
    u[:, ::3] = 0
    v = np.zeros_like(u)
    v[::2] = 255
    frames = [[y, u, v], [255 - y, 255 - u, 255 - v]]
    run_and_check(ctx, w, h, D.FMT_YUV420P, [(128, 32, D.FMT_NV12, method), (85, 21, D.FMT_YUV420P, method),
                                             (300, 70, D.FMT_NV12, method)], frames)


# A cross-section of the cases above on every kernel (the fallbacks forced onto geometries
# k_ladder7 would take: what a device batch whose planes are not 16-byte aligned runs on)
FALLBACK_CASES = [
    ("ladder", 384, 216, D.FMT_YUV420P, [(192, 108, D.FMT_NV12, BIC), (128, 72, D.FMT_NV12, BIC),
                                         (86, 48, D.FMT_NV12, BIC)]),
    ("lanczos-up", 100, 60, D.FMT_YUV420P, [(150, 90, D.FMT_YUV420P, LAN), (150, 90, D.FMT_NV12, LAN)]),
    ("odd", 333, 211, D.FMT_YUV420P, [(97, 55, D.FMT_YUV420P, D.SCALE_AREA), (97, 55, D.FMT_NV12, BIL)]),
    ("nv12", 258, 146, D.FMT_NV12, [(130, 74, D.FMT_NV12, LAN), (97, 51, D.FMT_YUV420P, BIC)]),
    ("p010", 258, 146, D.FMT_P010LE, [(130, 74, D.FMT_NV12, BIC), (258, 146, D.FMT_YUV420P, LAN)]),
    ("downscale", 520, 300, D.FMT_YUV420P, [(346, 200, D.FMT_NV12, D.SCALE_GAUSS), (171, 97, D.FMT_NV12, BIC),
                                            (104, 60, D.FMT_NV12, BIL)]),
    ("tall", 256, 1000, D.FMT_YUV420P, [(64, 900, D.FMT_NV12, BIC), (128, 250, D.FMT_YUV420P, LAN)]),
]


@pytest.mark.parametrize("case", FALLBACK_CASES, ids=[c[0] for c in FALLBACK_CASES])
def test_fallback_kernels(ctx, ladder_kernel, case):
    _name, sw, sh, sfmt, outs = case
    rng = np.random.default_rng(sw + sh + sfmt)
    frames = [random_frame(sw, sh, sfmt, rng), D.synth_host(sw, sh, sfmt, 0, 0x5EED, 1)]
    run_and_check(ctx, sw, sh, sfmt, outs, frames)


def test_many_batches_device_queue(ctx):
    """Persistent grid + work queue across several launches with different frame counts."""
    outs = [(96, 54, D.FMT_NV12, BIC), (64, 36, D.FMT_NV12, BIC)]
    g = D.Graph(ctx, D.make_spec(192, 108, D.FMT_YUV420P, outs, max_batch=3))
    for n in (1, 7, 3):
        frames = [D.synth_host(192, 108, D.FMT_YUV420P, 0, 77, 100 * n + f) for f in range(n)]
        got, _ = g.run_host(frames)
        for f in range(n):
            for k, o in enumerate(outs):
                want = oracle_frame(frames[f], 192, 108, D.FMT_YUV420P, *o)
                assert planes_equal(got[f][k], want), first_diff(got[f][k], want)
