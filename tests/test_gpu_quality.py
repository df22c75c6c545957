"""GPU parity: vf_psnr / vf_ssim kernels vs the CPU oracle.

SSE (hence MSE/PSNR) is integer-exact.  SSIM: per-window values are the same
f32 expression as vf_ssim.c; only the summation order differs (f64 on the
GPU), so the tolerance is the north-star 1e-4 (absolute on SSIM).
"""
import numpy as np
import pytest

import dtsffi as D
import orc
from _util import random_frame, planes_equal

pytestmark = pytest.mark.gpu
SSIM_TOL = 1e-4


def check_q(got, want):
    assert got["sse"] == want["sse"]
    for c in range(3):
        if np.isnan(want["ssim"][c]):
            assert np.isnan(got["ssim"][c])
            continue
        assert got["ssim"][c] == pytest.approx(want["ssim"][c], abs=SSIM_TOL)
        if np.isinf(want["psnr"][c]):
            assert np.isinf(got["psnr"][c])
        else:
            assert got["psnr"][c] == pytest.approx(want["psnr"][c], rel=1e-12)
    if not np.isnan(want["ssim_all"]):
        assert got["ssim_all"] == pytest.approx(want["ssim_all"], abs=SSIM_TOL)


# 64x260 / 128x520: a plane whose last block row is the apron row of a whole walk
# ((h >> 2) - 1 a multiple of 4 tiles x 16 block rows; 128x520 hits it in the chroma)
@pytest.mark.parametrize("w,h", [(64, 36), (37, 23), (258, 146), (1001, 67), (8, 8), (4, 4), (64, 260), (128, 520),
                                 (66, 1030)])
def test_quality_vs_oracle(ctx, w, h):
    import torch
    rng = np.random.default_rng(w * h)
    fr_a = [random_frame(w, h, D.FMT_YUV420P, rng) for _ in range(3)]
    fr_b = [[np.clip(p.astype(np.int16) + rng.integers(-6, 7, p.shape), 0, 255).astype(np.uint8) for p in f]
            for f in fr_a]
    fr_b[1] = [p.copy() for p in fr_a[1]]          # identical frame -> inf PSNR, SSIM 1
    got = gpu_quality(ctx, w, h, fr_a, fr_b, torch)
    for i in range(3):
        want = orc.quality_frame(w, h, fr_a[i], fr_b[i])
        check_q(got[i], want)
    if w >= 16 and h >= 16:       # chroma planes of >= 8x8 have SSIM windows
        assert got[1]["ssim_all"] == pytest.approx(1.0, abs=1e-12)


def gpu_quality(ctx, w, h, fa, fb, torch):
    n = len(fa)
    cw, ch = (w + 1) // 2, (h + 1) // 2
    pitch = [(w + 15) // 16 * 16, (cw + 15) // 16 * 16, (cw + 15) // 16 * 16]
    rows = [h, ch, ch]
    offs = [0, pitch[0] * h, pitch[0] * h + pitch[1] * ch]
    fsz = offs[2] + pitch[2] * ch

    def upload(frames):
        host = np.zeros((n, fsz), np.uint8)
        for f, planes in enumerate(frames):
            for p in range(3):
                img = host[f, offs[p]:offs[p] + pitch[p] * rows[p]].reshape(rows[p], pitch[p])
                img[:, :planes[p].shape[1]] = planes[p]
        t = torch.from_numpy(host).cuda()
        d = D.DevFrames()
        for p in range(3):
            d.data[p] = t.data_ptr() + offs[p]
            d.pitch[p] = pitch[p]
        d.frame_stride = fsz
        return t, d
    ta, da = upload(fa)
    tb, db = upload(fb)
    raw = torch.zeros((n, 6), dtype=torch.float64, device="cuda")   # 6 x 8 bytes = dts_qraw
    ctx.quality_device(w, h, D.FMT_YUV420P, da, db, n, raw.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    host = raw.cpu().numpy()
    recs = []
    for i in range(n):
        r = D.QRaw()
        b = host[i].tobytes()
        import ctypes
        ctypes.memmove(ctypes.addressof(r), b, ctypes.sizeof(r))
        recs.append(r)
    return D.qstat_finalize(w, h, recs)


def test_graph_quality_host_path(ctx):
    """cfg-4 shape at small scale: lanczos 2:1 + PSNR/SSIM vs a reference rendition."""
    sw, sh, w, h = 512, 288, 256, 144
    frames = [D.synth_host(sw, sh, D.FMT_YUV420P, 0, 5, f) for f in range(4)]
    ref = [orc.scale_frame(f, sw, sh, 0, w, h, 0, D.SCALE_BICUBIC) for f in frames]
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, [(w, h, D.FMT_YUV420P, D.SCALE_LANCZOS)],
                                 quality=D.Q_BOTH, quality_out=0))
    outs, qs = g.run_host(frames, qref=ref)
    for f in range(4):
        want_img = orc.scale_frame(frames[f], sw, sh, 0, w, h, 0, D.SCALE_LANCZOS)
        assert planes_equal(outs[f][0], want_img)
        check_q(qs[f], orc.quality_frame(w, h, want_img, ref[f]))


@pytest.mark.parametrize("w,h", [(64, 36), (130, 74), (854, 480), (64, 260), (128, 520)])
def test_quality_nv12_vs_oracle(ctx, w, h):
    """nv12 batches (cfg5's renditions): the kernel reads U / V from the interleaved
    plane; vf_psnr / vf_ssim take planar yuv420p, so the oracle gets the
    de-interleaved planes (the conversion ffmpeg inserts in front of them)."""
    import ctypes
    import torch
    rng = np.random.default_rng(w + h)
    fr_a = [random_frame(w, h, D.FMT_YUV420P, rng) for _ in range(2)]
    fr_b = [[np.clip(p.astype(np.int16) + rng.integers(-9, 10, p.shape), 0, 255).astype(np.uint8) for p in f]
            for f in fr_a]
    cw, ch = (w + 1) // 2, (h + 1) // 2
    py, puv = (w + 15) // 16 * 16, (2 * cw + 15) // 16 * 16
    fsz = py * h + puv * ch

    def upload(frames):
        host = np.zeros((len(frames), fsz), np.uint8)
        for f, (y, u, v) in enumerate(frames):
            host[f, :py * h].reshape(h, py)[:, :w] = y
            uv = host[f, py * h:].reshape(ch, puv)
            uv[:, 0:2 * cw:2] = u
            uv[:, 1:2 * cw:2] = v
        t = torch.from_numpy(host).cuda()
        d = D.DevFrames()
        d.data[0], d.pitch[0] = t.data_ptr(), py
        d.data[1], d.pitch[1] = t.data_ptr() + py * h, puv
        d.data[2], d.pitch[2] = None, 0
        d.frame_stride = fsz
        return t, d
    ta, da = upload(fr_a)
    tb, db = upload(fr_b)
    raw = torch.zeros((2, 6), dtype=torch.float64, device="cuda")
    ctx.quality_device(w, h, D.FMT_NV12, da, db, 2, raw.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    host = raw.cpu().numpy()
    for i in range(2):
        r = D.QRaw()
        ctypes.memmove(ctypes.addressof(r), host[i].tobytes(), ctypes.sizeof(r))
        got = D.qstat_finalize(w, h, [r])[0]
        check_q(got, orc.quality_frame(w, h, fr_a[i], fr_b[i]))


@pytest.mark.parametrize("fmt", [D.FMT_YUV420P, D.FMT_NV12])
def test_quality_host_entry_vs_oracle(ctx, fmt):
    """dts_quality_run_host (the Node worker's per-rendition quality): host frames of
    either 8-bit 4:2:0 layout against the oracle on the planar planes."""
    w, h = 130, 74
    src = [D.synth_host(2 * w, 2 * h, D.FMT_YUV420P, 0, 9, f) for f in range(3)]
    a = [orc.scale_frame(f, 2 * w, 2 * h, 0, w, h, fmt, D.SCALE_BICUBIC) for f in src]
    b = [orc.scale_frame(f, 2 * w, 2 * h, 0, w, h, fmt, D.SCALE_LANCZOS) for f in src]
    got = ctx.quality_host(w, h, fmt, a, b)

    def planar(p):
        if fmt != D.FMT_NV12:
            return p
        return [p[0], np.ascontiguousarray(p[1][:, 0::2]), np.ascontiguousarray(p[1][:, 1::2])]
    for i in range(3):
        check_q(got[i], orc.quality_frame(w, h, planar(a[i]), planar(b[i])))


@pytest.mark.parametrize("deint", [None, (0, 1)])
def test_graph_rendition_quality_host_path(ctx, deint):
    """Rendition quality (dts_output_spec.quality, ABI 6): the graph scales every rendition
    and, for the ones that ask, a lanczos reference of the same size from the same source
    frames, and scores them on the device -- the Node worker's per-segment quality with no
    rendition crossing PCIe twice.  More frames than max_batch (both host slots), mixed
    formats, one output without quality; with deint the references are made from the
    deinterlaced frames.  Every frame: SSE exact, SSIM 1e-4 vs the oracle."""
    sw, sh, n, batch = 384, 216, 7, 3
    src = [D.synth_host(sw, sh, D.FMT_YUV420P, 0, 21, f) for f in range(n + (2 if deint else 0))]
    outs = [(192, 108, D.FMT_NV12, D.SCALE_BICUBIC, None, (D.Q_BOTH, D.SCALE_LANCZOS)),
            (128, 72, D.FMT_YUV420P, D.SCALE_BILINEAR),
            (96, 54, D.FMT_YUV420P, D.SCALE_BICUBIC, None, (D.Q_PSNR, D.SCALE_BILINEAR))]
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, outs, max_batch=batch, deint=deint))
    got, qs = g.run_host(src)
    assert len(qs) == n and all(len(row) == 3 for row in qs)
    for f in range(n):
        frame = src[f + 1] if deint else src[f]
        if deint:
            frame = orc.yadif_frame(src[f], src[f + 1], src[f + 2], sw, sh, deint[0], deint[1], 0)
        for k, o in enumerate(outs):
            want = orc.scale_frame(frame, sw, sh, D.FMT_YUV420P, o[0], o[1], o[2], o[3])
            assert planes_equal(got[f][k], want), (f, k)
            if len(o) < 6:
                assert qs[f][k] is None
                continue
            ref = orc.scale_frame(frame, sw, sh, D.FMT_YUV420P, o[0], o[1], o[2], o[5][1])
            pl = (lambda p: [p[0], np.ascontiguousarray(p[1][:, 0::2]), np.ascontiguousarray(p[1][:, 1::2])]) \
                if o[2] == D.FMT_NV12 else (lambda p: p)
            check_q(qs[f][k], orc.quality_frame(o[0], o[1], pl(want), pl(ref)))
    g.close()


def test_graph_rendition_quality_device_path(ctx):
    """The same on the device path: qraw receives nframes x nout records, output-major."""
    import torch
    from bench import dev_batch, frame_bytes
    sw, sh, n = 512, 288, 5
    outs = [(256, 144, D.FMT_NV12, D.SCALE_BICUBIC, None, (D.Q_BOTH, D.SCALE_LANCZOS)),
            (170, 96, D.FMT_NV12, D.SCALE_BICUBIC, None, (D.Q_BOTH, D.SCALE_LANCZOS))]
    st = torch.cuda.current_stream().cuda_stream
    t = torch.empty((n, frame_bytes(sw, sh, D.FMT_YUV420P)), dtype=torch.uint8, device="cuda")
    sd, _ = dev_batch(t, sw, sh, D.FMT_YUV420P)
    ctx.synth_device(sw, sh, D.FMT_YUV420P, 0, 33, 0, sd, n, st)
    dts = []
    for o in outs:
        ot = torch.empty((n, frame_bytes(o[0], o[1], o[2])), dtype=torch.uint8, device="cuda")
        dts.append((ot, dev_batch(ot, o[0], o[1], o[2])[0]))
    raw = torch.zeros((len(outs) * n, 6), dtype=torch.float64, device="cuda")
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, outs, max_batch=2))
    g.run_device(sd, n, [d for (_t, d) in dts], qraw_ptr=raw.data_ptr(), stream=st)
    torch.cuda.synchronize()
    import ctypes
    host = raw.cpu().numpy()
    for k, o in enumerate(outs):
        recs = []
        for f in range(n):
            r = D.QRaw()
            ctypes.memmove(ctypes.addressof(r), host[k * n + f].tobytes(), ctypes.sizeof(r))
            recs.append(r)
        got = D.qstat_finalize(o[0], o[1], recs)
        for f in range(n):
            frame = D.synth_host(sw, sh, D.FMT_YUV420P, 0, 33, f)
            a = orc.scale_frame(frame, sw, sh, 0, o[0], o[1], o[2], o[3])
            b = orc.scale_frame(frame, sw, sh, 0, o[0], o[1], o[2], D.SCALE_LANCZOS)
            pl = lambda p: [p[0], np.ascontiguousarray(p[1][:, 0::2]), np.ascontiguousarray(p[1][:, 1::2])]
            check_q(got[f], orc.quality_frame(o[0], o[1], pl(a), pl(b)))
    g.close()
