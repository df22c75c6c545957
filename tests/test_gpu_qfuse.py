"""vf_psnr / vf_ssim fused into k_ladder7's V epilogue (ladder7.hip qrb7 + qfuse.hip k_qfix7 /
k_qfin7) against the separate k_quality pass over the same outputs and references
(dts_quality_run_device), and against the oracle (orc.quality_frame) on some frames.

SSE exact; SSIM window sums within 1e-6 per window of the separate pass (both sum f32
ssim_end1 values in f64, in different orders) and within 1e-4 of the oracle per frame.
Covers the three ways a graph asks for quality: external per-rendition references
(DTS_QREF_EXTERNAL, the cfg5 bench path), references the graph makes itself (ABI 6
qref_method = lanczos) and the graph's quality_out against one reference batch (cfg4);
widths that are not multiples of 16 / 4 (854 -> 427 chroma), heights not multiples of 16,
several batches per call, yuv420p and nv12 outputs and sources."""
import ctypes

import numpy as np
import pytest

import dtsffi as D
import orc

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fused(monkeypatch):
    """graphs made in these tests plan the fused path (DTS_QFUSE=1)"""
    monkeypatch.setenv("DTS_QFUSE", "1")

QREF_EXTERNAL = D.QREF_EXTERNAL
SSIM_TOL = 1e-4


def _sub(d, i0):
    e = D.DevFrames()
    for p in range(3):
        e.data[p] = (d.data[p] or 0) + i0 * d.frame_stride if d.data[p] else None
        e.pitch[p] = d.pitch[p]
    e.frame_stride = d.frame_stride
    return e


def _qraws(t, n, off=0):
    host = t.cpu().numpy()
    out = []
    for i in range(off, off + n):
        r = D.QRaw()
        ctypes.memmove(ctypes.addressof(r), host[i].tobytes(), ctypes.sizeof(r))
        out.append(r)
    return out


def _batch(w, h, fmt, n):
    import torch
    from bench import dev_batch, frame_bytes
    t = torch.zeros((n, frame_bytes(w, h, fmt)), dtype=torch.uint8, device="cuda")   # (row padding compared too)
    return t, dev_batch(t, w, h, fmt)[0]


def _nwin(w, h):
    pw = [w, (w + 1) // 2, (w + 1) // 2]
    ph = [h, (h + 1) // 2, (h + 1) // 2]
    return [max(0, ((pw[c] >> 2) - 1) * ((ph[c] >> 2) - 1)) for c in range(3)]


def _check_vs_separate(ctx, outs, refs, qraw, n, stride, stream):
    """each rendition k with a record: its fused records (qraw rows k * stride + f) vs k_quality's"""
    import torch
    for k, ((w, h, fmt), od, rd) in enumerate(outs):
        if rd is None:
            continue
        sep = torch.zeros((n, 6), dtype=torch.float64, device="cuda")
        ctx.quality_device(w, h, fmt, od, rd, n, sep.data_ptr(), stream)
        torch.cuda.synchronize()
        a, b = _qraws(qraw, n, k * stride), _qraws(sep, n)
        nw = _nwin(w, h)
        for f in range(n):
            for c in range(3):
                assert a[f].sse[c] == b[f].sse[c], (k, f, c, a[f].sse[c], b[f].sse[c])
                assert a[f].ssim_sum[c] == pytest.approx(b[f].ssim_sum[c], abs=1e-6 * max(nw[c], 1)), (k, f, c)


@pytest.mark.parametrize("sw,sh,sfmt,outs,nframes,batch", [
    (3840, 2160, D.FMT_YUV420P, [(1920, 1080, D.FMT_NV12), (1280, 720, D.FMT_NV12), (854, 480, D.FMT_NV12)], 5, 2),
    (1920, 1080, D.FMT_YUV420P, [(1280, 720, D.FMT_YUV420P), (854, 480, D.FMT_YUV420P), (640, 360, D.FMT_NV12)], 3, 8),
    (1920, 1080, D.FMT_NV12, [(960, 540, D.FMT_NV12), (426, 240, D.FMT_YUV420P)], 4, 3),
    (1280, 720, D.FMT_YUV420P, [(1280, 720, D.FMT_NV12), (636, 356, D.FMT_YUV420P)], 2, 2),
])
def test_fused_external_refs(ctx, sw, sh, sfmt, outs, nframes, batch):
    """DTS_QREF_EXTERNAL: every rendition scored against a batch the caller passes (the
    lanczos renditions of the same source here); records k * nframes + f"""
    import torch
    stream = torch.cuda.current_stream().cuda_stream
    _st, sd = _batch(sw, sh, sfmt, nframes)
    ctx.synth_device(sw, sh, sfmt, 0, 0x5EED, 7, sd, nframes, stream)
    spec_o = [(w, h, f, D.SCALE_BICUBIC, None, (D.Q_BOTH, QREF_EXTERNAL)) for (w, h, f) in outs]
    g = D.Graph(ctx, D.make_spec(sw, sh, sfmt, spec_o, max_batch=batch))
    rg = D.Graph(ctx, D.make_spec(sw, sh, sfmt, [(w, h, f, D.SCALE_LANCZOS) for (w, h, f) in outs], max_batch=batch))
    ob = [_batch(w, h, f, nframes) for (w, h, f) in outs]
    rb = [_batch(w, h, f, nframes) for (w, h, f) in outs]
    rg.run_device(sd, nframes, [d for (_t, d) in rb], stream=stream)
    qraw = torch.zeros((len(outs) * nframes, 6), dtype=torch.float64, device="cuda")
    g.run_device(sd, nframes, [d for (_t, d) in ob], qref=[d for (_t, d) in rb], qraw_ptr=qraw.data_ptr(),
                 stream=stream)
    torch.cuda.synchronize()
    _check_vs_separate(ctx, [(o, ob[k][1], rb[k][1]) for k, o in enumerate(outs)], None, qraw, nframes, nframes,
                       stream)
    # frame 0 of every rendition vs the oracle
    from bench import unpack_dev_frame
    for k, (w, h, fmt) in enumerate(outs):
        o = unpack_dev_frame(ob[k][0][0].cpu().numpy(), w, h, fmt)
        r = unpack_dev_frame(rb[k][0][0].cpu().numpy(), w, h, fmt)
        pl = (lambda p: [p[0], np.ascontiguousarray(p[1][:, 0::2]), np.ascontiguousarray(p[1][:, 1::2])]) \
            if fmt == D.FMT_NV12 else (lambda p: p)
        want = orc.quality_frame(w, h, pl(o), pl(r))
        gq = D.qstat_finalize(w, h, _qraws(qraw, 1, k * nframes))[0]
        assert gq["sse"] == want["sse"], k
        assert gq["ssim_all"] == pytest.approx(want["ssim_all"], abs=SSIM_TOL), k
    g.close()
    rg.close()


def test_fused_internal_refs_and_unfused_fallback(ctx, monkeypatch):
    """ABI 6 rendition quality (the graph makes lanczos references): fused records equal the
    DTS_QFUSE=0 graph's (separate k_quality pass) -- SSE exact, SSIM sums 1e-6 per window"""
    import torch
    stream = torch.cuda.current_stream().cuda_stream
    sw, sh, n = 3840, 2160, 3
    outs = [(1920, 1080, D.FMT_NV12), (854, 480, D.FMT_NV12)]
    _st, sd = _batch(sw, sh, D.FMT_YUV420P, n)
    ctx.synth_device(sw, sh, D.FMT_YUV420P, 0, 0x5EED, 3, sd, n, stream)
    spec = D.make_spec(sw, sh, D.FMT_YUV420P,
                       [(w, h, f, D.SCALE_BICUBIC, None, (D.Q_BOTH, D.SCALE_LANCZOS)) for (w, h, f) in outs],
                       max_batch=2)
    res = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("DTS_QFUSE", fuse)
        g = D.Graph(ctx, spec)
        ob = [_batch(w, h, f, n) for (w, h, f) in outs]
        qraw = torch.zeros((len(outs) * n, 6), dtype=torch.float64, device="cuda")
        g.run_device(sd, n, [d for (_t, d) in ob], qraw_ptr=qraw.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        res.append((qraw, [t.cpu() for (t, _d) in ob]))
        g.close()
    monkeypatch.setenv("DTS_QFUSE", "1")
    for k in range(len(outs)):
        assert torch.equal(res[0][1][k], res[1][1][k])       # the same renditions
    a, b = _qraws(res[0][0], len(outs) * n), _qraws(res[1][0], len(outs) * n)
    for i in range(len(outs) * n):
        nw = _nwin(*outs[i // n][:2])
        for c in range(3):
            assert a[i].sse[c] == b[i].sse[c], (i, c)
            assert a[i].ssim_sum[c] == pytest.approx(b[i].ssim_sum[c], abs=1e-6 * nw[c]), (i, c)


def test_fused_graph_quality_out(ctx):
    """cfg4's shape: one rendition (8K -> 4K lanczos), quality_out against one reference frame
    reused for every frame (frame_stride 0): records f"""
    import torch
    stream = torch.cuda.current_stream().cuda_stream
    sw, sh, n = 7680, 4320, 2
    w, h, fmt = 3840, 2160, D.FMT_YUV420P
    _st, sd = _batch(sw, sh, D.FMT_YUV420P, n)
    ctx.synth_device(sw, sh, D.FMT_YUV420P, 0, 0x5EED, 0, sd, n, stream)
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, [(w, h, fmt, D.SCALE_LANCZOS)], quality=D.Q_BOTH,
                                 max_batch=n))
    ot, od = _batch(w, h, fmt, n)
    rt, rd = _batch(w, h, fmt, 1)
    rd.frame_stride = 0
    ctx.synth_device(w, h, fmt, 0, 0x0EF, 0, rd, 1, stream)
    qraw = torch.zeros((n, 6), dtype=torch.float64, device="cuda")
    g.run_device(sd, n, [od], qref=rd, qraw_ptr=qraw.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    _check_vs_separate(ctx, [((w, h, fmt), od, rd)], None, qraw, n, 0, stream)
    g.close()
