"""GPU parity on exactly the paths bench.py times (BASELINE configs 2-5), at full size.

Each test drives dts_graph_run_device the way bench.py's step() does -- the same graph
specs, device-resident batches laid out by bench.dev_batch, the same reference plumbing
-- and checks every frame against the CPU oracle:
- cfg2: the 4K -> 1080p/720p/480p nv12 ladder, two launches of three frames, and one
  launch of 20 frames (frame quads 0-2 of k_ladder7's frame map on every XCD slot);
- cfg3: 4K p010 HDR10 -> 1080p SDR on the device path with more frames than one
  ladder -> tonemap chunk (max_batch 4, 9 frames: three chunks, both p010
  intermediates reused), vf_tonemap defaults;
- cfg4: 8K -> 4K lanczos with graph quality, every frame scored against its own 4K
  reference frame (bench's reference ring), two launches;
- cfg5: the ladder with every rendition scored against an external reference batch
  (DTS_QREF_EXTERNAL: the lanczos renditions, made by a second graph as bench does),
  two launches, records output-major.
Tolerances: integer outputs and SSE bit-exact, SSIM within 1e-4 (absolute), the HDR
float path within +-1 LSB with at most 1 % of samples off by one.
"""
import ctypes

import numpy as np
import pytest

import dtsffi as D
import orc
from _util import first_diff, planes_equal

pytestmark = pytest.mark.gpu
SSIM_TOL = 1e-4
LADDER = [(1920, 1080, D.FMT_NV12, D.SCALE_BICUBIC), (1280, 720, D.FMT_NV12, D.SCALE_BICUBIC),
          (854, 480, D.FMT_NV12, D.SCALE_BICUBIC)]


def _ring(w, h, fmt, n):
    import torch
    from bench import dev_batch, frame_bytes
    t = torch.zeros((n, frame_bytes(w, h, fmt)), dtype=torch.uint8, device="cuda")
    return t, dev_batch(t, w, h, fmt)[0]


def _at(d, i0):
    e = D.DevFrames()
    for p in range(3):
        e.data[p] = d.data[p] + i0 * d.frame_stride if d.data[p] else None
        e.pitch[p] = d.pitch[p]
    e.frame_stride = d.frame_stride
    return e


def _frame(t, i, w, h, fmt):
    from bench import unpack_dev_frame
    return unpack_dev_frame(t[i].cpu().numpy(), w, h, fmt)


def _qraws(t, rows):
    host = t.cpu().numpy()
    out = []
    for i in rows:
        r = D.QRaw()
        ctypes.memmove(ctypes.addressof(r), host[i].tobytes(), ctypes.sizeof(r))
        out.append(r)
    return out


def _planar(p, fmt):
    if fmt != D.FMT_NV12:
        return p
    return [p[0], np.ascontiguousarray(p[1][:, 0::2]), np.ascontiguousarray(p[1][:, 1::2])]


def _check_q(got, want, what):
    assert got["sse"] == want["sse"], what
    for c in range(3):
        assert got["ssim"][c] == pytest.approx(want["ssim"][c], abs=SSIM_TOL), (what, c)
    assert got["ssim_all"] == pytest.approx(want["ssim_all"], abs=SSIM_TOL), what


def test_cfg2_device_path_two_launches(ctx):
    import torch
    st = torch.cuda.current_stream().cuda_stream
    sw, sh, n, first = 3840, 2160, 3, 40
    _s, sd = _ring(sw, sh, D.FMT_YUV420P, 2 * n)
    ctx.synth_device(sw, sh, D.FMT_YUV420P, 0, 0x5EED, first, sd, 2 * n, st)
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, LADDER, max_batch=n))
    assert g.info.ladder_v5 == 3, "cfg2 runs on k_ladder7"
    outs = [_ring(w, h, fmt, n) for (w, h, fmt, _m) in LADDER]
    for step in range(2):
        g.run_device(_at(sd, step * n), n, [d for (_t, d) in outs], stream=st)
        torch.cuda.synchronize()
        for f in range(n):
            src = D.synth_host(sw, sh, D.FMT_YUV420P, 0, 0x5EED, first + step * n + f)
            for k, (w, h, fmt, m) in enumerate(LADDER):
                got = _frame(outs[k][0], f, w, h, fmt)
                want = orc.scale_frame(src, sw, sh, D.FMT_YUV420P, w, h, fmt, m)
                assert planes_equal(got, want), f"step {step} frame {f} out {k}: {first_diff(got, want)}"
    g.close()


def test_cfg2_device_path_full_frame_quads(ctx):
    """The headline launch shape at 4K: one launch of 20 frames, so k_ladder7's frame map
    (frame 8 fq + b % 8, ladder7.hip k_ladder7) reaches fq = 2 on all 8 XCD slots, the last
    quad partly filled; every frame of every rendition against the oracle."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from bench import unpack_dev_frame
    st = torch.cuda.current_stream().cuda_stream
    sw, sh, n, first = 3840, 2160, 20, 1000
    _s, sd = _ring(sw, sh, D.FMT_YUV420P, n)
    ctx.synth_device(sw, sh, D.FMT_YUV420P, 0, 0x5EED, first, sd, n, st)
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, LADDER, max_batch=n))
    assert g.info.ladder_v5 == 3, "cfg2 runs on k_ladder7"
    outs = [_ring(w, h, fmt, n) for (w, h, fmt, _m) in LADDER]
    g.run_device(sd, n, [d for (_t, d) in outs], stream=st)
    torch.cuda.synchronize()
    host = [t.cpu().numpy() for (t, _d) in outs]

    def check(f):
        src = D.synth_host(sw, sh, D.FMT_YUV420P, 0, 0x5EED, first + f)
        bad = []
        for k, (w, h, fmt, m) in enumerate(LADDER):
            got = unpack_dev_frame(host[k][f], w, h, fmt)
            want = orc.scale_frame(src, sw, sh, D.FMT_YUV420P, w, h, fmt, m)
            if not planes_equal(got, want):
                bad.append(f"frame {f} out {k}: {first_diff(got, want)}")
        return bad
    with ThreadPoolExecutor(8) as ex:
        bad = [b for r in ex.map(check, range(n)) for b in r]
    assert not bad, bad[:4]
    g.close()


def test_cfg3_device_path_multi_chunk(ctx):
    """More frames than one ladder -> tonemap chunk on the device path bench times."""
    import torch
    st = torch.cuda.current_stream().cuda_stream
    sw, sh, n, batch = 3840, 2160, 9, 4
    w, h, fmt = 1920, 1080, D.FMT_YUV420P
    tm = {"mode": D.TM_HABLE, "desat": 2.0, "peak": 0.0, "npl": 100.0}
    _s, sd = _ring(sw, sh, D.FMT_P010LE, n)
    ctx.synth_device(sw, sh, D.FMT_P010LE, 0, 0x5EED, 11, sd, n, st)
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_P010LE, [(w, h, fmt, D.SCALE_BICUBIC)], max_batch=batch,
                                 tonemap=tm))
    ot, od = _ring(w, h, fmt, n)
    g.run_device(sd, n, [od], stream=st)
    torch.cuda.synchronize()
    for f in range(n):
        src = D.synth_host(sw, sh, D.FMT_P010LE, 0, 0x5EED, 11 + f)
        mid = orc.scale_frame(src, sw, sh, D.FMT_P010LE, w, h, D.FMT_P010LE, D.SCALE_BICUBIC)
        want = orc.hdr_to_sdr(mid, w, h, fmt, D.TM_HABLE, float("nan"), 2.0, 0.0, 100.0)
        got = _frame(ot, f, w, h, fmt)
        nbad = ntot = 0
        for a, b in zip(got, want):
            d = np.abs(np.asarray(a).astype(np.int16) - np.asarray(b).astype(np.int16))
            assert d.max() <= 1, f"frame {f}: max diff {d.max()}"
            nbad += int((d > 0).sum())
            ntot += d.size
        assert nbad <= 0.01 * ntot, f"frame {f}: {nbad}/{ntot} samples off by one"
    g.close()


def test_cfg4_device_path_per_frame_references(ctx):
    """Every frame against its own reference (bench's reference ring), two launches."""
    import torch
    st = torch.cuda.current_stream().cuda_stream
    sw, sh, w, h, n = 7680, 4320, 3840, 2160, 2
    _s, sd = _ring(sw, sh, D.FMT_YUV420P, 2 * n)
    ctx.synth_device(sw, sh, D.FMT_YUV420P, 0, 0x5EED, 0, sd, 2 * n, st)
    _r, rd = _ring(w, h, D.FMT_YUV420P, 2 * n)
    ctx.synth_device(w, h, D.FMT_YUV420P, 0, 0x0EF, 0, rd, 2 * n, st)
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, [(w, h, D.FMT_YUV420P, D.SCALE_LANCZOS)],
                                 quality=D.Q_BOTH, max_batch=n))
    ot, od = _ring(w, h, D.FMT_YUV420P, n)
    qraw = torch.zeros((n, 6), dtype=torch.float64, device="cuda")
    for step in range(2):
        qraw.zero_()
        g.run_device(_at(sd, step * n), n, [od], qref=_at(rd, step * n), qraw_ptr=qraw.data_ptr(), stream=st)
        torch.cuda.synchronize()
        got_q = D.qstat_finalize(w, h, _qraws(qraw, range(n)))
        for f in range(n):
            i = step * n + f
            src = D.synth_host(sw, sh, D.FMT_YUV420P, 0, 0x5EED, i)
            ref = D.synth_host(w, h, D.FMT_YUV420P, 0, 0x0EF, i)
            want = orc.scale_frame(src, sw, sh, D.FMT_YUV420P, w, h, D.FMT_YUV420P, D.SCALE_LANCZOS)
            got = _frame(ot, f, w, h, D.FMT_YUV420P)
            assert planes_equal(got, want), f"frame {i}: {first_diff(got, want)}"
            _check_q(got_q[f], orc.quality_frame(w, h, want, ref), f"frame {i}")
    g.close()


def test_cfg5_device_path_external_references(ctx):
    """bench.py cfg5: DTS_QREF_EXTERNAL renditions, references from a lanczos graph, records
    k * nframes + f; two launches over different source batches."""
    import torch
    st = torch.cuda.current_stream().cuda_stream
    sw, sh, n = 3840, 2160, 3
    _s, sd = _ring(sw, sh, D.FMT_YUV420P, 2 * n)
    ctx.synth_device(sw, sh, D.FMT_YUV420P, 0, 0x5EED, 500, sd, 2 * n, st)
    gouts = [(w, h, fmt, m, None, (D.Q_BOTH, D.QREF_EXTERNAL)) for (w, h, fmt, m) in LADDER]
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, gouts, max_batch=n))
    qg = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, [(w, h, fmt, D.SCALE_LANCZOS) for (w, h, fmt, _m) in LADDER],
                                  max_batch=2 * n))
    refs = [_ring(w, h, fmt, 2 * n) for (w, h, fmt, _m) in LADDER]
    qg.run_device(sd, 2 * n, [d for (_t, d) in refs], stream=st)
    outs = [_ring(w, h, fmt, n) for (w, h, fmt, _m) in LADDER]
    qall = torch.zeros((len(LADDER) * n, 6), dtype=torch.float64, device="cuda")
    for step in range(2):
        qall.zero_()
        g.run_device(_at(sd, step * n), n, [d for (_t, d) in outs], qref=[_at(d, step * n) for (_t, d) in refs],
                     qraw_ptr=qall.data_ptr(), stream=st)
        torch.cuda.synchronize()
        for f in range(n):
            i = step * n + f
            src = D.synth_host(sw, sh, D.FMT_YUV420P, 0, 0x5EED, 500 + i)
            for k, (w, h, fmt, m) in enumerate(LADDER):
                want = orc.scale_frame(src, sw, sh, D.FMT_YUV420P, w, h, fmt, m)
                ref = orc.scale_frame(src, sw, sh, D.FMT_YUV420P, w, h, fmt, D.SCALE_LANCZOS)
                got = _frame(outs[k][0], f, w, h, fmt)
                assert planes_equal(got, want), f"frame {i} out {k}: {first_diff(got, want)}"
                assert planes_equal(_frame(refs[k][0], i, w, h, fmt), ref), f"reference {i} out {k}"
                gq = D.qstat_finalize(w, h, _qraws(qall, [k * n + f]))[0]
                _check_q(gq, orc.quality_frame(w, h, _planar(want, fmt), _planar(ref, fmt)), f"frame {i} out {k}")
    g.close()
    qg.close()


def test_external_references_refused_on_host_path(ctx):
    """The host path cannot take external reference batches: dts_graph_submit refuses the
    graph instead of returning records it never computed."""
    g = D.Graph(ctx, D.make_spec(128, 72, D.FMT_YUV420P,
                                 [(64, 36, D.FMT_YUV420P, D.SCALE_BICUBIC, None, (D.Q_BOTH, D.QREF_EXTERNAL))]))
    frames = [D.synth_host(128, 72, D.FMT_YUV420P, 0, 1, 0)]
    with pytest.raises(D.DtsError) as e:
        g.run_host(frames)
    assert e.value.code == D.E_UNSUPPORTED
    g.close()
