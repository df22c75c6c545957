"""GPU parity at the BASELINE configs' real geometry, and the host path with
quality on over many batches (both pinned slots / streams in flight).

Integer outputs and SSE bit-exact against the oracle; SSIM within the
north-star 1e-4 (absolute).  All calls go through the C-ABI (libdts.so).
"""
import numpy as np
import pytest

import dtsffi as D
import orc
from _util import first_diff, planes_equal

pytestmark = pytest.mark.gpu
SSIM_TOL = 1e-4


def check_q(got, want):
    assert got["sse"] == want["sse"]
    for c in range(3):
        assert got["ssim"][c] == pytest.approx(want["ssim"][c], abs=SSIM_TOL)
    assert got["ssim_all"] == pytest.approx(want["ssim_all"], abs=SSIM_TOL)
    assert got["psnr_avg"] == pytest.approx(want["psnr_avg"], rel=1e-12)


def test_host_path_quality_many_batches(ctx):
    """nframes > 3 x max_batch with PSNR/SSIM on: consecutive chunks run on the
    two host-path streams at once, each with its own quality partials (ADVICE
    r01: they used to share one scratch buffer).  Every frame is checked."""
    sw, sh, w, h = 512, 288, 256, 144
    n, batch = 14, 4
    frames = [D.synth_host(sw, sh, D.FMT_YUV420P, 0, 5, f) for f in range(n)]
    # a different reference per frame, so swapped partials cannot go unnoticed
    refs = [D.synth_host(w, h, D.FMT_YUV420P, 1, 100 + f, 0) for f in range(n)]
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, [(w, h, D.FMT_YUV420P, D.SCALE_LANCZOS)],
                                 quality=D.Q_BOTH, quality_out=0, max_batch=batch))
    for _rep in range(2):                     # the second submit reuses both slots' buffers
        outs, qs = g.run_host(frames, qref=refs)
        for f in range(n):
            want_img = orc.scale_frame(frames[f], sw, sh, 0, w, h, 0, D.SCALE_LANCZOS)
            assert planes_equal(outs[f][0], want_img), first_diff(outs[f][0], want_img)
            check_q(qs[f], orc.quality_frame(w, h, want_img, refs[f]))
    g.close()


def test_cfg4_8k_to_4k_lanczos_quality(ctx):
    """BASELINE config 4 at full size: 8K yuv420p -> 4K lanczos + per-frame
    vf_psnr / vf_ssim of the output against a 4K reference rendition."""
    sw, sh, w, h = 7680, 4320, 3840, 2160
    frames = [D.synth_host(sw, sh, D.FMT_YUV420P, 0, 0x5EED, 0)]
    refs = [D.synth_host(w, h, D.FMT_YUV420P, 0, 0x0EF, 0)]
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, [(w, h, D.FMT_YUV420P, D.SCALE_LANCZOS)],
                                 quality=D.Q_BOTH, quality_out=0))
    outs, qs = g.run_host(frames, qref=refs)
    want_img = orc.scale_frame(frames[0], sw, sh, 0, w, h, 0, D.SCALE_LANCZOS)
    assert planes_equal(outs[0][0], want_img), first_diff(outs[0][0], want_img)
    check_q(qs[0], orc.quality_frame(w, h, want_img, refs[0]))
    g.close()


def test_cfg1_1080p_to_720p_bicubic(ctx):
    """BASELINE config 1's filter (the CPU-worker plumbing case): 1080p yuv420p
    -> 720p bicubic yuv420p (libx264 is host-side and absent; only the pixel
    path is checked)."""
    sw, sh = 1920, 1080
    frames = [D.synth_host(sw, sh, D.FMT_YUV420P, 0, 0x5EED, f) for f in range(2)]
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, [(1280, 720, D.FMT_YUV420P, D.SCALE_BICUBIC)]))
    outs, _ = g.run_host(frames)
    for f in range(2):
        want = orc.scale_frame(frames[f], sw, sh, 0, 1280, 720, 0, D.SCALE_BICUBIC)
        assert planes_equal(outs[f][0], want), first_diff(outs[f][0], want)
    g.close()


def test_cfg2_ladder_4k_host_path_two_frames(ctx):
    """BASELINE config 2 through the host path (pinned H2D, one fused launch, D2H)."""
    sw, sh = 3840, 2160
    outs = [(1920, 1080, D.FMT_NV12, D.SCALE_BICUBIC), (1280, 720, D.FMT_NV12, D.SCALE_BICUBIC),
            (854, 480, D.FMT_NV12, D.SCALE_BICUBIC)]
    frames = [D.synth_host(sw, sh, D.FMT_YUV420P, 0, 0x5EED, f) for f in (3, 4)]
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, outs))
    got, _ = g.run_host(frames)
    for f in range(2):
        for k, (w, h, fmt, m) in enumerate(outs):
            want = orc.scale_frame(frames[f], sw, sh, 0, w, h, fmt, m)
            assert planes_equal(got[f][k], want), f"frame {f} out {k}: {first_diff(got[f][k], want)}"
    g.close()


@pytest.mark.parametrize("pin_src,pin_out", [(True, 16), (True, False), (False, 1), ("perm", 16)])
def test_host_path_pinned_frames(ctx, pin_src, pin_out):
    """ABI 7: frames in dts_host_alloc memory go to / come from the device by DMA straight
    from / into the caller's planes (no pass through the pinned rings); every combination
    of pinned and pageable sources / outputs over several chunks is bit-exact; with pinned
    outputs packed at their row bytes (pin_out 1) the 86 x 48 rendition's 86-byte rows differ
    from the device layout's 96-byte pitch, so that rendition goes through the ring and the
    others straight into the caller's frames.  Consecutive frames of one alloc_frames_pinned
    buffer cross as one DMA per run; "perm" hands the pinned frames over out of buffer order,
    so runs break (single frames by plane, a two-frame run at the end)."""
    sw, sh, n, batch = 384, 216, 7, 3
    outs_spec = [(192, 108, D.FMT_NV12, D.SCALE_BICUBIC), (128, 72, D.FMT_YUV420P, D.SCALE_LANCZOS),
                 (86, 48, D.FMT_NV12, D.SCALE_BICUBIC)]
    frames = [D.synth_host(sw, sh, D.FMT_YUV420P, 0, 77, f) for f in range(n)]
    keep = None
    if pin_src:
        pf, keep = D.alloc_frames_pinned(sw, sh, D.FMT_YUV420P, n)
        for a, b in zip(pf, frames):
            for pa, pb in zip(a, b):
                if pa is not None:
                    pa[...] = pb
        frames = pf
        if pin_src == "perm":
            frames = [pf[i] for i in (1, 0, 2, 4, 3, 5, 6)]
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, outs_spec, max_batch=batch))
    for _rep in range(2):
        outs, _ = g.run_host(frames, pinned_out=pin_out)
        for f in range(n):
            for k, (w, h, fmt, m) in enumerate(outs_spec):
                want = orc.scale_frame(frames[f], sw, sh, D.FMT_YUV420P, w, h, fmt, m)
                assert planes_equal(outs[f][k], want), f"frame {f} out {k}: {first_diff(outs[f][k], want)}"
    g.close()
    del keep


def test_pinned_outputs_outlive_the_next_call(ctx):
    """Pinned outputs of one run_host call stay valid after later pinned calls and after the
    PinnedBuffer object itself is dropped: every plane view keeps its allocation alive (ADVICE
    r05: the second call used to free the first call's buffers under the caller's views)."""
    import gc
    sw, sh, n = 256, 144, 3
    spec = [(128, 72, D.FMT_NV12, D.SCALE_BICUBIC), (64, 36, D.FMT_YUV420P, D.SCALE_BILINEAR)]
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, spec, max_batch=2))
    runs = []
    for seed in (5, 6, 7):
        frames = [D.synth_host(sw, sh, D.FMT_YUV420P, 0, seed, f) for f in range(n)]
        outs, _ = g.run_host(frames, pinned_out=True)
        runs.append((frames, outs))
        gc.collect()
    g.close()
    for frames, outs in runs:
        for f in range(n):
            for k, (w, h, fmt, m) in enumerate(spec):
                want = orc.scale_frame(frames[f], sw, sh, D.FMT_YUV420P, w, h, fmt, m)
                assert planes_equal(outs[f][k], want), (f, k)
    frames, buf = D.alloc_frames_pinned(64, 36, D.FMT_YUV420P, 2)
    del buf
    gc.collect()
    frames[1][0][...] = 9                       # the allocation is still there
    assert int(frames[1][0].sum()) == 9 * 64 * 36


def test_host_register_roundtrip(ctx):
    """dts_host_register / dts_host_unregister a caller range; frees of unknown pointers are
    ignored and a double unregister is an error."""
    import ctypes
    buf = np.zeros(1 << 20, np.uint8)
    L = D.lib()
    assert L.dts_host_register(ctypes.c_void_p(buf.ctypes.data), buf.nbytes) == 0
    assert L.dts_host_unregister(ctypes.c_void_p(buf.ctypes.data)) == 0
    assert L.dts_host_unregister(ctypes.c_void_p(buf.ctypes.data)) == D.E_INVAL
    L.dts_host_free(ctypes.c_void_p(buf.ctypes.data))          # not the library's: ignored
    p = D.PinnedBuffer(4096)
    p.array[:] = 7
    assert int(p.array.sum()) == 7 * 4096
    # overlapping ranges are refused (one record per pinned byte): inside an allocation, across
    # a registered range's start or end, and the same base twice
    assert L.dts_host_register(ctypes.c_void_p(p.ptr + 1024), 1024) == D.E_INVAL
    base = buf.ctypes.data
    assert L.dts_host_register(ctypes.c_void_p(base + 65536), 65536) == 0
    assert L.dts_host_register(ctypes.c_void_p(base + 65536), 4096) == D.E_INVAL
    assert L.dts_host_register(ctypes.c_void_p(base), 65536 + 1) == D.E_INVAL
    assert L.dts_host_register(ctypes.c_void_p(base + 65536 + 4096), 65536) == D.E_INVAL
    assert L.dts_host_register(ctypes.c_void_p(base), 65536) == 0          # adjacent: fine
    assert L.dts_host_unregister(ctypes.c_void_p(base)) == 0
    assert L.dts_host_unregister(ctypes.c_void_p(base + 65536)) == 0
    assert int(p.array.sum()) == 7 * 4096                                   # (the allocation untouched)
