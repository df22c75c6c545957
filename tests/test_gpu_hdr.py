"""GPU parity for p010 output and the HDR10 -> SDR path
(row a11, BASELINE config 3).

- p010 output (output.c yuv2p010lX_c / yuv2p010cX_c): bit-exact vs the oracle,
  on both ladder kernels, from every source format.
- HDR10 -> SDR: the ladder scales bit-exactly into a p010 intermediate, then
  the float tone-map kernel converts it.  Tolerance (north star, float path):
  every output sample within +-1 LSB of the double-precision restatement
  (oracle/vf_tonemap_ref.c) and at most 1 % of samples off by one.  Parity of
  that restatement vs zimg/ffmpeg is unpinned (neither exists here).
"""
import numpy as np
import pytest

import dtsffi as D
import orc
from _util import first_diff, oracle_frame, planes_equal, random_frame

pytestmark = pytest.mark.gpu

BIC, BIL, LAN = D.SCALE_BICUBIC, D.SCALE_BILINEAR, D.SCALE_LANCZOS
MAX_OFF_BY_ONE = 0.01


@pytest.fixture(params=["default", "v3"])
def ladder_kernel(request, monkeypatch):
    """The library's choice (258-wide planes are not k_ladder7's: k_ladder5 runs the 8-bit
    sources, k_ladder4 the p010 ones) and DTS_LADDER=3 (the v3 kernel, k_ladder4's own
    fallback for geometries it does not plan)."""
    if request.param == "default":
        monkeypatch.delenv("DTS_LADDER", raising=False)
        return request.param
    monkeypatch.setenv("DTS_LADDER", request.param[1])
    return request.param


@pytest.mark.parametrize("outs", [
    [(1920, 1080, D.FMT_P010LE, BIC)],
    [(1920, 1080, D.FMT_YUV420P, BIC), (1600, 900, D.FMT_NV12, BIL), (2560, 1440, D.FMT_P010LE, LAN)],
    [(2880, 1620, D.FMT_P010LE, BIC), (1920, 1080, D.FMT_NV12, LAN)],
])
def test_p010_sources_on_ladder7(ctx, outs):
    """p010 sources on k_ladder7's 16-bit walks (three raw-byte MFMA chains per K block,
    the p010 V epilogue, the ordered dither for 8-bit renditions): bit-exact vs the
    oracle on synthetic and fully random 16-bit words (the low 6 bits discarded, as
    p010LEToY_c's >> 6), including the 1080p intermediate of config 3."""
    sw, sh = 3840, 2160
    rng = np.random.default_rng(31)
    frames = [D.synth_host(sw, sh, D.FMT_P010LE, 0, 0x5EED, 2), random_frame(sw, sh, D.FMT_P010LE, rng)]
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_P010LE, outs))
    assert g.info.ladder_v5 == 3, "the graph should run on k_ladder7"
    got, _ = g.run_host(frames)
    for f, src in enumerate(frames):
        for k, o in enumerate(outs):
            want = oracle_frame(src, sw, sh, D.FMT_P010LE, o[0], o[1], o[2], o[3])
            assert planes_equal(got[f][k], want), f"frame {f} out {k} {o}: {first_diff(got[f][k], want)}"
    g.close()


@pytest.mark.parametrize("sfmt", [D.FMT_YUV420P, D.FMT_NV12, D.FMT_P010LE])
@pytest.mark.parametrize("method", [BIC, BIL, LAN])
def test_p010_output_bitexact(ctx, ladder_kernel, sfmt, method):
    rng = np.random.default_rng(100 + sfmt * 7 + method)
    sw, sh = 258, 146
    frames = [random_frame(sw, sh, sfmt, rng), D.synth_host(sw, sh, sfmt, 0, 0x5EED, 3)]
    outs = [(130, 74, D.FMT_P010LE, method), (97, 51, D.FMT_P010LE, method), (sw, sh, D.FMT_P010LE, method),
            (64, 36, D.FMT_NV12, method)]
    g = D.Graph(ctx, D.make_spec(sw, sh, sfmt, outs))
    got, _ = g.run_host(frames)
    for f, src in enumerate(frames):
        for k, o in enumerate(outs):
            want = oracle_frame(src, sw, sh, sfmt, o[0], o[1], o[2], o[3])
            assert planes_equal(got[f][k], want), f"frame {f} out {k} {o}: {first_diff(got[f][k], want)}"
    g.close()


def test_p010_identity_passthrough(ctx):
    """p010 -> p010 at 1:1 keeps the 10-bit samples (15-bit round trip is exact)."""
    rng = np.random.default_rng(5)
    src = random_frame(128, 64, D.FMT_P010LE, rng)
    g = D.Graph(ctx, D.make_spec(128, 64, D.FMT_P010LE, [(128, 64, D.FMT_P010LE, BIC)]))
    (out,), _ = g.run_host([src])
    for a, b in zip(out[0][:2], src[:2]):
        va = np.asarray(a).view(np.uint16) >> 6
        vb = np.asarray(b).copy().view(np.uint16) >> 6
        assert np.array_equal(va, vb)


def _check_tol(got, want, what):
    got, want = list(got), list(want)
    assert len(got) == len(want), f"{what}: {len(got)} planes vs {len(want)}"
    n = bad = 0
    for a, b in zip(got, want):
        assert (a is None) == (b is None), f"{what}: plane present in one frame only"
        if a is None:
            continue
        d = np.abs(np.asarray(a).astype(np.int16) - np.asarray(b).astype(np.int16))
        assert d.max() <= 1, f"{what}: max diff {d.max()} at {np.unravel_index(d.argmax(), d.shape)}"
        n += d.size
        bad += int((d > 0).sum())
    assert bad <= MAX_OFF_BY_ONE * n, f"{what}: {bad}/{n} samples off by one"


def _hdr_case(ctx, sw, sh, outs, frames, tm, full=False):
    g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_P010LE, outs, tonemap=tm, dst_range=int(full)))
    got, _ = g.run_host(frames)
    for f, src in enumerate(frames):
        for k, (w, h, fmt, m) in enumerate(outs):
            mid = orc.scale_frame(src, sw, sh, D.FMT_P010LE, w, h, D.FMT_P010LE, m)
            want = orc.hdr_to_sdr(mid, w, h, fmt, tm.get("mode", D.TM_HABLE), tm.get("param", float("nan")),
                                  tm.get("desat", 2.0), tm.get("peak", 0.0), tm.get("npl", 100.0), full)
            _check_tol(got[f][k], want, f"frame {f} out {k} tm {tm}")
    g.close()


@pytest.mark.parametrize("mode", ["hable", "mobius", "reinhard", "clip", "linear", "gamma", "none"])
def test_hdr_to_sdr_modes(ctx, mode):
    """config-3 shape at 1/10 scale: 384x216 p010 -> 192x108 SDR, every vf_tonemap curve."""
    frames = [D.synth_host(384, 216, D.FMT_P010LE, 0, 0x5EED, f) for f in range(2)]
    frames.append(random_frame(384, 216, D.FMT_P010LE, np.random.default_rng(9)))
    _hdr_case(ctx, 384, 216, [(192, 108, D.FMT_YUV420P, BIC), (128, 72, D.FMT_NV12, BIC)], frames,
              {"mode": D.TM_MODES[mode], "peak": 100.0 if mode != "hable" else 0.0})


@pytest.mark.parametrize("tm", [{"mode": D.TM_HABLE, "desat": 2.0}, {"mode": D.TM_HABLE, "npl": 203.0, "peak": 50.0},
                                {"mode": D.TM_MOBIUS, "param": 0.5, "peak": 12.0},
                                {"mode": D.TM_REINHARD, "param": 0.3, "peak": 40.0}])
def test_hdr_to_sdr_params(ctx, tm):
    frames = [D.synth_host(258, 146, D.FMT_P010LE, 0, 11, 2),
              random_frame(258, 146, D.FMT_P010LE, np.random.default_rng(3))]
    _hdr_case(ctx, 258, 146, [(130, 74, D.FMT_YUV420P, LAN)], frames, tm)


@pytest.mark.parametrize("mode", ["hable", "clip", "mobius"])
def test_hdr_to_sdr_full_range(ctx, mode):
    """The last zscale with r=pc (dst_range JPEG): the tone-map kernels' full-range quantiser
    (255 Y', 255 C + 128, chroma clamped at 255) vs the restatement, both column walks'
    edge handling included (130 x 74 is not a multiple of the walk's tiles)."""
    frames = [D.synth_host(384, 216, D.FMT_P010LE, 0, 0x5EED, 1),
              random_frame(384, 216, D.FMT_P010LE, np.random.default_rng(21))]
    _hdr_case(ctx, 384, 216, [(192, 108, D.FMT_YUV420P, BIC), (130, 74, D.FMT_NV12, BIL)], frames,
              {"mode": D.TM_MODES[mode], "peak": 100.0 if mode != "hable" else 0.0}, full=True)


def test_hdr_4k_to_1080p_one_frame(ctx):
    """The config-3 geometry itself, one frame (host path), with vf_tonemap's
    defaults (hable, desat 2.0, peak from the fallback): the graph a CPU worker's
    `tonemap=hable` runs."""
    frames = [D.synth_host(3840, 2160, D.FMT_P010LE, 0, 0x5EED, 0)]
    _hdr_case(ctx, 3840, 2160, [(1920, 1080, D.FMT_YUV420P, BIC)], frames, {"mode": D.TM_HABLE})


def test_hdr_many_frames_device_double_buffer(ctx):
    """More frames than one batch: the p010 intermediates are reused across chunks."""
    frames = [D.synth_host(130, 74, D.FMT_P010LE, 1, 77, f) for f in range(7)]
    spec = D.make_spec(130, 74, D.FMT_P010LE, [(64, 36, D.FMT_NV12, BIC)], max_batch=3,
                       tonemap={"mode": D.TM_HABLE})
    g = D.Graph(ctx, spec)
    got, _ = g.run_host(frames)
    for f, src in enumerate(frames):
        mid = orc.scale_frame(src, 130, 74, D.FMT_P010LE, 64, 36, D.FMT_P010LE, BIC)
        _check_tol(got[f][0], orc.hdr_to_sdr(mid, 64, 36, D.FMT_NV12, D.TM_HABLE), f"frame {f}")
    g.close()
