"""CPU checks of the HDR10 -> SDR restatement (oracle/vf_tonemap_ref.c) and of
the spec validation for HDR / p010-output graphs (no device needed).

Known answers that hold for any correct implementation of the zscale +
vf_tonemap chain: black stays black, neutral input stays neutral (Cb = Cr =
128 exactly), the bt2020 -> bt709 matrix maps white to white and matches the
published BT.2087 coefficients, luma is monotonic in the input code.
"""
import numpy as np
import pytest

import dtsffi as D
import orc


def _p010(w, h, y10, cb10, cr10):
    planes = D.alloc_frame(w, h, D.FMT_P010LE)
    planes[0].view(np.uint16)[...] = np.uint16(y10 << 6)
    uv = planes[1].view(np.uint16)
    uv[:, 0::2] = np.uint16(cb10 << 6)
    uv[:, 1::2] = np.uint16(cr10 << 6)
    return planes


def test_matrix_bt2087():
    m = orc.bt2020_to_bt709()
    want = np.array([[1.6605, -0.5876, -0.0728], [-0.1246, 1.1329, -0.0083], [-0.0182, -0.1006, 1.1187]])
    assert np.allclose(m, want, atol=1e-4)
    assert np.allclose(m.sum(axis=1), 1.0, atol=1e-9)


@pytest.mark.parametrize("mode", range(7))
def test_black_and_neutral(mode):
    for y10 in (64, 200, 400, 600, 940):
        out = orc.hdr_to_sdr(_p010(8, 4, y10, 512, 512), 8, 4, D.FMT_YUV420P, mode, peak=100.0)
        assert (out[1] == 128).all() and (out[2] == 128).all()
        if y10 == 64:
            assert (out[0] == 16).all()


def test_luma_monotonic_hable():
    prev = 0
    for y10 in range(64, 941, 16):
        y = int(orc.hdr_to_sdr(_p010(2, 2, y10, 512, 512), 2, 2, D.FMT_NV12, D.TM_HABLE)[0][0, 0])
        assert y >= prev
        prev = y
    assert prev > 200


def test_clip_100_nits_is_white():
    """PQ code of 100 cd/m^2 (E' = 0.5081) with npl = 100 and clip -> nominal white."""
    y10 = round(64 + 876 * 0.5081)
    out = orc.hdr_to_sdr(_p010(2, 2, y10, 512, 512), 2, 2, D.FMT_YUV420P, D.TM_CLIP)
    assert int(out[0][0, 0]) in (234, 235)


def test_full_range_output():
    """zscale r=pc (zimg full-range 8-bit: 255 Y', 255 C + 128): black is 0, clip's 100-nit
    white 254 / 255, neutral chroma 128, and every sample the r=tv one re-quantised to
    within 1."""
    for mode in (D.TM_HABLE, D.TM_CLIP):
        out = orc.hdr_to_sdr(_p010(8, 4, 64, 512, 512), 8, 4, D.FMT_YUV420P, mode, full=True)
        assert (out[0] == 0).all() and (out[1] == 128).all() and (out[2] == 128).all()
    y10 = round(64 + 876 * 0.5081)
    out = orc.hdr_to_sdr(_p010(2, 2, y10, 512, 512), 2, 2, D.FMT_YUV420P, D.TM_CLIP, full=True)
    assert int(out[0][0, 0]) in (254, 255)
    rng = np.random.default_rng(4)
    src = D.alloc_frame(64, 36, D.FMT_P010LE)
    for p in src[:2]:
        p.view(np.uint16)[...] = (rng.integers(64, 941, p.view(np.uint16).shape) << 6).astype(np.uint16)
    tv = orc.hdr_to_sdr(src, 64, 36, D.FMT_NV12, D.TM_CLIP)
    pc = orc.hdr_to_sdr(src, 64, 36, D.FMT_NV12, D.TM_CLIP, full=True)
    ty, py = tv[0].astype(np.float64), pc[0].astype(np.float64)
    assert np.abs((ty - 16) * 255 / 219 - py).max() <= 1.5
    tc, pcc = tv[1].astype(np.float64), pc[1].astype(np.float64)
    assert np.abs(np.clip((tc - 128) * 255 / 224 + 128, 0, 255) - pcc).max() <= 1.5
    assert py.max() > 235                           # the wider code range is used


def test_param_defaults():
    nan = float("nan")
    assert orc.lib().orc_tonemap_param(D.TM_GAMMA, nan) == pytest.approx(1.8)
    assert orc.lib().orc_tonemap_param(D.TM_MOBIUS, nan) == pytest.approx(0.3)
    assert orc.lib().orc_tonemap_param(D.TM_REINHARD, 0.5) == pytest.approx(1.0)
    assert orc.lib().orc_tonemap_param(D.TM_HABLE, nan) == 1.0


def test_spec_validation():
    ok = D.make_spec(3840, 2160, D.FMT_P010LE, [(1920, 1080, D.FMT_YUV420P, D.SCALE_BICUBIC)],
                     tonemap={"mode": D.TM_HABLE})
    info = D.graph_plan(ok)
    assert info.algo_bytes_per_frame == 3840 * 2160 * 3 + 1920 * 1080 * 3 // 2
    bad_src = D.make_spec(3840, 2160, D.FMT_YUV420P, [(1920, 1080, D.FMT_YUV420P, D.SCALE_BICUBIC)],
                          tonemap={"mode": D.TM_HABLE})
    with pytest.raises(D.DtsError):
        D.graph_plan(bad_src)
    bad_out = D.make_spec(3840, 2160, D.FMT_P010LE, [(1920, 1080, D.FMT_P010LE, D.SCALE_BICUBIC)],
                          tonemap={"mode": D.TM_HABLE})
    with pytest.raises(D.DtsError):
        D.graph_plan(bad_out)
    odd = D.make_spec(3840, 2160, D.FMT_P010LE, [(853, 480, D.FMT_YUV420P, D.SCALE_BICUBIC)],
                      tonemap={"mode": D.TM_HABLE})
    with pytest.raises(D.DtsError):
        D.graph_plan(odd)
    badmode = D.make_spec(3840, 2160, D.FMT_P010LE, [(1920, 1080, D.FMT_YUV420P, D.SCALE_BICUBIC)],
                          tonemap={"mode": 9})
    with pytest.raises(D.DtsError):
        D.graph_plan(badmode)
    # p010 output planned on both kernels; quality on a p010 output is not built
    p = D.make_spec(3840, 2160, D.FMT_YUV420P, [(1920, 1080, D.FMT_P010LE, D.SCALE_BICUBIC)])
    assert D.graph_plan(p).ladder_v4_mask == 3
    q = D.make_spec(3840, 2160, D.FMT_YUV420P, [(1920, 1080, D.FMT_P010LE, D.SCALE_BICUBIC)], quality=D.Q_BOTH)
    with pytest.raises(D.DtsError):
        D.graph_plan(q)


def test_oracle_p010_output_roundtrip():
    """oracle p010 -> p010 1:1 is the identity on the 10-bit samples."""
    rng = np.random.default_rng(2)
    src = D.alloc_frame(64, 32, D.FMT_P010LE)
    for p in src[:2]:
        p.view(np.uint16)[...] = (rng.integers(0, 1024, p.view(np.uint16).shape) << 6).astype(np.uint16)
    out = orc.scale_frame(src, 64, 32, D.FMT_P010LE, 64, 32, D.FMT_P010LE, D.SCALE_BICUBIC)
    assert np.array_equal(out[0], src[0]) and np.array_equal(out[1], src[1])
