"""CPU: known-answer tests pinning the oracle (oracle/liboracle.so).

The reference has no tests and FFmpeg is absent, so these are
the properties libswscale / vf_psnr / vf_ssim satisfy by construction
(SURVEY.md 4), plus the committed golden fixtures in test_golden.py.
"""
import math

import numpy as np
import pytest

import orc
from _util import planes_equal

BIL, BIC, LAN, POINT, AREA, GAUSS = 0x2, 0x4, 0x200, 0x10, 0x20, 0x80


def test_bilinear_2to1_is_triangle_1331():
    c, p = orc.init_filter(3840, 1920, BIL)
    assert c.shape[1] == 4
    assert list(c[5]) == [2048, 6144, 6144, 2048]
    assert p[5] == 9                                 # 2i - 1 (centred siting)


@pytest.mark.parametrize("method", [BIL, BIC, LAN, AREA, GAUSS])
@pytest.mark.parametrize("src,dst", [(3840, 1920), (3840, 1280), (3840, 854), (1920, 1280), (640, 1280),
                                     (37, 19), (100, 150)])
def test_rows_sum_to_one(method, src, dst):
    for one, align in ((1 << 14, 4), (1 << 12, 2)):
        c, p = orc.init_filter(src, dst, method, one=one, align=align)
        s = c.astype(np.int64).sum(1)
        assert np.all(s == one), (s.min(), s.max())
        assert np.all(p >= 0) and np.all(p + c.shape[1] <= max(src, c.shape[1]))
        assert np.all(np.diff(p) >= 0)              # filterPos monotonic


def test_unscaled_is_identity_filter():
    c, p = orc.init_filter(1920, 1920, BIC)
    # filterSize 1, padded to the x86 filterAlign (4) with zero taps under BITEXACT
    # (the right-border fix shifts the last windows left): each output = its own source sample
    for i in range(1920):
        taps = {int(p[i]) + j: int(v) for j, v in enumerate(c[i]) if v}
        assert taps == {i: 1 << 14}


def _frame(w, h, rng=None, const=None):
    cw, ch = (w + 1) // 2, (h + 1) // 2
    if const is not None:
        return [np.full((h, w), const[0], np.uint8), np.full((ch, cw), const[1], np.uint8),
                np.full((ch, cw), const[2], np.uint8)]
    return [rng.integers(0, 256, (h, w), dtype=np.uint8), rng.integers(0, 256, (ch, cw), dtype=np.uint8),
            rng.integers(0, 256, (ch, cw), dtype=np.uint8)]


@pytest.mark.parametrize("method", [BIL, BIC, LAN, POINT, AREA])
def test_constant_plane_stays_constant(method):
    src = _frame(97, 61, const=(123, 77, 201))
    out = orc.scale_frame(src, 97, 61, 0, 40, 23, 0, method)
    assert np.all(out[0] == 123) and np.all(out[1] == 77) and np.all(out[2] == 201)


def test_identity_and_nv12_roundtrip():
    rng = np.random.default_rng(0)
    src = _frame(64, 36, rng)
    same = orc.scale_frame(src, 64, 36, 0, 64, 36, 0, BIC)
    assert planes_equal(src, same)
    nv = orc.scale_frame(src, 64, 36, 0, 64, 36, 1, BIC)
    back = orc.nv12_to_planar(nv)
    assert planes_equal(src, back)


@pytest.mark.parametrize("method", [BIL, BIC])
def test_mirror_symmetry(method):
    rng = np.random.default_rng(3)
    src = _frame(96, 48, rng)
    mir = [np.ascontiguousarray(p[:, ::-1]) for p in src]
    a = orc.scale_frame(src, 96, 48, 0, 48, 24, 0, method)
    b = orc.scale_frame(mir, 96, 48, 0, 48, 24, 0, method)
    for pa, pb in zip(a, b):
        assert np.array_equal(pa, pb[:, ::-1])


def test_psnr_ssim_identities():
    rng = np.random.default_rng(5)
    a = _frame(64, 48, rng)
    q = orc.quality_frame(64, 48, a, a)
    assert q["sse"] == [0, 0, 0] and all(math.isinf(v) for v in q["psnr"]) and math.isinf(q["psnr_avg"])
    assert q["ssim"] == [1.0, 1.0, 1.0] and q["ssim_all"] == pytest.approx(1.0, abs=1e-15)
    b = [np.clip(p.astype(int) + 1, 0, 255).astype(np.uint8) for p in a]
    a2 = [np.clip(p, 0, 254) for p in a]
    b2 = [p + 1 for p in a2]
    q = orc.quality_frame(64, 48, a2, b2)
    assert q["psnr_avg"] == pytest.approx(10 * math.log10(255 ** 2), abs=1e-9)    # 48.1308 dB
    assert q["psnr"][0] == pytest.approx(48.1308036, abs=1e-6)
    assert b is not None


def test_dither_table_is_a_permutation():
    src = open(orc.HERE + "/swscale_ref.c").read()
    start = src.index("dither_8x8_128[9][8]")
    body = src[src.index("{", start) + 1: src.index("};", start)]
    vals = [int(v) for v in body.replace("{", " ").replace("}", " ").replace(",", " ").split()]
    assert len(vals) == 72 and vals[:8] == vals[64:]
    assert sorted(vals[:64]) == list(range(0, 128, 2))


def test_fps_map_properties():
    # 60 -> 30: every other frame; 30 -> 60: each frame twice; 24000/1001 -> 30
    assert list(orc.fps_map(10, (60, 1), (30, 1))) == [0, 2, 4, 6, 8]
    assert list(orc.fps_map(4, (30, 1), (60, 1))) == [0, 0, 1, 1, 2, 2, 3, 3]
    m = orc.fps_map(1001, (24000, 1001), (30, 1))
    assert len(m) == (1001 * 1001 * 30 + 12000) // 24000 and m[0] == 0 and np.all(np.diff(m) >= 0)
    assert m[-1] == 1000


def test_yadif_oracle_properties():
    """vf_yadif known answers: the kept field is copied; a static picture (prev =
    cur = next) whose odd rows equal their even neighbours is reproduced; a
    vertically constant plane stays constant."""
    import dtsffi as D
    w, h = 48, 20
    f = D.synth_host(w, h, D.FMT_YUV420P, 0, 3, 0)
    o = orc.yadif_frame(f, f, f, w, h, 0, 1, 0)
    assert np.array_equal(o[0][0::2], f[0][0::2])           # tff, first field: even rows kept
    o2 = orc.yadif_frame(f, f, f, w, h, 1, 1, 1)
    assert np.array_equal(o2[0][1::2], f[0][1::2])          # second field: odd rows kept
    c = [np.tile(np.arange(p.shape[1], dtype=np.uint8)[None, :] * 3, (p.shape[0], 1)) for p in f]
    for mode in range(4):
        oc = orc.yadif_frame(c, c, c, w, h, mode, 1, 0)
        assert planes_equal(oc, c)


@pytest.mark.parametrize("v,src_range,dst_range,luma,chroma", [
    (16, 0, 1, 0, 0), (235, 0, 1, 255, 250), (128, 0, 1, 130, 128),
    (0, 1, 0, 16, 16), (255, 1, 0, 235, 240), (128, 1, 0, 126, 128)])
def test_range_conversion_known_answers(v, src_range, dst_range, luma, chroma):
    """swscale.c lum/chrRangeToJpeg_c and *FromJpeg_c on a constant frame at 1:1:
    MPEG black / white 16 / 235 map to JPEG 0 / 255 and back, neutral chroma 128
    stays 128, JPEG chroma 255 maps to the MPEG chroma ceiling 240."""
    w, h = 64, 32
    f = [np.full((h, w), v, np.uint8), np.full((h // 2, w // 2), v, np.uint8), np.full((h // 2, w // 2), v, np.uint8)]
    out = orc.scale_frame(f, w, h, 0, w, h, 0, BIC, src_range=src_range, dst_range=dst_range)   # yuv420p
    assert set(np.unique(out[0])) == {luma}
    assert set(np.unique(out[1])) == {chroma} and set(np.unique(out[2])) == {chroma}
    same = orc.scale_frame(f, w, h, 0, w, h, 0, BIC, src_range=src_range, dst_range=src_range)
    assert planes_equal(same, f)      # equal ranges: no conversion
