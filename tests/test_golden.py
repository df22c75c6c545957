"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py
from the CPU oracle).  CPU: the oracle still reproduces them bit-exactly
(regression guard).  GPU: libdts reproduces them through the C-ABI (bit-exact;
+-1 LSB for the HDR float path).  Parity of the oracle vs FFmpeg itself is
unpinned."""
import glob
import os

import numpy as np
import pytest

import dtsffi as D
import orc
from _util import planes_equal

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SCALE = sorted(glob.glob(os.path.join(GOLD, "scale_*.npz")))


def _planes(z, prefix, n=3):
    return [z[f"{prefix}_p{i}"] if f"{prefix}_p{i}" in z else None for i in range(n)]


def _eq(a, b):
    return planes_equal(a, b)


def test_fixtures_present():
    assert len(SCALE) >= 4
    for n in ("quality_96x54.npz", "hdr_hable_64x36.npz", "yadif_48x20.npz"):
        assert os.path.exists(os.path.join(GOLD, n))


@pytest.mark.parametrize("path", SCALE, ids=os.path.basename)
def test_oracle_matches_golden_scale(path):
    z = np.load(path)
    sw, sh, sfmt, nout = (int(v) for v in z["meta"])
    src = _planes(z, "src")
    for k, (w, h, fmt, m) in enumerate(z["outs"]):
        assert _eq(orc.scale_frame(src, sw, sh, sfmt, int(w), int(h), int(fmt), int(m)), _planes(z, f"out{k}"))


def test_oracle_matches_golden_quality_hdr_yadif():
    z = np.load(os.path.join(GOLD, "quality_96x54.npz"))
    q = orc.quality_frame(96, 54, _planes(z, "a"), _planes(z, "b"))
    assert q["sse"] == [int(v) for v in z["sse"]] and q["ssim_all"] == float(z["ssim_all"])
    z = np.load(os.path.join(GOLD, "hdr_hable_64x36.npz"))
    assert _eq(orc.hdr_to_sdr(_planes(z, "src"), 64, 36, D.FMT_YUV420P, D.TM_HABLE, desat=0.0), _planes(z, "out"))
    z = np.load(os.path.join(GOLD, "yadif_48x20.npz"))
    fr = [_planes(z, f"in{i}") for i in range(3)]
    assert _eq(orc.yadif_frame(fr[0], fr[1], fr[2], 48, 20, 0, 1, 0), _planes(z, "out"))


@pytest.mark.gpu
@pytest.mark.parametrize("path", SCALE, ids=os.path.basename)
def test_gpu_matches_golden_scale(ctx, path):
    z = np.load(path)
    sw, sh, sfmt, nout = (int(v) for v in z["meta"])
    outs = [tuple(int(v) for v in o) for o in z["outs"]]
    g = D.Graph(ctx, D.make_spec(sw, sh, sfmt, outs))
    src = [None if p is None else np.ascontiguousarray(p) for p in _planes(z, "src")]
    got, _ = g.run_host([src])
    for k in range(nout):
        assert _eq(got[0][k], _planes(z, f"out{k}")), f"output {k}"
    g.close()


@pytest.mark.gpu
def test_gpu_matches_golden_quality_and_hdr(ctx):
    z = np.load(os.path.join(GOLD, "hdr_hable_64x36.npz"))
    g = D.Graph(ctx, D.make_spec(64, 36, D.FMT_P010LE, [(64, 36, D.FMT_YUV420P, D.SCALE_BICUBIC)],
                                 tonemap={"mode": D.TM_HABLE, "desat": 0.0}))   # as the fixture
    got, _ = g.run_host([_planes(z, "src")])
    assert len(got[0][0]) == len(_planes(z, "out"))
    for a, b in zip(got[0][0], _planes(z, "out")):
        assert np.abs(a.astype(int) - b.astype(int)).max() <= 1
    g.close()
    z = np.load(os.path.join(GOLD, "quality_96x54.npz"))
    g = D.Graph(ctx, D.make_spec(96, 54, D.FMT_YUV420P, [(96, 54, D.FMT_YUV420P, D.SCALE_BICUBIC)],
                                 quality=D.Q_BOTH))
    _, qs = g.run_host([_planes(z, "a")], qref=[_planes(z, "b")])
    assert qs[0]["sse"] == [int(v) for v in z["sse"]]
    assert abs(qs[0]["ssim_all"] - float(z["ssim_all"])) <= 1e-4
    g.close()
