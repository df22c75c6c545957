"""Regenerate the golden fixtures in this directory (tests/golden/*.npz).

The fixtures are inputs and expected outputs of the CPU oracle (oracle/,
a restatement of the FFmpeg 4.4 libswscale / vf_psnr / vf_ssim / vf_yadif C
paths and of zscale + vf_tonemap): they pin GPU == oracle and guard the
oracle against regressions.  They do NOT pin oracle == libswscale (no
ffmpeg exists in this image or on the GPU box: "parity unpinned").

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "distributed-transcoding-server_amd", "python"))

import dtsffi as D  # noqa: E402
import orc  # noqa: E402

# (name, src w, h, fmt, seed, pattern, [(w, h, fmt, method), ...])
SCALE_CASES = [
    ("ladder_bicubic_384x216", 384, 216, D.FMT_YUV420P, 0x5EED, 0,
     [(192, 108, D.FMT_NV12, D.SCALE_BICUBIC), (128, 72, D.FMT_NV12, D.SCALE_BICUBIC),
      (86, 48, D.FMT_NV12, D.SCALE_BICUBIC)]),
    ("odd_random_37x23", 37, 23, D.FMT_YUV420P, 7, 1,
     [(19, 11, D.FMT_YUV420P, D.SCALE_LANCZOS), (50, 31, D.FMT_NV12, D.SCALE_BILINEAR)]),
    ("p010_to_p010_nv12_130x74", 130, 74, D.FMT_P010LE, 11, 1,
     [(64, 36, D.FMT_P010LE, D.SCALE_BICUBIC), (97, 51, D.FMT_NV12, D.SCALE_LANCZOS)]),
    ("nv12_upscale_64x36", 64, 36, D.FMT_NV12, 3, 0,
     [(100, 60, D.FMT_YUV420P, D.SCALE_BICUBIC), (64, 36, D.FMT_YUV420P, D.SCALE_POINT)]),
]


def planes_dict(prefix, planes):
    return {f"{prefix}_p{i}": np.ascontiguousarray(p) for i, p in enumerate(planes) if p is not None}


def main():
    for name, sw, sh, sfmt, seed, pat, outs in SCALE_CASES:
        src = D.synth_host(sw, sh, sfmt, pat, seed, 0)
        d = {"meta": np.array([sw, sh, sfmt, len(outs)], np.int64),
             "outs": np.array([list(o) for o in outs], np.int64)}
        d.update(planes_dict("src", src))
        for k, (w, h, fmt, m) in enumerate(outs):
            d.update(planes_dict(f"out{k}", orc.scale_frame(src, sw, sh, sfmt, w, h, fmt, m)))
        np.savez_compressed(os.path.join(HERE, f"scale_{name}.npz"), **d)
    # quality (vf_psnr / vf_ssim) of two 8-bit frames
    a = D.synth_host(96, 54, D.FMT_YUV420P, 0, 1, 0)
    b = D.synth_host(96, 54, D.FMT_YUV420P, 0, 1, 3)
    q = orc.quality_frame(96, 54, a, b)
    d = {"sse": np.array(q["sse"], np.uint64), "ssim": np.array(q["ssim"]), "ssim_all": np.array(q["ssim_all"]),
         "psnr_avg": np.array(q["psnr_avg"])}
    d.update(planes_dict("a", a))
    d.update(planes_dict("b", b))
    np.savez_compressed(os.path.join(HERE, "quality_96x54.npz"), **d)
    # HDR10 -> SDR (float path, double oracle) and yadif
    src = D.synth_host(64, 36, D.FMT_P010LE, 0, 5, 0)
    d = planes_dict("src", src)
    d.update(planes_dict("out", orc.hdr_to_sdr(src, 64, 36, D.FMT_YUV420P, D.TM_HABLE, desat=0.0)))
    np.savez_compressed(os.path.join(HERE, "hdr_hable_64x36.npz"), **d)
    fr = [D.synth_host(48, 20, D.FMT_YUV420P, 1, 9, i) for i in range(3)]
    d = {}
    for i, f in enumerate(fr):
        d.update(planes_dict(f"in{i}", f))
    d.update(planes_dict("out", orc.yadif_frame(fr[0], fr[1], fr[2], 48, 20, 0, 1, 0)))
    np.savez_compressed(os.path.join(HERE, "yadif_48x20.npz"), **d)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
