"""GPU parity of BASELINE config 5's per-segment work.

The cfg5 job: a 4K source cut into segments, each segment run through the
3-rung nv12 bicubic ABR ladder, every rendition scored with vf_psnr / vf_ssim
against a lanczos reference rendition of the same size, and each segment's
per-frame records reduced to one record (the running sums vf_psnr / vf_ssim
keep) that the GPUs gather (database.js:97-129: segments carry their results).

Here: 2 segments of 5 frames each through graphs with max_batch = 2 (so every
segment spans 3 ladder launches), on the device path, then
- every rendition frame bit-exact vs the oracle, every frame's SSE exact and
  SSIM within 1e-4 vs orc.quality_frame on the de-interleaved planes;
- every segment record (dts_qraw_sum_device) vs the sum of the oracle's
  per-frame records: SSE exact, SSIM sums within 1e-4 per frame;
- the job-level averages (dts_qstat_stream on the sum of both segment records)
  vs the oracle's mean MSE / mean SSIM.
"""
import ctypes
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import dtsffi as D
import orc
from _util import first_diff, planes_equal

pytestmark = pytest.mark.gpu

SW, SH = 3840, 2160
LADDER = [(1920, 1080, D.FMT_NV12, D.SCALE_BICUBIC), (1280, 720, D.FMT_NV12, D.SCALE_BICUBIC),
          (854, 480, D.FMT_NV12, D.SCALE_BICUBIC)]
SEGMENTS, SEG_FRAMES, BATCH = 2, 5, 2
SSIM_TOL = 1e-4


def _planar(planes):
    """nv12 -> Y, U, V (vf_psnr / vf_ssim take planar yuv420p; ffmpeg converts ahead of them)."""
    return [planes[0], np.ascontiguousarray(planes[1][:, 0::2]), np.ascontiguousarray(planes[1][:, 1::2])]


def _oracle_frame(idx):
    src = D.synth_host(SW, SH, D.FMT_YUV420P, 0, 0x5EED, idx)
    outs, recs = [], []
    for (w, h, fmt, m) in LADDER:
        o = orc.scale_frame(src, SW, SH, D.FMT_YUV420P, w, h, fmt, m)
        r = orc.scale_frame(src, SW, SH, D.FMT_YUV420P, w, h, fmt, D.SCALE_LANCZOS)
        outs.append(o)
        recs.append(orc.quality_frame(w, h, _planar(o), _planar(r)))
    return outs, recs


def _sub(d, i0):
    """Frames i0.. of a DevFrames batch."""
    e = D.DevFrames()
    for p in range(3):
        e.data[p] = (d.data[p] or 0) + i0 * d.frame_stride if d.data[p] else None
        e.pitch[p] = d.pitch[p]
    e.frame_stride = d.frame_stride
    return e


def _qraws(t, n):
    host = t.cpu().numpy()
    out = []
    for i in range(n):
        r = D.QRaw()
        ctypes.memmove(ctypes.addressof(r), host[i].tobytes(), ctypes.sizeof(r))
        out.append(r)
    return out


def test_cfg5_segments_ladder_quality_and_records(ctx):
    import torch
    from bench import dev_batch, frame_bytes, unpack_dev_frame
    n = SEGMENTS * SEG_FRAMES
    stream = torch.cuda.current_stream().cuda_stream
    src_t = torch.empty((n, frame_bytes(SW, SH, D.FMT_YUV420P)), dtype=torch.uint8, device="cuda")
    sd, _ = dev_batch(src_t, SW, SH, D.FMT_YUV420P)
    ctx.synth_device(SW, SH, D.FMT_YUV420P, 0, 0x5EED, 0, sd, n, stream)
    lad = D.Graph(ctx, D.make_spec(SW, SH, D.FMT_YUV420P, LADDER, max_batch=BATCH))
    ref = D.Graph(ctx, D.make_spec(SW, SH, D.FMT_YUV420P, [(w, h, f, D.SCALE_LANCZOS) for (w, h, f, _m) in LADDER],
                                   max_batch=BATCH))
    outs, refs = [], []
    for (w, h, fmt, _m) in LADDER:
        for lst in (outs, refs):
            t = torch.empty((n, frame_bytes(w, h, fmt)), dtype=torch.uint8, device="cuda")
            lst.append((t, dev_batch(t, w, h, fmt)[0]))
    qraw = [torch.zeros((n, 6), dtype=torch.float64, device="cuda") for _ in LADDER]     # dts_qraw = 48 B
    seg = [torch.zeros((SEGMENTS, 6), dtype=torch.float64, device="cuda") for _ in LADDER]
    for s in range(SEGMENTS):
        f0 = s * SEG_FRAMES
        # the segment through both graphs in max_batch launches
        for b0 in range(f0, f0 + SEG_FRAMES, BATCH):
            m = min(BATCH, f0 + SEG_FRAMES - b0)
            lad.run_device(_sub(sd, b0), m, [_sub(d, b0) for (_t, d) in outs], stream=stream)
            ref.run_device(_sub(sd, b0), m, [_sub(d, b0) for (_t, d) in refs], stream=stream)
        # per rendition: the segment's per-frame records, then its one record
        for k, (w, h, fmt, _m) in enumerate(LADDER):
            ctx.quality_device(w, h, fmt, _sub(outs[k][1], f0), _sub(refs[k][1], f0), SEG_FRAMES,
                               qraw[k].data_ptr() + f0 * 48, stream)
            ctx.qraw_sum_device(qraw[k].data_ptr() + f0 * 48, SEG_FRAMES, seg[k].data_ptr() + s * 48, stream)
    torch.cuda.synchronize()

    with ThreadPoolExecutor(8) as ex:
        want = list(ex.map(_oracle_frame, range(n)))
    for k, (w, h, fmt, _m) in enumerate(LADDER):
        got_q = D.qstat_finalize(w, h, _qraws(qraw[k], n))
        host = outs[k][0].cpu().numpy()
        for i in range(n):
            img = unpack_dev_frame(host[i], w, h, fmt)
            assert planes_equal(img, want[i][0][k]), f"rung {k} frame {i}: {first_diff(img, want[i][0][k])}"
            wq, gq = want[i][1][k], got_q[i]
            assert gq["sse"] == wq["sse"], (k, i)
            for c in range(3):
                assert gq["ssim"][c] == pytest.approx(wq["ssim"][c], abs=SSIM_TOL), (k, i, c)
            assert gq["ssim_all"] == pytest.approx(wq["ssim_all"], abs=SSIM_TOL), (k, i)
        # segment records vs the sums of the oracle's frame records
        recs = _qraws(seg[k], SEGMENTS)
        pw = [w, (w + 1) // 2, (w + 1) // 2]
        ph = [h, (h + 1) // 2, (h + 1) // 2]
        nw = [((pw[c] >> 2) - 1) * ((ph[c] >> 2) - 1) for c in range(3)]
        for s in range(SEGMENTS):
            fr = range(s * SEG_FRAMES, (s + 1) * SEG_FRAMES)
            for c in range(3):
                assert recs[s].sse[c] == sum(want[i][1][k]["sse"][c] for i in fr), (k, s, c)
                assert recs[s].ssim_sum[c] / nw[c] == pytest.approx(
                    sum(want[i][1][k]["ssim"][c] for i in fr), abs=SSIM_TOL * SEG_FRAMES), (k, s, c)
        # the job (both segments): vf_psnr's mean-MSE PSNR and vf_ssim's mean SSIM
        job = D.qstat_stream(w, h, D.qraw_sum_host(recs), n)
        area = sum(pw[c] * ph[c] for c in range(3))
        mse = [sum(want[i][1][k]["sse"][c] for i in range(n)) / (n * pw[c] * ph[c]) for c in range(3)]
        mse_avg = sum(mse[c] * pw[c] * ph[c] / area for c in range(3))
        assert job["psnr_avg"] == pytest.approx(10 * np.log10(255 * 255 / mse_avg), rel=1e-12)
        for c in range(3):
            assert job["mse"][c] == pytest.approx(mse[c], rel=1e-12)
            assert job["ssim"][c] == pytest.approx(np.mean([want[i][1][k]["ssim"][c] for i in range(n)]),
                                                   abs=SSIM_TOL)
        assert job["ssim_all"] == pytest.approx(np.mean([want[i][1][k]["ssim_all"] for i in range(n)]), abs=SSIM_TOL)
    lad.close()
    ref.close()
