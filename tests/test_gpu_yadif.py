"""GPU parity of the vf_yadif deinterlacer: bit-exact vs
the CPU restatement (oracle/vf_yadif_ref.c) for every mode, both field
orders, odd sizes, and the sequence ends (prev/next clones)."""
import numpy as np
import pytest

import dtsffi as D
import orc
from _util import random_frame, planes_equal

pytestmark = pytest.mark.gpu


def _packed(w, h):
    cw, ch = (w + 1) // 2, (h + 1) // 2
    return [(0, w, h), (w * h, cw, ch), (w * h + cw * ch, cw, ch)], w * h + 2 * cw * ch


def _to_dev(frames, w, h):
    import torch
    planes, size = _packed(w, h)
    host = np.zeros((len(frames), size), np.uint8)
    for i, f in enumerate(frames):
        for (off, pw, ph), p in zip(planes, f):
            host[i, off:off + pw * ph] = np.ascontiguousarray(p).reshape(-1)
    t = torch.from_numpy(host).cuda()
    return t, _dev(t, w, h)


def _dev(t, w, h):
    planes, _ = _packed(w, h)
    d = D.DevFrames()
    for p, (off, pw, _ph) in enumerate(planes):
        d.data[p] = t.data_ptr() + off
        d.pitch[p] = pw
    d.frame_stride = t.stride(0)
    return d


def _from_dev(row, w, h):
    planes, _ = _packed(w, h)
    return [row[off:off + pw * ph].reshape(ph, pw) for (off, pw, ph) in planes]


@pytest.mark.parametrize("w,h", [(64, 36), (130, 74), (37, 23), (720, 480)])
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("tff", [1, 0])
def test_yadif_vs_oracle(ctx, w, h, mode, tff):
    import torch
    if w < 16:
        pytest.skip("yadif needs w >= 16")
    rng = np.random.default_rng(w * 7 + h + mode * 3 + tff)
    n = 4
    frames = [D.synth_host(w, h, D.FMT_YUV420P, 0, 9, i) if i % 2 else random_frame(w, h, D.FMT_YUV420P, rng)
              for i in range(n)]
    seq_t, seq = _to_dev(frames, w, h)
    fields = 2 if mode & 1 else 1
    _, size = _packed(w, h)
    out_t = torch.zeros((n * fields, size), dtype=torch.uint8, device="cuda")
    ctx.yadif_device(w, h, mode, tff, seq, n, 0, n, _dev(out_t, w, h), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = out_t.cpu().numpy()
    # the oracle needs shared pitches: use the packed planes of the same host copy
    host = seq_t.cpu().numpy()
    hp = [_from_dev(host[i], w, h) for i in range(n)]
    for i in range(n):
        for s in range(fields):
            want = orc.yadif_frame(hp[max(i - 1, 0)], hp[i], hp[min(i + 1, n - 1)], w, h, mode, tff, s)
            got = _from_dev(out[i * fields + s], w, h)
            for p in range(3):
                assert np.array_equal(got[p], want[p]), \
                    f"frame {i} field {s} plane {p}: {int((got[p] != want[p]).sum())} diffs"


def test_yadif_subrange_and_validation(ctx):
    """first/count select outputs inside a longer sequence; bad arguments fail loudly."""
    import torch
    w, h, n = 96, 54, 6
    frames = [D.synth_host(w, h, D.FMT_YUV420P, 1, 5, i) for i in range(n)]
    seq_t, seq = _to_dev(frames, w, h)
    _, size = _packed(w, h)
    out_t = torch.zeros((2, size), dtype=torch.uint8, device="cuda")
    ctx.yadif_device(w, h, 0, 1, seq, n, 3, 2, _dev(out_t, w, h), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    host = seq_t.cpu().numpy()
    hp = [_from_dev(host[i], w, h) for i in range(n)]
    for j in range(2):
        i = 3 + j
        want = orc.yadif_frame(hp[i - 1], hp[i], hp[min(i + 1, n - 1)], w, h, 0, 1, 0)
        got = _from_dev(out_t[j].cpu().numpy(), w, h)
        assert planes_equal(got, want)
    with pytest.raises(D.DtsError):
        ctx.yadif_device(w, h, 0, 1, seq, n, 5, 2, _dev(out_t, w, h))
    with pytest.raises(D.DtsError):
        ctx.yadif_device(8, h, 0, 1, seq, n, 0, 1, _dev(out_t, w, h))


@pytest.mark.parametrize("mode,tff", [(0, 1), (2, 0)])
def test_graph_yadif_then_ladder(ctx, mode, tff):
    """The graph's deinterlace stage (dts_graph_spec.deint): yadif on the device batch,
    then the ladder, bit-exact against orc.yadif_frame followed by orc.scale_frame.
    The host path chunks by max_batch = 2, so chunk edges take their neighbours
    from the one-frame context the caller supplies around the segment."""
    import dtsffi as Dm
    sw, sh = 384, 216
    rng = np.random.default_rng(mode * 7 + tff)
    seq = [random_frame(sw, sh, Dm.FMT_YUV420P, rng) for _ in range(7)]
    outs = [(192, 108, Dm.FMT_NV12, Dm.SCALE_BICUBIC), (128, 72, Dm.FMT_YUV420P, Dm.SCALE_LANCZOS)]
    g = Dm.Graph(ctx, Dm.make_spec(sw, sh, Dm.FMT_YUV420P, outs, max_batch=2, deint=(mode, tff)))
    got, _ = g.run_host(seq[1:7])                    # segment = seq[2..5], context seq[1] and seq[6]
    assert len(got) == 4
    for j in range(4):
        i = 2 + j
        de = orc.yadif_frame(seq[i - 1], seq[i], seq[i + 1], sw, sh, mode, tff, 0)
        for k, (w, h, fmt, m) in enumerate(outs):
            want = orc.scale_frame(de, sw, sh, Dm.FMT_YUV420P, w, h, fmt, m)
            assert planes_equal(got[j][k], want), (mode, tff, j, k)
    g.close()
    with pytest.raises(Dm.DtsError):                   # frame-rate modes only; 8-bit planar sources only
        Dm.Graph(ctx, Dm.make_spec(sw, sh, Dm.FMT_YUV420P, outs, deint=(1, 1)))
    with pytest.raises(Dm.DtsError):
        Dm.Graph(ctx, Dm.make_spec(sw, sh, Dm.FMT_NV12, outs, deint=(0, 1)))


def _aligned_seq(frames, w, h, n_extra_out=0):
    """frames laid out by bench.dev_batch (pitches of 256 B, planes 16-byte aligned): the
    temporal-walk kernel's domain (k_yadif_t)"""
    import torch
    from bench import dev_batch, frame_bytes
    fb = frame_bytes(w, h, D.FMT_YUV420P)
    t = torch.zeros((len(frames), fb), dtype=torch.uint8, device="cuda")
    d, _ = dev_batch(t, w, h, D.FMT_YUV420P)
    host = np.zeros((len(frames), fb), np.uint8)
    for i, f in enumerate(frames):
        for p in range(3):
            off = d.data[p] - t.data_ptr()
            rows, cols = f[p].shape
            host[i, off:off + rows * d.pitch[p]].reshape(rows, d.pitch[p])[:, :cols] = f[p]
    t.copy_(torch.from_numpy(host))
    return t, d


@pytest.mark.parametrize("w,h,n,first,count", [(720, 480, 5, 0, 5), (130, 74, 4, 0, 4), (1000, 36, 3, 0, 3),
                                               (1920, 1080, 20, 1, 18), (3840, 2160, 3, 0, 3), (16, 6, 3, 0, 3),
                                               (264, 45, 3, 0, 3)])
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("tff", [1, 0])
def test_yadif_temporal_walk_vs_oracle(ctx, w, h, n, first, count, mode, tff):
    """k_yadif_t (16-byte aligned sequences: every frame tile staged once, a ring of prev /
    cur / next in LDS): bit-exact vs the oracle in every mode and field order; tiles at every
    plane edge, widths not multiples of 16, walks longer than one workgroup's (16 frames) and
    starting inside the sequence (first > 0: the graph path's context frame); odd heights put the
    two-row threads' boundary (rows y - 2 .. y + 4 inside the plane, else the one-row code) at
    every offset from the bottom edge."""
    import torch
    from bench import dev_batch, frame_bytes, unpack_dev_frame
    if w >= 1920 and (mode, tff) not in [(0, 1), (1, 0), (2, 0)]:
        pytest.skip("large frames: a subset of modes")
    rng = np.random.default_rng(w + h + 31 * mode + tff)
    frames = [random_frame(w, h, D.FMT_YUV420P, rng) if i % 3 == 0 else D.synth_host(w, h, D.FMT_YUV420P, 0, 13, i)
              for i in range(n)]
    seq_t, seq = _aligned_seq(frames, w, h)
    fields = 2 if mode & 1 else 1
    out_t = torch.zeros((count * fields, frame_bytes(w, h, D.FMT_YUV420P)), dtype=torch.uint8, device="cuda")
    od, _ = dev_batch(out_t, w, h, D.FMT_YUV420P)
    ctx.yadif_device(w, h, mode, tff, seq, n, first, count, od, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = out_t.cpu().numpy()
    for j in range(count):
        i = first + j
        for s in range(fields):
            want = orc.yadif_frame(frames[max(i - 1, 0)], frames[i], frames[min(i + 1, n - 1)], w, h, mode, tff, s)
            got = unpack_dev_frame(out[j * fields + s], w, h, D.FMT_YUV420P)
            for p in range(3):
                assert np.array_equal(got[p], want[p]), \
                    f"frame {i} field {s} plane {p}: {int((got[p] != want[p]).sum())} diffs"
