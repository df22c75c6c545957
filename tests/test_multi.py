"""N > 1 path on CPU: bench.py's per-rank segment sharding and its only
collectives (record all-gather + wall-time max-reduce), run with the gloo
backend at world sizes 2 and 4 (the GPU box runs the same code over RCCL)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = 32 * (rank + 1)
        total, wall, recs = bench.gather_records(frames, 1000 + rank, 0.5 + rank, world, torch.device("cpu"))
        out[rank] = (total, wall, recs, bench.segment_base(rank))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gather_records_gloo(world):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for rank in range(world):
        total, wall, recs, base = out[rank]
        assert total == sum(32 * (r + 1) for r in range(world))
        assert wall == pytest.approx(world - 0.5)         # max over ranks
        assert recs == [(32 * (r + 1), 1000 + r) for r in range(world)]
    assert len({out[r][3] for r in range(world)}) == world  # disjoint segments per rank


def _qworker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sse, ssim = _segment_records(rank)
        gs, gq = bench.gather_quality(sse, ssim, world)
        out[rank] = (gs.numpy().tolist(), gq.numpy().tolist())
    finally:
        dist.destroy_process_group()


def _segment_records(rank, nseg=3, nrung=3):
    """Deterministic per-segment quality records of one rank (u64 SSE in int64, f64 SSIM sums)."""
    g = torch.Generator().manual_seed(100 + rank)
    sse = torch.randint(0, 1 << 40, (nseg, nrung, 3), generator=g, dtype=torch.int64)
    ssim = torch.rand((nseg, nrung, 3), generator=g, dtype=torch.float64) * 1e5
    return sse, ssim


@pytest.mark.parametrize("world", [2, 4])
def test_gather_quality_gloo(world):
    """cfg5's quality-stat all-gather (RCCL on the GPU box) at world sizes 2 and 4 on gloo:
    every rank ends with every rank's segment records in rank (= segment) order, equal
    to what a single rank holding all the segments would have."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_qworker, args=(world, _free_port(), out), nprocs=world, join=True)
    want_sse = torch.cat([_segment_records(r)[0] for r in range(world)])
    want_ssim = torch.cat([_segment_records(r)[1] for r in range(world)])
    for rank in range(world):
        gs, gq = out[rank]
        assert gs == want_sse.tolist()
        assert gq == want_ssim.tolist()
    sys.path.insert(0, ROOT)
    import bench
    single = bench.gather_quality(want_sse, want_ssim, 1)
    assert torch.equal(single[0], want_sse) and torch.equal(single[1], want_ssim)


def test_job_quality_matches_per_frame_finish():
    """Segment sums -> vf_psnr/vf_ssim averages: one frame per segment of a single
    rendition must equal dts_qstat_finalize's mse_avg / ssim_all over the same records."""
    sys.path.insert(0, ROOT)
    import bench
    import dtsffi as D
    w, h = 64, 36
    recs = []
    for s in range(4):
        r = D.QRaw()
        for c in range(3):
            r.sse[c] = 1000 * (s + 1) + 7 * c
            r.ssim_sum[c] = 50.0 + s + c
        recs.append(r)
    sse = torch.tensor([[list(r.sse)] for r in recs], dtype=torch.int64)
    ssim = torch.tensor([[list(r.ssim_sum)] for r in recs], dtype=torch.float64)
    got = bench.job_quality([(w, h, D.FMT_YUV420P, D.SCALE_BICUBIC)], sse, ssim, 1)[0]
    per = D.qstat_finalize(w, h, recs)
    mse_avg = sum(q["mse_avg"] for q in per) / 4
    ssim_all = sum(q["ssim_all"] for q in per) / 4
    import math
    assert got["psnr_avg"] == pytest.approx(round(10 * math.log10(255 * 255 / mse_avg), 4))
    assert got["ssim_all"] == pytest.approx(round(ssim_all, 6))
    assert got["frames"] == 4


def test_gather_records_single():
    sys.path.insert(0, ROOT)
    import bench
    total, wall, recs = bench.gather_records(7, 3, 0.25, 1, torch.device("cpu"))
    assert (total, wall, recs) == (7, 0.25, [(7, 3)])


@pytest.mark.gpu
def test_bench_two_ranks_one_device():
    """bench.py's N > 1 path on hardware (no 8-GPU node has run it yet): two ranks launched by
    torch.distributed.run exactly as the driver launches them, each with its own libdts context
    on device 0 (DTS_BENCH_SHARE_DEVICE=1: RCCL needs one device per rank, so the collectives go
    over gloo), cfg5 -- per-rank segments, every segment's rendition-quality records all-gathered,
    the wall time max-reduced.  Rank 0's line must count both ranks' frames and segments and
    verify its renditions and quality records against the oracle."""
    steps, batch = 2, 16
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--workload", "cfg5", "--steps", str(steps), "--warmup", "1",
           "--batch", str(batch), "--ring", str(2 * batch), "--no-cpu"]
    env = dict(os.environ, DTS_BENCH_SHARE_DEVICE="1", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1                                   # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == 2
    assert line["verified_vs_oracle"] is True
    q = line["quality"]
    assert q["segments"] == 2 * steps and q["frames_per_segment"] == batch
    assert [r["rendition"] for r in q["renditions"]] == ["1920x1080", "1280x720", "854x480"]
    for rend in q["renditions"]:
        assert rend["frames"] == 2 * steps * batch
        assert 0.0 < rend["ssim_all"] <= 1.0 and rend["psnr_avg"] > 20.0
    # frames of both ranks over the slower rank's wall time
    assert line["value"] == pytest.approx(2 * steps * batch / (line["ms_per_step"] * steps / 1e3), rel=0.02)
