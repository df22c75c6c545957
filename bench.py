#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: frames/s and % HBM roofline of the
4K -> 1080p/720p/480p ABR ladder (scale + nv12 convert, bicubic) on MI355X.

One process per GPU (torch.distributed over RCCL when WORLD_SIZE > 1).  Each
rank owns its own segments of a synthetic 4K source (weak scaling: no data-path
collective); the only collective is the post-run RCCL all-gather of the
per-segment records (frames, output checksums) plus the timing max-reduce.

A step = one ladder launch over one batch of B source frames that are already
resident in HBM (a ring of R >= 64 frames = 796 MB > the 256 MB Infinity
Cache, so the source really streams from HBM).  value = all ranks' frames /
max-over-ranks wall time of the K timed steps.

roofline.achieved = algorithmic bytes per frame (read the 4:2:0 source once,
write each nv12 rendition once: 17,549,280 B) x B / the ladder
kernel's average duration, timed with HIP events on the stream the kernel is
launched on.  cpu_baseline = the CPU oracle (plain-C restatement of the
libswscale C path, oracle/) on a bounded sample of the same workload on the
host cores; ffmpeg itself is not installed on the box.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch  # noqa: E402  (import before libdts so both share torch's HIP runtime)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-transcoding-server_amd", "python"))
import dtsffi as D  # noqa: E402

METRIC = "frames/s and % HBM roofline, 4K→ABR ladder scale+convert, 1/2/4/8 MI355X"
HBM_PEAK = 8.0e12       # B/s, MI355X HBM3E (MI355X_MICROARCH.md chip table)
SRC_W, SRC_H = 3840, 2160
LADDER = [(1920, 1080, D.FMT_NV12, D.SCALE_BICUBIC), (1280, 720, D.FMT_NV12, D.SCALE_BICUBIC),
          (854, 480, D.FMT_NV12, D.SCALE_BICUBIC)]


def dev_batch(t, w, h, fmt, pitch_align=256):
    """Lay frames of (w, h, fmt) into rows of the 2-D uint8 tensor t (frame = row)."""
    shapes = D.plane_shapes(w, h, fmt)
    d = D.DevFrames()
    off = 0
    for p, s in enumerate(shapes):
        if s is None:
            d.data[p], d.pitch[p] = None, 0
            continue
        pitch = (s[1] + pitch_align - 1) // pitch_align * pitch_align
        d.data[p] = t.data_ptr() + off
        d.pitch[p] = pitch
        off += pitch * s[0]
    d.frame_stride = t.stride(0)
    return d, off


def frame_bytes(w, h, fmt, pitch_align=256):
    off = 0
    for s in D.plane_shapes(w, h, fmt):
        if s is not None:
            off += (s[1] + pitch_align - 1) // pitch_align * pitch_align * s[0]
    return (off + 4095) // 4096 * 4096


def cpu_baseline(budget_s, threads):
    """Oracle (C restatement of libswscale, single frame per thread) on host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    from concurrent.futures import ThreadPoolExecutor
    frames = [D.synth_host(SRC_W, SRC_H, D.FMT_YUV420P, 0, 0x5EED, i) for i in range(threads)]

    def one(i):
        src = frames[i % len(frames)]
        for (w, h, fmt, m) in LADDER:
            orc.scale_frame(src, SRC_W, SRC_H, 0, w, h, fmt, m)
        return 1
    done = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t0 < budget_s:
            done += sum(ex.map(one, range(done, done + threads)))
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{done} synthetic 4K yuv420p frames through the 3-rung bicubic nv12 ladder by the CPU "
                      f"oracle (plain-C libswscale C-path restatement, ctypes, 1 frame per thread) in {dt:.1f} s; "
                      "ffmpeg is not installed on the box"}


def hip_runtimes():
    """Which libamdhip64 files this process mapped (must be exactly one)."""
    libs = set()
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                libs.add(line.split()[-1])
    return sorted(libs)


def verify_first_frame(src_index, outs):
    """Bit-exact check of frame 0 of the last batch against the CPU oracle."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import orc
    host = D.synth_host(SRC_W, SRC_H, D.FMT_YUV420P, 0, 0x5EED, src_index)
    for k, (w, h, fmt, m) in enumerate(LADDER):
        want = orc.scale_frame(host, SRC_W, SRC_H, 0, w, h, fmt, m)
        raw = outs[k][0].cpu().numpy()
        off = 0
        for p, shp in enumerate(D.plane_shapes(w, h, fmt)):
            if shp is None:
                continue
            pitch = (shp[1] + 255) // 256 * 256
            plane = raw[off:off + pitch * shp[0]].reshape(shp[0], pitch)[:, :shp[1]]
            off += pitch * shp[0]
            if not np.array_equal(plane, want[p]):
                return False
    return True


def load_traffic():
    """(HBM bytes per frame, profile tag) from the newest committed rocprofv3 PMC
    summary (tools/prof_summary.py writes profiles/pmc_latest.json), or (None, None)."""
    path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(path):
        return None, None
    try:
        with open(path) as f:
            j = json.load(f)
        return j.get("hbm_bytes_per_frame"), j.get("tag")
    except Exception:
        return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="source frames per step (one ladder launch)")
    ap.add_argument("--ring", type=int, default=96, help="device-resident source frames per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    stream = torch.cuda.Stream(dev)          # a real (non-null) HIP stream shared by torch events and libdts
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    assert sptr, "libdts needs a non-null stream handle"

    torch.zeros(1, device=dev)           # initialise torch's HIP runtime before libdts loads
    ctx = D.Context(local)
    runtimes = hip_runtimes()
    if len(runtimes) != 1:
        print(f"WARNING: {len(runtimes)} HIP runtimes mapped: {runtimes}", file=sys.stderr)
    g = D.Graph(ctx, D.make_spec(SRC_W, SRC_H, D.FMT_YUV420P, LADDER))
    info = g.info
    B, R = args.batch, max(args.ring, 2 * args.batch)
    R = (R // B) * B

    # device-resident source ring: this rank's segments (frame index offset by rank)
    sfb = frame_bytes(SRC_W, SRC_H, D.FMT_YUV420P)
    src = torch.empty((R, sfb), dtype=torch.uint8, device=dev)
    sd, _ = dev_batch(src, SRC_W, SRC_H, D.FMT_YUV420P)
    first = rank * 1_000_000
    ctx.synth_device(SRC_W, SRC_H, D.FMT_YUV420P, 0, 0x5EED, first, sd, R, sptr)
    outs, ods = [], []
    for (w, h, fmt, _m) in LADDER:
        t = torch.empty((B, frame_bytes(w, h, fmt)), dtype=torch.uint8, device=dev)
        d, _ = dev_batch(t, w, h, fmt)
        outs.append(t)
        ods.append(d)

    def batch_src(step):
        i0 = (step * B) % R
        d = D.DevFrames()
        for p in range(3):
            d.data[p] = (sd.data[p] or 0) + i0 * sd.frame_stride
            d.pitch[p] = sd.pitch[p]
        d.frame_stride = sd.frame_stride
        return d

    for s in range(args.warmup):
        g.run_device(batch_src(s), B, ods, stream=sptr)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s in range(args.steps):
        ev[s][0].record(stream)
        g.run_device(batch_src(args.warmup + s), B, ods, stream=sptr)
        ev[s][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps

    # segment records: frames + an output checksum per rank, gathered over RCCL
    rec = torch.tensor([float(args.steps * B), float(sum(int(o.sum().item()) for o in outs) % (1 << 40))],
                       dtype=torch.float64, device=dev)
    wall_t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(wall_t, op=dist.ReduceOp.MAX)
        gathered = [torch.zeros_like(rec) for _ in range(world)]
        dist.all_gather(gathered, rec)
        frames_total = sum(int(r[0].item()) for r in gathered)
    else:
        frames_total = int(rec[0].item())
    wall_max = float(wall_t.item())

    verified = None
    if rank == 0 and not args.no_verify:
        last = args.warmup + args.steps - 1
        verified = verify_first_frame(first + (last * B) % R, outs)
    if rank == 0:
        fps = frames_total / wall_max
        algo = info.algo_bytes_per_frame
        achieved = algo * B / (kern_ms * 1e-3)
        traffic_pf, traffic_tag = load_traffic()
        # PMC bytes (FETCH_SIZE + WRITE_SIZE, Infinity-Cache hits included) per launch over this run's
        # kernel time, in the unit of `achieved`
        traffic = round(traffic_pf * B / (kern_ms * 1e-3) / 1e9, 1) if traffic_pf else None
        line = {
            "metric": METRIC, "value": round(fps, 1), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall_max * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": f"synthetic testsrc2-like 4K yuv420p (seed 0x5EED), device-resident ring of {R} frames per GPU",
            "config": {"workload": "cfg2: 4K60 8-bit yuv420p -> 1080p/720p/854x480 nv12 ABR ladder, bicubic "
                                   "(SWS_BITEXACT|ACCURATE_RND semantics), one fused launch per batch",
                       "src": f"{SRC_W}x{SRC_H} yuv420p", "outputs": ["1920x1080 nv12", "1280x720 nv12",
                                                                      "854x480 nv12"],
                       "batch_frames": B, "parallelism": f"segments x{world} (one process per GPU)"},
            "mpixel_per_s": round(fps * SRC_W * SRC_H / 1e6, 1),
            "verified_vs_oracle": verified, "hip_runtime": runtimes,
            "algo_bytes_per_frame": algo,
            "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4),
                         "traffic": traffic, "traffic_bytes_per_frame": traffic_pf,
                         "traffic_profile": traffic_tag, "kernel_ms_per_launch": round(kern_ms, 4),
                         "frames_per_launch": B},
        }
        if world == 1 and not args.no_cpu:
            threads = min(16, os.cpu_count() or 1)
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, threads)
        print(json.dumps(line), flush=True)
    g.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
