#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: frames/s and % HBM roofline of the
4K -> 1080p/720p/480p ABR ladder (scale + nv12 convert, bicubic) on MI355X.

One process per GPU (torch.distributed over RCCL when WORLD_SIZE > 1).  Each
rank owns its own segments of a synthetic 4K source (weak scaling: no data-path
collective); the only collective is the post-run RCCL all-gather of the
per-segment records (frames, output checksums) plus the timing max-reduce.

A step = one ladder launch over one batch of B source frames (cfg2: 512, less
than one 600-frame segment) that are already resident in HBM (a ring of R >= 2B
frames: 12.7 GB of 4K frames >> the 256 MB Infinity Cache, so the source really
streams from HBM).  value = all ranks' frames /
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
import math
import os
import sys
import time

import torch  # noqa: E402  (import before libdts so both share torch's HIP runtime)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-transcoding-server_amd", "python"))
import dtsffi as D  # noqa: E402

METRIC = "frames/s and % HBM roofline, 4K→ABR ladder scale+convert, 1/2/4/8 MI355X"
FMTS = {D.FMT_YUV420P: "yuv420p", D.FMT_NV12: "nv12", D.FMT_P010LE: "p010le"}
HBM_PEAK = 8.0e12       # B/s, MI355X HBM3E (MI355X_MICROARCH.md chip table)
SRC_W, SRC_H = 3840, 2160
LADDER = [(1920, 1080, D.FMT_NV12, D.SCALE_BICUBIC), (1280, 720, D.FMT_NV12, D.SCALE_BICUBIC),
          (854, 480, D.FMT_NV12, D.SCALE_BICUBIC)]

# BASELINE.json configs measurable on one GPU.  cfg2 is the metric's workload (the
# default bench line); cfg3 / cfg4 are extra lines (--workload) with their own
# algorithmic bytes.
WORKLOADS = {
    # BASELINE config 1's filtergraph on the GPU: 1080p30 yuv420p -> 720p bicubic (the
    # reference's libx264 encode is host work and absent from the image)
    "cfg1": {"src": (1920, 1080, D.FMT_YUV420P), "outs": [(1280, 720, D.FMT_YUV420P, D.SCALE_BICUBIC)],
             "tonemap": None, "quality": False, "batch": 512,
             "desc": "cfg1: 1080p30 yuv420p -> 720p yuv420p bicubic (the scale of the reference's one-worker "
                     "plumbing case; libx264 is out of scope)"},
    "cfg2": {"src": (SRC_W, SRC_H, D.FMT_YUV420P), "outs": LADDER, "tonemap": None, "quality": False,
             "batch": 512,                 # frames per launch (< one 600-frame segment): 256 -> 159.5k,
                                           # 512 -> 164.8k fps (the launch tail amortised)
             "desc": "cfg2: 4K60 8-bit yuv420p -> 1080p/720p/854x480 nv12 ABR ladder, bicubic "
                     "(SWS_BITEXACT|ACCURATE_RND semantics), one fused launch per batch"},
    "cfg3": {"src": (SRC_W, SRC_H, D.FMT_P010LE), "outs": [(1920, 1080, D.FMT_YUV420P, D.SCALE_BICUBIC)],
             # one launch = one 10 s 4K60 segment (600 frames, the JobChunk unit; round 5: 256-frame
             # launches 86.9 k fps, 600 90.0 k -- the launch tail)
             "tonemap": {"mode": D.TM_HABLE, "desat": 2.0, "peak": 0.0, "npl": 100.0}, "quality": False,
             "batch": 600, "ring": 600,
             "desc": "cfg3: 4K60 10-bit p010 HDR10 (PQ, bt2020nc) -> SDR bt709 8-bit 1080p yuv420p: bit-exact "
                     "bicubic scale to p010 + float zscale/vf_tonemap hable (+-1 LSB), one 10 s segment "
                     "(600 frames) per launch"},
    "cfg4": {"src": (7680, 4320, D.FMT_YUV420P), "outs": [(3840, 2160, D.FMT_YUV420P, D.SCALE_LANCZOS)],
             # one launch = one 10 s segment of 8K30 (300 frames: the JobChunk unit, as cfg5's
             # 600-frame 4K60 segments); round 5: 64-frame launches left a 1.5-wave launch tail
             "tonemap": None, "quality": True, "batch": 300, "ring": 300,
             "desc": "cfg4: 8K30 yuv420p -> 4K lanczos + per-frame vf_psnr/vf_ssim of the output vs its own 4K "
                     "reference frame (a device-resident reference ring as long as the source ring), one "
                     "10 s segment (300 frames) per launch"},
    # BASELINE config 5 on one GPU: a step is one 600-frame segment of the cfg2 ladder plus
    # vf_psnr/vf_ssim of every rendition against a reference rendition of the same size
    # (the source scaled with lanczos: computed once, outside the timed region); the
    # per-segment records (u64 sse[rung][3], f64 ssim_sum[rung][3]) are all-gathered over
    # RCCL at the end
    "cfg5": {"src": (SRC_W, SRC_H, D.FMT_YUV420P), "outs": LADDER, "tonemap": None, "quality": False,
             "rung_quality": True, "batch": 600, "ring": 600,
             "desc": "cfg5: 2-hour 4K60 ABR ladder as 600-frame segments sharded over GPUs (weak scaling): "
                     "1080p/720p/854x480 nv12 bicubic + per-rung vf_psnr/vf_ssim vs lanczos reference "
                     "renditions; per-segment quality records all-gathered over RCCL"},
    # not a BASELINE config: cfg2's ladder from an nv12 source (hardware decoders' output
    # format; k_ladder7 de-interleaves the chroma in its A operand reads)
    "cfg2nv12": {"src": (SRC_W, SRC_H, D.FMT_NV12), "outs": LADDER, "tonemap": None, "quality": False,
                 "batch": 512,
                 "desc": "cfg2 from nv12: 4K60 8-bit nv12 -> 1080p/720p/854x480 nv12 ABR ladder, bicubic"},
    # not a BASELINE config: the vf_yadif kernel on a 4K sequence
    "yadif": {"src": (SRC_W, SRC_H, D.FMT_YUV420P), "outs": [(SRC_W, SRC_H, D.FMT_YUV420P, 0)], "tonemap": None,
              "quality": False, "yadif": 0, "batch": 64,
              "desc": "yadif: vf_yadif mode 0 (send_frame, tff) over a device-resident 4K yuv420p sequence"},
}


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


def planar420(planes, fmt):
    """Y, U, V of an 8-bit 4:2:0 frame (nv12 de-interleaved: vf_psnr / vf_ssim take planar
    yuv420p, so ffmpeg converts nv12 before them)."""
    if fmt != D.FMT_NV12:
        return planes
    uv = planes[1]
    return [planes[0], uv[:, 0::2].copy(), uv[:, 1::2].copy()]


def oracle_outputs(wl, src, qref=None, prev=None, nxt=None):
    """The CPU oracle's outputs (and quality record) for one source frame of workload wl."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    sw, sh, sfmt = wl["src"]
    if wl.get("yadif") is not None:
        return [orc.yadif_frame(prev if prev is not None else src, src, nxt if nxt is not None else src, sw, sh,
                                wl["yadif"], 1, 0)], None
    outs = []
    for (w, h, fmt, m) in wl["outs"]:
        if wl["tonemap"]:
            t = wl["tonemap"]
            mid = orc.scale_frame(src, sw, sh, sfmt, w, h, D.FMT_P010LE, m)
            outs.append(orc.hdr_to_sdr(mid, w, h, fmt, t["mode"], float("nan"), t["desat"], t["peak"], t["npl"]))
        else:
            outs.append(orc.scale_frame(src, sw, sh, sfmt, w, h, fmt, m))
    q = None
    if wl["quality"] and qref is not None:
        w, h = wl["outs"][0][:2]
        q = orc.quality_frame(w, h, outs[0], qref)
    if wl.get("rung_quality"):             # cfg5: every rendition vs its lanczos reference rendition
        q = [orc.quality_frame(w, h, planar420(o, fmt),
                               planar420(orc.scale_frame(src, sw, sh, sfmt, w, h, fmt, D.SCALE_LANCZOS), fmt))
             for (w, h, fmt, _m), o in zip(wl["outs"], outs)]
    return outs, q


def cpu_baseline(wl_name, budget_s, threads):
    """Oracle (C restatement of libswscale / vf_*, single frame per thread) on host cores."""
    from concurrent.futures import ThreadPoolExecutor
    wl = WORKLOADS[wl_name]
    sw, sh, sfmt = wl["src"]
    frames = [D.synth_host(sw, sh, sfmt, 0, 0x5EED, i) for i in range(threads)]
    qref = None
    if wl["quality"]:
        w, h, fmt, _ = wl["outs"][0]
        qref = D.synth_host(w, h, fmt, 0, 0x0EF, 0)

    def one(i):
        oracle_outputs(wl, frames[i % len(frames)], qref)
        return 1
    done = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t0 < budget_s:
            done += sum(ex.map(one, range(done, done + threads)))
    dt = time.perf_counter() - t0
    nproc = os.cpu_count() or threads
    return {"value": done / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "nproc": nproc, "per_core": round(done / dt / threads, 3),
            "all_cores_linear_est": round(done / dt / threads * nproc, 1),
            "sample": f"{done} synthetic {sw}x{sh} source frames through the {wl_name} graph by the CPU "
                      f"oracle (plain-C libswscale / vf_* restatement, ctypes, 1 frame per thread) in {dt:.1f} s "
                      f"on {threads} threads = every CPU this process may use (sched_getaffinity; the box's share "
                      f"for one GPU, of nproc = {nproc}); all_cores_linear_est scales per_core to nproc; "
                      "ffmpeg is not installed on the box"}


def cpu_share():
    """CPUs this process may run on: sched_getaffinity, capped by the box's
    per-GPU share (OMP_NUM_THREADS, which the GPU box sets) when that is set."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def hip_runtimes():
    """Which libamdhip64 files this process mapped (must be exactly one)."""
    libs = set()
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                libs.add(line.split()[-1])
    return sorted(libs)


def unpack_dev_frame(raw, w, h, fmt):
    """Plane list of frame row `raw` laid out by dev_batch."""
    planes, off = [], 0
    for shp in D.plane_shapes(w, h, fmt):
        if shp is None:
            planes.append(None)
            continue
        pitch = (shp[1] + 255) // 256 * 256
        planes.append(raw[off:off + pitch * shp[0]].reshape(shp[0], pitch)[:, :shp[1]])
        off += pitch * shp[0]
    return planes


def verify_frame(wl, src_index, outs, j=0, qref_host=None, qraw=None, ring_first=None, ring_len=None,
                 rung_qraws=None):
    """Frame j of the last batch (source frame src_index) against the CPU oracle: bit-exact
    for the integer paths, +-1 LSB for the HDR float path, 1e-4 for SSIM."""
    import numpy as np
    sw, sh, sfmt = wl["src"]
    host = D.synth_host(sw, sh, sfmt, 0, 0x5EED, src_index)
    prev = nxt = None
    if wl.get("yadif") is not None:        # neighbours inside the ring (clamped at its ends)
        prev = D.synth_host(sw, sh, sfmt, 0, 0x5EED, max(src_index - 1, ring_first))
        nxt = D.synth_host(sw, sh, sfmt, 0, 0x5EED, min(src_index + 1, ring_first + ring_len - 1))
    want, wq = oracle_outputs(wl, host, qref_host, prev, nxt)
    for k, (w, h, fmt, m) in enumerate(wl["outs"]):
        got = unpack_dev_frame(outs[k][j].cpu().numpy(), w, h, fmt)
        for a, b in zip(got, want[k]):
            if a is None:
                continue
            d = np.abs(a.astype(np.int16) - b.astype(np.int16))
            if d.max() > (1 if wl["tonemap"] else 0):
                return False
    if rung_qraws is not None:             # cfg5: each rendition's record vs the oracle's (lanczos reference)
        for k, (w, h, fmt, _m) in enumerate(wl["outs"]):
            oq = wq[k]
            r = D.QRaw.from_buffer_copy(rung_qraws[k][j].cpu().numpy().tobytes())
            gq = D.qstat_finalize(w, h, [r])[0]
            if gq["sse"] != oq["sse"] or abs(gq["ssim_all"] - oq["ssim_all"]) > 1e-4:
                return False
    if wq is not None and qraw is not None and not wl.get("rung_quality"):
        w, h = wl["outs"][0][:2]
        r = D.QRaw.from_buffer_copy(qraw[j].cpu().numpy().tobytes())
        gq = D.qstat_finalize(w, h, [r])[0]
        if gq["sse"] != wq["sse"] or abs(gq["ssim_all"] - wq["ssim_all"]) > 1e-4:
            return False
    return True


def load_traffic(workload):
    """(HBM bytes per frame, profile tag) of this workload's step from its newest committed
    rocprofv3 PMC summary (tools/prof_wl.py writes profiles/pmc_<workload>.json: FETCH_SIZE x2 +
    WRITE_SIZE summed over the step's kernels, per frame), or (None, None)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(path):
        return None, None
    try:
        with open(path) as f:
            j = json.load(f)
        return j.get("hbm_bytes_per_frame"), j.get("tag")
    except Exception:
        return None, None


def gather_quality(sse, ssim, world):
    """cfg5's quality-stat gather, the path's only data collective: every rank's
    per-segment records -- int64 sse[seg][rung][3] and float64 ssim_sum[seg][rung][3],
    fixed size, equal segment counts on every rank (weak scaling) -- all-gathered over
    RCCL (gloo in the CPU tests).  Returns both concatenated in rank order, which is
    segment order (rank r owns segments segment_base(r) ...), on the host."""
    if world > 1:
        sse, ssim = _coll(sse), _coll(ssim)
        gs = [torch.zeros_like(sse) for _ in range(world)]
        gq = [torch.zeros_like(ssim) for _ in range(world)]
        dist.all_gather(gs, sse.contiguous())
        dist.all_gather(gq, ssim.contiguous())
        sse, ssim = torch.cat(gs), torch.cat(gq)
    return sse.cpu(), ssim.cpu()


def _coll(t):
    """A collective's operand on the process group's device: as is over RCCL, on the host
    over gloo (the CPU tests and the one-GPU rehearsal, DTS_BENCH_SHARE_DEVICE)."""
    return t.cpu() if dist.get_backend() == "gloo" else t


def job_quality(outs, sse, ssim, frames_per_segment):
    """vf_psnr / vf_ssim end-of-stream averages per rendition from the gathered segment
    records: mse per plane = sum(sse) / (frames * plane pixels), ssim per plane =
    sum(ssim_sum) / (frames * 4x4-window count), combined over planes by area as the
    per-frame statistics are (dts_qstat_finalize)."""
    def psnr(m):
        return float("inf") if m == 0 else 10 * math.log10(255 * 255 / m)
    res = []
    n = sse.shape[0] * frames_per_segment
    for k, (w, h, _fmt, _m) in enumerate(outs):
        pw = [w, (w + 1) >> 1, (w + 1) >> 1]
        ph = [h, (h + 1) >> 1, (h + 1) >> 1]
        area = sum(a * b for a, b in zip(pw, ph))
        mse = [int(sse[:, k, c].sum()) / (n * pw[c] * ph[c]) for c in range(3)]
        ssimp = [float(ssim[:, k, c].sum()) / (n * ((pw[c] >> 2) - 1) * ((ph[c] >> 2) - 1)) for c in range(3)]
        mse_avg = sum(mse[c] * pw[c] * ph[c] / area for c in range(3))
        ssim_all = sum(ssimp[c] * pw[c] * ph[c] / area for c in range(3))
        res.append({"rendition": f"{w}x{h}", "frames": n, "psnr": [round(psnr(m), 4) for m in mse],
                    "psnr_avg": round(psnr(mse_avg), 4), "ssim": [round(x, 6) for x in ssimp],
                    "ssim_all": round(ssim_all, 6)})
    return res


def segment_base(rank):
    """First synthetic frame index of this rank's segments: ranks own disjoint
    segments of the source (weak scaling, no data exchange)."""
    return rank * 1_000_000


def gather_records(frames, checksum, wall, world, dev):
    """The only collectives of the path: all-gather of the per-rank segment
    records (frames, output checksum) and the max-reduce of the wall time.
    Works on any backend (RCCL on the GPU box, gloo in the CPU tests).
    Returns (total frames, max wall seconds, [(frames, checksum) per rank])."""
    rec = torch.tensor([float(frames), float(checksum)], dtype=torch.float64, device=dev)
    wall_t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        rec, wall_t = _coll(rec), _coll(wall_t)
        dist.all_reduce(wall_t, op=dist.ReduceOp.MAX)
        gathered = [torch.zeros_like(rec) for _ in range(world)]
        dist.all_gather(gathered, rec)
    else:
        gathered = [rec]
    records = [(int(r[0].item()), int(r[1].item())) for r in gathered]
    return sum(r[0] for r in records), float(wall_t.item()), records


def run_e2e(args, wl, ctx, sptr):
    """The host-memory path end to end (dts_graph_submit / dts_graph_wait, the Node worker's
    path): source frames in pageable host memory -> pinned rings (host threads) -> H2D ->
    ladder -> D2H -> the caller's output frames, two slots / streams in flight.  PCIe and
    host copies included: the rate a worker sees, not the kernel's."""
    import numpy as np
    sw, sh, sfmt = wl["src"]
    chunk = args.e2e_batch
    g = D.Graph(ctx, D.make_spec(sw, sh, sfmt, wl["outs"], max_batch=chunk, tonemap=wl["tonemap"]))
    nsrc = args.e2e_frames                   # distinct host source frames, cycled
    srcs = [D.synth_host(sw, sh, sfmt, 0, 0x5EED, i) for i in range(nsrc)]
    per = args.e2e_submit                    # frames per submit (several chunks: both slots busy)
    keep = []
    if args.e2e_pinned:
        # ABI 7: frames in dts_host_alloc memory -- the library DMAs straight from / into them
        pf, buf = D.alloc_frames_pinned(sw, sh, sfmt, nsrc)
        keep.append(buf)
        for a, b in zip(pf, srcs):
            for pa, pb in zip(a, b):
                if pa is not None:
                    pa[...] = pb
        srcs = pf
        per_out = []
        for (w, h, fmt, _m) in wl["outs"]:
            fr, buf = D.alloc_frames_pinned(w, h, fmt, per)
            keep.append(buf)
            per_out.append(fr)
        outs = [[per_out[k][f] for k in range(len(wl["outs"]))] for f in range(per)]
    else:
        outs = [[D.alloc_frame(w, h, fmt) for (w, h, fmt, _m) in wl["outs"]] for _ in range(per)]
    nout = len(wl["outs"])
    dst = (D.Frame * (per * nout))(*[D.frame_struct(outs[f][k]) for f in range(per) for k in range(nout)])
    src_arr = [(D.Frame * per)(*[D.frame_struct(srcs[(i * per + f) % nsrc]) for f in range(per)])
               for i in range(max(1, nsrc // per))]
    L = D.lib()

    def step(i):
        D.check(L.dts_graph_submit(g.h, src_arr[i % len(src_arr)], per, dst, None, None), "submit")
        D.check(L.dts_graph_wait(g.h), "wait")
    for i in range(args.warmup):
        step(i)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    wall = time.perf_counter() - t0
    fps = args.steps * per / wall
    io = g.info.src_frame_bytes + sum(g.info.out_frame_bytes[k] for k in range(nout))
    ok = True
    if not args.no_verify:                   # the last submit's first frame vs the oracle
        want, _ = oracle_outputs(wl, srcs[((args.warmup + args.steps - 1) % len(src_arr)) * per % nsrc])
        for k in range(nout):
            for a, b in zip(outs[0][k], want[k]):
                if a is not None and not np.array_equal(a, b):
                    ok = False
    g.close()
    src_b = g.info.src_frame_bytes
    out_b = sum(g.info.out_frame_bytes[k] for k in range(nout))
    return {"metric": f"frames/s end to end (host memory -> GPU -> host memory), {args.workload}",
            "value": round(fps, 1), "unit": "frames/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall * 1e3 / args.steps, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": f"{nsrc} synthetic host frames, cycled",
            "config": {"workload": wl["desc"], "frames_per_submit": per, "chunk_frames": chunk,
                       "host_frames": "pinned (dts_host_alloc: direct DMA)" if args.e2e_pinned
                       else "pageable (packed through the library's pinned rings)",
                       "host_threads": os.environ.get("DTS_HOST_THREADS", "hardware threads (<= 16)")},
            "pcie_bytes_per_frame": io, "host_io_GBps": round(fps * io / 1e9, 2),
            "h2d_GBps": round(fps * src_b / 1e9, 2), "d2h_GBps": round(fps * out_b / 1e9, 2),
            "verified_vs_oracle": ok if not args.no_verify else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="source frames per step (one ladder launch); default per workload (cfg2: 256)")
    ap.add_argument("--ring", type=int, default=96, help="device-resident source frames per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--e2e", action="store_true",
                    help="time the host-memory path (dts_graph_submit / wait) instead of device-resident batches")
    # (round 5, tools/e2e.sh: submits of 512 frames in chunks of 64 3,174-3,270 fps against 2,918-3,032 for
    # 128 / 32, pageable or pinned alike)
    ap.add_argument("--e2e-batch", type=int, default=64, help="--e2e: frames per device chunk (max_batch)")
    ap.add_argument("--e2e-submit", type=int, default=512, help="--e2e: frames per submit")
    ap.add_argument("--e2e-frames", type=int, default=256, help="--e2e: distinct host source frames")
    ap.add_argument("--e2e-pinned", action="store_true",
                    help="--e2e: host frames in dts_host_alloc memory (direct DMA, no ring copies)")
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS),
                    help="cfg2 = the BASELINE metric's workload (default line); cfg3 / cfg4 = extra lines")
    args = ap.parse_args()
    wl = WORKLOADS[args.workload]
    sw, sh, sfmt = wl["src"]
    if args.batch is None:
        # frames per launch: a 10 s 60 fps segment is 600 frames; 256 keeps the persistent grid's
        # tail (its last, partly idle round of items) small (batch sweep r01v7: 32 -> 256 = +22 %)
        args.batch = wl.get("batch", 256)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DTS_BENCH_SHARE_DEVICE=1: a rehearsal of the N > 1 path on a one-GPU box -- every rank on
    # device 0 with its own libdts context, the collectives over gloo (RCCL needs one device per
    # rank).  Its rate is not a scaling number; the driver's multi-GPU runs never set it.
    share = os.environ.get("DTS_BENCH_SHARE_DEVICE") == "1"
    if share:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if share:
            dist.init_process_group("gloo")
        else:
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
    if args.e2e:
        line = run_e2e(args, wl, ctx, sptr)
        if rank == 0:
            print(json.dumps(line), flush=True)
        ctx.close()
        return
    B, R = args.batch, max(args.ring, 2 * args.batch)
    if "ring" in wl and args.ring == ap.get_default("ring"):
        R = max(wl["ring"], B)                 # cfg5: one segment resident (7.4 GB), re-read every step
    R = (R // B) * B
    rungq = bool(wl.get("rung_quality"))
    yadif = wl.get("yadif")
    if yadif is None:
        # cfg5: every rendition scored against its reference batch (DTS_QREF_EXTERNAL), in the graph:
        # the ladder launch, then the k_quality pass over each rendition and its reference
        gouts = [(w, h, fmt, m, None, (D.Q_BOTH, D.QREF_EXTERNAL)) if rungq else (w, h, fmt, m)
                 for (w, h, fmt, m) in wl["outs"]]
        g = D.Graph(ctx, D.make_spec(sw, sh, sfmt, gouts, quality=D.Q_BOTH if wl["quality"] else D.Q_NONE,
                                     max_batch=B, tonemap=wl["tonemap"]))
        algo_bytes = g.info.algo_bytes_per_frame
        if rungq:                          # + each rendition's reference read once
            algo_bytes += sum(g.info.out_frame_bytes[k] for k in range(len(wl["outs"])))
    else:
        g = None
        # each frame of the sequence is new once (prev/next re-reads hit cache) + one output frame
        algo_bytes = 2 * (sw * sh + 2 * ((sw + 1) // 2) * ((sh + 1) // 2))

    # device-resident source ring: this rank's segments (frame index offset by rank)
    sfb = frame_bytes(sw, sh, sfmt)
    src = torch.empty((R, sfb), dtype=torch.uint8, device=dev)
    sd, _ = dev_batch(src, sw, sh, sfmt)
    first = segment_base(rank)
    ctx.synth_device(sw, sh, sfmt, 0, 0x5EED, first, sd, R, sptr)
    outs, ods = [], []
    for (w, h, fmt, _m) in wl["outs"]:
        t = torch.empty((B, frame_bytes(w, h, fmt)), dtype=torch.uint8, device=dev)
        d, _ = dev_batch(t, w, h, fmt)
        outs.append(t)
        ods.append(d)
    qref = qrd = qraw = None
    if wl["quality"]:
        # cfg4: every source frame has its own 4K reference frame (reference i = synthetic frame
        # first + i, seed 0x0EF), a device-resident ring as long as the source ring (R x 12.6 MB
        # >> the 256 MB Infinity Cache): the reference streams from HBM like the source does
        w, h, fmt, _m = wl["outs"][0]
        qref = torch.empty((R, frame_bytes(w, h, fmt)), dtype=torch.uint8, device=dev)
        qrd, _ = dev_batch(qref, w, h, fmt)
        ctx.synth_device(w, h, fmt, 0, 0x0EF, first, qrd, R, sptr)
        qraw = torch.zeros((B, ctypes.sizeof(D.QRaw)), dtype=torch.uint8, device=dev)

    # cfg5: reference renditions (the ring scaled with lanczos) and per-rung quality records
    qrefs, qraws, seg_sse, seg_ssim = [], [], [], []
    if rungq:
        ref_outs = [(w, h, fmt, D.SCALE_LANCZOS) for (w, h, fmt, _m) in wl["outs"]]
        qg = D.Graph(ctx, D.make_spec(sw, sh, sfmt, ref_outs, max_batch=B))
        # the graph's records: rendition k's frame f at row k * B + f
        qall = torch.zeros((len(wl["outs"]) * B, ctypes.sizeof(D.QRaw)), dtype=torch.uint8, device=dev)
        for k, (w, h, fmt, _m) in enumerate(wl["outs"]):
            t = torch.empty((R, frame_bytes(w, h, fmt)), dtype=torch.uint8, device=dev)
            d, _ = dev_batch(t, w, h, fmt)
            qrefs.append((t, d))
            qraws.append(qall[k * B:(k + 1) * B])
        for i0 in range(0, R, B):
            sdi = D.DevFrames()
            for p in range(3):
                sdi.data[p] = (sd.data[p] or 0) + i0 * sd.frame_stride
                sdi.pitch[p] = sd.pitch[p]
            sdi.frame_stride = sd.frame_stride
            dsts = []
            for (t, d) in qrefs:
                dd = D.DevFrames()
                for p in range(3):
                    dd.data[p] = (d.data[p] or 0) + i0 * d.frame_stride
                    dd.pitch[p] = d.pitch[p]
                dd.frame_stride = d.frame_stride
                dsts.append(dd)
            qg.run_device(sdi, B, dsts, stream=sptr)
        torch.cuda.synchronize(dev)
        qg.close()

    def qref_batch(k, step):
        t, d = qrefs[k]
        i0 = (step * B) % R
        dd = D.DevFrames()
        for p in range(3):
            dd.data[p] = (d.data[p] or 0) + i0 * d.frame_stride
            dd.pitch[p] = d.pitch[p]
        dd.frame_stride = d.frame_stride
        return dd

    def ring_at(ring, step):
        i0 = (step * B) % R
        d = D.DevFrames()
        for p in range(3):
            d.data[p] = (ring.data[p] or 0) + i0 * ring.frame_stride if ring.data[p] else None
            d.pitch[p] = ring.pitch[p]
        d.frame_stride = ring.frame_stride
        return d

    def batch_src(step):
        return ring_at(sd, step)

    def step(i):
        if g is None:                      # prev/next of the batch's frames come from the same ring
            ctx.yadif_device(sw, sh, yadif, 1, sd, R, (i * B) % R, B, ods[0], sptr)
            return
        if rungq:                          # the ladder with every rendition scored against its reference
            g.run_device(batch_src(i), B, ods, qref=[qref_batch(k, i) for k in range(len(ods))],
                         qraw_ptr=qall.data_ptr(), stream=sptr)
        else:
            g.run_device(batch_src(i), B, ods, qref=ring_at(qrd, i) if qrd is not None else None,
                         qraw_ptr=qraw.data_ptr() if qraw is not None else 0, stream=sptr)
        if rungq:
            # the segment's record (computed in warmup too, so torch's reduction kernels are
            # loaded before the timed region)
            sse = torch.stack([q.view(torch.int64)[:, :3].sum(0) for q in qraws])
            ssim = torch.stack([q.view(torch.float64)[:, 3:].sum(0) for q in qraws])
            if i >= args.warmup:
                seg_sse.append(sse)
                seg_ssim.append(ssim)

    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s in range(args.steps):
        ev[s][0].record(stream)
        step(args.warmup + s)
        ev[s][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps

    # segment records: frames + an output checksum per rank, gathered over RCCL
    checksum = sum(int(o.sum().item()) for o in outs) % (1 << 40)
    frames_total, wall_max, _records = gather_records(args.steps * B, checksum, wall, world, dev)
    jq = None
    if rungq:                              # the per-segment quality records of every rank, in segment order
        all_sse, all_ssim = gather_quality(torch.stack(seg_sse), torch.stack(seg_ssim), world)
        jq = {"segments": int(all_sse.shape[0]), "frames_per_segment": B,
              "renditions": job_quality(wl["outs"], all_sse, all_ssim, B)}

    verified = None
    if rank == 0 and not args.no_verify:
        # the first and the last frame of the last batch (the last one sits in the launch's
        # highest frame quad: k_ladder7 maps frame 8 fq + b % 8)
        last = args.warmup + args.steps - 1
        verified = True
        for j in sorted({0, B - 1}):
            si = first + (last * B) % R + j
            qhost = None
            if wl["quality"]:              # the reference of that frame
                w, h, fmt, _m = wl["outs"][0]
                qhost = D.synth_host(w, h, fmt, 0, 0x0EF, si)
            verified = verified and verify_frame(wl, si, outs, j, qhost, qraw, ring_first=first, ring_len=R,
                                                 rung_qraws=qraws if rungq else None)
    if rank == 0:
        fps = frames_total / wall_max
        algo = algo_bytes
        achieved = algo * B / (kern_ms * 1e-3)
        traffic_pf, traffic_tag = load_traffic(args.workload)
        # PMC bytes (FETCH_SIZE + WRITE_SIZE, Infinity-Cache hits included) per launch over this run's
        # kernel time, in the unit of `achieved`
        traffic = round(traffic_pf * B / (kern_ms * 1e-3) / 1e9, 1) if traffic_pf else None
        line = {
            "metric": METRIC if args.workload == "cfg2" else f"frames/s and % HBM roofline, {args.workload}",
            "value": round(fps, 1), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall_max * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8" if not wl["tonemap"] else "u16 scale + f32 tonemap",
            "data": f"synthetic testsrc2-like {sw}x{sh} {FMTS[sfmt]} (seed 0x5EED), device-resident ring of {R} "
                    "frames per GPU",
            "config": {"workload": wl["desc"], "src": f"{sw}x{sh} {FMTS[sfmt]}",
                       "outputs": [f"{w}x{h} {FMTS[fmt]}" for (w, h, fmt, _m) in wl["outs"]],
                       "batch_frames": B, "frames_per_launch": B,
                       "parallelism": f"segments x{world} (one process per GPU)"},
            "mpixel_per_s": round(fps * sw * sh / 1e6, 1),
            "verified_vs_oracle": verified, "hip_runtime": runtimes,
            "algo_bytes_per_frame": algo,
            "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4),
                         "traffic": traffic, "traffic_bytes_per_frame": traffic_pf,
                         "traffic_profile": traffic_tag, "kernel_ms_per_launch": round(kern_ms, 4),
                         "frames_per_launch": B},
        }
        if share and world > 1:
            line["config"]["parallelism"] += " -- rehearsal: every rank on device 0, collectives over gloo"
        if jq is not None:
            line["quality"] = jq
        if wl["quality"]:
            # cfg4: the three streams of the algorithmic bytes, per frame (the reference now streams
            # from HBM too: one distinct reference frame per source frame)
            rb = g.info.out_frame_bytes[0]
            line["roofline"]["bytes_per_frame_split"] = {
                "source_read": g.info.src_frame_bytes, "output_write": rb, "reference_read": rb}
        if world == 1 and not args.no_cpu:
            threads = cpu_share()
            line["cpu_baseline"] = cpu_baseline(args.workload, args.cpu_seconds, threads)
        print(json.dumps(line), flush=True)
    if g is not None:
        g.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
