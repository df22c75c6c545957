#!/usr/bin/env python3
"""Occupancy probe (diagnostic): k_ladder7 on a 4K -> 1080p nv12 bicubic graph, whose
walks are the half-width 1080p variants only (76 VGPRs) when DTS_L7_NARROW=1, so a
library built with DTS_L7_WPE=5/6 (tools/build_v7var.sh) runs them at 5/6 waves per
SIMD without spills in the code that executes.  Prints frames/s.  Env: DTS_LIB,
DTS_L7_*; args: frames per launch, launches."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-transcoding-server_amd", "python"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import dtsffi as D  # noqa: E402
from bench import dev_batch, frame_bytes  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
sw, sh = 3840, 2160
outs = [(1920, 1080, D.FMT_NV12, D.SCALE_BICUBIC)]
ctx = D.Context(0)
g = D.Graph(ctx, D.make_spec(sw, sh, D.FMT_YUV420P, outs, max_batch=B))
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
src = torch.empty((2 * B, frame_bytes(sw, sh, D.FMT_YUV420P)), dtype=torch.uint8, device=dev)
sd, _ = dev_batch(src, sw, sh, D.FMT_YUV420P)
ctx.synth_device(sw, sh, D.FMT_YUV420P, 0, 0x5EED, 0, sd, 2 * B, stream.cuda_stream)
out = torch.empty((B, frame_bytes(1920, 1080, D.FMT_NV12)), dtype=torch.uint8, device=dev)
od, _ = dev_batch(out, 1920, 1080, D.FMT_NV12)


def batch(i):
    d = D.DevFrames()
    for p in range(3):
        d.data[p] = (sd.data[p] or 0) + (i % 2) * B * sd.frame_stride
        d.pitch[p] = sd.pitch[p]
    d.frame_stride = sd.frame_stride
    return d


for i in range(3):
    g.run_device(batch(i), B, [od], stream=stream.cuda_stream)
torch.cuda.synchronize(dev)
t0 = time.perf_counter()
for i in range(N):
    g.run_device(batch(i), B, [od], stream=stream.cuda_stream)
torch.cuda.synchronize(dev)
dt = time.perf_counter() - t0
print(f"{os.environ.get('PROBE_TAG', '')} plan v{g.info.ladder_v5} groups {g.info.njobs} lds {g.info.lds_bytes}: "
      f"{B * N / dt:.0f} frames/s")
