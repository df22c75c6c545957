#!/usr/bin/env python3
"""Per-phase cycle breakdown of k_ladder5 (diagnostic build lib/libdts_stamp.so).
Runs a few cfg2 launches through bench-like device buffers and prints the
average s_memtime cycles per wave per step of each phase of the step loop."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DTS_LIB"] = os.path.join(ROOT, "distributed-transcoding-server_amd", "lib", os.environ.get("STAMP_LIB", "libdts_stamp.so"))
sys.path.insert(0, ROOT)
sys.argv = ["bench.py", "--steps", "3", "--warmup", "1", "--no-cpu", "--no-verify"] + sys.argv[1:]
import bench  # noqa: E402
import dtsffi as D  # noqa: E402

lib = D.lib()
lib.dts_debug_ladder5_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
bench.main()
lib.dts_debug_ladder5_stamps(buf, 0)
names = ["V(b-1)", "H(b)", "dma(b+2)", "vstep", "dma wait", "barrier"]
waves_steps = buf[15]      # lane 0 of every wave adds its item's step count
tot = sum(buf[k] for k in range(6))
print(f"wave-steps {waves_steps}, cycles per wave-step {tot / max(1, waves_steps):.0f}")
for k, n in enumerate(names):
    print(f"  {n:12s} {buf[k] / max(1, waves_steps):8.0f} cycles/wave-step  {100.0 * buf[k] / max(1, tot):5.1f} %")
