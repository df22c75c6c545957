#!/usr/bin/env python3
"""Per-phase cycle breakdown of k_ladder7 (diagnostic build lib/libdts_stamp7.so, tools/build_stamp7.sh).
Runs a few cfg2 launches through bench.py and prints, per variant, the average s_memtime
cycles per wave per granule of each phase of the walk.  Diagnostic only."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DTS_LIB"] = os.path.join(ROOT, "distributed-transcoding-server_amd", "lib",
                                     os.environ.get("STAMP_LIB", "libdts_stamp7.so"))
sys.path.insert(0, ROOT)
sys.argv = ["bench.py", "--steps", "3", "--warmup", "1", "--no-cpu", "--no-verify"] + sys.argv[1:]
import bench  # noqa: E402
import dtsffi as D  # noqa: E402

lib = D.lib()
lib.dts_debug_ladder7_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
NV = 33                                 # kL7Variants + 1 rows (the last: staging-only waves)
buf = (ctypes.c_ulonglong * (8 * NV))()
bench.main()
lib.dts_debug_ladder7_stamps(buf, 0)
names = ["vm wait", "barrier", "dma issue", "H", "V", "tail"]
for v in range(NV):
    row = buf[8 * v: 8 * v + 8]
    gran, waves = row[6], row[7]
    if not waves:
        continue
    tot = sum(row[:6])
    print(f"variant {v}: waves {waves}, granules/wave {gran / waves:.0f}, cycles/granule {tot / gran:.0f}, "
          f"cycles/wave {tot / waves:.0f}")
    for k, n in enumerate(names):
        print(f"    {n:10s} {row[k] / gran:8.0f} cycles/granule  {100.0 * row[k] / max(1, tot):5.1f} %")
