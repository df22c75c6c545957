#!/usr/bin/env python3
"""Condense a tools/profile.sh run (gpurun_out/prof_<tag>/) into profiles/<tag>_*.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats
summary, copied verbatim) and profiles/<tag>_pmc.json: per-launch PMC totals of
the ladder kernel plus HBM bytes corrected per MI355X_MICROARCH.md (FETCH_SIZE
is reported in KiB and counts half the bytes of 16-B-per-lane streaming
reads -> x2; WRITE_SIZE exact for wide stores; Infinity-Cache hits are
counted as fetches, so this is an upper bound on HBM reads).
"""
import collections
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 32
kname = sys.argv[3] if len(sys.argv) > 3 else "k_ladder"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out", f"prof_{tag}")
dst = os.path.join(root, "profiles")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))

tot = collections.defaultdict(float)
launches = collections.Counter()
for sub in sorted(os.listdir(src)):
    if not sub.startswith("pmc_"):
        continue
    path = os.path.join(src, sub, f"{sub}_counter_collection.csv")
    if not os.path.exists(path):
        continue
    for r in csv.DictReader(open(path)):
        if kname not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        launches[(sub, r["Counter_Name"])] += 1
per = {}
for c, v in tot.items():
    n = max(n for (s, cc), n in launches.items() if cc == c)
    per[c] = v / n
out = {"tag": tag, "kernel": kname, "frames_per_launch": frames, "per_launch": per}
if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
    rd = per["FETCH_SIZE"] * 1024 * 2
    wr = per["WRITE_SIZE"] * 1024
    out["hbm_read_bytes_per_launch"] = rd
    out["hbm_write_bytes_per_launch"] = wr
    out["hbm_bytes_per_frame"] = (rd + wr) / frames
    out["note"] = ("FETCH_SIZE KiB x1024 x2 (gfx950 16-B streaming-read correction), WRITE_SIZE KiB x1024; "
                   "Infinity-Cache hits are included in FETCH_SIZE (upper bound on HBM reads)")
stats = list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))))
for s in stats:
    if kname in s["Name"]:
        out["avg_kernel_ns"] = float(s["AverageNs"])
        out["calls"] = int(s["Calls"])
json.dump(out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
json.dump(out, open(os.path.join(dst, "pmc_latest.json"), "w"), indent=1)   # read by bench.py
print(json.dumps(out, indent=1))
