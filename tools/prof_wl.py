#!/usr/bin/env python3
"""Condense tools/prof_wl.sh output (gpurun_out/prof_<tag>_<wl>/) into profiles/<tag>_<wl>.json
and profiles/pmc_<wl>.json (the file bench.py reads for roofline.traffic).

Per step of the workload (the last (steps + warmup) steps' libdts dispatches; setup dispatches
such as k_synth and cfg5's reference-rendition launch are dropped):
  - each kernel's dispatches per step, average duration (kernel trace) and PMC bytes;
  - traffic per frame = FETCH_SIZE KiB x 1024 x 2 (gfx950 16-B streaming-read correction,
    MI355X_MICROARCH.md; Infinity-Cache hits are counted as fetches, so this is an upper bound on
    HBM reads) + WRITE_SIZE KiB x 1024, summed over the step's kernels, / frames per step;
  - clock = GRBM_GUI_ACTIVE per dispatch / 8 XCDs / the dispatch's traced duration;
  - the bench line printed by the profiled process itself (same run as the trace).
usage: tools/prof_wl.py TAG WORKLOAD [STEPS WARMUP]
"""
import collections
import csv
import glob
import json
import os
import shutil
import statistics
import sys

tag, wl = sys.argv[1], sys.argv[2]
S = int(sys.argv[3]) + int(sys.argv[4]) if len(sys.argv) > 4 else 10
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out", f"prof_{tag}_{wl}")
dst = os.path.join(root, "profiles")


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("dts::", "")
    return n.split("(")[0]


def step_rows(rows):
    """The libdts dispatches of the last S steps, in dispatch order."""
    rows = [r for r in rows if "dts::" in r["Kernel_Name"] and "k_synth" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0)))
    per_step = max(1, round(len(rows) / S))
    return rows[-per_step * S:], per_step


def one(path_glob):
    f = glob.glob(os.path.join(src, path_glob), recursive=True)
    return f[0] if f else None


def bench_line(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    return None


kt_csv = one("kt/**/*kernel_trace.csv")
trace = list(csv.DictReader(open(kt_csv)))
for r in trace:
    r["Kernel_Name"] = r.get("Kernel_Name", r.get("Kernel-Name", ""))
    r["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
tr, per_step = step_rows(trace)
line = bench_line(os.path.join(src, "kt.log"))
B = line["roofline"]["frames_per_launch"]
kern = collections.OrderedDict()
for r in tr:
    k = kern.setdefault(short(r["Kernel_Name"]), {"dispatches": 0, "ns": []})
    k["dispatches"] += 1
    k["ns"].append(r["ns"])
step_ns = sum(r["ns"] for r in tr) / S

pmc = collections.defaultdict(lambda: collections.defaultdict(float))
for sub in ("fetch", "write", "grbm", "sq1", "sq2"):
    f = one(f"{sub}/**/*counter_collection.csv")
    if not f:
        continue
    rows = list(csv.DictReader(open(f)))
    by_disp = collections.OrderedDict()
    for r in rows:
        by_disp.setdefault(r["Dispatch_Id"], []).append(r)
    disp = [{"Kernel_Name": rs[0]["Kernel_Name"], "Dispatch_Id": d, "rs": rs} for d, rs in by_disp.items()]
    sel, _ = step_rows(disp)
    for d in sel:
        for r in d["rs"]:
            pmc[short(d["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])

out = {"tag": tag, "workload": wl, "steps_profiled": S, "frames_per_step": B, "dispatches_per_step": per_step,
       "kernels": {}, "note": __doc__.split("\n\n")[0]}
tot_rd = tot_wr = 0.0
have_bytes = True
for name, k in kern.items():
    n = k["dispatches"]
    e = {"dispatches_per_step": n / S, "avg_ns": round(statistics.mean(k["ns"]), 1),
         "ms_per_step": round(sum(k["ns"]) / S / 1e6, 4)}
    c = pmc.get(name, {})
    for cn, v in sorted(c.items()):
        e.setdefault("pmc_per_dispatch", {})[cn] = v / n
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rd, wr = c["FETCH_SIZE"] * 1024 * 2 / S, c["WRITE_SIZE"] * 1024 / S
        e["read_bytes_per_frame"] = round(rd / B)
        e["write_bytes_per_frame"] = round(wr / B)
        tot_rd += rd
        tot_wr += wr
    else:
        have_bytes = False
    if "GRBM_GUI_ACTIVE" in c:
        e["clock_ghz"] = round(c["GRBM_GUI_ACTIVE"] / n / 8 / statistics.mean(k["ns"]), 3)
    out["kernels"][name] = e
algo = line["algo_bytes_per_frame"]
out["step_kernel_ms"] = round(step_ns / 1e6, 4)
out["algo_bytes_per_frame"] = algo
out["frac_from_trace"] = round(algo * B / (step_ns * 1e-9) / 8e12, 4)
if have_bytes:
    out["traffic_bytes_per_frame"] = round((tot_rd + tot_wr) / B)
    out["read_bytes_per_frame"] = round(tot_rd / B)
    out["write_bytes_per_frame"] = round(tot_wr / B)
    out["traffic_ratio"] = round((tot_rd + tot_wr) / B / algo, 3)
out["line_in_profiled_run"] = {k: line.get(k) for k in ("value", "ms_per_step")}
out["line_in_profiled_run"]["kernel_ms_per_launch"] = line["roofline"]["kernel_ms_per_launch"]
out["line_in_profiled_run"]["frac"] = line["roofline"]["frac"]
os.makedirs(dst, exist_ok=True)
json.dump(out, open(os.path.join(dst, f"{tag}_{wl}.json"), "w"), indent=1)
if have_bytes:
    json.dump({"tag": tag, "workload": wl, "hbm_bytes_per_frame": out["traffic_bytes_per_frame"],
               "read_bytes_per_frame": out["read_bytes_per_frame"],
               "write_bytes_per_frame": out["write_bytes_per_frame"]},
              open(os.path.join(dst, f"pmc_{wl}.json"), "w"), indent=1)
# the unprofiled bench line of the same box and build (prof_wl.sh LINE=1): its traffic from this profile
lp = os.path.join(src, "line.log")
if os.path.exists(lp) and bench_line(lp) is not None:
    bl = bench_line(lp)
    if have_bytes:
        r = bl["roofline"]
        r["traffic_bytes_per_frame"] = out["traffic_bytes_per_frame"]
        r["traffic"] = round(out["traffic_bytes_per_frame"] * r["frames_per_launch"] /
                             (r["kernel_ms_per_launch"] * 1e-3) / 1e9, 1)
        r["traffic_profile"] = f"{tag}_{wl}"
    json.dump(bl, open(os.path.join(dst, f"{tag}_bench_{wl}.json"), "w"))
    out["unprofiled_line"] = {"value": bl["value"], "kernel_ms_per_launch": bl["roofline"]["kernel_ms_per_launch"],
                              "frac": bl["roofline"]["frac"]}
    json.dump(out, open(os.path.join(dst, f"{tag}_{wl}.json"), "w"), indent=1)
st = one("kt/**/*kernel_stats.csv")
if st:
    shutil.copy(st, os.path.join(dst, f"{tag}_{wl}_kernel_stats.csv"))
print(json.dumps({k: out[k] for k in out if k not in ("kernels", "note")}))
for n, e in out["kernels"].items():
    print(f"  {n}: {e.get('dispatches_per_step')}/step {e['ms_per_step']} ms/step "
          f"rd {e.get('read_bytes_per_frame')} wr {e.get('write_bytes_per_frame')} clk {e.get('clock_ghz')}")
