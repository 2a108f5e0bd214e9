#!/usr/bin/env python3
"""Recomputes bench.py's roofline fraction from a rocprofv3 kernel-trace summary: the dominant path
kernel's average duration (kernel_stats.csv) with the per-launch work of the same run's bench line
(path_stats: FLOP or bytes per ray segment, rays per launch).
usage: tools/roofline_from_profile.py KERNEL_STATS.csv BENCH_LINE.json"""
import csv
import json
import sys

stats, line = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(stats)))
# the timed path kernel: the scene-specialised build, else the uninstrumented generic kernel with
# the most calls (the instrumented variant and the AUTO calibration probe run once each)
paths = [r for r in rows if r["Name"] == "rt_path_const" or ("path_kernel" in r["Name"] and int(r["Calls"]) > 1)]
k = max(paths, key=lambda r: float(r["TotalDurationNs"]))
avg_ms = float(k["AverageNs"]) / 1e6
d = json.loads(open(line).read())
ps, rf = d["path_stats"], d["roofline"]
work = ps["flop_per_ray"] if rf["unit"] == "TFLOP/s" else ps["bytes_per_ray"]
scale = 1e12 if rf["unit"] == "TFLOP/s" else 1e9
achieved = work * ps["rays_per_launch"] / (avg_ms * 1e-3) / scale
print(json.dumps({"kernel": k["Name"][:60], "calls": int(k["Calls"]), "rocprof_avg_ms": round(avg_ms, 3),
                  "bench_kernel_ms_same_run": d["kernel_ms"], "ms_per_step_same_run": d["ms_per_step"],
                  "work_per_ray": work, "rays_per_launch": ps["rays_per_launch"], "unit": rf["unit"],
                  "achieved": round(achieved, 3), "peak": rf["peak"], "frac": round(achieved / rf["peak"], 4)}))
