#!/usr/bin/env python3
"""Summarise tools/ab_c4.sh output: per variant the kernel time, rays, and per-launch counters per
ray segment.  usage: tools/ab_c4_summary.py gpurun_out/ab_TAG"""
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
print(f"{'variant':16s} {'kern ms':>8s} {'Grays/s':>8s} {'WRITE GB':>9s} {'lookups/ray':>11s} {'L2req/ray':>9s} "
      f"{'L2lat':>6s} {'TA busy':>7s} {'L2 hit':>7s} {'nodes':>6s} {'tris':>6s}")
for d in sorted(glob.glob(os.path.join(root, "*"))):
    v = os.path.basename(d)
    try:
        b = json.loads(open(os.path.join(d, "bench.json")).read().strip().splitlines()[-1])
    except Exception:
        continue
    rays = b["path_stats"]["rays_per_launch"]
    c = {}
    for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        last = {}
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "path_kernel_bvh" not in k or "true" in k.split("<", 1)[1].split(">")[0].split(",")[3]:
                continue
            last.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = \
                last.get(int(r["Dispatch_Id"]), {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if last:
            c.update(last[max(last)])
    g = c.get("GRBM_GUI_ACTIVE", 0.0)
    print(f"{v:16s} {b['kernel_ms']:8.2f} {rays / b['kernel_ms'] / 1e6:8.3f} "
          f"{c.get('WRITE_SIZE', float('nan')) * 1024 / 1e9:9.2f} "
          f"{c.get('TCP_TOTAL_CACHE_ACCESSES_sum', float('nan')) / rays:11.2f} "
          f"{c.get('TCP_TCC_READ_REQ_sum', float('nan')) / rays:9.2f} "
          f"{c.get('TCP_TCC_READ_REQ_LATENCY_sum', float('nan')) / max(1, c.get('TCP_TCC_READ_REQ_sum', 1)):6.0f} "
          f"{c.get('TA_BUSY_avr', float('nan')) / (g / 8) if g else float('nan'):7.3f} "
          f"{c.get('TCC_HIT_sum', float('nan')) / max(1, c.get('TCC_REQ_sum', 1)):7.3f} "
          f"{b['path_stats']['per_ray']['nodes']:6.2f} {b['path_stats']['per_ray']['tris']:6.2f}")
