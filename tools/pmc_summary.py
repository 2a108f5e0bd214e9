#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of the path kernel: per-dispatch counters of the timed
(non-instrumented) launches and derived ratios.  usage: tools/pmc_summary.py DIR [kernel-substring]"""
import collections
import csv
import glob
import os
import sys

import json

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].endswith(".json") else None  # None: either path kernel
PATH_KERNELS = ("path_kernel", "rt_path_const")  # generic template instances, the scene-specialised build
json_out = next((a for a in sys.argv[2:] if a.endswith(".json")), None)
agg = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for f in glob.glob(os.path.join(d, "pmc*", "pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        kname = r["Kernel_Name"]
        i = kname.find("path_kernel")
        tmpl = kname[i:].split(">")[0] if i >= 0 else ""
        # template arguments: path_kernel<CULL, LDS, STATS, VN>, path_kernel_bvh<WIDTH, STACK, LDS, STATS, VN>
        targs = [a.strip() for a in tmpl.split("<", 1)[1].split(",")] if "<" in tmpl else []
        stats_arg = targs[3] if tmpl.startswith("path_kernel_bvh") and len(targs) > 3 else \
            (targs[2] if len(targs) > 2 else "false")
        hit = (sub in kname) if sub else any(k in kname for k in PATH_KERNELS)
        if hit and stats_arg != "true":  # skip the instrumented (STATS) variant and probes
            key = (os.path.basename(os.path.dirname(f)), int(r["Dispatch_Id"]))
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            names[key] = r["Kernel_Name"][:70]
by_pass = collections.defaultdict(list)
for (p, disp), v in sorted(agg.items()):
    by_pass[p].append(v)
tot = {}
for p, lst in by_pass.items():
    last = lst[-1]  # the last timed dispatch of that pass
    tot.update(last)
for k in sorted(tot):
    print(f"{k:24s} {tot[k]:.6g}")
if "SQ_INSTS_VALU" in tot and "SQ_WAVES" in tot:
    print("VALU instr per wave", tot["SQ_INSTS_VALU"] / tot["SQ_WAVES"])
    print("SALU/VALU", tot["SQ_INSTS_SALU"] / tot["SQ_INSTS_VALU"])
if "GRBM_GUI_ACTIVE" in tot and "SQ_INSTS_VALU" in tot:
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs: cycles per SIMD = GRBM / 8
    simd_cycles = tot["GRBM_GUI_ACTIVE"] / 8
    per_simd = tot["SQ_INSTS_VALU"] / 1024  # 256 CUs x 4 SIMDs
    print("VALU wave-instructions per SIMD-cycle", per_simd / simd_cycles,
          "(issue-bound near 1/3.4: 2-cycle fp32 add/mul/fma mixed with 4-cycle SGPR-operand, compare, "
          "select and min/max forms, tools/micro/valu_forms.hip)")
if "SQ_THREAD_CYCLES_VALU" in tot and "SQ_ACTIVE_INST_VALU" in tot:
    print("VALU lane utilisation", tot["SQ_THREAD_CYCLES_VALU"] / (64 * tot["SQ_ACTIVE_INST_VALU"]))
if "TA_BUSY_avr" in tot and "GRBM_GUI_ACTIVE" in tot:
    # the vector-memory pipeline; TA_BUSY_avr is per CU, GRBM_GUI_ACTIVE summed over 8 XCDs
    print("TA busy fraction", tot["TA_BUSY_avr"] / (tot["GRBM_GUI_ACTIVE"] / 8))
if "TCP_TOTAL_CACHE_ACCESSES_sum" in tot and "TCP_TCC_READ_REQ_sum" in tot:
    print("L1 (TCP) hit rate", 1 - tot["TCP_TCC_READ_REQ_sum"] / tot["TCP_TOTAL_CACHE_ACCESSES_sum"])
if "TCP_TCC_READ_REQ_LATENCY_sum" in tot and tot.get("TCP_TCC_READ_REQ_sum", 0) > 1e7:  # (C2/C3: too few to average)
    print("L1 -> L2 read latency (cycles)", tot["TCP_TCC_READ_REQ_LATENCY_sum"] / tot["TCP_TCC_READ_REQ_sum"])
if "TCP_PENDING_STALL_CYCLES_sum" in tot and "GRBM_GUI_ACTIVE" in tot:
    print("L1 pending-stall fraction", tot["TCP_PENDING_STALL_CYCLES_sum"] / 256 / (tot["GRBM_GUI_ACTIVE"] / 8))
if json_out and "FETCH_SIZE" in tot and "WRITE_SIZE" in tot:
    # rocprofv3 reports kB; on gfx950 FETCH_SIZE counts half the bytes of wide reads (MI355X_MICROARCH.md, HBM)
    rec = {"fetch_size_kb": tot["FETCH_SIZE"], "write_size_kb": tot["WRITE_SIZE"],
           "traffic_bytes": 2 * tot["FETCH_SIZE"] * 1024 + tot["WRITE_SIZE"] * 1024,
           "note": "per path-kernel launch; FETCH_SIZE doubled per the gfx950 correction", "source": d}
    # the compute view's hardware figures (bench.py roofline.counter_view): FP32 FLOP counter per
    # launch (x 64 lanes per wave-level count), VALU issue rate and lane utilisation
    if "SQ_INSTS_VALU_FLOPS_FP32" in tot:
        rec["valu_flops_fp32"] = tot["SQ_INSTS_VALU_FLOPS_FP32"]
    if "GRBM_GUI_ACTIVE" in tot and "SQ_INSTS_VALU" in tot:
        rec["valu_issue_per_simd_cycle"] = round(tot["SQ_INSTS_VALU"] / 1024 / (tot["GRBM_GUI_ACTIVE"] / 8), 4)
    if "SQ_THREAD_CYCLES_VALU" in tot and "SQ_ACTIVE_INST_VALU" in tot:
        rec["valu_lane_utilisation"] = round(tot["SQ_THREAD_CYCLES_VALU"] / (64 * tot["SQ_ACTIVE_INST_VALU"]), 4)
    json.dump(rec, open(json_out, "w"), indent=1)
    print("wrote", json_out, rec["traffic_bytes"])
