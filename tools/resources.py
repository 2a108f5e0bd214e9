#!/usr/bin/env python3
"""Register / occupancy / LDS report of the path kernels (compiles kernels_path.hip for gfx950)."""
import re
import subprocess
import sys

extra = sys.argv[1:]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "--offload-arch=gfx950", "-x", "hip", "-c",
       "raytracercore_amd/csrc/kernels_path.hip", "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        k = re.search(r"N_1\d+(\w+?)I(.*?)EEEv", cur)
        cur = (k.group(1) + "<" + k.group(2) + ">") if k else cur[:40]
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    print(f"{k:40s} VGPR {v.get('VGPRs','?'):>4} SGPR {v.get('SGPRs','?'):>4} spillV {v.get('VGPRs Spill','?'):>3} "
          f"spillS {v.get('SGPRs Spill','?'):>3} occ {v.get('Occupancy','?')} LDS {v.get('LDS Size','?')}")
