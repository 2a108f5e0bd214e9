#!/usr/bin/env python3
"""Static instruction mix of one kernel by source function: compiles nothing, reads a -g -S
listing.  usage: tools/isa_by_line.py LISTING.s KERNEL_SYMBOL_PREFIX SOURCE.hip"""
import collections
import re
import sys

listing, ksym, src = sys.argv[1:4]
lines = open(src).read().split("\n")
# function extents: a line starting a definition "...name(" at column 0 or "__device__ ... name("
func_at = {}
cur = "?"
for i, l in enumerate(lines, 1):
    m = re.match(r"^(?:template.*)?(?:__device__|__global__|static|inline).*?\b(\w+)\s*\(", l)
    if m and not l.strip().endswith(";"):
        cur = m.group(1)
    m2 = re.match(r"^\s+path_kernel\(", l)
    if m2:
        cur = "path_kernel"
    func_at[i] = cur
files = {}
inside = False
count = collections.Counter()
loc_line, loc_file = 0, 0
for l in open(listing):
    if l.startswith(ksym):
        inside = True
        continue
    if inside and l.startswith(".Lfunc_end"):
        break
    if l.startswith("\t.file"):
        m = re.match(r'\t\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[int(m.group(1))] = (m.group(3) or m.group(2))
        continue
    if not inside:
        continue
    m = re.match(r"\s+\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        loc_file, loc_line = int(m.group(1)), int(m.group(2))
        continue
    m = re.match(r"\s+([vs]_\w+|global_\w+|ds_\w+|buffer_\w+)", l)
    if not m:
        continue
    op = m.group(1)
    kind = "VALU" if op.startswith("v_") else "SALU" if op.startswith("s_") else "MEM"
    fname = files.get(loc_file, "?")
    where = func_at.get(loc_line, "?") if fname.endswith(src.split("/")[-1]) else fname.split("/")[-1]
    count[(where, kind)] += 1
tot = collections.Counter()
for (w, k), n in count.items():
    tot[w] += n
for w, n in tot.most_common():
    print(f"{w:28s} VALU {count[(w,'VALU')]:5d}  SALU {count[(w,'SALU')]:5d}  MEM {count[(w,'MEM')]:4d}")
