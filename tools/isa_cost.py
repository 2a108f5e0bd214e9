#!/usr/bin/env python3
"""Static issue-cost estimate of one kernel by source function, with the gfx950 VALU cost table
measured by tools/micro/valu_forms.hip (cycles per wave64 instruction per SIMD at full
occupancy): 2 for fp32 add/sub/mul/fma/fmac and int add/sub/xor/and/or/shift on VGPRs and inline
constants; 4 with an SGPR operand and for compares, cndmask, min/max/med3, int mul, 3-operand
int ops, conversions, readlane/writelane; 8 for transcendentals.  Loops over primitives count
once.  usage: tools/isa_cost.py LISTING.s KERNEL_SYMBOL_PREFIX SOURCE.hip [LINE_FROM LINE_TO]"""
import collections
import re
import sys

listing, ksym, src = sys.argv[1:4]
lines = open(src).read().split("\n")
func_at, cur = {}, "?"
for i, l in enumerate(lines, 1):
    m = re.match(r"^(?:template.*)?(?:__device__|__global__|static|inline).*?\b(\w+)\s*\(", l)
    if m and not l.strip().endswith(";"):
        cur = m.group(1)
    if re.match(r"^\s+path_kernel(_bvh)?\(", l):
        cur = "path_kernel"
    func_at[i] = cur
FAST = re.compile(r"^v_(add|sub|subrev|mul|fma|fmac|fmaak|fmamk)_f32|^v_(add|sub|subrev)_u32|^v_(xor|and|or|not)_b32"
                  r"|^v_(lshlrev|lshrrev|ashrrev)_b32|^v_mov_b32|^v_pk_mov")
TRANS = re.compile(r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32")
cost = collections.Counter()
count = collections.Counter()
inside, file_no, line_no, main_file = False, 0, 0, None
files = {}
for l in open(listing):
    m = re.match(r"\s*\.file\s+(\d+)\s+\"([^\"]*)\"(?:\s+\"([^\"]*)\")?", l)
    if m:
        files[int(m.group(1))] = (m.group(3) or m.group(2))
    if l.startswith(ksym):
        inside = True
        continue
    if not inside:
        continue
    if l.startswith(".Lfunc_end"):
        break
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        file_no, line_no = int(m.group(1)), int(m.group(2))
        continue
    m = re.match(r"\s+([sv]_\w+|global_\w+|buffer_\w+|ds_\w+|scratch_\w+|flat_\w+)\s*(.*)", l)
    if not m:
        continue
    op, args = m.group(1), m.group(2)
    fname = files.get(file_no, "?")
    key = func_at.get(line_no, "?") if fname.endswith(src.split("/")[-1]) else fname.split("/")[-1]
    if op.startswith("v_"):
        if TRANS.match(op):
            c = 8
        elif FAST.match(op) and not re.search(r"\bs\[?\d|vcc|exec", args.split(";")[0]):
            c = 2
        elif op.startswith("v_pk_"):
            c = 4.5
        else:
            c = 4
        cost[(key, "VALU")] += c
        count[(key, "VALU")] += 1
    elif op.startswith("s_"):
        count[(key, "SALU")] += 1
    else:
        count[(key, "MEM")] += 1
rows = sorted({k for k, _ in count}, key=lambda k: -cost[(k, "VALU")])
tot = sum(cost.values())
for k in rows:
    print(f"{k:28s} VALU {count[(k, 'VALU')]:5d} instr {cost[(k, 'VALU')]:7.0f} cyc ({100 * cost[(k, 'VALU')] / tot:4.1f}%)"
          f"  SALU {count[(k, 'SALU')]:4d}  MEM {count[(k, 'MEM')]:3d}")
print(f"total VALU cycles (static) {tot:.0f}")
