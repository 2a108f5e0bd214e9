#!/usr/bin/env python3
"""Census of a kernel's VALU instructions by source section and instruction class.

Reads the disassembly of a code object built with -g (tools/jit_isa.py HEADER 0 OUT -g for the
scene-specialised kernel), attributes every VALU instruction by its inline chain (llvm-symbolizer -i)
to the innermost kernels_path.hip function that is not a one-line helper (dot, madd, rcp, ...:
their instructions count for the caller; rtcore_rng.h code counts as "rng"), and counts the
instructions per class with the gfx950 issue costs of DESIGN.md §3.2 (tools/micro/valu_forms.hip):

  arith   fp32 add/sub/mul/fma/fmac/fmaak/fmamk, int add/sub/xor/and/or/not, shifts: 2 cycles,
          4 with an SGPR operand (counted as `arith_s`)
  cmp     v_cmp*                                   4
  cnd     v_cndmask                                4
  minmax  v_min*/v_max*/v_med3*                    4
  mov     v_mov (2), v_readlane/v_writelane/readfirstlane (4)
  trans   rcp/rsq/sqrt/exp/log/sin/cos             8
  other   3-operand int ops, conversions, mul_lo/hi, ldexp, bfe, ...  4

A static census: loops count once (the bounce.txt specialised query is straight-line code).
usage: tools/isa_census.py CODE_OBJECT.co [KERNEL_SYMBOL_SUBSTRING]
"""
import collections
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin/"
# one-line helpers whose instructions are charged to the function that calls them
HELPERS = {"dot", "dot3", "dot4", "xyz", "v3", "madd", "kfma", "kmul", "known_zero", "cross", "rcp", "fsqrt", "normalize",
           "vmin", "vmax", "vmin3", "vmax3", "vmax0", "vmax1", "operator+", "operator-", "operator*", "xf_point", "xf_dir",
           "pack_sg", "next_u", "pin4", "ubyte", "cswap", "slab_rcp", "slab_rcp_lean", "cam_frustum", "cam_dof",
           "renormalise_at"}
ARITH = re.compile(r"^v_(add|sub|subrev|mul|fma|fmac|fmaak|fmamk)_f32|^v_(add|sub|subrev)_(u32|i32|co_u32|co_ci_u32)"
                   r"|^v_(xor|and|or|not)_b32|^v_(lshlrev|lshrrev|ashrrev)_b32")
TRANS = re.compile(r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32")
MINMAX = re.compile(r"^v_(min|max|med3|min3|max3)")
MOV = re.compile(r"^v_(mov|readlane|writelane|readfirstlane)")
CLASSES = ["arith", "arith_s", "cmp", "cnd", "minmax", "mov", "trans", "other"]


def cls(op, args):
    if op.startswith("v_cmp"):
        return "cmp", 4
    if op.startswith("v_cndmask"):
        return "cnd", 4
    if MINMAX.match(op):
        return "minmax", 4
    if TRANS.match(op):
        return "trans", 8
    if MOV.match(op):
        return "mov", 2 if op.startswith("v_mov") else 4
    if ARITH.match(op):
        return ("arith_s", 4) if re.search(r"\bs\[?\d", args) else ("arith", 2)
    return "other", 4


def section(block):
    frames = block.split("\n")
    chain = []  # innermost first: (function short name, location)
    for k in range(0, len(frames) - 1, 2):
        fn, loc = frames[k], frames[k + 1]
        short = re.sub(r"\(.*", "", fn.replace("(anonymous namespace)", "anon"))  # drop the argument list
        short = re.sub(r"<[^<>]*>", "", re.sub(r"<[^<>]*>", "", short))  # template arguments (two levels)
        short = short.split("::")[-1].split(" ")[-1]
        chain.append((short, loc))
    for short, loc in chain:
        if "rtcore_rng.h" in loc:
            return "rng"
        if "kernels_path.hip" in loc and short not in HELPERS:
            return short
    return chain[-1][0] if chain else "?"


def main():
    co = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else None  # a kernel symbol (substring); default: every function
    dis = subprocess.run([LLVM + "llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True, text=True,
                         check=True).stdout
    insts = []
    inside = want is None
    for l in dis.split("\n"):
        m = re.match(r"^[0-9A-Fa-f]+ <(.*)>:", l)
        if m and want is not None:
            inside = want in m.group(1)
            continue
        m = re.match(r"\s+(v_\w+)\s*(.*?)//\s*([0-9A-Fa-f]+):", l)
        if m and inside:
            insts.append((m.group(1), m.group(2), int(m.group(3), 16)))
    sym = subprocess.run([LLVM + "llvm-symbolizer", "--obj=" + co, "-i", "-C"],
                         input="\n".join(hex(a) for _, _, a in insts) + "\n", capture_output=True, text=True,
                         check=True).stdout
    blocks = sym.strip("\n").split("\n\n")
    assert len(blocks) == len(insts), (len(blocks), len(insts))
    count = collections.defaultdict(collections.Counter)
    cyc = collections.Counter()
    for (op, args, _), blk in zip(insts, blocks):
        key = section(blk)
        c, k = cls(op, args)
        count[key][c] += 1
        cyc[key] += k
    tot_n = sum(sum(v.values()) for v in count.values())
    tot_c = sum(cyc.values())
    print(f"{'section':20s} {'VALU':>5s} {'cycles':>7s} " + " ".join(f"{c:>7s}" for c in CLASSES))
    allc = collections.Counter()
    for key in sorted(count, key=lambda k: -cyc[k]):
        v = count[key]
        allc.update(v)
        print(f"{key:20s} {sum(v.values()):5d} {cyc[key]:7d} " + " ".join(f"{v[c]:7d}" for c in CLASSES))
    print(f"{'TOTAL':20s} {tot_n:5d} {tot_c:7d} " + " ".join(f"{allc[c]:7d}" for c in CLASSES))
    non = allc["cmp"] + allc["cnd"] + allc["minmax"] + allc["mov"]
    print(f"compares + selects + min/max + moves: {non} of {tot_n} VALU ({100 * non / max(1, tot_n):.1f} %)")


if __name__ == "__main__":
    main()
