"""Cost experiments on the path kernels, kept out of the product source.

Copies raytracercore_amd/csrc (and include/) into raytracercore_amd/variants/NAME/tree, applies the
named textual patches below to the copy of kernels_path.hip, and builds the library there
(raytracercore_amd/variants/NAME/librtcore_hip.so; load it with RTCORE_LIB=<path>).  The copy's
sources are what its scene-specialised builds embed, so the patches reach them too.

usage: python tools/exp_patch.py NAME PATCH[,PATCH...] ["EXTRA hipcc flags"]
       python tools/exp_patch.py --list
A patch is a list of (anchor, replacement) pairs; every anchor must occur exactly once.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "raytracercore_amd", "csrc")

TRACE_CALL = ("            trace_brute<CULL, STATS>(sc, groups, tests, rects, frames, boxes, xf, S.o, S.d, S.prev, b, cnt.tris,\n"
              "                                     cnt.sphs, cnt.nodes);\n")
BOUNCE_CALL = "            bounce<VN>(L, S, sc, R, vnormals, tests, pq->prims_d, b);\n"
RAYS_LINE = "        wave_rays += (unsigned)__popcll(__ballot(L.live)); // one Scene.RayTrace per live lane\n"

NODE_LOAD = '                    const Node4Q q = (ref & RT_HOT_BIT) ? lds_hot[ref & ~RT_HOT_BIT] : Node4Q(nodes4[ref]);\n'
HOT_ON = '    static const bool on = !(getenv("RTCORE_HOT_NODES") && getenv("RTCORE_HOT_NODES")[0] == \'0\'); // A/B switch\n'

PATCHES = {
    # every camera ray misses: the per-sample overhead alone
    "NO_TRACE": [(TRACE_CALL, "")],
    # a second bounce on a copy of the sample: the shading section's cost
    "DUP_SHADE": [(BOUNCE_CALL,
                   "            {\n"
                   "                Sample S2 = S;\n"
                   "                S2.rng.x ^= (unsigned)S.bounce;\n"
                   "                V3 c2;\n"
                   "                shade<VN>(sc, R.prims, R.mats, R.xfs, vnormals, tests, pq->prims_d, b, S2, c2);\n"
                   "                if (c2.x + S2.d.x == 1234.5f) pq->partial[0].x = 1.0f;\n"
                   "            }\n" + BOUNCE_CALL)],
    # a second camera sample on a copy: the sample start's cost
    "DUP_START": [(RAYS_LINE,
                   "        if (L.live) {\n"
                   "            Sample S2 = S;\n"
                   "            S2.rng.x ^= (unsigned)S.bounce;\n"
                   "            start_sample<true>(*cp, L.fx, L.fy, S2);\n"
                   "            if (S2.o.x + S2.d.y == 1234.5f) pq->partial[0].x = 1.0f;\n"
                   "        }\n" + RAYS_LINE)],
    # no depth of field in the sample start
    "NO_DOF": [("    if (cam_dof(cam)) {\n", "    if (false) {\n")],
    # the bounce direction never renormalised (round 3's brute-force form)
    "NO_RENORM": [("    S.d = out_dir * (renormalise_at<SLOT>(s, S.bounce + 1) ? fmaf(-0.5f, dot(out_dir, out_dir), 1.5f) : 1.0f);\n",
                   "    S.d = SLOT ? normalize(out_dir) : out_dir;\n")],
    # the renormalisation test as a plain remainder in every kernel
    "RENORM_MOD3": [("    if (SLOT) return (unsigned)i % 3u == 0u;\n", "    return (unsigned)i % 3u == 0u;\n")],
    # wide BVH visit without the child-count test (empty slots have inverted boxes; C4 -0.6 %, kept for safety)
    "WIDE_NO_NC": [("        D = ((K < nc) & (tmin <= fminf(tmax * 1.00000024f, tmax_best))) ? tmin : __builtin_huge_valf();         \\\n",
                    "        D = (tmin <= fminf(tmax * 1.00000024f, tmax_best)) ? tmin : __builtin_huge_valf();         \\\n")],
    # work items of one wave: the samples of one pixel (chunk-major) instead of one sample of the
    # 64 pixels of an 8x8 block (C4 ray-coherence probe: a wave's primary rays then meet one point)
    "SAMPLE_MAJOR": [("    const unsigned q = item & 63u, t = item >> 6;\n",
                      "    const unsigned q = (item >> p.log2_chunks) & 63u, t = ((item >> (p.log2_chunks + 6)) << p.log2_chunks) | (item & (unsigned)(p.n_chunks - 1));\n")],
    # leaf step: a record past the leaf's end is loaded from the leaf's first record instead (same
    # instructions, no spare line): the cost of the spare records' lines
    "NO_SPARE_LINE": [("        r[j][0] = rows[3 * (k + j)];\n"
                       "        r[j][1] = rows[3 * (k + j) + 1];\n"
                       "        r[j][2] = rows[3 * (k + j) + 2];\n",
                       "        const int kk = (j == 0 || k + j < kend) ? k + j : k;\n"
                       "        r[j][0] = rows[3 * kk];\n"
                       "        r[j][1] = rows[3 * kk + 1];\n"
                       "        r[j][2] = rows[3 * kk + 2];\n")],
    # leaf rows loaded non-temporally (streamed past L2, so the nodes stay there longer)
    "NT_ROWS": [("        r[j][0] = rows[3 * (k + j)];\n"
                 "        r[j][1] = rows[3 * (k + j) + 1];\n"
                 "        r[j][2] = rows[3 * (k + j) + 2];\n",
                 "        {\n"
                 "            typedef float ntf4 __attribute__((ext_vector_type(4)));\n"
                 "            typedef __attribute__((address_space(1))) const ntf4 gf4;\n"
                 "            gf4* g = (gf4*)(uintptr_t)(rows + 3 * (k + j));\n"
                 "            ntf4 a0 = __builtin_nontemporal_load(g), a1 = __builtin_nontemporal_load(g + 1),\n"
                 "                 a2 = __builtin_nontemporal_load(g + 2);\n"
                 "            r[j][0] = make_float4(a0.x, a0.y, a0.z, a0.w);\n"
                 "            r[j][1] = make_float4(a1.x, a1.y, a1.z, a1.w);\n"
                 "            r[j][2] = make_float4(a2.x, a2.y, a2.z, a2.w);\n"
                 "        }\n")],
    # wide nodes loaded non-temporally
    "NT_NODES": [("                    const Node4Q q = (ref & RT_HOT_BIT) ? lds_hot[ref & ~RT_HOT_BIT] : Node4Q(nodes4[ref]);\n"
                  "                    [[maybe_unused]] const int sp0 = sp;\n",
                  "                    Node4Q q;\n"
                  "                    if (ref & RT_HOT_BIT) q = lds_hot[ref & ~RT_HOT_BIT];\n"
                  "                    else {\n"
                  "                        typedef float ntf4 __attribute__((ext_vector_type(4)));\n"
                  "                        typedef __attribute__((address_space(1))) const ntf4 gf4;\n"
                  "                        gf4* g = (gf4*)(uintptr_t)(nodes4 + ref);\n"
                  "                        ntf4 a0 = __builtin_nontemporal_load(g), a1 = __builtin_nontemporal_load(g + 1),\n"
                  "                             a2 = __builtin_nontemporal_load(g + 2), a3 = __builtin_nontemporal_load(g + 3);\n"
                  "                        q.a = make_float4(a0.x, a0.y, a0.z, a0.w);\n"
                  "                        q.b = make_float4(a1.x, a1.y, a1.z, a1.w);\n"
                  "                        q.c = make_float4(a2.x, a2.y, a2.z, a2.w);\n"
                  "                        q.d = make_float4(a3.x, a3.y, a3.z, a3.w);\n"
                  "                    }\n"
                  "                    [[maybe_unused]] const int sp0 = sp;\n")],
    # round 6, C4 visit VALU: no hot-node table (no LDS-or-global select per visit)
    "WIDE_NOHOT": [(NODE_LOAD, "                    const Node4Q q = nodes4[ref];\n"),
                   (HOT_ON, "    static const bool on = false;\n")],
    # ... and the node read through a buffer resource with a 32-bit byte offset (no 64-bit address math)
    "WIDE_BUFLOAD": [(NODE_LOAD,
                      "                    Node4Q q;\n"
                      "                    {\n"
                      "                        typedef float v4f __attribute__((ext_vector_type(4)));\n"
                      "                        const __amdgpu_buffer_rsrc_t rs =\n"
                      "                            __builtin_amdgcn_make_buffer_rsrc((void*)pq->nodes4, (short)0, -1, 0x00020000);\n"
                      "                        const unsigned off = (unsigned)ref << 6;\n"
                      "                        const v4f a0 = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);\n"
                      "                        const v4f a1 = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0);\n"
                      "                        const v4f a2 = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 32, 0, 0);\n"
                      "                        const v4f a3 = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 48, 0, 0);\n"
                      "                        q.a = make_float4(a0.x, a0.y, a0.z, a0.w);\n"
                      "                        q.b = make_float4(a1.x, a1.y, a1.z, a1.w);\n"
                      "                        q.c = make_float4(a2.x, a2.y, a2.z, a2.w);\n"
                      "                        q.d = make_float4(a3.x, a3.y, a3.z, a3.w);\n"
                      "                    }\n"),
                     (HOT_ON, "    static const bool on = false;\n")],
    # the buffer-resource node read with the hot-node table kept (LDS for the top of the tree)
    "WIDE_BUFLOAD_HOT": [(NODE_LOAD,
                          "                    Node4Q q;\n"
                          "                    if (ref & RT_HOT_BIT) q = lds_hot[ref & ~RT_HOT_BIT];\n"
                          "                    else {\n"
                          "                        typedef float v4f __attribute__((ext_vector_type(4)));\n"
                          "                        const __amdgpu_buffer_rsrc_t rs =\n"
                          "                            __builtin_amdgcn_make_buffer_rsrc((void*)pq->nodes4, (short)0, -1, 0x00020000);\n"
                          "                        const unsigned off = (unsigned)ref << 6;\n"
                          "                        const v4f a0 = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);\n"
                          "                        const v4f a1 = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0);\n"
                          "                        const v4f a2 = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 32, 0, 0);\n"
                          "                        const v4f a3 = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 48, 0, 0);\n"
                          "                        q.a = make_float4(a0.x, a0.y, a0.z, a0.w);\n"
                          "                        q.b = make_float4(a1.x, a1.y, a1.z, a1.w);\n"
                          "                        q.c = make_float4(a2.x, a2.y, a2.z, a2.w);\n"
                          "                        q.d = make_float4(a3.x, a3.y, a3.z, a3.w);\n"
                          "                    }\n")],
    # the leaf step's rows through a buffer resource too (32-bit byte offsets)
    "LEAF_BUFLOAD": [("        r[j][0] = rows[3 * (k + j)];\n"
                      "        r[j][1] = rows[3 * (k + j) + 1];\n"
                      "        r[j][2] = rows[3 * (k + j) + 2];\n",
                      "        {\n"
                      "            typedef float v4f __attribute__((ext_vector_type(4)));\n"
                      "            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)rows, (short)0, -1, 0x00020000);\n"
                      "            const unsigned off = (unsigned)(k + j) * 48u;\n"
                      "            const v4f a0 = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);\n"
                      "            const v4f a1 = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0);\n"
                      "            const v4f a2 = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 32, 0, 0);\n"
                      "            r[j][0] = make_float4(a0.x, a0.y, a0.z, a0.w);\n"
                      "            r[j][1] = make_float4(a1.x, a1.y, a1.z, a1.w);\n"
                      "            r[j][2] = make_float4(a2.x, a2.y, a2.z, a2.w);\n"
                      "        }\n")],
    # the 4-child sort without its last exchange (the two middle pushes in either order)
    "WIDE_SORT4": [("    cswap(d1, r1, d2, r2);\n", "")],
    # the direction's signs computed once per query (after the shading phase) instead of per visit
    "WIDE_SIGNS": [("                                           const TravStack& stk, bool& pop)\n",
                    "                                           const TravStack& stk, bool& pop, bool sgx, bool sgy, bool sgz)\n"),
                   ("    const uint32_t nx = id.x >= 0.0f ? lx : hx, fx = id.x >= 0.0f ? hx : lx;\n"
                    "    const uint32_t ny = id.y >= 0.0f ? ly : hy, fy = id.y >= 0.0f ? hy : ly;\n"
                    "    const uint32_t nz = id.z >= 0.0f ? lz : hz, fz = id.z >= 0.0f ? hz : lz;\n",
                    "    const uint32_t nx = sgx ? lx : hx, fx = sgx ? hx : lx;\n"
                    "    const uint32_t ny = sgy ? ly : hy, fy = sgy ? hy : ly;\n"
                    "    const uint32_t nz = sgz ? lz : hz, fz = sgz ? hz : lz;\n"),
                   ("    V3 id{0, 0, 0};\n    Best b{", "    V3 id{0, 0, 0};\n    bool sgx = true, sgy = true, sgz = true;\n    Best b{"),
                   ("            id = v3(slab_rcp(S.d.x), slab_rcp(S.d.y), slab_rcp(S.d.z));\n",
                    "            id = v3(slab_rcp(S.d.x), slab_rcp(S.d.y), slab_rcp(S.d.z));\n"
                    "            sgx = id.x >= 0.0f;\n            sgy = id.y >= 0.0f;\n            sgz = id.z >= 0.0f;\n"),
                   ("                    wide_visit<STACK>(q, id, oi, b.t, ref, sp, stk, pop);\n",
                    "                    wide_visit<STACK>(q, id, oi, b.t, ref, sp, stk, pop, sgx, sgy, sgz);\n"),
                   ("                wide_visit<STACK>(q, id, S.o * id, b.t, ref, sp, stk, pop);\n",
                    "                wide_visit<STACK>(q, id, S.o * id, b.t, ref, sp, stk, pop, id.x >= 0.0f, id.y >= 0.0f, id.z >= 0.0f);\n"),
                   ("                wide_visit<STACK>(q, id, oi, b.t, ref, sp, stk, pop);\n",
                    "                wide_visit<STACK>(q, id, oi, b.t, ref, sp, stk, pop, id.x >= 0.0f, id.y >= 0.0f, id.z >= 0.0f);\n")],
    # no literal folding of zero scene fields in the specialised build
    "NO_KFOLD": [("    return __builtin_constant_p(c) && c == 0.0f;\n", "    return false;\n")],
}


def apply(src: str, names: list[str]) -> str:
    for name in names:
        for anchor, repl in PATCHES[name]:
            n = src.count(anchor)
            if n != 1:
                sys.exit(f"patch {name}: anchor found {n} times:\n{anchor}")
            src = src.replace(anchor, repl)
    return src


def main() -> None:
    if len(sys.argv) >= 2 and sys.argv[1] == "--list":
        print("\n".join(sorted(PATCHES)))
        return
    if len(sys.argv) < 3:
        sys.exit(__doc__)
    name, names = sys.argv[1], [p for p in sys.argv[2].split(",") if p and p != "NONE"]
    extra = sys.argv[3] if len(sys.argv) > 3 else ""
    for p in names:
        if p not in PATCHES:
            sys.exit(f"unknown patch {p} (known: {', '.join(sorted(PATCHES))})")
    out = os.path.join(ROOT, "raytracercore_amd", "variants", name)
    tree = os.path.join(out, "tree")
    shutil.rmtree(tree, ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tree, "include"))
    dst = os.path.join(tree, "raytracercore_amd", "csrc")  # the repository's layout (source_hash.py)
    shutil.copytree(CSRC, dst, ignore=shutil.ignore_patterns("_obj*"))
    kp = os.path.join(dst, "kernels_path.hip")
    with open(kp) as f:
        src = f.read()
    with open(kp, "w") as f:
        f.write(apply(src, names))
    jobs = str(min(16, os.cpu_count() or 8))
    subprocess.run(["make", "-s", "-C", dst, "-j" + jobs, "OUT=" + out, "EXTRA=" + extra], check=True)
    print(os.path.join(out, "librtcore_hip.so"))


if __name__ == "__main__":
    main()
