// kernels_path.hip -- the persistent fp32 path-tracing kernel for gfx950.
//
// One launch renders `spp` samples for every pixel of a tile.  Work items are
// (sample chunk, pixel) pairs dealt out by a wave-aggregated atomic; each lane owns one item
// at a time and regenerates a new camera path the iteration after its previous path ends,
// so every loop iteration issues exactly one closest-hit query (Scene.RayTrace) per live
// lane.  Per item the lane accumulates its chunk's samples in registers and writes one
// 16-byte partial; a second kernel folds the partials into fp64 accumulators in a fixed
// order, so results do not depend on scheduling.
//
// Per path this restates Raytracer.GetCameraRay + GetColor (Raytracer.cs:51-287):
//   camera jitter and depth of field, the bounce loop with RandomShine (rough normal),
//   Fresnel / total internal reflection, the luminance-weighted transmit / specular /
//   diffuse / emission choice, tint *= colour * max(totalLum, 1), and the miss rules
//   (primary miss -> Placeholder/miss, secondary miss -> AmbientRGB untinted).
// The closest-hit query restates Scene.RayTrace semantics (Scene.cs:65-120, Primitive.cs:46-75)
// in fp32: strict-closest hit, Invert flipping Inside only, one-sided culling, and
// Util.RayHitMatches' self-hit rejection (Util.cs:179-192) restated as: a flat primitive
// is never re-hit by the ray leaving it; a sphere re-hit keeps only the far root when the
// ray heads into it (DESIGN.md §Self-hit rule).
//
// Brute-force traversal walks the primitive records with a wave-uniform index: the records
// come through the scalar data cache (s_load) into SGPRs and every lane tests every
// primitive branch-free.  BVH traversal keeps a per-lane stack in LDS.
#include "../../include/rtcore_rng.h"
#include "rt_kernels.h"
#ifdef RT_SCENE_CONST
// rt_jit.cpp generates this header per scene (and camera, for the grouped order): the launch's
// PathScene and its brute-force records as 32-bit words (kSceneW, kGroupsW, kRectsW, kFramesW,
// kTestsW, kXfW, kCameraW) and the camera switches (RT_SCENE_CAMERA_KIND / _DOF).  Every record
// field then folds into the instructions (literal operands cost what a VGPR operand does on
// gfx950, an SGPR operand twice that), the primitive loops unroll and the per-record flag branches
// resolve at compile time.  Included first, so that every macro it defines is seen by the code.
#include "rt_scene_const.h"
#endif

namespace rtc {
namespace {

struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 xyz(float4 a) { return V3{a.x, a.y, a.z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ float dot(V3 a, V3 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, a.z * b.z)); }
// Products with a scene or camera field.  In the scene-specialised build those fields are literals,
// and IEEE rules keep fmaf(0, x, y) as an instruction (x could be infinite, and y + 0 is not y for
// y = -0): axis-aligned cameras, rotation frames and two-sided rectangles carried ~20 such terms per
// query on bounce.txt.  A term whose literal factor is zero is dropped there; the generic kernel
// computes the same values except for the sign of an exact zero (x is always finite here).
__device__ __forceinline__ bool known_zero(float c)
{
#if defined(RT_SCENE_CONST)
    return __builtin_constant_p(c) && c == 0.0f;
#else
    (void)c;
    return false;
#endif
}
__device__ __forceinline__ float kfma(float a, float b, float c) { return (known_zero(a) || known_zero(b)) ? c : fmaf(a, b, c); }
__device__ __forceinline__ float kmul(float a, float b) { return (known_zero(a) || known_zero(b)) ? -0.0f : a * b; }
__device__ __forceinline__ float dot4(float4 r, V3 p) { return kfma(r.x, p.x, kfma(r.y, p.y, kfma(r.z, p.z, r.w))); }
__device__ __forceinline__ float dot3(float4 r, V3 p) { return kfma(r.x, p.x, kfma(r.y, p.y, kmul(r.z, p.z))); }
__device__ __forceinline__ V3 cross(V3 a, V3 b)
{
    return {fmaf(a.y, b.z, -a.z * b.y), fmaf(a.z, b.x, -a.x * b.z), fmaf(a.x, b.y, -a.y * b.x)};
}
__device__ __forceinline__ V3 madd(V3 a, float s, V3 c) { return {kfma(a.x, s, c.x), kfma(a.y, s, c.y), kfma(a.z, s, c.z)}; }
__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ V3 normalize(V3 a) { return a * __builtin_amdgcn_rsqf(dot(a, a)); }
__device__ __forceinline__ V3 xf_point(const float4* m, V3 p) { return {dot4(m[0], p), dot4(m[1], p), dot4(m[2], p)}; }
__device__ __forceinline__ V3 xf_dir(const float4* m, V3 p) { return {dot3(m[0], p), dot3(m[1], p), dot3(m[2], p)}; }

struct Best {
    float t; // world distance (Hit.Distance)
    int sg;  // slot << 1 | geometric inside (before Invert; selects the flipped normal); -1 = none
};
__device__ __forceinline__ int pack_sg(int slot, bool gin) { return (slot << 1) | (int)gin; }

// Triangle via the affine inverse record (TestRec): w(t) = 0 gives t, then (u, v).
// Inside (Moller-Trumbore's 1/det < 0, Triangle.cs:127) <=> d . n > 0 <=> dw > 0.
// Every kernel names the primitive a ray leaves by its slot (SLOT: id = slot, Sample.prev = slot): a
// hit-able primitive has exactly one slot in each order, the records of compact leaves carry no ID,
// and a box names its faces' slots by face index (sg0 / 2 + f) without a table.
__device__ __forceinline__ void hit_tri_rows(float4 r0, float4 r1, float4 r2, uint32_t fl, int id, int slot, V3 o, V3 d,
                                             int prev, Best& b)
{
    const float dw = dot3(r2, d);
    const float t = -dot4(r2, o) * rcp(dw);
    const float u = fmaf(t, dot3(r0, d), dot4(r0, o));
    const float v = fmaf(t, dot3(r1, d), dot4(r1, o));
    const bool gin = dw > 0.0f;
    bool ok = (t >= 0.0f) & (t < b.t) & (u >= 0.0f) & (v >= 0.0f) & (id != prev);
    ok &= (fl & F_MIRROR) ? ((u <= 1.0f) & (v <= 1.0f)) : (u + v <= 1.0f);
    if (!(fl & F_TWOSIDED)) ok &= !(gin ^ ((fl & F_INVERT) != 0)); // one-sided: cull Inside
    b.t = ok ? t : b.t;
    b.sg = ok ? pack_sg(slot, gin) : b.sg;
}
template <bool SLOT = false>
__device__ __forceinline__ void hit_tri(const TestRec& R, int slot, V3 o, V3 d, int prev, Best& b)
{
    hit_tri_rows(R.r0, R.r1, R.r2, __float_as_uint(R.meta.y), SLOT ? slot : __float_as_int(R.meta.x), slot, o, d, prev, b);
}

// Sphere (Sphere.cs:50-155).  Primitive.RayTrace returns the first surviving root: the close
// one (Inside = false) if it lies ahead and is not culled, otherwise the far one.
// WSKIP: the rest of the test is skipped, by a wave-uniform branch, when no lane's line meets the
// sphere and no lane leaves it.  The grouped brute-force order takes it (die.txt's pips, r = 0.15:
// C3 25.65 -> 23.56 ms), the flat order not (bounce.txt's large spheres: C2 18.43 -> 18.65 ms;
// the branch costs more than the waves that skip save); RT_SPH_WAVE_SKIP = 0 / 1 forces it off /
// on for both.  The box test skips its face choice the same way when no lane meets the box ahead
// (RT_BOX_WAVE_SKIP, default on: C2 18.43 -> 17.85 ms, bounce.txt's light box and rotated cube).
// Neither changes a result: the skipped part can report no hit.
#ifndef RT_SPH_WAVE_SKIP
#define RT_SPH_WAVE_SKIP -1
#endif
#ifndef RT_BOX_WAVE_SKIP
#define RT_BOX_WAVE_SKIP 1
#endif
template <bool WSKIP = false, class XfP> // XfP: const XformF*, generic or in the constant address space
__device__ __forceinline__ void hit_sph_rows(float4 r0, float4 r1, uint32_t fl, int id, int slot, V3 o, V3 d, int prev,
                                             XfP xf, Best& b)
{
    V3 oo = o, dd = d;
    float k = 1.0f; // object-space ray parameter -> world distance
    if (fl & F_TRANSFORMED) {
        const XformF X = xf[__float_as_int(r1.y)];
        oo = xf_point(X.to_world, o);
        const V3 dl = xf_dir(X.to_world, d);
        k = __builtin_amdgcn_rsqf(dot(dl, dl)); // |to_obj * dd| = 1 / |to_world * d|
        dd = dl * k;
    }
    const V3 oc = oo - xyz(r0);
    const float bb = dot(oc, dd);
    const V3 l = madd(dd, -bb, oc);
    const float disc = r1.x - dot(l, l);
    const bool self = id == prev;
    if (WSKIP && !__any((disc >= 0.0f) | self)) return;
    const float sq = fsqrt(fmaxf(disc, 0.0f));
    // self-hit: the root at the bounce point is skipped; the other root is -2 (oc.dd)
    const float tn = self ? -1.0f : -bb - sq;
    const float tf = self ? -2.0f * bb : sq - bb;
    const bool any = self ? (bb < 0.0f) : ((disc >= 0.0f) & (tf >= 0.0f));
    const bool two = (fl & F_TWOSIDED) != 0, inv = (fl & F_INVERT) != 0;
    const bool use_close = any & (tn >= 0.0f) & (two | !inv);
    const bool use_far = !use_close & any & (two | inv);
    const float tc = use_close ? tn : tf;
    const float tw = tc * k;
    const bool ok = (use_close | use_far) & (tw < b.t);
    b.t = ok ? tw : b.t;
    b.sg = ok ? pack_sg(slot, use_far) : b.sg;
}
template <bool SLOT = false, bool WSKIP = false, class XfP>
__device__ __forceinline__ void hit_sph(const TestRec& R, int slot, V3 o, V3 d, int prev, XfP xf, Best& b)
{
    hit_sph_rows<WSKIP>(R.r0, R.r1, __float_as_uint(R.meta.y), SLOT ? slot : __float_as_int(R.meta.x), slot, o, d, prev,
                        xf, b);
}

// Plane (Plane.cs:36-66), including the NearlyEqual branch for rays in the plane.
template <bool SLOT = false>
__device__ __forceinline__ void hit_plane(const TestRec& R, int slot, V3 o, V3 d, int prev, Best& b)
{
    const int id = SLOT ? slot : __float_as_int(R.meta.x);
    const uint32_t fl = __float_as_uint(R.meta.y);
    const V3 n = xyz(R.r0);
    const float pd = R.r0.w;
    const float rd = dot(o, n), den = dot(d, n);
    const float t = (pd - rd) / den;
    const bool flat = den == 0.0f;
    const bool any = flat ? ((pd == rd) | (fmaxf(pd, rd) < 0.0f)) : (t >= -1e-24f);
    const float dist = flat ? 0.0f : fabsf(t);
    const bool gin = flat ? true : (den > 0.0f);
    bool ok = any & (id != prev) & (dist < b.t);
    if (!(fl & F_TWOSIDED)) ok &= !(gin ^ ((fl & F_INVERT) != 0));
    b.t = ok ? dist : b.t;
    b.sg = ok ? pack_sg(slot, gin) : b.sg;
}

// Axis-aligned rectangle on plane `AXIS` (RectRec): the same hit as the Mirror parallelogram
// test (u, v in [0, 1]^2) with the extents in world units.  id = 1 / d, oi = o / d.  The side
// of the hit (Inside) is not tracked here: the shading step recomputes it from the normal.
// SUB: oi holds o itself and t = (c - o) / d (one fewer live vector than the fma form)
template <int AXIS, bool SUB = false>
__device__ __forceinline__ void hit_rect(const RectRec& R, int sg, V3 o, V3 d, V3 id, V3 oi, int prev, Best& b)
{
    const float ida = AXIS == 0 ? id.x : AXIS == 1 ? id.y : id.z;
    const float oia = AXIS == 0 ? oi.x : AXIS == 1 ? oi.y : oi.z;
    const float da = AXIS == 0 ? d.x : AXIS == 1 ? d.y : d.z;
    const float d1 = AXIS == 0 ? d.y : d.x, o1 = AXIS == 0 ? o.y : o.x;
    const float d2 = AXIS == 2 ? d.y : d.z, o2 = AXIS == 2 ? o.y : o.z;
    const float t = SUB ? (R.c - oia) * ida : fmaf(R.c, ida, -oia);
    // |p - mid| <= half on both in-plane axes (false for NaN)
    const bool in1 = fabsf(fmaf(t, d1, o1) - R.m1) <= R.h1;
    const bool in2 = fabsf(fmaf(t, d2, o2) - R.m2) <= R.h2;
    // 0 <= t < best as one unsigned compare of the bit patterns (b.t >= 0; NaN and -t fail)
    const bool near = __float_as_uint(t) < __float_as_uint(b.t);
    const bool ok = near & in1 & in2 & (kmul(R.cull, da) <= 0.0f) & ((R.sg >> 1) != prev); // prev: a slot
    b.t = ok ? t : b.t; // the shading step rebuilds the hit point from t
    b.sg = ok ? sg : b.sg;
}

template <int AXIS, bool SUB = false, class RectP>
__device__ __forceinline__ void rect_group(RectP r, int n, V3 o, V3 d, V3 id, V3 oi, int prev, Best& b)
{
    for (; n >= 2; n -= 2, r += 2) {
        const RectRec r0 = r[0], r1 = r[1];
        hit_rect<AXIS, SUB>(r0, r0.sg, o, d, id, oi, prev, b);
        hit_rect<AXIS, SUB>(r1, r1.sg, o, d, id, oi, prev, b);
    }
    if (n > 0) {
        const RectRec r0 = r[0];
        hit_rect<AXIS, SUB>(r0, r0.sg, o, d, id, oi, prev, b);
    }
}

// Min / max as the bare VALU instructions.  fminf / fmaxf of values the compiler cannot prove
// canonical (here: slab distances that pass through the sphere tests' divergent branches) get a
// v_max_f32 x, x, x quieting each operand first; our operands are never signalling NaNs, and a
// quiet NaN operand is ignored either way (IEEE minNum), so the bare instruction is the same min.
__device__ __forceinline__ float vmin(float a, float b)
{
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmax(float a, float b)
{
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ __forceinline__ float vmax3(float a, float b, float c)
{
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float vmin3(float a, float b, float c)
{
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float vmax0(float a)
{
    float r;
    asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(a));
    return r;
}
__device__ __forceinline__ float vmax1(float a)
{
    float r;
    asm("v_max_f32 %0, 1.0, %1" : "=v"(r) : "v"(a));
    return r;
}

// Closed box (BoxRec): one slab test gives the entry and exit distances and faces; each is a
// hit when it lies in [0, best), its face keeps hits from that side (culling) and it is not the
// face the ray leaves (self-hit).  The entry wins when both are hits.  Equivalent to testing the
// six faces as rectangles (a convex box is met at most twice), up to ties on its edges.
// SUB: oi holds o itself (frame-local rays), as in hit_rect.
template <bool SUB>
__device__ __forceinline__ void hit_box(const BoxRec& B, V3 o, V3 d, V3 id, V3 oi, int prev, Best& b)
{
    const float lx = SUB ? (B.lo.x - oi.x) * id.x : fmaf(B.lo.x, id.x, -oi.x);
    const float hx = SUB ? (B.hi.x - oi.x) * id.x : fmaf(B.hi.x, id.x, -oi.x);
    const float ly = SUB ? (B.lo.y - oi.y) * id.y : fmaf(B.lo.y, id.y, -oi.y);
    const float hy = SUB ? (B.hi.y - oi.y) * id.y : fmaf(B.hi.y, id.y, -oi.y);
    const float lz = SUB ? (B.lo.z - oi.z) * id.z : fmaf(B.lo.z, id.z, -oi.z);
    const float hz = SUB ? (B.hi.z - oi.z) * id.z : fmaf(B.hi.z, id.z, -oi.z);
    const float nx = vmin(lx, hx), ny = vmin(ly, hy), nz = vmin(lz, hz);
    const float fx = vmax(lx, hx), fy = vmax(ly, hy), fz = vmax(lz, hz);
    const float te = vmax3(nx, ny, nz), tx = vmin3(fx, fy, fz);
    const bool meet = te <= tx;
    if (RT_BOX_WAVE_SKIP && !__any(meet & (tx >= 0.0f))) return; // no lane meets the box ahead
    // the ray enters axis a's slab by its lower plane (side 0) when d[a] > 0
    const int sx = (int)(__float_as_uint(d.x) >> 31), sy = (int)(__float_as_uint(d.y) >> 31),
              sz = (int)(__float_as_uint(d.z) >> 31);
    const uint32_t keep = B.keep;
    const uint32_t rel_prev = (uint32_t)(prev - (B.sg0 >> 1)); // the face slot the ray leaves, relative to face 0
    bool ok_e = false, ok_x = false;
    int fe = 0, fo = 0;
    if (keep & 0x3Fu) { // some face keeps entry hits (wave-uniform)
        fe = te == nx ? sx : (te == ny ? 2 + sy : 4 + sz);
        // the keep bit is tested unconditionally: selecting on "every face keeps" cost more, and
        // folding that case in the scene-specialised build measured no change (round 3)
        ok_e = meet & (__float_as_uint(te) < __float_as_uint(b.t)) & ((uint32_t)fe != rel_prev) &
               (((keep >> fe) & 1u) != 0);
    }
    if (keep & 0x3F00u) { // some face keeps exit hits
        fo = tx == fx ? 1 - sx : (tx == fy ? 3 - sy : 5 - sz);
        ok_x = meet & (__float_as_uint(tx) < __float_as_uint(b.t)) & ((uint32_t)fo != rel_prev) &
               (((keep >> (8 + fo)) & 1u) != 0);
    }
    const bool ok = ok_e | ok_x;
    b.t = ok ? (ok_e ? te : tx) : b.t;
    b.sg = ok ? B.sg0 + 2 * (ok_e ? fe : fo) : b.sg;
}

// 1/d for the box tests, with |d| clamped to >= 2^-64 so that an axis-parallel ray (d = 0 on an
// axis, e.g. a diffuse bounce whose angle draw is exactly 0) gives large finite slab distances of
// the right sign instead of 0 * inf = NaN, which the min/max chains would ignore (a box the ray
// runs parallel to and outside of would then count as hit, and the query would visit every node).
__device__ __forceinline__ float slab_rcp(float d)
{
    return rcp(fabsf(d) >= 5.421010862e-20f ? d : __builtin_copysignf(5.421010862e-20f, d));
}
// The brute-force kernels' form: the reciprocal clamped to +-2^64 by one v_med3 instead of a
// compare, a select and a sign insert before it; the same value for every finite or zero d
// (1/(+-0) = +-inf clamps to +-2^64 = 1/(+-2^-64)).  A NaN d (a vertex-normal triangle's NaN
// normal) gets a finite +-2^64 here, so a box test could report a hit for it: path_body ends such
// a query as a miss, as the reference's BVH root test does.
__device__ __forceinline__ float slab_rcp_lean(float d)
{
    return __builtin_amdgcn_fmed3f(rcp(d), -0x1p64f, 0x1p64f);
}

// BARE (the brute-force kernels' group boxes): the per-axis min / max as bare instructions (vmin,
// vmax), which drops the compiler's NaN quieting of their operands; same values.
template <bool BARE = false>
__device__ __forceinline__ bool slab(float4 lo, float4 hi, V3 oi, V3 id, float tmax, float& tnear)
{
    // t = box * (1/d) - o * (1/d); NaN from 0*inf is ignored by fminf/fmaxf (conservative)
    const float tx0 = fmaf(lo.x, id.x, -oi.x), tx1 = fmaf(hi.x, id.x, -oi.x);
    const float ty0 = fmaf(lo.y, id.y, -oi.y), ty1 = fmaf(hi.y, id.y, -oi.y);
    const float tz0 = fmaf(lo.z, id.z, -oi.z), tz1 = fmaf(hi.z, id.z, -oi.z);
    const float nx = BARE ? vmin(tx0, tx1) : fminf(tx0, tx1), fx = BARE ? vmax(tx0, tx1) : fmaxf(tx0, tx1);
    const float ny = BARE ? vmin(ty0, ty1) : fminf(ty0, ty1), fy = BARE ? vmax(ty0, ty1) : fmaxf(ty0, ty1);
    const float nz = BARE ? vmin(tz0, tz1) : fminf(tz0, tz1), fz = BARE ? vmax(tz0, tz1) : fmaxf(tz0, tz1);
    const float tmin = BARE ? vmax3(nx, ny, vmax0(nz)) : fmaxf(fmaxf(nx, ny), fmaxf(nz, 0.0f));
    const float tmx = BARE ? vmin3(fx, fy, vmin(fz, tmax)) : fminf(fminf(fx, fy), fminf(fz, tmax));
    tnear = tmin;
    return tmin <= tmx * 1.00000024f;
}

// Every primitive, group by group (GroupRec: x-rects | y-rects | z-rects | triangles | spheres).
// The loop indices are wave-uniform, so the records arrive through scalar loads.  With CULL a
// group is skipped when no lane of the wave meets its box before its current closest hit, and
// with it the G.skip records that follow it (a super record: the box of a subtree of groups, no
// primitives of its own).  The skip is a wave-uniform bound (skip_to), not a jump of the loop
// index, so the scene-specialised build still unrolls the loop.
// The record pointers are in the constant address space (RT_AS_CONST) or generic.
// boxes: the frame array viewed as BoxRecs (they share it).
template <bool CULL, bool STATS, class SceneT, class GroupP, class TestP, class RectP, class FrameP, class BoxP, class XfP>
__device__ __forceinline__ void trace_brute(const SceneT& s, GroupP groups, TestP tests, RectP rects, FrameP frames,
                                            BoxP boxes, XfP xf, V3 o, V3 d, int prev, Best& b, unsigned& n_flat,
                                            unsigned& n_sph, unsigned& n_node)
{
    const V3 id = v3(slab_rcp_lean(d.x), slab_rcp_lean(d.y), slab_rcp_lean(d.z));
    const V3 oi = o * id;
    const int n_groups = CULL ? s.n_groups : 1; // the flat order is one group (1/d and o/d die after its rects)
    int skip_to = 0;
#ifdef RT_SCENE_CONST
#pragma unroll // the scene-specialised build: every group's tests in line, their records literals
#endif
    for (int g = 0; g < n_groups; g++) {
        if (CULL && g < skip_to) continue;
        const GroupRec G = groups[g];
        if (CULL) {
            if (STATS) n_node++; // the group's box: a node of a shallow tree (SURVEY 8(d) N_node)
            float tn;
            if (!__any(slab<true>(G.lo, G.hi, oi, id, b.t, tn))) {
                skip_to = g + 1 + G.skip;
                continue;
            }
        }
        if (STATS) { // primitive tests actually made (groups the wave skipped are not counted)
            n_flat += G.n_rect[0] + G.n_rect[1] + G.n_rect[2] + G.n_flat_extra + (G.n_tri_sph & 0xFFFF);
            n_sph += G.n_tri_sph >> 16;
        }
        RectP r = rects + __float_as_int(G.lo.w);
        rect_group<0>(r, G.n_rect[0], o, d, id, oi, prev, b);
        r += G.n_rect[0];
        rect_group<1>(r, G.n_rect[1], o, d, id, oi, prev, b);
        r += G.n_rect[1];
        rect_group<2>(r, G.n_rect[2], o, d, id, oi, prev, b);
        for (int j = G.frame_first + G.n_frames; j < G.frame_first + G.n_frames + G.n_boxes; j++) {
            const BoxRec B = boxes[j];
            hit_box<false>(B, o, d, id, oi, prev, b);
        }
        // rectangles in a common affine frame: the ray mapped once, then the same rect tests (t is
        // invariant under the map; a local d of 0 gives an infinite or NaN t, which never hits)
        for (int f = G.frame_first; f < G.frame_first + G.n_frames; f++) {
            const FrameRec F = frames[f];
            const V3 lo = v3(dot4(F.r0, o), dot4(F.r1, o), dot4(F.r2, o));
            const V3 ld = v3(dot3(F.r0, d), dot3(F.r1, d), dot3(F.r2, d));
            const V3 lid = v3(rcp(ld.x), rcp(ld.y), rcp(ld.z));
            RectP fr = rects + F.rect_first;
            rect_group<0, true>(fr, F.n_rect[0], lo, ld, lid, lo, prev, b);
            fr += F.n_rect[0];
            rect_group<1, true>(fr, F.n_rect[1], lo, ld, lid, lo, prev, b);
            fr += F.n_rect[1];
            rect_group<2, true>(fr, F.n_rect[2], lo, ld, lid, lo, prev, b);
            if (F.box >= 0) {
                const BoxRec B = boxes[F.box];
                hit_box<true>(B, lo, ld, lid, lo, prev, b);
            }
        }
        int i = __float_as_int(G.hi.w);
        int end = i + (G.n_tri_sph & 0xFFFF);
        if (i < end) {
            TestRec cur = tests[i];
            for (; i < end; i++) {
                const TestRec nxt = tests[i + 1];
                hit_tri<true>(cur, i, o, d, prev, b);
                cur = nxt;
            }
        }
        end = i + (G.n_tri_sph >> 16);
        if (i < end) {
            TestRec cur = tests[i];
            for (; i < end; i++) {
                const TestRec nxt = tests[i + 1];
                hit_sph<true, RT_SPH_WAVE_SKIP < 0 ? CULL : RT_SPH_WAVE_SKIP != 0>(cur, i, o, d, prev, xf, b);
                cur = nxt;
            }
        }
    }
}

template <bool SLOT = false, class XfP>
__device__ __forceinline__ void hit_any(const TestRec& R, int slot, V3 o, V3 d, int prev, XfP xf, Best& b)
{
    switch (__float_as_uint(R.meta.y) & KIND_MASK) {
    case RT_PRIM_TRIANGLE: hit_tri<SLOT>(R, slot, o, d, prev, b); break;
    case RT_PRIM_SPHERE: hit_sph<SLOT>(R, slot, o, d, prev, xf, b); break;
    default: hit_plane<SLOT>(R, slot, o, d, prev, b); break;
    }
}

// The pending leaf of a BVH query is one register: the leaf code (rt_internal.h) whose count field
// holds the primitives still to test, minus one; -1 when no leaf is pending.  A leaf step decodes
// its slots and, for a compact leaf, the record flags its primitives share (leaf_flags);
// kLeafGeneric for a generic leaf (flags from each record's meta row).
constexpr uint32_t kLeafGeneric = 0xFFFFFFFFu;
__device__ __forceinline__ void leaf_decode(int pend, int& k, int& kend, uint32_t& lfl)
{
    const bool compact = (pend & kLeafCompact) != 0;
    k = compact ? (pend >> 2) & (kLeafCompactMaxFirst - 1) : pend >> 3;
    kend = k + (pend & (compact ? 3 : 7)) + 1;
    lfl = compact ? leaf_flags(((uint32_t)pend >> 25) & 31u) : kLeafGeneric;
}
// after a step of n primitives: the first slot advanced by n and the count field lowered by n, or -1
__device__ __forceinline__ int leaf_advance(int pend, int n)
{
    const bool compact = (pend & kLeafCompact) != 0;
    const int left = pend & (compact ? 3 : 7);
    return left >= n ? pend + (compact ? (n << 2) - n : (n << 3) - n) : -1;
}



// One visit of a 4-wide quantised node (Node4Q): slab tests of the four children against
// dequantised planes t = q * (2^e / d) + (origin - o) / d, nearest hit child next, the other hit
// children pushed far-to-near.  pop stays true when no child is hit.
__device__ __forceinline__ float ubyte(uint32_t v, int k) { return (float)((v >> (8 * k)) & 255u); }
__device__ __forceinline__ void cswap(float& da, int& ra, float& db, int& rb)
{
    const bool sw = db < da;
    const float t = da;
    const int r = ra;
    da = sw ? db : da;
    ra = sw ? rb : ra;
    db = sw ? t : db;
    rb = sw ? r : rb;
}
// Per-lane traversal stack: the first STACK entries in LDS (stride 256 = the block's lanes), deeper
// entries in a global overflow area (stride = all lanes of the grid), reached only by rare deep
// paths; the host bounds the depth any ray can need by STACK + RT_STACK_OVF.
// The two parts are typed by address space: with plain pointers the compiler merged the LDS and the
// overflow access of push / pop into one flat access through a selected pointer (a flat store or
// load, plus the pointer arithmetic, on every push and pop, and through the texture addresser).
// The bases are wave-uniform and the lane's offset is formed at use: per-lane pointers held across
// the loop were spilled to scratch and reloaded at every push (C4 52.4 -> 66.6 ms).
#define RT_STACK_OVF 44 // = kStackOverflow (rt_kernels.h); with the 16-entry LDS stacks, 60 entries in all
typedef __attribute__((address_space(3))) int LdsInt;
typedef __attribute__((address_space(1))) int GlobalInt;
struct TravStack {
    LdsInt* lds;    // the block's stack array (entry e of thread t at e * 256 + t)
    GlobalInt* ovf; // the grid's overflow area (entry e of global thread g at e * grid threads + g)
};
__device__ __forceinline__ TravStack make_stack(int* lds_base, int* ovf_base)
{
    return TravStack{(LdsInt*)lds_base, (GlobalInt*)ovf_base};
}
__device__ __forceinline__ unsigned ovf_slot(int e)
{
    return (unsigned)e * (gridDim.x * 256u) + blockIdx.x * 256u + threadIdx.x;
}
template <int STACK>
__device__ __forceinline__ void push(const TravStack& st, int& sp, int v)
{
    if (sp < STACK) st.lds[sp * 256 + (int)threadIdx.x] = v;
    else st.ovf[ovf_slot(sp - STACK)] = v;
    sp++;
}
template <int STACK>
__device__ __forceinline__ int pop_ref(const TravStack& st, int& sp)
{
    --sp;
    return sp < STACK ? st.lds[sp * 256 + (int)threadIdx.x] : st.ovf[ovf_slot(sp - STACK)];
}

__device__ __forceinline__ void pin4(float4& f)
{
    typedef float F4 __attribute__((ext_vector_type(4)));
    F4 v = {f.x, f.y, f.z, f.w};
    asm volatile("" : "+v"(v));
    f = make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void pin_rec(TestRec& t)
{
    pin4(t.r0);
    pin4(t.r1);
    pin4(t.r2);
    pin4(t.meta);
}
template <int STACK>
__device__ __forceinline__ void wide_visit(const Node4Q& q, V3 id, V3 oi, float best, int& ref, int& sp,
                                           const TravStack& stk, bool& pop)
{
    const uint32_t ex = __float_as_uint(q.a.w);
    const float ax = __builtin_amdgcn_ldexpf(id.x, (int)(ex & 255u) - 128);
    const float ay = __builtin_amdgcn_ldexpf(id.y, (int)((ex >> 8) & 255u) - 128);
    const float az = __builtin_amdgcn_ldexpf(id.z, (int)((ex >> 16) & 255u) - 128);
    const float bx = fmaf(q.a.x, id.x, -oi.x), by = fmaf(q.a.y, id.y, -oi.y), bz = fmaf(q.a.z, id.z, -oi.z);
    const uint32_t lx = __float_as_uint(q.b.x), hx = __float_as_uint(q.b.y);
    const uint32_t ly = __float_as_uint(q.b.z), hy = __float_as_uint(q.b.w);
    const uint32_t lz = __float_as_uint(q.c.x), hz = __float_as_uint(q.c.y);
    // near / far planes by the direction's sign
    const uint32_t nx = id.x >= 0.0f ? lx : hx, fx = id.x >= 0.0f ? hx : lx;
    const uint32_t ny = id.y >= 0.0f ? ly : hy, fy = id.y >= 0.0f ? hy : ly;
    const uint32_t nz = id.z >= 0.0f ? lz : hz, fz = id.z >= 0.0f ? hz : lz;
    const int nc = __float_as_int(q.d.z);
    float d0, d1, d2, d3;
    int r0 = __float_as_int(q.c.z), r1 = __float_as_int(q.c.w), r2 = __float_as_int(q.d.x), r3 = __float_as_int(q.d.y);
    const float tmax_best = best * 1.00000024f;
#define RT_WIDE_CHILD(K, D)                                                                                       \
    {                                                                                                             \
        const float tmin = fmaxf(fmaxf(fmaxf(fmaf(ubyte(nx, K), ax, bx), fmaf(ubyte(ny, K), ay, by)),              \
                                       fmaf(ubyte(nz, K), az, bz)), 0.0f);                                         \
        const float tmax = fminf(fminf(fmaf(ubyte(fx, K), ax, bx), fmaf(ubyte(fy, K), ay, by)),                   \
                                 fmaf(ubyte(fz, K), az, bz));                                                      \
        D = ((K < nc) & (tmin <= fminf(tmax * 1.00000024f, tmax_best))) ? tmin : __builtin_huge_valf();         \
    } // (K < nc) without short-circuit: "&&" made each child a divergent branch.  The test stays although
      // an empty slot's box is inverted (quantize_node4): inverted only up to the fp32 rounding of the
      // planes, and a hit on an empty slot would push RT_NODE4_EMPTY (round 4: dropping it saved 0.6 %)
    RT_WIDE_CHILD(0, d0)
    RT_WIDE_CHILD(1, d1)
    RT_WIDE_CHILD(2, d2)
    RT_WIDE_CHILD(3, d3)
#undef RT_WIDE_CHILD
    cswap(d0, r0, d1, r1);
    cswap(d2, r2, d3, r3);
    cswap(d0, r0, d2, r2);
    cswap(d1, r1, d3, r3);
    cswap(d1, r1, d2, r2);
    const float inf = __builtin_huge_valf();
    if (d0 < inf) {
        if (d3 < inf) push<STACK>(stk, sp, r3);
        if (d2 < inf) push<STACK>(stk, sp, r2);
        if (d1 < inf) push<STACK>(stk, sp, r1);
        ref = r0;
        pop = false;
    }
}

struct Counters {
    unsigned nodes, tris, sphs;                                  // per lane
    unsigned ovf_pushes, max_sp;                                 // per lane: stack entries written past the LDS part; deepest stack
    unsigned outer;                                              // per lane: faces of the BVH order's outer group tested
    unsigned q_steps, max_steps;                                 // per lane: steps of the current / longest query
    unsigned long long cyc_start, cyc_trace, cyc_shade, iters; // per wave (uniform)
};

// q = x / d, r = x % d through the fp32 reciprocal plus one correction step (exact for the
// quotients used here, all far below 2^22).
__device__ __forceinline__ void divmod(unsigned x, unsigned d, float inv_d, unsigned& q, unsigned& r)
{
    q = (unsigned)((float)x * inv_d);
    r = x - q * d;
    if ((int)r < 0) {
        q--;
        r += d;
    } else if (r >= d) {
        q++;
        r -= d;
    }
}

struct Sample {
    V3 o, d, tint;
    int bounce;
    int prev;
    rt_rng rng;
};

__device__ __forceinline__ float next_u(rt_rng& r) { return rt_rng_next_float(&r); }

// Vec4D.CreateHorizon(pole, z, theta) (Vec4D.cs:52-58) as the equivalent Rodrigues form:
// pole*z + (c*cos(theta) + (pole x c)*sin(theta)) * s, c = normalize(pole x z^) or x^.
// The frame (c, pole x c) depends on the pole only, so one bounce builds it once for both
// the rough normal and the diffuse direction (both turn about the hit normal).
struct Frame {
    V3 c, bn;
};
__device__ __forceinline__ Frame make_frame(V3 pole)
{
    V3 c = v3(pole.y, -pole.x, 0.0f);
    const float cl = fmaf(c.x, c.x, c.y * c.y);
    c = (cl == 0.0f) ? v3(1.0f, 0.0f, 0.0f) : c * __builtin_amdgcn_rsqf(cl);
    return Frame{c, cross(pole, c)};
}
__device__ __forceinline__ V3 horizon(const Frame& f, V3 pole, float z, float s, float turn)
{
    const float cs = __builtin_amdgcn_cosf(turn), sn = __builtin_amdgcn_sinf(turn); // argument in turns
    const V3 h = madd(f.c, cs, f.bn * sn);
    return madd(h, s, pole * z);
}

// 2 * acos(u) / pi for u in [0, 1): sqrt(1 - u) * P(u), the degree-7 fit of Abramowitz &
// Stegun 4.4.46 (|error| <= 2e-8 rad) scaled by 2 / pi; as accurate as fp32 acosf here.
__device__ __forceinline__ float acos_turn2(float u)
{
    float p = fmaf(u, -0.0008037268f, 0.0042463113f);
    p = fmaf(u, p, -0.0108786384f);
    p = fmaf(u, p, 0.0196663830f);
    p = fmaf(u, p, -0.0319419540f);
    p = fmaf(u, p, 0.0566457845f);
    p = fmaf(u, p, -0.1366178393f);
    p = fmaf(u, p, 1.0f);
    return fsqrt(1.0f - u) * p;
}

struct Ray3 {
    V3 o, d;
};
// The camera's kind and depth-of-field switch: compile-time constants in a camera-independent
// scene-specialised build (rt_jit.cpp), else read from the camera record.
template <class CamT>
__device__ __forceinline__ bool cam_frustum(const CamT& c)
{
#ifdef RT_SCENE_CAMERA_KIND
    (void)c;
    return RT_SCENE_CAMERA_KIND == RT_CAMERA_FRUSTUM;
#else
    return c.kind == RT_CAMERA_FRUSTUM;
#endif
}
template <class CamT>
__device__ __forceinline__ bool cam_dof(const CamT& c)
{
#ifdef RT_SCENE_CAMERA_DOF
    (void)c;
    return RT_SCENE_CAMERA_DOF != 0;
#else
    return c.dof != 0.0f;
#endif
}
template <class CamT> // CameraF, or CameraF in the constant address space (scalar loads)
__device__ __forceinline__ Ray3 camera_ray(const CamT& c, float x, float y)
{
    Ray3 r;
    if (cam_frustum(c)) {
        const float ox = fmaf(x, c.tan_x_per_px, -c.tan_x); // tan_x * (x - w2) / w2
        const float oy = fmaf(y, c.tan_y_per_px, -c.tan_y);
        r.d = normalize(madd(xyz(c.up), oy, madd(xyz(c.side), ox, xyz(c.look))));
        r.o = xyz(c.position);
    } else {
        r.o = madd(xyz(c.up), (y - c.h2) * c.v_mult, madd(xyz(c.side), (x - c.w2) * c.h_mult, xyz(c.position)));
        r.d = normalize(xyz(c.look));
    }
    r.o = madd(r.d, c.image_plane, r.o);
    return r;
}

// Raytracer.GetCameraRay (Raytracer.cs:262-282)
// LEAN (the brute-force kernels): x + U as one fma of the integer draw (U = h * 2^-24 exactly, so the
// single rounding is the add's: the same value); the BVH kernels keep the add (their register
// allocation moved spills into the traversal loop with it, C4 44.4 -> 55.9 ms)
template <bool LEAN = false, class CamT>
__device__ __forceinline__ void start_sample(const CamT& cam, int x, int y, Sample& S)
{
    const float sx = LEAN ? fmaf((float)rt_rng_next24(&S.rng), 0x1p-24f, (float)x) : (float)x + next_u(S.rng);
    const float sy = LEAN ? fmaf((float)rt_rng_next24(&S.rng), 0x1p-24f, (float)y) : (float)y + next_u(S.rng);
    const Ray3 r = camera_ray(cam, sx, sy);
    S.o = r.o;
    S.d = r.d;
    if (cam_dof(cam)) {
        const V3 focus = madd(r.d, cam.focal_length - cam.image_plane, r.o);
        const float dist = fsqrt(next_u(S.rng)) * cam.dof;
        const float turn = next_u(S.rng);
        const float ox = __builtin_amdgcn_cosf(turn) * dist, oy = __builtin_amdgcn_sinf(turn) * dist;
        const Ray3 r2 = camera_ray(cam, sx + ox, sy + oy);
        S.o = r2.o;
        S.d = normalize(focus - r2.o);
    }
    S.tint = v3(1.0f, 1.0f, 1.0f);
    S.bounce = 0;
    S.prev = -1;
}

// 1 - z^2 for z = 2^a (a <= 0) without cancellation: 1 - 2^(2a) = -expm1(2a ln 2) by its series
// near z = 1, else directly; both forms evaluated and selected (no divergent branch).  LEAN (the
// brute-force kernels) takes the direct form as 1 - z z from the z already computed (z^2 <= 0.958
// there, so the product's rounding costs a few ulp of the difference) instead of a second exp2.
template <bool LEAN>
__device__ __forceinline__ float one_minus_exp2_2a(float a, float z)
{
    const float x = 2.0f * a * 0.69314718055994531f;
    const float series = -x * fmaf(x, fmaf(x, fmaf(x, 1.0f / 24.0f, 1.0f / 6.0f), 0.5f), 1.0f);
    const float direct = LEAN ? fmaf(-z, z, 1.0f) : 1.0f - __builtin_amdgcn_exp2f(2.0f * a);
    return x > -0.0625f ? series : direct;
}

// Triangle.RayTraceAVXFaster (Triangle.cs:77-146) in fp64, in the reference's operation order
// (FMA crosses, hadd sums), on the ray that leaves a vertex-normal triangle from its own hit
// point o = fma(e01, u, fma(e02, v, v0)) (Triangle.cs:131).  The reference's next query meets the
// same triangle at t ~ 0 whenever the rounding residual of t is >= 0; RayHitMatches then decides
// whether that is the same hit (Util.cs:179-192).  For a flat triangle it always is (the face
// normal and the geometric side agree); a smooth normal (Triangle.GetNormal, :209-224) can send the
// ray under the geometric surface, and then it is not.  The kernel evaluates the same fp64
// expression on its own hit point.
__host__ __device__ __noinline__ bool vn_rehit_test(const PrimD& P, double u, double v, V3 dir, bool& inside,
                                                   double* t_out = nullptr, double* o_out = nullptr)
{
    const Vec4d a = P.a, e1 = P.b, e2 = P.c;
    const double d[4] = {(double)dir.x, (double)dir.y, (double)dir.z, 0.0};
    const double o[4] = {__builtin_fma(e1.x, u, __builtin_fma(e2.x, v, a.x)), __builtin_fma(e1.y, u, __builtin_fma(e2.y, v, a.y)),
                         __builtin_fma(e1.z, u, __builtin_fma(e2.z, v, a.z)), __builtin_fma(e1.w, u, __builtin_fma(e2.w, v, a.w))};
    const double off[4] = {o[0] - a.x, o[1] - a.y, o[2] - a.z, o[3] - a.w};
    const double b1[4] = {e1.x, e1.y, e1.z, e1.w}, c2[4] = {e2.x, e2.y, e2.z, e2.w};
    auto crs = [](const double* l, const double* r, double* out) { // SIMDHelpers.Cross
        out[0] = __builtin_fma(l[1], r[2], -(l[2] * r[1]));
        out[1] = __builtin_fma(l[2], r[0], -(l[0] * r[2]));
        out[2] = __builtin_fma(l[0], r[1], -(l[1] * r[0]));
        out[3] = __builtin_fma(l[3], r[3], -(l[3] * r[3]));
    };
    auto hs = [](const double* x, const double* y) { return (x[0] * y[0] + x[1] * y[1]) + (x[2] * y[2] + x[3] * y[3]); };
    double s1[4], s2[4];
    crs(off, b1, s1);
    crs(d, c2, s2);
    const double uu = hs(off, s2), vv = hs(d, s1), tt = hs(c2, s1), det = hs(b1, s2);
    const double inv = 1.0 / det;
    const double invz = (inv == inv) ? inv : 0.0;
    const double u2 = uu * invz, v2 = vv * invz, t2 = tt * invz;
    bool rej = (u2 < 0) | (v2 < 0) | (t2 < 0);
    rej |= (P.flags & F_MIRROR) ? ((u2 > 1) | (v2 > 1)) : ((u2 + v2) > 1);
    inside = invz < 0;
    if (t_out) *t_out = t2;
    if (o_out) {
        o_out[0] = o[0];
        o_out[1] = o[1];
        o_out[2] = o[2];
    }
    return !rej;
}

// Raytracer.cs:74-75: `if (i % 3 == 0) ray = Ray.Directional(...)` at the start of bounce i.  Here
// i <= Recursion; for the (usual) recursion depths below 32 the brute-force kernels test one bit of a
// constant.  The BVH kernels (SLOT) take the plain remainder: the bit test's extra scene read moved
// their register spills (C4 wide kernel 17 -> 23 VGPRs spilled).
template <bool SLOT, class SceneT>
__device__ __forceinline__ bool renormalise_at(const SceneT& s, int i)
{
    if (SLOT) return (unsigned)i % 3u == 0u;
    return s.recursion < 32 ? ((0x49249249u >> (unsigned)i) & 1u) != 0 : (unsigned)i % 3u == 0u;
}

// The closest hit a query starts from: none, or the re-hit of a vertex-normal triangle that
// shade() found the reference makes (encoded in Sample.prev <= -2 as -2 - sg).
template <bool VN, class SceneT>
__device__ __forceinline__ Best query_start(const SceneT& s, int prev)
{
    if (VN && s.n_vn > 0 && prev <= -2) return Best{0.0f, -2 - prev};
    return Best{__builtin_huge_valf(), -1};
}

// One bounce of Raytracer.GetColor after the closest-hit query.  Returns 0 to continue the
// path, 1 if the sample ended with colour `col`, 2 if it ended as a miss (Placeholder).
template <bool VN, bool PIN = false, bool SLOT = false, class SceneT, class VnP, class TestP>
__device__ __forceinline__ int shade(const SceneT& s, const PrimF* __restrict__ prims, const MatF* __restrict__ mats,
                                     const XformF* __restrict__ xfs, VnP vnormals, TestP tests, const PrimD* prims_d,
                                     const Best& b, Sample& S, V3& col)
{
    if (b.sg < 0) {
        if (S.bounce == 0 || s.ambient_miss) return 2;
        col = v3(s.ambient_r, s.ambient_g, s.ambient_b);
        return 1;
    }
    bool gin = (b.sg & 1) != 0;
    PrimF P = prims[b.sg >> 1];
    if (PIN) { // records from global memory: every field in flight at once (see pin_rec)
        pin4(P.a);
        pin4(P.b);
        pin4(P.d);
    }
    const uint32_t fl = __float_as_uint(P.b.w);
    const int id = __float_as_int(P.a.w);
    const MatF& M = mats[__float_as_int(P.d.w)]; // the primitive's material (deduplicated table)
    const uint32_t kind = fl & KIND_MASK;
    const V3 emis = xyz(M.emission);
    if (s.debug_geom) { // Raytracer.cs:93-98
        col = xyz(M.specular) + xyz(M.diffuse) + emis;
        return 1;
    }
    if (S.bounce >= s.recursion) {
        col = S.tint * emis;
        return 1;
    }
    // hit position and normal facing the incoming ray: one straight-line form for every kind
    // (world point o + t d), with transformed spheres and vertex-normal triangles on a separate
    // (rare) path.  The rectangle tests do not track the side of their hit, so a rectangle's
    // Inside is recomputed here (Moller-Trumbore's inside = d . N > 0), and an axis-aligned one's
    // hit point is put on its plane.
    V3 pos = madd(S.d, b.t, S.o);
    const bool sph = (s.facts & FACT_SPHERE) && kind == RT_PRIM_SPHERE;
    V3 n;
    if (SLOT) { // the BVH kernels (records in global memory: the three rows a, b, d only)
        const uint32_t axis = (fl & F_AXIS_MASK) >> F_AXIS_SHIFT; // axis-aligned rectangle: on its plane
        if (axis | (fl & F_FRAME_RECT)) gin = dot(S.d, xyz(P.d)) > 0.0f;
        pos.x = axis == 1 ? P.a.x : pos.x;
        pos.y = axis == 2 ? P.a.y : pos.y;
        pos.z = axis == 3 ? P.a.z : pos.z;
        n = sph ? (pos - xyz(P.a)) * P.b.y : xyz(P.d);
    } else { // the brute-force kernels (records in LDS): the same by arithmetic on the shading row c
        // c.xyz: one-hot plane axis of an axis-aligned rectangle (the hit point moves onto the plane
        // through v0 = P.a), c.w: 1/r of a sphere, whose P.d holds -centre/r (normal = p/r - c/r), 0
        // for the flat kinds, whose P.d is the face normal
        const float4 Pc = prims[b.sg >> 1].c;
        pos = v3(fmaf(Pc.x, P.a.x - pos.x, pos.x), fmaf(Pc.y, P.a.y - pos.y, pos.y), fmaf(Pc.z, P.a.z - pos.z, pos.z));
        n = madd(pos, Pc.w, xyz(P.d));
        if (fl & (F_AXIS_MASK | F_FRAME_RECT)) gin = dot(S.d, xyz(P.d)) > 0.0f;
    }
    float bu = 0.0f, bv = 0.0f; // vertex-normal triangle: the barycentrics of the hit
    if ((s.facts & (FACT_XF | FACT_VN)) && (fl & (F_TRANSFORMED | F_HASNORMALS))) {
        if (sph) { // ellipsoid: the world normal is an affine map of the world hit point
            n = normalize(xf_point(xfs[__float_as_int(P.b.z)].normal, pos));
        } else if (s.facts & FACT_VN) { // Triangle.GetNormal quirk: Normal is never set -> NaN when inside
            const VnP vn = vnormals + 3 * id;
            const TestRec R = tests[b.sg >> 1]; // barycentrics (u, v) = rows 0, 1 of M (p, 1)
            bu = dot4(R.r0, pos);
            bv = dot4(R.r1, pos);
            n = normalize(madd(xyz(vn[2]), bu + bv, madd(xyz(vn[1]), bv, xyz(vn[0]) * bu)));
            if (gin) n = v3(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""));
        }
    }
    const V3 nrm = gin ? -n : n;
    const bool inside = gin ^ ((fl & F_INVERT) != 0);

    // RandomShine (Raytracer.cs:51-56): z = U^(1/shininess), theta = U * 2pi
    const float shin = M.shininess;
    float z = 1.0f, sz = 0.0f;
    if (!(s.facts & FACT_INF_SHININESS) || !(__builtin_isinf(shin) && shin > 0.0f)) {
        const float a = __builtin_amdgcn_logf(next_u(S.rng)) * M.inv_shininess; // log2(U) / shininess
        z = __builtin_amdgcn_exp2f(a);
        sz = fsqrt(one_minus_exp2_2a<!SLOT>(a, z));
    }
    const Frame fr = make_frame(nrm);
    const V3 rough = horizon(fr, nrm, z, sz, next_u(S.rng));

    const float diff_lum = M.diffuse.w, emis_lum = M.emission.w;
    float spec_lum = M.specular.w, refr_lum = M.refraction.w;
    const float cs = -dot(rough, S.d);
    float cos_out = 0.0f, ior_ratio = 0.0f;
    // (luminances are never NaN: for them x > 0 is the integer compare of the bits, which needs no
    // quieting of the LDS-loaded operands as the max the compiler made of the float form did)
    const bool some_lum = SLOT ? ((refr_lum > 0.0f) | (spec_lum > 0.0f))
                               : ((__float_as_int(refr_lum) > 0) | (__float_as_int(spec_lum) > 0));
    if ((s.facts & FACT_IOR) && some_lum && M.ior != 0.0f &&
        cs >= 0.0f) { // Raytracer.cs:120-161
        ior_ratio = inside ? M.eta_exit : M.eta_enter; // eta = iorIn / iorOut
        const float sin_out = ior_ratio * fsqrt(1.0f - cs * cs);
        if (sin_out >= 1.0f) {
            refr_lum = 0.0f;
        } else {
            cos_out = fsqrt(1.0f - sin_out * sin_out);
            // unpolarised Fresnel with numerator and denominator divided by iorOut:
            // rs = (cs - eta co) / (cs + eta co), rp = (eta cs - co) / (eta cs + co), one reciprocal
            const float ra = fmaf(-ior_ratio, cos_out, cs), rb = fmaf(ior_ratio, cos_out, cs);
            const float pa = fmaf(ior_ratio, cs, -cos_out), pb = fmaf(ior_ratio, cs, cos_out);
            const float ratio = (ra * ra * pb * pb + pa * pa * rb * rb) * rcp(rb * rb * pb * pb) * 0.5f;
            spec_lum *= ratio;
            refr_lum *= 1.0f - ratio;
        }
    } else {
        refr_lum = 0.0f;
    }
    const float total = diff_lum + spec_lum + refr_lum + emis_lum;
    if (total <= 0.0f) {
        col = S.tint * emis;
        return 1;
    }
    // the choice (Raytracer.cs:177-229): refraction -> specular -> diffuse -> emission, by
    // subtracting luminances from U * total; then one direction formula per kind of event
    float ray_rand = next_u(S.rng) * total;
    const bool transmit = refr_lum != 0.0f && (ray_rand -= refr_lum) <= 0.0f;
    const bool specular = !transmit && spec_lum != 0.0f && (ray_rand -= spec_lum) <= 0.0f;
    const bool diffuse = !transmit && !specular && diff_lum != 0.0f && (ray_rand -= diff_lum) <= 0.0f;
    if (!(transmit | specular | diffuse)) { // emission
        col = S.tint * emis;
        return 1;
    }
    V3 out_dir, new_tint;
    if (diffuse) {
        const float dz = acos_turn2(next_u(S.rng)); // 2 acos(U) / pi (Raytracer.cs:215)
        const float ds = fsqrt(fmaxf(0.0f, 1.0f - dz * dz));
        out_dir = horizon(fr, nrm, dz, ds, next_u(S.rng));
        new_tint = xyz(M.diffuse);
    } else {
        // transmission: (d + rough cs) eta - rough cos_out; reflection: d + rough 2 cs
        const float al = transmit ? ior_ratio : 1.0f;
        const float be = transmit ? cs * ior_ratio - cos_out : 2.0f * cs;
        out_dir = madd(rough, be, S.d * al);
        if (specular && !(dot(out_dir, nrm) > 0.0f)) { // a specular ray into the surface ends the path
            col = S.tint * emis;
            return 1;
        }
        new_tint = transmit ? (inside ? v3(1.0f, 1.0f, 1.0f) : xyz(M.refraction)) : xyz(M.specular);
    }
    S.o = pos;
    // GetColor renormalises the direction at the start of bounces i = 0, 3, 6, 9, ... only
    // (Raytracer.cs:74-75, Ray.Directional); the ray leaving this bounce is traced as bounce
    // S.bounce + 1.  The reflected, transmitted and CreateHorizon directions are unit vectors up to
    // rounding, so one Newton step of 1/|d| (1.5 - 0.5 |d|^2, relative error (|d|^2 - 1)^2) is the
    // normalisation to fp32 precision, without the reciprocal square root.
    S.d = out_dir * (renormalise_at<SLOT>(s, S.bounce + 1) ? fmaf(-0.5f, dot(out_dir, out_dir), 1.5f) : 1.0f);
    S.prev = b.sg >> 1; // the primitive the ray leaves, named by its slot (every kernel)
    if (VN && s.n_vn > 0 && kind == RT_PRIM_TRIANGLE && (fl & F_HASNORMALS)) {
        // does the reference's next query meet this triangle again (vn_rehit_test), and is that a
        // new hit?  Primitive.RayTrace culls it first when one-sided (Primitive.cs:56-64).  A NaN
        // direction (a diffuse bounce about GetNormal's NaN) never gets past the BVH root
        // (BVH.cs:301-303: far >= 0 fails), so it meets nothing.
        bool gin2;
        if (!__builtin_isnan(S.d.x + S.d.y + S.d.z) && vn_rehit_test(prims_d[id], (double)bu, (double)bv, S.d, gin2) &&
            ((fl & F_TWOSIDED) || !(gin2 ^ ((fl & F_INVERT) != 0)))) {
            const bool front = dot(out_dir, nrm) > 0.0f; // Ray.Direction . prev.Normal (false for NaN)
            if (front ? (gin2 == gin) : (gin2 != gin))  // Inside compared after Invert on both sides
                S.prev = -2 - ((b.sg & ~1) | (int)gin2);
        }
    }
    S.tint = S.tint * (new_tint * (SLOT ? fmaxf(total, 1.0f) : vmax1(total)));
    S.bounce++;
    return 0;
}

#ifndef RT_PATH_WAVES
#define RT_PATH_WAVES 7 // minimum waves per SIMD the register allocator must allow (brute force; 6 -> 7: C2 28.4 -> 27.5 ms)
#endif
#ifndef RT_GROUPED_WAVES
#define RT_GROUPED_WAVES 7 // the same for the grouped brute-force kernel
#endif
#ifndef RT_WIDE_STACK
#define RT_WIDE_STACK 16 // LDS entries of the wide BVH kernel's traversal stack (then global overflow): 7 blocks per CU
#endif
#ifndef RT_BVH_SPEC
#define RT_BVH_SPEC 1 // speculative BVH traversal with wave-wide leaf steps (p.spec); 0: the mixed-step loop (C4 69.8 -> 62.1 ms)
#endif
#ifndef RT_SPEC_PRIMS
#define RT_SPEC_PRIMS 2 // leaf primitives per leaf step, both traversal loops (<= kTestSpares + 1)
#endif
#ifndef RT_BVH_WAVES
#define RT_BVH_WAVES 7 // the same for the BVH kernels (C4: 4 waves with a 40-entry LDS stack 80.7 ms, 5 waves with 24 entries
                       // 72.0 ms; with the launch record read at use, 6 waves with 20 entries (8 VGPRs spilled) 57.2-58.6
                       // against 60.7-61.3 ms at 5 / 24; 7 waves with 16 entries spilled 27 VGPRs: 70.1 ms.  Round 3,
                       // after compact leaves (one register of pending-leaf state) and o/d recomputed per node visit:
                       // 6 waves / 20 entries 45.9 ms (2 spilled), 7 waves / 16 entries 45.0 ms (17 spilled))
#endif
#ifndef RT_BVH2_WAVES
#define RT_BVH2_WAVES 6 // the BVH2 kernel (24-entry LDS stack: at most 6 blocks per CU)
#endif

// LDS staging of the shading records (PrimF per slot, MatF per ID, XformF): the per-lane gathers
// after each closest-hit query become LDS reads instead of dependent global loads.
struct ShadeRecs {
    const PrimF* prims;
    const MatF* mats;
    const XformF* xfs;
};
template <bool LDS, class SceneT>
__device__ __forceinline__ ShadeRecs stage_scene(const SceneT& s, const PrimF* prims_g, const MatF* mats_g,
                                                 const XformF* xf, float4* lds_scene)
{
    if (!LDS) return ShadeRecs{prims_g, mats_g, xf};
    const int n_p = s.n_slots * (int)(sizeof(PrimF) / 16), n_m = s.n_mats * (int)(sizeof(MatF) / 16),
              n_x = s.n_xf * (int)(sizeof(XformF) / 16);
    const float4* gp = reinterpret_cast<const float4*>(prims_g);
    const float4* gm = reinterpret_cast<const float4*>(mats_g);
    const float4* gx = reinterpret_cast<const float4*>(xf);
    for (int i = threadIdx.x; i < n_p; i += blockDim.x) lds_scene[i] = gp[i];
    for (int i = threadIdx.x; i < n_m; i += blockDim.x) lds_scene[n_p + i] = gm[i];
    for (int i = threadIdx.x; i < n_x; i += blockDim.x) lds_scene[n_p + n_m + i] = gx[i];
    __syncthreads();
    return ShadeRecs{reinterpret_cast<const PrimF*>(lds_scene), reinterpret_cast<const MatF*>(lds_scene + n_p),
                     reinterpret_cast<const XformF*>(lds_scene + n_p + n_m)};
}

__device__ __forceinline__ int scene_lds_float4s(const PathScene& s)
{
    return s.n_slots * (int)(sizeof(PrimF) / 16) + s.n_mats * (int)(sizeof(MatF) / 16) +
           s.n_xf * (int)(sizeof(XformF) / 16);
}

// One lane's work: the open work item (a chunk of samples of one pixel), its running sums and
// the sample in flight.  The wave's item pool [pool_next, pool_end) is wave-uniform.
struct Lane {
    bool active, item_open, live;
    unsigned item;
    int fx, fy, s_next;
    rt_key2 pkey; // rt_rng_pixel_key of the open item's pixel
    float ar, ag, ab;
    unsigned cnt; // item bookkeeping: samples (bits 0-7) | misses (8-15) | samples left (16-31)
    unsigned pool_next, pool_end;
    unsigned split_j; // lane 0: item ranges (after its own) this wave found spent (PathParams::n_split)
};

__device__ __forceinline__ void lane_init(Lane& L)
{
    L.active = true;
    L.item_open = L.live = false;
    L.item = 0;
    L.fx = L.fy = L.s_next = 0;
    L.pkey = rt_key2{0u, 0u};
    L.ar = L.ag = L.ab = 0.0f;
    L.cnt = 0;
    L.pool_next = L.pool_end = 0;
    L.split_j = 0;
}

// Lanes without a sample in flight close finished items and take new ones from the wave's
// pool (one atomic per p.pool items: chunks of one 8x8 block), then start the next camera sample
// of their item.
// NT: store the item partials non-temporally (the BVH kernels: their 16-B-per-sample partial
// stream would otherwise push the scene out of the Infinity Cache; C4 52.74-52.86 -> 52.30-52.37
// ms; the brute-force kernels keep normal stores, die.txt C3 27.5 -> 27.7-27.8 ms with them)
// The BVH (NT) kernels hold as little per lane as they can: at 7 waves per SIMD every register the
// refill and shading phases keep live spilled (round 5: 19 VGPRs, 21 GB of scratch writes per C4
// launch against 2.1 GB of partials).  Four changes, each computing the same values, took that to
// 2 (profiles/r06/c4_ab.txt, one call: C4 42.99 -> 38.52 ms, WRITE_SIZE 21.2 -> 2.7 GB per launch):
// * a lane's rank in the item dispenser by v_mbcnt (lanes_below), not a popcount of
//   m & ((1 << lane) - 1), whose 64-bit lane mask the compiler hoisted out of the loop and spilled;
// * the pixel's frame x and y in one register (L.fx = x | y << 16); since the xorshift stream (round 6),
//   in none: decoded from the item again at each sample start (item_pixel), as is the sample index
//   (item_sample; C4 scratch 24 -> 8 B per lane);
// * the pixel's RNG key derived again at each sample start instead of held per lane;
// * 1/d of every lane's query rebuilt after the shading phase instead of held through it.
// The brute-force kernels keep their layout (they read the pixel key from the scene's table).
__device__ __forceinline__ unsigned lanes_below(unsigned long long m)
{
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
// A work item's pixel: item = ((block << log2_chunks) + chunk) * 64 + pixel of the 8x8 block, tile
// coordinates (px, py), its chunk c, and its frame coordinates (fx, fy; a band set maps tile rows to
// frame rows).
template <class ParT>
__device__ __forceinline__ void item_pixel(unsigned item, const ParT& p, int& px, int& py, int& c, int& fx, int& fy)
{
    const unsigned q = item & 63u, t = item >> 6;
    c = (int)(t & (unsigned)(p.n_chunks - 1));
    unsigned by, bx;
    const unsigned blk = t >> p.log2_chunks;
    if (p.magic_bx != 0) { // multiply-high division (exact here, make_params checks)
        by = __umulhi(blk, p.magic_bx);
        bx = blk - by * (unsigned)p.blocks_x;
    } else {
        divmod(blk, (unsigned)p.blocks_x, p.inv_blocks_x, by, bx);
    }
    px = (int)bx * 8 + (int)(q & 7);
    py = (int)by * 8 + (int)(q >> 3);
    fx = p.x0 + px;
    fy = p.y0 + py;
    if (p.band > 0) { // band set: tile row py -> frame row (wave-uniform branch)
        unsigned bq, br;
        if (p.band_log2 >= 0) {
            bq = (unsigned)py >> p.band_log2;
            br = (unsigned)py & (unsigned)(p.band - 1);
        } else {
            divmod((unsigned)py, (unsigned)p.band, p.inv_band, bq, br);
        }
        fy = p.y0 + ((int)bq * p.band_stride + p.band_offset) * p.band + (int)br;
    }
}

// The next sample of the lane's item.  The BVH (NT) kernels hold no register for it: the item's
// first sample (its chunk, from the item index) plus the samples it finished (samples + misses).
template <bool NT, class ParT>
__device__ __forceinline__ int item_sample(const Lane& L, const ParT& p)
{
    if (!NT) return L.s_next;
    const int c = (int)((L.item >> 6) & (unsigned)(p.n_chunks - 1));
    return c * p.chunk + (int)(L.cnt & 0xFFu) + (int)((L.cnt >> 8) & 0xFFu);
}
template <bool NT, class ParT, class SceneT, class CamT>
__device__ __forceinline__ void refill(Lane& L, Sample& S, const ParT& p, const SceneT& s, const CamT& cam, int lane,
                                      unsigned total)
{
    const bool need = L.active && !L.live && (!L.item_open || L.cnt < 65536u);
    if (need && L.item_open) {
        const float4 part = make_float4(L.ar, L.ag, L.ab, __uint_as_float((L.cnt & 0xFFu) | ((L.cnt & 0xFF00u) << 8)));
        if (NT) {
            typedef float nt_f4 __attribute__((ext_vector_type(4)));
            const nt_f4 v = {part.x, part.y, part.z, part.w};
            __builtin_nontemporal_store(v, reinterpret_cast<nt_f4*>(&p.partial[L.item]));
        } else {
            p.partial[L.item] = part;
        }
        L.item_open = false;
        L.ar = L.ag = L.ab = 0.0f; // the next item starts from zero
    }
    const unsigned long long m = __ballot(need);
    if (m) {
        const unsigned k = (unsigned)__popcll(m), avail = L.pool_end - L.pool_next;
        unsigned fresh = 0;
        if (k > avail) { // wave-uniform: one atomic refills the pool
            if (lane == 0) {
                if (p.n_split <= 1) {
                    fresh = atomicAdd(p.counter, (unsigned)p.pool);
                } else {
                    // the range of this workgroup's XCD first, then the others in turn (L.split_j: the
                    // ranges this wave found spent); all spent -> total, which ends the lane
                    fresh = total;
                    const unsigned g0 = blockIdx.x & (unsigned)(p.n_split - 1);
                    for (; L.split_j < (unsigned)p.n_split; L.split_j++) {
                        const unsigned g = (g0 + L.split_j) & (unsigned)(p.n_split - 1);
                        const unsigned f = atomicAdd(p.counter + kSplitStride * g, (unsigned)p.pool);
                        if (f < p.split_start[g + 1] - p.split_start[g]) {
                            fresh = p.split_start[g] + f;
                            break;
                        }
                    }
                }
            }
            fresh = __builtin_amdgcn_readfirstlane(fresh);
        }
        if (need) {
            const unsigned r = NT ? lanes_below(m) : (unsigned)__popcll(m & ((1ull << lane) - 1ull));
            L.item = r < avail ? L.pool_next + r : fresh + (r - avail);
            if (L.item >= total) {
                L.active = false;
            } else {
                int px, py, c, fx, fy;
                item_pixel(L.item, p, px, py, c, fx, fy);
                if (px < p.w && py < p.h && c * p.chunk < p.spp) {
                    L.item_open = true;
                    const int s0 = c * p.chunk;
                    if (!NT) L.s_next = s0; // (the BVH kernels derive it: item_sample)
                    L.cnt = (unsigned)(min(p.spp, s0 + p.chunk) - s0) << 16; // chunk <= 64
                    if (!NT) { // (the BVH kernels decode the item again at each sample start)
                        L.fx = fx;
                        L.fy = fy;
                    }
                    // the frame width from the launch record (a scene-specialised build's constant
                    // scene leaves it out, so one build serves every frame size)
                    const unsigned long long pix = (unsigned long long)fy * (unsigned long long)p.scene.width +
                                                   (unsigned long long)fx;
                    // the brute-force kernels read the key from the scene's table (the same value:
                    // two hash rounds fewer per item open, which runs in most iterations)
                    if (!NT && p.pkeys) L.pkey = p.pkeys[pix];
                    else if (!NT) L.pkey = rt_rng_pixel_key(p.seed_key, pix);
                }
            }
        }
        if (k > avail) {
            L.pool_next = fresh + (k - avail);
            L.pool_end = fresh + (unsigned)p.pool;
        } else {
            L.pool_next += k;
        }
    }
    if (L.active && L.item_open && !L.live && L.cnt >= 65536u) {
        int fx = L.fx, fy = L.fy;
        if (NT) { // the pixel and its key again at every sample start: three registers fewer held
            int px, py, c;
            item_pixel(L.item, p, px, py, c, fx, fy);
            L.pkey = rt_rng_pixel_key(p.seed_key, (unsigned long long)fy * (unsigned long long)p.scene.width +
                                                      (unsigned long long)fx);
        }
        S.rng = rt_rng_from_pixel_key(L.pkey, p.sample_base + (unsigned long long)item_sample<NT>(L, p));
        start_sample<!NT>(cam, fx, fy, S);
        L.live = true;
    }
}

// After a closest-hit query: one bounce of GetColor; a finished sample goes into the item's sums.
template <bool VN, bool PIN = false, bool SLOT = false, class SceneT, class VnP, class TestP>
__device__ __forceinline__ void bounce(Lane& L, Sample& S, const SceneT& s, const ShadeRecs& R, VnP vnormals, TestP tests,
                                       const PrimD* prims_d, const Best& b)
{
    V3 col;
    const int r = shade<VN, PIN, SLOT>(s, R.prims, R.mats, R.xfs, vnormals, tests, prims_d, b, S, col);
    if (r != 0) {
        const bool hit = r == 1;
        L.ar += hit ? col.x : 0.0f;
        L.ag += hit ? col.y : 0.0f;
        L.ab += hit ? col.z : 0.0f;
        L.cnt += hit ? 1u - 65536u : 256u - 65536u; // one more sample or miss, one fewer left
        if (!SLOT) L.s_next++; // (the BVH kernels derive it from cnt: item_sample)
        L.live = false;
        if (!SLOT) {
            // The sample is over: its ray state is dead until the next start_sample writes all of it.
            // Saying so (an empty asm that "defines" the registers) lets the register allocator give
            // these values the registers the continuing lanes' new ray state takes, instead of
            // copying the 12 sample registers out and back at this divergent join (23 moves per
            // iteration in the bounce.txt listing; measured: C2 unchanged, C3 27.31-27.40 ->
            // 27.25-27.31 ms).  The BVH kernels, whose finished lanes wait for the batched shading
            // phase, keep the plain form.
            asm volatile("" : "=v"(S.o.x), "=v"(S.o.y), "=v"(S.o.z), "=v"(S.d.x), "=v"(S.d.y), "=v"(S.d.z),
                         "=v"(S.tint.x), "=v"(S.tint.y), "=v"(S.tint.z), "=v"(S.bounce), "=v"(S.prev),
                         "=v"(S.rng.x));
        }
    }
}

template <bool STATS, class ParT>
__device__ __forceinline__ void flush_counts(unsigned long long wave_rays, const Counters& cnt, const ParT& p,
                                             int lane)
{
    // one 64-bit add per wave for the ray count (and the optional traversal counters)
    if (lane == 0) atomicAdd(p.rays, wave_rays);
    if (STATS) {
        unsigned long long a = cnt.nodes, t = cnt.tris, q = cnt.sphs;
        for (int off = 32; off > 0; off >>= 1) {
            a += __shfl_down(a, off);
            t += __shfl_down(t, off);
            q += __shfl_down(q, off);
        }
        if (lane == 0) {
            atomicAdd(p.stats + 0, a);
            atomicAdd(p.stats + 1, t);
            atomicAdd(p.stats + 2, q);
            atomicAdd(p.stats + 3, cnt.cyc_start);
            atomicAdd(p.stats + 4, cnt.cyc_trace);
            atomicAdd(p.stats + 5, cnt.cyc_shade);
            atomicAdd(p.stats + 6, cnt.iters);
        }
        unsigned long long mx = cnt.max_steps, ov = cnt.ovf_pushes, ms = cnt.max_sp, ot = cnt.outer;
        for (int off = 32; off > 0; off >>= 1) {
            mx = max(mx, (unsigned long long)__shfl_down(mx, off));
            ov += __shfl_down(ov, off);
            ms = max(ms, (unsigned long long)__shfl_down(ms, off));
            ot += __shfl_down(ot, off);
        }
        if (lane == 0) {
            atomicMax(p.stats + 7, mx);
            atomicAdd(p.stats + 8, ov);
            atomicMax(p.stats + 9, ms);
            atomicAdd(p.stats + 10, ot);
        }
    }
}

// The camera and the launch parameters in the constant address space: uniform reads become
// scalar loads (the kernels never write them).
#ifdef __HIP_DEVICE_COMPILE__
#define RT_AS_CONST __attribute__((address_space(4)))
#else
#define RT_AS_CONST // the host pass only needs the types
#endif
typedef RT_AS_CONST const CameraF CameraC;
typedef RT_AS_CONST const PathParams ParamsC;

// Brute-force megakernel: every loop iteration issues one closest-hit query per live lane
// (the scene's records arrive through scalar loads) and shades it.
template <bool CULL, bool LDS, bool STATS, bool VN>
__device__ __forceinline__ void path_body(const CameraF* __restrict__ camp, const PathParams* __restrict__ pp)
{
    // everything but the LDS staging is read from the launch record *pp (fill_launch) in the
    // constant address space, by scalar loads where it is used (the by-value arguments are the
    // BVH kernels'; held in SGPRs for the whole kernel they spilled into VGPR lanes here)
    const ParamsC& P0 = *(const ParamsC*)pp;
    extern __shared__ float4 lds_scene[];
    const ShadeRecs R = stage_scene<LDS>(P0.scene, P0.prims, P0.mats, P0.xf, lds_scene);
    const int lane = threadIdx.x & 63;
    const unsigned total = (unsigned)P0.n_chunks * (unsigned)P0.n_pad;
    Lane L;
    lane_init(L);
    Sample S;
    S.prev = -1;
    S.bounce = 0;
    Counters cnt{};
    unsigned long long wave_rays = 0; // wave-uniform

    while (true) {
        unsigned long long t0 = 0, t1 = 0, t2 = 0;
        if (STATS) t0 = __builtin_readcyclecounter();
        // The camera and the launch record are read per iteration through scalar loads from an
        // opaque pointer: that keeps the compiler from holding ~28 camera words and the scene
        // fields in SGPRs for the whole kernel (they spilled into VGPR lanes and scratch).  The
        // pointers are in the constant address space: through a generic pointer the compiler
        // cannot rule out the kernel's own stores and emits per-lane flat loads instead.
        const CameraC* cp = (const CameraC*)camp;
        asm volatile("" : "+s"(cp));
        const ParamsC* pq = (const ParamsC*)pp;
        asm volatile("" : "+s"(pq));
#ifdef RT_SCENE_CONST
        const PathScene& sc = *(const PathScene*)kSceneW;
#else
        const auto& sc = pq->scene;
#endif
#if defined(RT_SCENE_CONST) && RT_SCENE_CONST_CAMERA
        refill<false>(L, S, *pq, sc, *(const CameraF*)kCameraW, lane, total); // the camera compiled in too
#else
        refill<false>(L, S, *pq, sc, *cp, lane, total);
#endif
        if (!__any(L.active)) break;
        if (STATS) t1 = __builtin_readcyclecounter();
        wave_rays += (unsigned)__popcll(__ballot(L.live)); // one Scene.RayTrace per live lane
        if (L.live) {
#ifdef RT_SCENE_CONST // scene-specialised build (rt_jit.cpp): the records are compile-time constants
            const auto tests = (const TestRec*)kTestsW;
            const auto rects = (const RectRec*)kRectsW;
            const auto frames = (const FrameRec*)kFramesW;
            const auto boxes = (const BoxRec*)kFramesW;
            const auto groups = (const GroupRec*)kGroupsW;
            const auto xf = (const XformF*)kXfW;
#else
            const auto tests = (const RT_AS_CONST TestRec*)pq->tests;
            const auto rects = (const RT_AS_CONST RectRec*)pq->rects;
            const auto frames = (const RT_AS_CONST FrameRec*)pq->frames;
            const auto boxes = (const RT_AS_CONST BoxRec*)pq->frames;
            const auto groups = (const RT_AS_CONST GroupRec*)pq->groups;
            const auto xf = (const RT_AS_CONST XformF*)pq->xf;
#endif
            const auto vnormals = (const RT_AS_CONST float4*)pq->vnormals;
            Best b = query_start<VN>(sc, S.prev);
            trace_brute<CULL, STATS>(sc, groups, tests, rects, frames, boxes, xf, S.o, S.d, S.prev, b, cnt.tris,
                                     cnt.sphs, cnt.nodes);
            const int pln0 = sc.n_bvh;
            for (int i = pln0; i < pln0 + sc.n_pln; i++) {
                const TestRec tr = tests[i];
                hit_plane<true>(tr, i, S.o, S.d, S.prev, b);
            }
            // A NaN direction (a diffuse bounce about GetNormal's NaN normal, only in scenes with
            // vertex-normal triangles) fails the reference's BVH root test (BVH.cs:301-303: far >= 0
            // is false for NaN) and meets nothing.  The brute-force records would not all say so: a
            // box's slab reciprocals stay finite for NaN (slab_rcp_lean), so a NaN ray inside a room
            // box met its exit face.
            if (VN && __builtin_isnan(S.d.x + S.d.y + S.d.z)) b = Best{__builtin_huge_valf(), -1};
            if (STATS) t2 = __builtin_readcyclecounter();
            bounce<VN>(L, S, sc, R, vnormals, tests, pq->prims_d, b);
        } else if (STATS) {
            t2 = __builtin_readcyclecounter();
        }
        if (STATS) {
            const unsigned long long t3 = __builtin_readcyclecounter();
            cnt.cyc_start += t1 - t0;
            cnt.cyc_trace += t2 - t1;
            cnt.cyc_shade += t3 - t2;
            cnt.iters++;
        }
    }
    flush_counts<STATS>(wave_rays, cnt, *(const ParamsC*)pp, lane);
}

template <bool CULL, bool LDS, bool STATS, bool VN>
__global__ void __launch_bounds__(256, CULL ? RT_GROUPED_WAVES : RT_PATH_WAVES)
    path_kernel(PathScene, const CameraF* __restrict__ camp, const PathParams* __restrict__ pp, const TestRec*,
                const RectRec*, const FrameRec*, const PrimF*, const NodeF*, const Node4Q*, const GroupRec*,
                const XformF*, const MatF*, const float4*)
{
    path_body<CULL, LDS, STATS, VN>(camp, pp); // the other arguments are the BVH kernels' (same launch)
}

// The BVH order's outer group (DevScene::groups_bvh): the world rects and closed boxes left out of
// the tree, tested by the lanes whose query ended, as the brute-force kernels test a group.
template <bool STATS, class GroupP, class RectP, class BoxP>
__device__ __forceinline__ void test_outer(GroupP groups, RectP rects, BoxP boxes, V3 o, V3 d, int prev, Best& b,
                                           unsigned& n_tests)
{
    const V3 id = v3(slab_rcp_lean(d.x), slab_rcp_lean(d.y), slab_rcp_lean(d.z));
    const V3 oi = o * id;
    const GroupRec G = groups[0];
    if (STATS) n_tests += G.n_rect[0] + G.n_rect[1] + G.n_rect[2] + G.n_flat_extra;
    RectP r = rects + __float_as_int(G.lo.w);
    rect_group<0>(r, G.n_rect[0], o, d, id, oi, prev, b);
    r += G.n_rect[0];
    rect_group<1>(r, G.n_rect[1], o, d, id, oi, prev, b);
    r += G.n_rect[1];
    rect_group<2>(r, G.n_rect[2], o, d, id, oi, prev, b);
    for (int j = G.frame_first + G.n_frames; j < G.frame_first + G.n_frames + G.n_boxes; j++) {
        const BoxRec B = boxes[j];
        hit_box<false>(B, o, d, id, oi, prev, b);
    }
}

// One leaf step of the BVH kernels: RT_SPEC_PRIMS primitives of the pending leaf pend, their
// loads issued together.  Every leaf reads the 48-B rows of its records (3 loads per primitive); a
// compact leaf's flags come with its reference (lfl), a generic leaf's from each record's meta row
// (one more 4-B load).  The BVH order holds triangles and spheres only (planes follow it), and both
// arrays carry kTestSpares zero records after the last slot.
template <bool STATS, class TestP, class RowP, class XfP>
__device__ __forceinline__ void test_leaf(TestP tests, RowP rows, XfP xf, int pend, V3 o, V3 d, int prev, Best& b,
                                          unsigned& n_tri, unsigned& n_sph)
{
    int k, kend;
    uint32_t lfl;
    leaf_decode(pend, k, kend, lfl);
    float4 r[RT_SPEC_PRIMS][3];
    uint32_t fl[RT_SPEC_PRIMS];
#pragma unroll
    for (int j = 0; j < RT_SPEC_PRIMS; j++) {
        r[j][0] = rows[3 * (k + j)];
        r[j][1] = rows[3 * (k + j) + 1];
        r[j][2] = rows[3 * (k + j) + 2];
    }
    if (lfl == kLeafGeneric) {
#pragma unroll
        for (int j = 0; j < RT_SPEC_PRIMS; j++) fl[j] = __float_as_uint(tests[k + j].meta.y);
    } else {
#pragma unroll
        for (int j = 0; j < RT_SPEC_PRIMS; j++) fl[j] = lfl;
    }
    // all rows in registers before the kind dispatch: otherwise the compiler sinks row loads into the
    // triangle / sphere branches, one more round trip per step (C4 49.9 -> 48.9 ms, 64-B records)
#pragma unroll
    for (int j = 0; j < RT_SPEC_PRIMS; j++) {
        pin4(r[j][0]);
        pin4(r[j][1]);
        pin4(r[j][2]);
    }
#pragma unroll
    for (int j = 0; j < RT_SPEC_PRIMS; j++) {
        if (j == 0 || k + j < kend) {
            const bool sph = (fl[j] & KIND_MASK) == RT_PRIM_SPHERE;
            if (STATS) {
                if (sph) n_sph++;
                else n_tri++;
            }
            if (sph) hit_sph_rows(r[j][0], r[j][1], fl[j], k + j, k + j, o, d, prev, xf, b);
            else hit_tri_rows(r[j][0], r[j][1], r[j][2], fl[j], k + j, k + j, o, d, prev, b);
        }
    }
}

// BVH megakernel with decoupled traversal.  A loop iteration advances the traversing lanes by
// one step: with RT_BVH_SPEC a wave-wide node step or leaf step (up to two primitives), lanes
// keeping a reached leaf pending while they visit further nodes; without it, one node visit or
// one leaf step per lane.  Lanes whose query finished wait, and the shading / new-sample phase
// runs only once at least p.refill lanes wait (or none is still traversing).  So one long
// traversal no longer holds the other 63 lanes of its wave, and the divergent shading code is
// paid once per batch of finished queries.
template <int WIDTH, int STACK, bool LDS, bool STATS, bool VN>
__global__ void __launch_bounds__(256, WIDTH == 4 ? RT_BVH_WAVES : RT_BVH2_WAVES)
    path_kernel_bvh(PathScene, const CameraF* __restrict__ camp, const PathParams* __restrict__ pp, const TestRec*,
                    const RectRec*, const FrameRec*, const PrimF*, const NodeF*, const Node4Q*, const GroupRec*,
                    const XformF*, const MatF*, const float4*)
{
    // As in the brute-force kernels, the camera and the launch record are read through opaque
    // constant-address-space pointers where they are used (held whole-kernel in SGPRs, they
    // spilled 58 SGPRs into VGPR lanes here); the other arguments are unused.
    const ParamsC& P0 = *(const ParamsC*)pp;
    __shared__ int stack_mem[STACK * 256];
    extern __shared__ float4 lds_scene[];
    const TravStack stk = make_stack(stack_mem, P0.stack_ovf);
    const ShadeRecs R = stage_scene<LDS>(P0.scene, P0.prims, P0.mats, P0.xf, lds_scene);
    // hot wide nodes after the staged shading records (dynamic LDS; see path_lds_bytes)
    Node4Q* lds_hot = reinterpret_cast<Node4Q*>(lds_scene + (LDS ? scene_lds_float4s(P0.scene) : 0));
    if (WIDTH == 4 && P0.scene.n_hot4 > 0) {
        const float4* src = reinterpret_cast<const float4*>(P0.scene.hot4);
        float4* dst = reinterpret_cast<float4*>(lds_hot);
        for (int i = threadIdx.x; i < P0.scene.n_hot4 * 4; i += blockDim.x) dst[i] = src[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const unsigned total = (unsigned)P0.n_chunks * (unsigned)P0.n_pad;
    Lane L;
    lane_init(L);
    Sample S;
    S.prev = -1;
    S.bounce = 0;
    Counters cnt{};
    unsigned long long wave_rays = 0; // wave-uniform
    // traversal state of the lane's current query
    bool trav = false, done = false;
    [[maybe_unused]] bool more = false; // RT_BVH_SPEC: ref still holds a reference to process (stack not exhausted)
    int ref = 0, sp = 0;
    int pend = -1; // the pending leaf (leaf_decode), -1 for none
    // 1/d of the query; o/d is recomputed per node visit (three multiplies) instead of being held
    // across the loop (VGPR spills of the C4 kernel 13 -> 2 at 6 waves per SIMD; recomputing 1/d as
    // well, three clamped reciprocals per visit, measured slower: 45.9 -> 46.2 ms)
    V3 id{0, 0, 0};
    Best b{__builtin_huge_valf(), -1};

    while (true) {
        const ParamsC* pq = (const ParamsC*)pp;
        asm volatile("" : "+s"(pq));
        const CameraC* cp = (const CameraC*)camp;
        asm volatile("" : "+s"(cp));
        const ParamsC& p = *pq;
        const auto& s = pq->scene;
        const auto tests = (const RT_AS_CONST TestRec*)pq->tests;
        const auto rows = (const RT_AS_CONST float4*)pq->rows;
        const auto xf = (const RT_AS_CONST XformF*)pq->xf;
        const auto vnormals = (const RT_AS_CONST float4*)pq->vnormals;
        const auto nodes = (const RT_AS_CONST NodeF*)pq->nodes;
        const auto nodes4 = (const RT_AS_CONST Node4Q*)pq->nodes4;
        const unsigned long long waiting = __ballot(!trav && (L.active || L.live));
        const unsigned long long busy = __ballot(trav);
        if (!waiting && !busy) break;
        // The threshold is at most half the lanes still holding work, so that a wave whose item pool
        // ran dry does not hold its finished lanes until every query ends (C4 38.24-38.28 -> 38.10-38.15
        // ms, profiles/r06/ab_refill_adapt.log)
        const int refill_at = min(p.refill, (__popcll(waiting | busy) + 1) >> 1);
        if (!busy || __popcll(waiting) >= refill_at) {
            wave_rays += (unsigned)__popcll(__ballot(done)); // one Scene.RayTrace per finished query
            if (done) { // the query finished: the outer records and planes (outside the BVH), then one bounce
                // (a NaN direction, from a vertex-normal triangle, meets nothing: see path_body).  Here,
                // not at the query's start: there it held the query's best hit through the traversal
                // and measured 48.35 against 38.52 ms (profiles/r06/c4_ab.txt, lowreg_ostart)
                if (s.n_groups > 0 && !(VN && __builtin_isnan(S.d.x + S.d.y + S.d.z)))
                    test_outer<STATS>((const RT_AS_CONST GroupRec*)pq->groups, (const RT_AS_CONST RectRec*)pq->rects,
                                      (const RT_AS_CONST BoxRec*)pq->frames, S.o, S.d, S.prev, b, cnt.outer);
                for (int i = s.n_bvh; i < s.n_bvh + s.n_pln; i++) {
                    const TestRec tr = tests[i];
                    hit_plane<true>(tr, i, S.o, S.d, S.prev, b);
                }
                if (STATS && p.ray_log) { // rt_debug_ray_log: the query and its closest hit
                    const unsigned q = atomicAdd(p.ray_log_n, 1u);
                    if (q < p.ray_log_cap) {
                        float4* r = p.ray_log + 3 * (size_t)q;
                        r[0] = make_float4(S.o.x, S.o.y, S.o.z, __int_as_float(S.prev));
                        int px, py, c, fx, fy;
                        item_pixel(L.item, p, px, py, c, fx, fy);
                        r[1] = make_float4(S.d.x, S.d.y, S.d.z, __int_as_float(fy * p.scene.width + fx));
                        r[2] = make_float4(b.t, __int_as_float(b.sg), __int_as_float(S.bounce), 0.0f);
                    }
                }
                bounce<VN, !LDS, true>(L, S, s, R, vnormals, tests, pq->prims_d, b);
                done = false;
            }
            refill<true>(L, S, p, s, *cp, lane, total);
            if (L.live && !trav) { // start the next query
                ref = s.root;
                sp = 0;
                pend = -1;
                more = true;
                if (ref < 0) { // the root itself is a leaf
                    pend = ~ref;
                    more = false;
                }
                b = query_start<VN>(s, S.prev);
                trav = true;
            }
            // 1/d of every lane's query rebuilt after the shading phase, so that the three registers
            // are free inside it (the traversing lanes recompute the same values)
            id = v3(slab_rcp(S.d.x), slab_rcp(S.d.y), slab_rcp(S.d.z));
        }
#if RT_BVH_SPEC
        // Speculative traversal (Aila & Laine 2009): a lane that reaches a leaf keeps it pending and
        // goes on visiting nodes.  Leaf primitives are tested in wave-wide leaf steps, taken once
        // p.spec lanes are blocked (a second leaf reached, or no node left) or no lane can visit a
        // node, so an iteration is one kind of step instead of both.  Node culling uses the best hit
        // so far (the pending leaf not yet tested): more visits, the same closest hit.
#ifndef RT_SPEC_RUNAHEAD
#define RT_SPEC_RUNAHEAD 1 // 0: a lane with a pending leaf waits for the leaf step instead of visiting on
#endif
        const bool can_node = trav && more && ref >= 0 && (RT_SPEC_RUNAHEAD || pend < 0);
        const bool blocked = trav && pend >= 0 && !can_node;
        const bool leaf_step = __ballot(can_node) == 0 || __popcll(__ballot(blocked)) >= p.spec; // wave-uniform
        if (STATS) { // lane slots of this iteration (the BVH kernels reuse the brute-force cycle counters):
                     // testing a leaf | traversing but idle in this step's kind | waiting for the shading phase
            const unsigned n_trav = (unsigned)__popcll(__ballot(trav));
            const unsigned n_node = leaf_step ? 0u : (unsigned)__popcll(__ballot(can_node));
            const unsigned n_leaf = leaf_step ? (unsigned)__popcll(__ballot(trav && pend >= 0)) : 0u;
            cnt.cyc_start += n_leaf;
            cnt.cyc_trace += n_trav - n_node - n_leaf;
            cnt.cyc_shade += (unsigned)__popcll(__ballot(!trav && (L.active || L.live)));
        }
        if (trav) {
            if (leaf_step) {
                if (pend >= 0) { // RT_SPEC_PRIMS primitives of the pending leaf, their loads issued together
                    test_leaf<STATS>(tests, rows, xf, pend, S.o, S.d, S.prev, b, cnt.tris, cnt.sphs);
                    pend = leaf_advance(pend, RT_SPEC_PRIMS);
                }
            } else if (can_node) {
                bool pop = true;
                const V3 oi = S.o * id;
                if (WIDTH == 4) {
                    const Node4Q q = (ref & RT_HOT_BIT) ? lds_hot[ref & ~RT_HOT_BIT] : Node4Q(nodes4[ref]);
                    [[maybe_unused]] const int sp0 = sp;
                    wide_visit<STACK>(q, id, oi, b.t, ref, sp, stk, pop);
                    if (STATS) {
                        cnt.ovf_pushes += (unsigned)max(0, sp - max(sp0, STACK));
                        cnt.max_sp = max(cnt.max_sp, (unsigned)sp);
                    }
                } else {
                    const NodeF n = nodes[ref];
                    float tl, tr;
                    const bool hl = slab(n.lmin, n.lmax, oi, id, b.t, tl);
                    const bool hr = slab(n.rmin, n.rmax, oi, id, b.t, tr);
                    const int cl = __float_as_int(n.lmin.w), cr = __float_as_int(n.rmin.w);
                    if (hl && hr) {
                        const bool lf = tl <= tr;
                        push<STACK>(stk, sp, lf ? cr : cl);
                        ref = lf ? cl : cr;
                        pop = false;
                    } else if (hl | hr) {
                        ref = hl ? cl : cr;
                        pop = false;
                    }
                }
                if (STATS) cnt.nodes++;
                if (pop) {
                    if (sp > 0) ref = pop_ref<STACK>(stk, sp);
                    else more = false;
                }
            }
            // a leaf reference becomes the pending leaf once the previous one is tested, and the
            // next reference is popped so that traversal goes on past it
            if (more && ref < 0 && pend < 0) {
                pend = ~ref;
                if (sp > 0) ref = pop_ref<STACK>(stk, sp);
                else more = false;
            }
            if (!more && pend < 0) {
                trav = false;
                done = true;
            }
        }
#else
        if (trav) { // one traversal step: one node visit, or one primitive of the current leaf
            bool pop = true; // child references are node indices or ~leaf codes (any int)
            if (pend >= 0) { // RT_SPEC_PRIMS primitives, their loads issued together
                test_leaf<STATS>(tests, rows, xf, pend, S.o, S.d, S.prev, b, cnt.tris, cnt.sphs);
                pend = leaf_advance(pend, RT_SPEC_PRIMS);
                pop = pend < 0;
            } else if (WIDTH == 4) {
                // the top of the tree comes from LDS, the rest from global memory
                const Node4Q q = (ref & RT_HOT_BIT) ? lds_hot[ref & ~RT_HOT_BIT] : Node4Q(nodes4[ref]);
                wide_visit<STACK>(q, id, S.o * id, b.t, ref, sp, stk, pop);
                if (STATS) cnt.nodes++;
            } else {
                const NodeF n = nodes[ref];
                if (STATS) cnt.nodes++;
                float tl, tr;
                const V3 oi = S.o * id;
                const bool hl = slab(n.lmin, n.lmax, oi, id, b.t, tl);
                const bool hr = slab(n.rmin, n.rmax, oi, id, b.t, tr);
                const int cl = __float_as_int(n.lmin.w), cr = __float_as_int(n.rmin.w);
                if (hl && hr) {
                    const bool lf = tl <= tr;
                    push<STACK>(stk, sp, lf ? cr : cl);
                    ref = lf ? cl : cr;
                    pop = false;
                } else if (hl | hr) {
                    ref = hl ? cl : cr;
                    pop = false;
                }
            }
            if (pop) {
                if (sp > 0) {
                    ref = pop_ref<STACK>(stk, sp);
                } else {
                    trav = false;
                    done = true;
                }
            }
            if (trav && ref < 0 && pend < 0) pend = ~ref; // entering a leaf
        }
#endif
        if (STATS) {
            cnt.iters++;
            if (trav) cnt.q_steps++;
            if (done) {
                cnt.max_steps = max(cnt.max_steps, cnt.q_steps);
                cnt.q_steps = 0;
            }
        }
    }
    flush_counts<STATS>(wave_rays, cnt, P0, lane);
}

#ifndef __HIPCC_RTC__ // the host side and the other kernels (not part of a hiprtc build)
// Trace-only kernel (rt_debug_trace_rays): the wide BVH kernel's speculative traversal over a
// list of logged queries, with no shading phase and no path state, so that each lane takes the
// next ray as soon as its query ends.  It measures the traversal stage of a wavefront split
// (Laine, Karras & Aila 2013) against the megakernel on the same rays.
template <int STACK, int WAVES, bool STATS>
__global__ void __launch_bounds__(256, WAVES) trace_rays_kernel(TraceRaysParams p)
{
    __shared__ int stack_mem[STACK * 256];
    const TravStack stk = make_stack(stack_mem, p.stack_ovf);
    const int lane = threadIdx.x & 63;
    const RT_AS_CONST TestRec* tests = (const RT_AS_CONST TestRec*)p.tests;
    const RT_AS_CONST float4* rows = (const RT_AS_CONST float4*)p.rows;
    const RT_AS_CONST Node4Q* nodes4 = (const RT_AS_CONST Node4Q*)p.nodes4;
    const RT_AS_CONST XformF* xf = (const RT_AS_CONST XformF*)p.xf;
    bool trav = false, more = false, exhausted = false;
    int ref = 0, sp = 0, pend = -1, prev = -1;
    unsigned n_tri = 0, n_sph = 0;
    unsigned idx = 0, pool_next = 0, pool_end = 0; // the wave's pool of ray indices (uniform)
    V3 o{0, 0, 0}, d{0, 0, 0}, id{0, 0, 0}, oi{0, 0, 0};
    Best b{__builtin_huge_valf(), -1};
    unsigned long long n_node = 0, n_leaf = 0, n_slots = 0;
    while (true) {
        const bool need = !trav && !exhausted;
        const unsigned long long m = __ballot(need);
        if (m) { // lanes without a query take the next rays (one atomic per 256 rays per wave)
            const unsigned kk = (unsigned)__popcll(m), avail = pool_end - pool_next;
            unsigned fresh = 0;
            if (kk > avail) {
                if (lane == 0) fresh = atomicAdd(p.counter, 256u);
                fresh = __builtin_amdgcn_readfirstlane(fresh);
            }
            if (need) {
                const unsigned r = (unsigned)__popcll(m & ((1ull << lane) - 1ull));
                idx = r < avail ? pool_next + r : fresh + (r - avail);
                if (idx >= p.n) {
                    exhausted = true;
                } else {
                    const float4 r0 = p.rays[3 * (size_t)idx], r1 = p.rays[3 * (size_t)idx + 1];
                    o = v3(r0.x, r0.y, r0.z);
                    d = v3(r1.x, r1.y, r1.z);
                    prev = __float_as_int(r0.w);
                    id = v3(slab_rcp(d.x), slab_rcp(d.y), slab_rcp(d.z));
                    oi = o * id;
                    ref = p.root4;
                    sp = 0;
                    pend = -1;
                    more = true;
                    if (ref < 0) {
                        pend = ~ref;
                        more = false;
                    }
                    b = Best{__builtin_huge_valf(), -1};
                    trav = true;
                }
            }
            if (kk > avail) {
                pool_next = fresh + (kk - avail);
                pool_end = fresh + 256u;
            } else {
                pool_next += kk;
            }
        }
        if (!__any(trav)) break;
        const bool can_node = trav && more && ref >= 0;
        const bool blocked = trav && pend >= 0 && !can_node;
        const bool leaf_step = __ballot(can_node) == 0 || __popcll(__ballot(blocked)) >= p.spec;
        if (STATS) {
            n_slots += 64;
            if (leaf_step) n_leaf += (trav && pend >= 0) ? 1 : 0;
            else n_node += can_node ? 1 : 0;
        }
        if (trav) {
            if (leaf_step) {
                if (pend >= 0) {
                    test_leaf<false>(tests, rows, xf, pend, o, d, prev, b, n_tri, n_sph);
                    pend = leaf_advance(pend, RT_SPEC_PRIMS);
                }
            } else if (can_node) {
                bool pop = true;
                const Node4Q q = nodes4[ref];
                wide_visit<STACK>(q, id, oi, b.t, ref, sp, stk, pop);
                if (pop) {
                    if (sp > 0) ref = pop_ref<STACK>(stk, sp);
                    else more = false;
                }
            }
            if (more && ref < 0 && pend < 0) {
                pend = ~ref;
                if (sp > 0) ref = pop_ref<STACK>(stk, sp);
                else more = false;
            }
            if (!more && pend < 0) {
                trav = false;
                if (p.outer)
                    test_outer<false>((const RT_AS_CONST GroupRec*)p.outer, (const RT_AS_CONST RectRec*)p.outer_rects,
                                      (const RT_AS_CONST BoxRec*)p.outer_boxes, o, d, prev, b, n_tri);
                p.hits[idx] = make_float2(b.t, __int_as_float(b.sg));
            }
        }
    }
    if (STATS) {
        for (int off = 32; off > 0; off >>= 1) {
            n_node += __shfl_down(n_node, off);
            n_leaf += __shfl_down(n_leaf, off);
        }
        if (lane == 0) {
            atomicAdd(p.stats + 0, n_node);
            atomicAdd(p.stats + 1, n_leaf);
            atomicAdd(p.stats + 2, n_slots);
        }
    }
}

// plane: element stride between the R, G and B planes of sum (>= w*h; a gather slot may be taller
// than the band set written into it)
__global__ void accumulate_kernel(PathParams p, double* sum, uint32_t* samples, uint32_t* misses, size_t plane)
{
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= p.w || y >= p.h) return;
    const size_t blk = (size_t)((y >> 3) * p.blocks_x + (x >> 3));
    const int q = (y & 7) * 8 + (x & 7);
    const size_t i = (size_t)y * p.w + x;
    double r = sum[i], g = sum[plane + i], bl = sum[2 * plane + i];
    uint32_t ns = 0, nm = 0;
    const int used = (p.spp + p.chunk - 1) / p.chunk; // chunks past spp hold no partial
    for (int c = 0; c < used; c++) {
        const float4 v = p.partial[(((blk << p.log2_chunks) + c) << 6) + q];
        r += v.x;
        g += v.y;
        bl += v.z;
        const uint32_t k = __float_as_uint(v.w);
        ns += k & 0xFFFFu;
        nm += k >> 16;
    }
    sum[i] = r;
    sum[plane + i] = g;
    sum[2 * plane + i] = bl;
    samples[i] += ns;
    misses[i] += nm;
}

// SampleSet.GetOutput / GetColorCode (SampleSet.cs:50-113) per pixel of planar accumulators.
__device__ __forceinline__ uint32_t color_code(double r, double g, double b, double a)
{
    auto q = [](double v) { // Util.Clamp to [0, 1], then (int)(v * 255)
        v = v > 0.0 ? v : 0.0;
        v = v < 1.0 ? v : 1.0;
        return (uint32_t)(int32_t)(v * 255);
    };
    return (q(a) << 24) | (q(r) << 16) | (q(g) << 8) | q(b);
}

__global__ void tonemap_kernel(int w, int h, const double* __restrict__ sum, const uint32_t* __restrict__ samples,
                               const uint32_t* __restrict__ misses, double br, double bg, double bb, double back_alpha,
                               double exposure, int32_t* __restrict__ argb)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = w * h;
    if (i >= n) return;
    const uint32_t ns = samples[i], nm = misses[i];
    if (ns == 0) {
        argb[i] = (int32_t)color_code(br * exposure, bg * exposure, bb * exposure, back_alpha);
        return;
    }
    const double total = (double)ns + (double)nm;
    const double mult = exposure / ns;
    double r = sum[i] * mult, g = sum[n + i] * mult, b = sum[2 * (size_t)n + i] * mult, a = 1;
    const double bam = nm / total, bk = bam * back_alpha;
    r += (br - r) * bk;
    g += (bg - g) * bk;
    b += (bb - b) * bk;
    a += (back_alpha - a) * bam;
    const double gamma = 1 / 2.2;
    argb[i] = (int32_t)color_code(pow(r, gamma), pow(g, gamma), pow(b, gamma), a);
}

// One pass of Raytracer.Render (1 spp): DoubleColor[w, h] with Placeholder (-1) on a primary miss,
// in the caller's order x * h + y, as fp32 -- a sample's colour is fp32 in the kernel, so the host
// widens it to double exactly, and the PCIe copy is 12 B per pixel instead of 24.
__global__ void colors_1spp_kernel(PathParams p, float* __restrict__ out)
{
    const size_t npix = (size_t)p.w * p.h;
    const size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= npix) return;
    const int x = (int)(o / (size_t)p.h), y = (int)(o - (size_t)x * p.h);
    const int q = ((y >> 3) * p.blocks_x + (x >> 3)) * 64 + (y & 7) * 8 + (x & 7); // 1 spp: one chunk
    const float4 v = p.partial[q];
    const bool miss = (__float_as_uint(v.w) & 0xFFFFu) == 0;
    out[3 * o + 0] = miss ? -1.0f : v.x;
    out[3 * o + 1] = miss ? -1.0f : v.y;
    out[3 * o + 2] = miss ? -1.0f : v.z;
}

// Planar row-major tile accumulators -> the caller's SampleSet order (C# [x, y]: x * h + y), one
// 32-B record per pixel (DoubleColor, samples, misses), so that the host-buffer entry point copies
// one contiguous image in chunks and adds each chunk sequentially as it lands.
__global__ void tile_host_layout_kernel(int w, int h, const double* __restrict__ sum, const uint32_t* __restrict__ ns,
                                        const uint32_t* __restrict__ ms, TileRec* __restrict__ out)
{
    const size_t npix = (size_t)w * h;
    const size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= npix) return;
    const size_t x = o / (size_t)h, y = o - x * (size_t)h;
    const size_t i = y * (size_t)w + x;
    TileRec r;
    r.r = sum[i];
    r.g = sum[npix + i];
    r.b = sum[2 * npix + i];
    r.samples = ns[i];
    r.misses = ms[i];
    out[o] = r;
}

// ---- compact leaves (rt_internal.h): 48-B rows and homogeneous leaf references --------------
__global__ void rows_kernel(const TestRec* __restrict__ tests, int n, float4* __restrict__ rows)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const TestRec t = tests[i];
    rows[3 * (size_t)i] = t.r0;
    rows[3 * (size_t)i + 1] = t.r1;
    rows[3 * (size_t)i + 2] = t.r2;
}

// A generic leaf whose primitives (at most 4, all of them at slots below 2^23) share their kind
// (triangle or sphere) and test flags becomes a compact leaf; any other reference is returned
// unchanged.  (A leaf reaching past slot 2^23 stays generic: leaf_advance adds to the first-slot
// field, whose carry would run into the flag bits.)
__device__ int compact_ref(int ref, const TestRec* __restrict__ tests)
{
    if (ref >= 0 || ref == RT_NODE4_EMPTY) return ref;
    const int code = ~ref;
    if (code & kLeafCompact) return ref;
    const int first = code >> 3, count = (code & 7) + 1;
    if (count > 4 || first + count > kLeafCompactMaxFirst) return ref;
    uint32_t key = 0;
    for (int j = 0; j < count; j++) {
        const uint32_t fl = __float_as_uint(tests[first + j].meta.y), kind = fl & KIND_MASK;
        if (kind != RT_PRIM_TRIANGLE && kind != RT_PRIM_SPHERE) return ref;
        const uint32_t lf = (kind == RT_PRIM_SPHERE ? 1u : 0u) | ((fl >> 1) & 0xEu) | ((fl >> 2) & 0x10u);
        if (j > 0 && lf != key) return ref;
        key = lf;
    }
    return ~(kLeafCompact | (int)(key << 25) | (first << 2) | (count - 1));
}

__global__ void compact_nodes_kernel(NodeF* __restrict__ n2, int n_n2, Node4Q* __restrict__ n4, int n_n4,
                                     const TestRec* __restrict__ tests)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_n2) {
        NodeF& n = n2[i];
        n.lmin.w = __int_as_float(compact_ref(__float_as_int(n.lmin.w), tests));
        n.rmin.w = __int_as_float(compact_ref(__float_as_int(n.rmin.w), tests));
    }
    if (i < n_n4) {
        Node4Q& q = n4[i];
        q.c.z = __int_as_float(compact_ref(__float_as_int(q.c.z), tests));
        q.c.w = __int_as_float(compact_ref(__float_as_int(q.c.w), tests));
        q.d.x = __int_as_float(compact_ref(__float_as_int(q.d.x), tests));
        q.d.y = __int_as_float(compact_ref(__float_as_int(q.d.y), tests));
    }
}

using PathKernel = void (*)(PathScene, const CameraF*, const PathParams*, const TestRec*, const RectRec*, const FrameRec*, const PrimF*,
                            const NodeF*, const Node4Q*, const GroupRec*, const XformF*, const MatF*, const float4*);

// vn: the scene has vertex-normal triangles (their re-hit test, vn_rehit_test, is fp64 code that
// costs the other scenes' kernels registers, so it is compiled only into separate instances)
template <bool CULL, bool LDS>
PathKernel pick_brute(bool stats, bool vn)
{
    if (vn) return stats ? path_kernel<CULL, LDS, true, true> : path_kernel<CULL, LDS, false, true>;
    return stats ? path_kernel<CULL, LDS, true, false> : path_kernel<CULL, LDS, false, false>;
}
template <int WIDTH, int STACK, bool LDS>
PathKernel pick_bvh(bool stats, bool vn)
{
    if (vn) return stats ? path_kernel_bvh<WIDTH, STACK, LDS, true, true> : path_kernel_bvh<WIDTH, STACK, LDS, false, true>;
    return stats ? path_kernel_bvh<WIDTH, STACK, LDS, true, false> : path_kernel_bvh<WIDTH, STACK, LDS, false, false>;
}

// variant = kernel * 2 + lds; kernel 0 brute force (flat), 1 brute force (grouped, culled),
// 2 BVH2 (24-entry LDS stack), 3 wide BVH (RT_WIDE_STACK-entry LDS stack); both overflow to global memory
PathKernel pick(int variant, bool stats, bool vn)
{
    switch (variant) {
    case 1: return pick_brute<false, true>(stats, vn);
    case 2: return pick_brute<true, false>(stats, vn);
    case 3: return pick_brute<true, true>(stats, vn);
    case 4: return pick_bvh<2, 24, false>(stats, vn);
    case 5: return pick_bvh<2, 24, true>(stats, vn);
    case 6: return pick_bvh<4, RT_WIDE_STACK, false>(stats, vn);
    case 7: return pick_bvh<4, RT_WIDE_STACK, true>(stats, vn);
    default: return pick_brute<false, false>(stats, vn);
    }
}

PathScene make_path_scene(const DevScene& s)
{
    PathScene ps;
    for (int k = 0; k < 3; k++) ps.n_rect[k] = s.n_rect[k];
    ps.n_tri = s.n_tri;
    ps.n_sph = s.n_sph;
    ps.n_pln = s.n_pln;
    ps.n_bvh = s.pln0_bf; // set per order by launch_path
    ps.n_slots = ps.n_bvh + s.n_pln;
    ps.n_mats = s.n_mats;
    ps.n_xf = s.n_xf;
    ps.n_vn = s.n_vn;
    ps.facts = s.facts;
    ps.root = s.root;
    ps.width = s.width;
    ps.recursion = s.recursion;
    ps.debug_geom = s.debug_geom;
    ps.ambient_miss = s.ambient_miss;
    ps.air_ior = s.air_ior;
    ps.ambient_r = s.ambient.x;
    ps.ambient_g = s.ambient.y;
    ps.ambient_b = s.ambient.z;
    return ps;
}

#endif // __HIPCC_RTC__
} // namespace

#ifndef __HIPCC_RTC__
int path_wide_stack() { return RT_WIDE_STACK; }

int debug_vn_rehit(const double v0[3], const double e01[3], const double e02[3], int mirror, double u, double v,
                   const float dir[3], int* inside, double* t, double o[3])
{
    PrimD P{};
    P.a = Vec4d{v0[0], v0[1], v0[2], 1.0};
    P.b = Vec4d{e01[0], e01[1], e01[2], 0.0};
    P.c = Vec4d{e02[0], e02[1], e02[2], 0.0};
    P.flags = mirror ? F_MIRROR : 0u;
    bool in = false;
    const bool hit = vn_rehit_test(P, u, v, V3{dir[0], dir[1], dir[2]}, in, t, o);
    *inside = in ? 1 : 0;
    return hit ? 1 : 0;
}

size_t path_lds_bytes(const DevScene& s)
{
    const size_t slots = (size_t)std::max(std::max(s.pln0_bf, s.pln0_gr), s.pln0_bvh) + s.n_pln;
    return slots * sizeof(PrimF) + (size_t)s.n_mats * sizeof(MatF) + (size_t)s.n_xf * sizeof(XformF);
}

int path_variant(int kernel, bool lds) { return kernel * 2 + (lds ? 1 : 0); }

bool hot_nodes_enabled()
{
    static const bool on = !(getenv("RTCORE_HOT_NODES") && getenv("RTCORE_HOT_NODES")[0] == '0'); // A/B switch
    return on;
}

size_t path_dyn_lds(const DevScene& s, int variant)
{
    size_t b = (variant & 1) ? path_lds_bytes(s) : 0;
    if ((variant >> 1) == 3 && s.n_hot4 > 0 && hot_nodes_enabled()) b += (size_t)s.n_hot4 * sizeof(Node4Q);
    return b;
}

int path_blocks_per_cu(int variant, size_t dyn_lds, bool stats, bool vn)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(pick(variant, stats, vn)), 256,
                                                     dyn_lds) != hipSuccess ||
        n < 1)
        n = 1;
    return n;
}

void fill_launch(const DevScene& s, int variant, PathParams& p)
{
    PathScene ps = make_path_scene(s);
    const int kernel = variant >> 1;
    ps.hot4 = nullptr;
    ps.n_hot4 = 0;
    if (kernel == 3) { // the wide kernel walks the collapsed tree, its top from the hot table
        ps.root = s.root4;
        if (s.n_hot4 > 0 && hot_nodes_enabled()) {
            ps.root = s.root4_hot;
            ps.hot4 = s.hot4;
            ps.n_hot4 = s.n_hot4;
        }
    }
    const bool grouped = kernel == 1, bvh = kernel >= 2;
    ps.n_groups = grouped ? s.n_groups_gr : bvh ? s.n_outer : 1;
    ps.n_bvh = bvh ? s.pln0_bvh : grouped ? s.pln0_gr : s.pln0_bf;
    ps.n_slots = ps.n_bvh + s.n_pln;
    p.scene = ps;
    p.tests = bvh ? s.tests_bvh : grouped ? s.tests_gr : s.tests_bf;
    p.rows = bvh ? s.rows_bvh : nullptr;
    p.rects = bvh ? s.rects_bvh : grouped ? s.rects_gr : s.rects_bf;
    p.frames = bvh ? s.frames_bvh : grouped ? s.frames_gr : s.frames_bf;
    p.prims = bvh ? s.prims_bvh : grouped ? s.prims_gr : s.prims_bf;
    p.groups = bvh ? s.groups_bvh : grouped ? s.groups_gr : s.groups_bf;
    p.nodes = s.nodes;
    p.nodes4 = s.nodes4;
    p.xf = s.xf;
    p.mats = s.mats;
    p.vnormals = s.vnormals;
    p.prims_d = s.prims_d;
}

hipError_t launch_path(const DevScene& s, const CameraF* d_cam, const PathParams* d_params, int variant,
                       int grid_blocks, hipStream_t stream, bool stats)
{
    PathParams h{}; // the same launch record as the device copy: the BVH kernels take it as arguments
    fill_launch(s, variant, h);
    PathScene ps = h.scene;
    const CameraF* ca = d_cam;
    const PathParams* pa = d_params;
    const TestRec* tests = h.tests;
    const RectRec* rects = h.rects;
    const FrameRec* frames = h.frames;
    const PrimF* prims = h.prims;
    const NodeF* nodes = s.nodes;
    const Node4Q* nodes4 = s.nodes4;
    const GroupRec* groups = h.groups;
    const XformF* xf = h.xf;
    const MatF* mats = h.mats;
    const float4* vn = h.vnormals;
    void* args[] = {&ps, &ca, &pa, &tests, &rects, &frames, &prims, &nodes, &nodes4, &groups, &xf, &mats, &vn};
    const size_t dyn = path_dyn_lds(s, variant);
    return hipLaunchKernel(reinterpret_cast<const void*>(pick(variant, stats, s.n_vn > 0)), dim3(grid_blocks), dim3(256), args, dyn,
                           stream);
}

hipError_t launch_accumulate(const PathParams& p, double* d_sum, uint32_t* d_samples, uint32_t* d_misses, hipStream_t stream,
                             size_t plane)
{
    if (plane == 0) plane = (size_t)p.w * p.h;
    dim3 grid((p.w + 15) / 16, (p.h + 15) / 16);
    hipLaunchKernelGGL(accumulate_kernel, grid, dim3(256), 0, stream, p, d_sum, d_samples, d_misses, plane);
    return hipGetLastError();
}

hipError_t launch_tonemap(int w, int h, const double* d_sum, const uint32_t* d_samples, const uint32_t* d_misses,
                          rt_color back, double back_alpha, double exposure, int32_t* d_argb, hipStream_t stream)
{
    const int n = w * h;
    hipLaunchKernelGGL(tonemap_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, w, h, d_sum, d_samples, d_misses,
                       back.r, back.g, back.b, back_alpha, exposure, d_argb);
    return hipGetLastError();
}

hipError_t launch_tile_host_layout(int w, int h, const double* d_sum, const uint32_t* d_samples,
                                  const uint32_t* d_misses, TileRec* d_out, hipStream_t stream)
{
    const size_t npix = (size_t)w * h;
    if (npix == 0) return hipSuccess;
    hipLaunchKernelGGL(tile_host_layout_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, stream, w, h, d_sum,
                       d_samples, d_misses, d_out);
    return hipGetLastError();
}

using TraceKernel = void (*)(TraceRaysParams);
TraceKernel pick_trace(int waves, bool stats)
{
    if (waves >= 8) return stats ? trace_rays_kernel<16, 8, true> : trace_rays_kernel<16, 8, false>;
    if (waves == 7) return stats ? trace_rays_kernel<16, 7, true> : trace_rays_kernel<16, 7, false>;
    return stats ? trace_rays_kernel<20, 6, true> : trace_rays_kernel<20, 6, false>;
}

int trace_rays_blocks_per_cu(int waves)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(pick_trace(waves, false)), 256, 0) !=
            hipSuccess ||
        n < 1)
        n = 1;
    return n;
}

hipError_t launch_trace_rays(const TraceRaysParams& p, int waves, int grid_blocks, hipStream_t stream)
{
    hipLaunchKernelGGL(pick_trace(waves, p.stats != nullptr), dim3(grid_blocks), dim3(256), 0, stream, p);
    return hipGetLastError();
}

hipError_t compact_leaves(const TestRec* d_tests, int n_records, float4* d_rows, NodeF* d_nodes, int n_nodes,
                          Node4Q* d_nodes4, int n_nodes4, bool rewrite, hipStream_t stream)
{
    if (n_records > 0)
        hipLaunchKernelGGL(rows_kernel, dim3((n_records + 255) / 256), dim3(256), 0, stream, d_tests, n_records, d_rows);
    const int n = std::max(n_nodes, n_nodes4);
    if (rewrite && n > 0)
        hipLaunchKernelGGL(compact_nodes_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_nodes, n_nodes, d_nodes4,
                           n_nodes4, d_tests);
    return hipGetLastError();
}

__global__ void pixel_keys_kernel(rt_key2 seed_key, int w, int h, rt_key2* __restrict__ out)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)w * (size_t)h) return;
    out[i] = rt_rng_pixel_key(seed_key, (unsigned long long)i);
}

hipError_t launch_pixel_keys(rt_key2 seed_key, int w, int h, rt_key2* out, hipStream_t stream)
{
    const size_t n = (size_t)w * (size_t)h;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(pixel_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, seed_key, w, h, out);
    return hipGetLastError();
}

hipError_t launch_colors_1spp(const PathParams& p, float* d_out, hipStream_t stream)
{
    const size_t npix = (size_t)p.w * p.h;
    if (npix == 0) return hipSuccess;
    hipLaunchKernelGGL(colors_1spp_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, stream, p, d_out);
    return hipGetLastError();
}

#endif // __HIPCC_RTC__
} // namespace rtc

#ifdef RT_SCENE_CONST
// The entry point of a scene-specialised build (rt_jit.cpp): RT_SCENE_CONST_GROUPED selects the
// grouped (culling) or the flat brute-force kernel; LDS staging of the shading records.
extern "C" __global__ void __launch_bounds__(256, RT_SCENE_CONST_GROUPED ? RT_GROUPED_WAVES : RT_PATH_WAVES)
    rt_path_const(const rtc::CameraF* __restrict__ camp, const rtc::PathParams* __restrict__ pp)
{
    rtc::path_body<RT_SCENE_CONST_GROUPED != 0, true, false, RT_SCENE_CONST_VN != 0>(camp, pp);
}
#endif
