// rt_internal.h -- internal data layout of the MI355X path-tracing core.
//
// Two device representations of one scene are built on the host:
//   * the EXACT fp64 set (PrimD + RefNode): the reference's own agglomerative BVH
//     (Acceleration/BVH.cs:193-236) flattened in depth-first order, used by the
//     DebugRaycaster-equivalent primary-ID kernel that must match the reference's
//     closest-hit query bit for bit (Scene.cs:65-111);
//   * the FAST fp32 set (PrimF + NodeF): a binned-SAH BVH2 whose nodes carry both child
//     boxes (one 64-B line per visit), used by the persistent path-tracing kernel.
#pragma once
#ifndef __HIPCC_RTC__ // hiprtc (the scene-specialised kernels, rt_jit.cpp) provides these itself
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "../../include/rtcore.h"

namespace rtc {

// ---- flags packed into PrimF / PrimD -------------------------------------------------
enum : uint32_t {
    KIND_MASK = 3u,     // rt_prim_kind in bits 0-1
    F_MIRROR = 1u << 2,
    F_TWOSIDED = 1u << 3,
    F_INVERT = 1u << 4,
    F_HASNORMALS = 1u << 5,
    F_TRANSFORMED = 1u << 6,
    F_AXIS_SHIFT = 7,   // axis-aligned rectangle: (axis + 1) in bits 7-8, 0 = general
    F_AXIS_MASK = 3u << 7,
    F_FRAME_RECT = 1u << 9, // brute-force slot tested as a rectangle of a FrameRec (shading: Inside from N . d)
};

// Scene facts (PathScene.facts): what the scene's primitives and materials use at all.  In a
// scene-specialised build they are constants, so the shading code of features the scene does not
// use (Fresnel, infinite shininess, ellipsoid and vertex normals, sphere normals) folds away.
enum : uint32_t {
    FACT_INF_SHININESS = 1u << 0, // some material has Shininess = +inf (RandomShine draws no z)
    FACT_IOR = 1u << 1,           // some material has a RefractiveIndex (Fresnel / TIR)
    FACT_XF = 1u << 2,            // a transformed sphere (ellipsoid normal)
    FACT_SPHERE = 1u << 3,        // some sphere
    FACT_VN = 1u << 4,            // a vertex-normal triangle (smooth normal, GetNormal's NaN quirk)
    FACT_ALL = 0x1Fu,
};

// Axis-aligned rectangle (a Mirror parallelogram whose edges follow two coordinate axes, e.g.
// every Cube face, Cube.cs:90-116): the plane coordinate on `axis`, the extents on the two
// other axes (in x, y, z order) and the one-sided culling rule folded into one factor:
// a hit is kept iff cull * d[axis] <= 0 (0 = two-sided; Primitive.cs:56-61).
struct alignas(16) RectRec {
    float m1, m2;   // mid-points on the first and second remaining axes (one aligned SGPR pair:
    float h1, h2;   // the in-plane test is one packed subtract), half-widths likewise
    float c;        // plane coordinate
    float cull;     // 0 two-sided, else +-1: sign(N[axis]), negated for Invert
    int32_t id;     // primitive ID
    int32_t sg;     // slot << 1 (the Best.sg of a hit)
};

// Parallelograms whose edges follow the axes of one common affine frame (the six faces of a
// transformed `cube`, Cube.cs:90-116, whose vertices the loader bakes into world space,
// Triangle.cs:68-74) are tested as axis-aligned rectangles in that frame: the ray is mapped
// once per frame (rows r0..r2: world -> local, t is unchanged by an affine map), then each face
// is a RectRec in local coordinates.  The rects of frame f are rects[rect_first ..) in local
// axis order x | y | z.
struct alignas(16) FrameRec {
    float4 r0, r1, r2;          // local = (r_k . p + r_k.w)
    int32_t rect_first;
    int16_t n_rect[3];
    int16_t box;                // index of the frame's BoxRec in the same array, or -1
};

// Six rectangles that close an axis-aligned box (in world space, or in a frame) are tested
// together by one slab test: the candidates are the face the ray enters by and the face it
// leaves by, each kept under its face's culling rule and self-hit rule, entry first (a convex
// box is met at most twice).  Faces f = 2 axis + side (side 0 = the lower plane) occupy slots
// sg0 / 2 + f (the kernels name a face by that slot); their primitive IDs are id0 + (perm >> 4 f & 15)
// (kept for inspection).  Stored in the FrameRec array
// (same 64-B size) so that the kernel needs no further argument.
struct alignas(16) BoxRec {
    float4 lo;                  // xyz: lower planes, w = bitcast id0
    float4 hi;                  // xyz: upper planes, w = bitcast perm
    uint32_t keep;              // bit f: face f kept as an entry hit, bit 8 + f: as an exit hit
    int32_t sg0;                // slot of face 0, << 1
    int32_t pad[6];
};
static_assert(sizeof(BoxRec) == sizeof(FrameRec), "boxes share the frame array");

// ---- exact fp64 scene (primary-ID pass) -----------------------------------------------
struct alignas(16) Vec4d {
    double x, y, z, w;
};

struct alignas(16) PrimD {      // 256 B
    Vec4d a, b, c, d;           // tri: v0, e01, e02, N | sphere: center, (r, r^2) | plane: N, (dist)
    Vec4d vn[3];                // triangle vertex normals (HasNormals)
    uint32_t flags;
    int32_t xf;                 // index into XformD for transformed spheres, else -1
    int32_t pad[6];
};

struct alignas(16) XformD {     // MatrixToWorld, MatrixToObject, MatrixToNormal (row-major)
    double to_world[16];
    double to_obj[16];
    double to_normal[16];
};

struct alignas(16) RefNode {    // 80 B, depth-first pre-order; left child = this + 1
    Vec4d mn, mx;
    int32_t right;              // index of the right child (internal) or -1
    int32_t prim;               // leaf: primitive index, internal: -1
    int32_t skip;               // BVH<T>.SkipVolume (BVH.cs:44-48)
    int32_t pad;
};

// ---- fast fp32 scene (path tracing) --------------------------------------------------
struct alignas(16) PrimF {      // 64 B
    float4 a; // tri: v0.xyz, id | sphere: c.xyz, id | plane: N.xyz, id
    float4 b; // tri: e01.xyz, flags | sphere: (r, 1/r, xf, flags) | plane: (dist, 0, 0, flags)
    float4 c; // the brute-force kernels' shading row: one-hot plane axis of an axis-aligned rectangle
              // slot (xyz), 1/r of an untransformed sphere (w); 0 otherwise
    float4 d; // tri and plane: N.xyz | untransformed sphere: -centre / r; w: material index
};

struct alignas(16) XformF {     // rows 0-2 (last row is 0 0 0 1)
    float4 to_world[3];         // Sphere.MatrixToWorld: world -> object space (the reference's names)
    float4 normal[3];           // world hit point -> unnormalised world normal: the affine composite
                                // MatrixToNormal * (MatrixToWorld * p - centre) / r (Sphere.cs:50-155)
};

struct alignas(16) MatF {       // one per distinct material (PrimF.d.w indexes it), 80 B
    float4 emission;            // rgb, luminance
    float4 diffuse;             // rgb, luminance
    float4 specular;            // rgb (Shininess<=0 -> black), luminance
    float4 refraction;          // rgb (Shininess<=0 -> black), luminance
    float shininess;            // may be +inf
    float ior;                  // RefractiveIndex
    uint32_t flags;
    float inv_shininess;        // 1 / Shininess (RandomShine's exponent)
    float eta_enter, eta_exit;  // AirRefractiveIndex / RefractiveIndex and its inverse (0 when no IOR)
    float pad[2];
};

// A group of the brute-force slot order (64 B): its primitives' box (fp32, rounded outward) and
// typed ranges -- world rects (x | y | z) in RectRec order from rect_first, then n_frames
// FrameRecs and n_boxes world BoxRecs from frame_first (the frames' rects follow the world rects),
// then triangles and spheres in slot order from tri_slot.  The grouped kernel skips a group when no lane of the wave meets its
// box; the flat order is one group whose box is never tested.
struct alignas(16) GroupRec {
    float4 lo;     // xyz, w = bitcast rect_first
    float4 hi;     // xyz, w = bitcast tri_slot
    int32_t n_rect[3];
    int32_t n_tri_sph; // n_tri | n_sph << 16
    int32_t frame_first;
    int16_t n_frames, n_boxes; // FrameRecs, then world BoxRecs, from frame_first
    int32_t n_flat_extra;      // faces tested through frames and boxes (statistics)
    int32_t skip;              // super record (no primitives): the records after it that its box
                               // holds, skipped with it; 0 for a group of primitives
};

// Intersection record of the fp32 kernel (64 B), one per primitive slot:
//   triangle: rows r0..r2 of the affine inverse of [e01 e02 n | v0], so that
//             (u, v, w) = M (p, 1): w = 0 on the plane, (u, v) = the barycentrics the
//             reference's Moller-Trumbore test computes (Triangle.cs:77-146)
//   sphere:   r0 = (centre, radius), r1 = (radius^2, bitcast xf index, 0, 0)
//   plane:    r0 = (normal, origin distance)
//   meta = (bitcast primitive ID, bitcast flags, 0, 0)
struct alignas(16) TestRec {
    float4 r0, r1, r2, meta;
};

struct Node4Q;

// Scalar fields of the path kernel (pointers are passed as separate __restrict__ arguments
// so that the wave-uniform primitive loop is served by scalar loads).
struct PathScene {
    // brute-force slot order: x-rects | y-rects | z-rects | triangles | spheres | planes
    int32_t n_rect[3];
    int32_t n_tri, n_sph, n_pln;
    int32_t n_bvh;               // primitives in the BVH (all but planes); planes follow them
    int32_t n_slots;             // n_bvh + n_pln (PrimF records)
    int32_t n_mats;              // MatF records (distinct materials)
    int32_t n_xf;                // XformF records
    int32_t n_vn;                // triangles with vertex normals (Triangle.HasNormals); 0 removes their path
    uint32_t facts;              // FACT_* of the scene
    int32_t n_groups;            // brute force: GroupRec records; BVH kernels: outer groups (0 or 1)
    int32_t root;                // child reference of the BVH root
    const Node4Q* hot4;          // wide kernel: the top nodes, staged in LDS (child refs | RT_HOT_BIT)
    int32_t n_hot4;
    int32_t width;               // frame width (RNG pixel index)
    int32_t recursion;
    int32_t debug_geom;
    int32_t ambient_miss;
    float air_ior;
    float ambient_r, ambient_g, ambient_b;
};

// Child reference in a NodeF: >= 0 internal node index, < 0 leaf = ~code, where code is
//   generic leaf: first << 3 | (count - 1)            (first < 2^27; 64-B TestRecs, kind and flags per record)
//   compact leaf: kLeafCompact | lf << 25 | first << 2 | (count - 1)   (count <= 4, first < 2^23)
// A compact leaf's primitives share their kind and test flags, held in the reference (lf: bit 0 sphere,
// bit 1 Mirror, 2 TwoSided, 3 Invert, 4 transformed), so the leaf step reads only their 48-B rows
// (the TestRec without its meta row: 3 vector loads per primitive instead of 4).  The builders emit
// generic leaves; compact_leaves (kernels_path.hip) rewrites every homogeneous one after the upload.
constexpr int kLeafCompact = 1 << 30;
constexpr int kLeafCompactMaxFirst = 1 << 23;
constexpr int kLeafGenericMaxSlots = 1 << 27; // slots a generic leaf code can address (rt_scene_create refuses more)
__host__ __device__ inline void leaf_range(int ref, int& first, int& count)
{
    const int code = ~ref;
    const bool compact = (code & kLeafCompact) != 0;
    first = compact ? (code >> 2) & (kLeafCompactMaxFirst - 1) : code >> 3;
    count = (code & (compact ? 3 : 7)) + 1;
}
// the record flags (KIND_MASK | F_MIRROR | F_TWOSIDED | F_INVERT | F_TRANSFORMED) of a compact leaf
__host__ __device__ inline uint32_t leaf_flags(uint32_t lf)
{
    return ((lf & 1u) ? 1u : 0u) /* RT_PRIM_SPHERE */ | ((lf & 0xEu) << 1) | ((lf & 0x10u) << 2);
}
struct alignas(16) NodeF {      // 64 B: both children's boxes
    float4 lmin; // xyz, w = bitcast int left child
    float4 lmax; // xyz, w unused
    float4 rmin; // xyz, w = bitcast int right child
    float4 rmax;
};

// 4-wide BVH node with 8-bit quantised child boxes (64 B, one visit = one record):
//   a = (origin.xyz, exponents: (e_x + 128) | (e_y + 128) << 8 | (e_z + 128) << 16)
//   b = (qlo_x, qhi_x, qlo_y, qhi_y), c = (qlo_z, qhi_z, child0, child1), d = (child2, child3, n_children, 0)
// q* hold one byte per child (child k in bits 8k..8k+7): plane = origin + q * 2^e, rounded outward.
// Child references as in NodeF (>= 0 wide-node index, < 0 leaf code); unused slots are
// RT_NODE4_EMPTY with an inverted box.
#define RT_NODE4_EMPTY ((int32_t)0x80000000)
// A child reference with this bit set names a node of the hot table (the top of the wide tree in
// breadth-first order, copied into LDS by the wide kernel) instead of the global node array.
#define RT_HOT_BIT 0x40000000
struct alignas(16) Node4Q {
    float4 a, b, c, d;
};

__host__ __device__ inline float bits_f(uint32_t u)
{
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}

// Quantise up to four child boxes (fp32, lo/hi per axis) into a Node4Q.  Shared by the host
// collapse (bvh_sah.cpp) and the GPU builder (bvh_gpu.hip), in fp64: the exponent is the smallest
// e with origin + 255 * 2^e >= the node's upper plane in fp32, and each child plane is rounded
// outward until its fp32 dequantised value contains the child box.
__host__ __device__ inline Node4Q quantize_node4(const float lo[4][3], const float hi[4][3], const int refs_in[4],
                                                 int nc)
{
    float org[3];
    int ex[3];
    uint32_t qlo[3] = {0, 0, 0}, qhi[3] = {0, 0, 0};
    for (int a = 0; a < 3; a++) {
        float nlo = __builtin_huge_valf(), nhi = -__builtin_huge_valf();
        for (int k = 0; k < nc; k++) {
            nlo = lo[k][a] < nlo ? lo[k][a] : nlo;
            nhi = hi[k][a] > nhi ? hi[k][a] : nhi;
        }
        org[a] = nlo;
        const double ext = (double)nhi - (double)nlo;
        int e = ext > 0 ? (int)ceil(log2(ext / 255.0)) : -100;
        e = e > -100 ? e : -100;
        while ((double)(float)((double)org[a] + 255.0 * ldexp(1.0, e)) < (double)nhi) e++;
        ex[a] = e;
        const double sc = ldexp(1.0, e);
        for (int k = 0; k < 4; k++) {
            uint32_t lo8 = 255, hi8 = 0; // empty slot: inverted box
            if (k < nc) {
                double ql = floor(((double)lo[k][a] - (double)org[a]) / sc);
                double qh = ceil(((double)hi[k][a] - (double)org[a]) / sc);
                ql = ql < 0.0 ? 0.0 : (ql > 255.0 ? 255.0 : ql);
                qh = qh < 0.0 ? 0.0 : (qh > 255.0 ? 255.0 : qh);
                // the fp32 dequantised planes must contain the child box
                while (ql > 0 && (float)((double)org[a] + ql * sc) > lo[k][a]) ql -= 1;
                while (qh < 255 && (float)((double)org[a] + qh * sc) < hi[k][a]) qh += 1;
                lo8 = (uint32_t)ql;
                hi8 = (uint32_t)qh;
            }
            qlo[a] |= lo8 << (8 * k);
            qhi[a] |= hi8 << (8 * k);
        }
    }
    int refs[4] = {RT_NODE4_EMPTY, RT_NODE4_EMPTY, RT_NODE4_EMPTY, RT_NODE4_EMPTY};
    for (int k = 0; k < nc; k++) refs[k] = refs_in[k];
    const uint32_t exps = (uint32_t)(ex[0] + 128) | ((uint32_t)(ex[1] + 128) << 8) | ((uint32_t)(ex[2] + 128) << 16);
    Node4Q q;
    q.a = make_float4(org[0], org[1], org[2], bits_f(exps));
    q.b = make_float4(bits_f(qlo[0]), bits_f(qhi[0]), bits_f(qlo[1]), bits_f(qhi[1]));
    q.c = make_float4(bits_f(qlo[2]), bits_f(qhi[2]), bits_f((uint32_t)refs[0]), bits_f((uint32_t)refs[1]));
    q.d = make_float4(bits_f((uint32_t)refs[2]), bits_f((uint32_t)refs[3]), bits_f((uint32_t)nc), 0.0f);
    return q;
}

struct CameraF {                // post-InitRender state in fp32 (path kernel)
    float4 position, look, side, up;
    float w2, h2, tan_x, tan_y, h_mult, v_mult, image_plane, dof, focal_length;
    float tan_x_per_px, tan_y_per_px; // tan_x / w2, tan_y / h2 (frustum: ox = x * this - tan_x)
    int32_t kind;
};

struct CameraD {                // post-InitRender state in fp64 (exact kernel)
    Vec4d position, look, side, up;
    double w2, h2, tan_x, tan_y, h_mult, v_mult, image_plane, dof, focal_length;
    int32_t kind;
    int32_t pad;
};

// Everything the kernels need (device pointers + scene fields).
struct DevScene {
    // fast set; slot order is [triangles | spheres | planes] for brute force and
    // [BVH leaf order | planes] for the BVH, with matching TestRec / PrimF arrays
    const TestRec* tests_bf;
    const RectRec* rects_bf;    // world rects of the groups, then their frames' rects
    const FrameRec* frames_bf;
    const PrimF* prims_bf;
    const GroupRec* groups_bf;  // one group: the whole flat order
    // the grouped brute-force order (same records, group-major slot order)
    const TestRec* tests_gr;
    const RectRec* rects_gr;
    const FrameRec* frames_gr;
    const PrimF* prims_gr;
    const GroupRec* groups_gr;
    int32_t n_groups_gr;
    int32_t n_rect[3];
    int32_t n_tri, n_sph, n_pln; // flat-order slots: n_tri counts general triangles (frame rects included)
    int32_t pln0_bf, pln0_gr, pln0_bvh; // first plane slot of the flat, grouped and BVH orders
    const TestRec* tests_bvh;
    const float4* rows_bvh;     // the BVH order's TestRecs without the meta row (3 float4 per slot): compact leaves
    const PrimF* prims_bvh;
    // outer records of the BVH order (host builder, large scenes): one GroupRec of world rects and
    // closed boxes left out of the tree, tested when a query ends; n_outer = 0 or 1 groups
    const RectRec* rects_bvh;
    const FrameRec* frames_bvh;
    const GroupRec* groups_bvh;
    int32_t n_outer;
    const NodeF* nodes;
    int32_t n_nodes;
    int32_t root;               // child reference of the root (may be a leaf)
    const Node4Q* nodes4;       // the same tree collapsed to 4-wide quantised nodes
    int32_t n_nodes4;
    int32_t root4;
    const Node4Q* hot4;         // the top n_hot4 wide nodes, breadth-first, refs among them | RT_HOT_BIT
    int32_t n_hot4;
    int32_t root4_hot;          // root reference when the hot table is used
    const XformF* xf;
    const MatF* mats;
    const float4* vnormals;     // 3 per primitive ID (HasNormals triangles)
    int32_t n_mats;             // MatF records (distinct materials)
    int32_t n_xf;               // XformF records
    int32_t n_vn;               // triangles with vertex normals
    uint32_t facts;             // FACT_* (materials and primitive kinds in use)
    // exact set
    const PrimD* prims_d;
    const XformD* xf_d;
    const RefNode* ref_nodes;
    int32_t n_ref_nodes;
    // scene fields
    int32_t width, height;
    int32_t recursion;
    int32_t debug_geom;
    float air_ior;
    float3 ambient;
    int32_t ambient_miss;
};

} // namespace rtc
