// kernels_exact.hip -- the exact fp64 primary-ray pass (DebugRaycaster Primitives mode).
//
// Restates, per pixel, camera.GetRay(x, y).Offset(camera.imagePlane)
// (DebugRaycaster.cs:241; FrustumCamera.cs:33-41; OrthoCamera.cs:33-38) followed by
// Scene.RayTrace(ray, null) (Scene.cs:65-111): the reference BVH's IntersectLeaves
// (BVH.cs:295-331: every pierced leaf in depth-first order, AABB.IntersectAVX,
// SkipVolume reuse), the stable insertion sort by Near (Util.cs:262-280), the
// `Near > previous.Far` early break and the strict `<` replacement, with
// Primitive.RayTrace (Primitive.cs:46-75) over Triangle.RayTraceAVXFaster
// (Triangle.cs:77-146), Sphere.RayTraceAVX (Sphere.cs:50-155) and Plane.DoRayTrace
// (Plane.cs:36-66).  Every operation keeps the reference's order and FMA use, and the file
// is compiled with -ffp-contract=off, so the result is bit-identical to an fp64 host
// restatement on the same inputs.
#include "rt_kernels.h"
#include "rt_refmath.h"

namespace rtc {

struct HitD {
    int prim;
    double dist;
    bool inside;
};

__device__ static int tri_trace_d(const PrimD& p, Vec4d o, Vec4d d, HitD* out)
{
    Vec4d off = sub(o, p.a);
    Vec4d s1 = cross_fma(off, p.b);
    Vec4d s2 = cross_fma(d, p.c);
    double uu = hsum(mul(off, s2)), vv = hsum(mul(d, s1)), tt = hsum(mul(p.c, s1)), det = hsum(mul(p.b, s2));
    double inv = 1.0 / det;
    double invz = (inv == inv) ? inv : 0.0;
    double u = uu * invz, v = vv * invz, t = tt * invz;
    bool rej = (u < 0) | (v < 0);
    if (p.flags & F_MIRROR)
        rej |= (u > 1) | (v > 1);
    else
        rej |= ((u + v) > 1);
    rej |= (t < 0);
    if (rej) return 0;
    out[0].dist = t;
    out[0].inside = invz < 0;
    return 1;
}

__device__ static int sphere_trace_d(const PrimD& p, const XformD* xf, Vec4d o, Vec4d d, HitD* out)
{
    Vec4d oo = o, od = d;
    const bool tr = (p.flags & F_TRANSFORMED) != 0;
    if (tr) {
        oo = mat_vec(xf[p.xf].to_world, o);
        od = normalize_v(mat_vec(xf[p.xf].to_world, d));
    }
    Vec4d off = sub(oo, p.a);
    double b = -2 * dot_v(off, od);
    double c = dot_v(off, off) - p.b.y;
    double radix = sqrt((b * b) - (4 * c));
    double dfar = (b + radix) / 2, dclose = (b - radix) / 2;
    if (tr) {
        Vec4d pfar = mat_vec(xf[p.xf].to_obj, fma4(dfar, od, oo));
        Vec4d pclose = mat_vec(xf[p.xf].to_obj, fma4(dclose, od, oo));
        dfar = dot_v(d, sub(pfar, o));
        dclose = dot_v(d, sub(pclose, o));
    }
    if (!(dfar >= 0)) return 0;
    if (!(dclose >= 0)) {
        out[0] = HitD{0, dfar, true};
        return 1;
    }
    out[0] = HitD{0, dclose, false};
    out[1] = HitD{0, dfar, true};
    return 2;
}

__device__ static bool nearly_equal_d(double a, double b, double delta) // Util.cs:41-51
{
    const double min_normal = 4.9406564584124654e-324 * 1e7;
    if (delta == 0) return true;
    delta = fabs(delta);
    return delta <= min_normal || delta / net_max(a, b) < 1e-24;
}

__device__ static int plane_trace_d(const PrimD& p, Vec4d o, Vec4d d, HitD* out)
{
    double ray_dist = dot_s(o, p.a);
    double denom = dot_s(d, p.a);
    const double od = p.b.x;
    if (nearly_equal_d(denom, 0, denom - 0) && nearly_equal_d(od, ray_dist, od - ray_dist)) {
        out[0] = HitD{0, 0.0, true};
        return 1;
    }
    if (denom == 0) return 0;
    double dist = (od - ray_dist) / denom;
    if (dist >= -1e-24) {
        Vec4d hp = add(o, scale(d, dist));
        out[0] = HitD{0, length_s(sub(hp, o)), dot_s(p.a, d) > 0};
        return 1;
    }
    return 0;
}

// Primitive.RayTrace with a null skip hit (primary rays): first hit that survives culling.
__device__ static bool prim_raytrace_d(const DevScene& s, int pi, Vec4d o, Vec4d d, HitD& h)
{
    const PrimD& p = s.prims_d[pi];
    HitD hits[2];
    int n;
    switch (p.flags & KIND_MASK) {
    case RT_PRIM_TRIANGLE: n = tri_trace_d(p, o, d, hits); break;
    case RT_PRIM_SPHERE: n = sphere_trace_d(p, s.xf_d, o, d, hits); break;
    default: n = plane_trace_d(p, o, d, hits); break;
    }
    for (int i = 0; i < n; i++) {
        bool inside = hits[i].inside;
        if (p.flags & F_INVERT) inside = !inside;
        if (inside && !(p.flags & F_TWOSIDED)) continue;
        h = HitD{pi, hits[i].dist, inside};
        return true;
    }
    return false;
}

constexpr int kLeafCap = 64;
constexpr int kStackCap = 96;

__device__ static int cmp_near(double a, double b) // double.CompareTo
{
    if (a < b) return -1;
    if (a > b) return 1;
    if (a == b) return 0;
    return (a != a) ? ((b != b) ? 0 : -1) : 1;
}

struct LeafItem {
    int node;
    double nr, fr;
};

// The leaf scan of Scene.RayTracePrimitives (Scene.cs:74-91) over leaves given in sorted order.
struct LeafScan {
    int best = -1;
    double best_d = 0, prev_far = 0;
    bool have_prev = false;
    // returns false once the `Near > previous.Far` break is reached
    __device__ bool visit(const DevScene& s, const LeafItem& it, Vec4d o, Vec4d d)
    {
        if (have_prev && it.nr > prev_far) return false;
        HitD h;
        if (prim_raytrace_d(s, s.ref_nodes[it.node].prim, o, d, h) && (best < 0 || h.dist < best_d)) {
            best = h.prim;
            best_d = h.dist;
            prev_far = it.fr;
            have_prev = true;
        }
        return true;
    }
};

// (near, DFS ordinal) in the order of the stable insertion sort with double.CompareTo
__device__ static bool key_less(double an, int ao, double bn, int bo)
{
    const int c = cmp_near(an, bn);
    return c < 0 || (c == 0 && ao < bo);
}

// BVH<T>.IntersectLeaves (BVH.cs:295-331) as an explicit depth-first walk: calls f(item, ordinal)
// for every pierced leaf in the order the reference appends them.
template <class F>
__device__ static bool walk_leaves(const DevScene& s, Vec4d o, Vec4d d, F&& f)
{
    LeafItem stack[kStackCap];
    int sp = 0, ord = 0;
    stack[sp++] = LeafItem{0, 0.0, 0.0};
    while (sp > 0) {
        LeafItem it = stack[--sp];
        const RefNode& n = s.ref_nodes[it.node];
        if (!n.skip) {
            aabb_hit_ref(n.mn, n.mx, o, d, it.nr, it.fr);
            if (!(it.fr >= 0)) continue;
        }
        if (n.prim >= 0) {
            f(it, ord++);
            continue;
        }
        if (sp + 2 > kStackCap) return false;
        stack[sp++] = LeafItem{n.right, it.nr, it.fr};
        stack[sp++] = LeafItem{it.node + 1, it.nr, it.fr};
    }
    return true;
}

// Same result when more than kLeafCap leaves are pierced (large meshes): the leaves are taken in
// sorted order by repeated selection, one depth-first walk per leaf the scan consumes (the scan
// usually stops after a few leaves), so no list is stored.
__device__ static int ref_raytrace_select(const DevScene& s, Vec4d o, Vec4d d)
{
    LeafScan scan;
    double cur_n = 0;
    int cur_o = -1;
    bool first = true;
    while (true) {
        LeafItem next{-1, 0.0, 0.0};
        int next_o = -1;
        const bool ok = walk_leaves(s, o, d, [&](const LeafItem& it, int ord) {
            if (!first && !key_less(cur_n, cur_o, it.nr, ord)) return; // already consumed
            if (next_o < 0 || key_less(it.nr, ord, next.nr, next_o)) {
                next = it;
                next_o = ord;
            }
        });
        if (!ok) return -2;
        if (next_o < 0 || !scan.visit(s, next, o, d)) break;
        cur_n = next.nr;
        cur_o = next_o;
        first = false;
    }
    return scan.best;
}

// Returns the primitive ID, -1 on a miss, -2 if the traversal stack overflowed.
__device__ int ref_raytrace(const DevScene& s, Vec4d o, Vec4d d)
{
    if (s.n_ref_nodes == 0) return -1;
    LeafItem leaves[kLeafCap];
    int nl = 0;
    bool overflow = false;
    const bool ok = walk_leaves(s, o, d, [&](const LeafItem& it, int) {
        if (nl < kLeafCap) leaves[nl++] = it;
        else overflow = true;
    });
    if (!ok) return -2;
    if (overflow) return ref_raytrace_select(s, o, d);
    for (int i = 1; i < nl; i++) { // Util.InsertSort, stable
        LeafItem a = leaves[i];
        int j = i - 1;
        while (j >= 0 && cmp_near(a.nr, leaves[j].nr) < 0) {
            leaves[j + 1] = leaves[j];
            j--;
        }
        leaves[j + 1] = a;
    }
    LeafScan scan;
    for (int i = 0; i < nl; i++)
        if (!scan.visit(s, leaves[i], o, d)) break;
    return scan.best;
}

// BVH<T>.GetIntersectionCount (BVH.cs:352-363), DebugRaycaster BoundingVolumes mode: the nodes
// whose own box the ray meets (Volume.Intersect(ray).far >= 0), descending only through them.
__device__ int ref_bvh_count(const DevScene& s, Vec4d o, Vec4d d)
{
    if (s.n_ref_nodes == 0) return 0;
    int stack[kStackCap];
    int sp = 0, count = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const int i = stack[--sp];
        const RefNode& n = s.ref_nodes[i];
        double nr, fr;
        aabb_hit_ref(n.mn, n.mx, o, d, nr, fr);
        if (!(fr >= 0)) continue;
        count++;
        if (n.prim >= 0) continue;
        if (sp + 2 > kStackCap) return -2;
        stack[sp++] = n.right;
        stack[sp++] = i + 1;
    }
    return count;
}

__device__ static void camera_ray_d(const CameraD& c, double x, double y, Vec4d& o, Vec4d& d)
{
    if (c.kind == RT_CAMERA_FRUSTUM) {
        double ox = c.tan_x * ((x - c.w2) / c.w2);
        double oy = c.tan_y * ((y - c.h2) / c.h2);
        Vec4d dir = add(add(c.look, scale(c.side, ox)), scale(c.up, oy));
        o = c.position;
        d = normalize_v(dir);
    } else {
        o = add(add(c.position, scale(c.side, (x - c.w2) * c.h_mult)), scale(c.up, (y - c.h2) * c.v_mult));
        d = normalize_v(c.look);
    }
    o = add(o, scale(d, c.image_plane)); // Ray.Offset (Ray.cs:59-62)
}

// mode 0: primary hit IDs (Primitives mode), mode 1: BVH node counts (BoundingVolumes mode)
__global__ void __launch_bounds__(64) primary_ids_kernel(DevScene s, CameraD cam, int x0, int y0, int w, int h, int mode,
                                                         int32_t* ids)
{
    int x = blockIdx.x * 8 + (threadIdx.x & 7);
    int y = blockIdx.y * 8 + (threadIdx.x >> 3);
    if (x >= w || y >= h) return;
    Vec4d o, d;
    camera_ray_d(cam, (double)(x0 + x), (double)(y0 + y), o, d);
    ids[(size_t)y * w + x] = mode == 0 ? ref_raytrace(s, o, d) : ref_bvh_count(s, o, d);
}

hipError_t launch_primary_ids(const DevScene& s, const CameraD& cam, int x0, int y0, int w, int h, int mode,
                              int32_t* d_ids, hipStream_t stream)
{
    dim3 grid((w + 7) / 8, (h + 7) / 8);
    hipLaunchKernelGGL(primary_ids_kernel, grid, dim3(64), 0, stream, s, cam, x0, y0, w, h, mode, d_ids);
    return hipGetLastError();
}

} // namespace rtc
