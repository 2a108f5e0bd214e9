// oracle_prims.cpp -- primitives, bounds, cameras and ray/primitive intersection in fp64.
// TEST INFRASTRUCTURE (see oracle.h).  Follows the AVX2+FMA paths the reference takes
// when SIMDHelpers.Enabled (Vectors/SIMDHelpers.cs:15).
#include "oracle_scene.h"

namespace orc {

// ---------------------------------------------------------------- Triangle ----
void Prim::recalc_triangle()
{
    // Triangle.Recalculate (Triangle.cs:54-66)
    e01 = vp[1] - vp[0];
    e02 = vp[2] - vp[0];
    if (!has_normals) {
        normal = normalize(cross(e01, e02));
        // Vert.WithNormal -> new Vertex(pos, normal) normalises again (Vertex.cs:11-15,22-25)
        for (int i = 0; i < 3; i++) vn[i] = normalize(normal);
    }
}

V4 Prim::get_center() const
{
    switch (kind) {
    case kTri: return (vp[0] + vp[1] + vp[2]) / 3; // Triangle.cs:226-229
    case kSphere: return transformed ? mvmul(to_obj, center) : center; // Sphere.cs:212-218
    default: return v4(0, 0, 0, 1) + pnormal * origin_dist; // Plane.cs:24-27
    }
}

double Prim::max_center_distance(V4 dir) const
{
    if (kind == kTri) { // Triangle.cs:231-263
        V4 c = get_center();
        double dist = 0;
        V4 a = vp[0] - c, b = vp[1] - c, d = vp[2] - c, v3{0, 0, 0, 0};
        if (mirror) v3 = vp[0] + e01 + e02 - c;
        bool zero = eq3(dir, v4(0, 0, 0, 0));
        auto f = [&](V4 v) { return zero ? length(v) : dot(v, dir); };
        dist = net_max(f(a), dist);
        dist = net_max(f(b), dist);
        dist = net_max(f(d), dist);
        if (!eq3(v3, v4(0, 0, 0, 0))) dist = net_max(f(v3), dist);
        return dist;
    }
    if (kind == kSphere) { // Sphere.cs:220-232
        if (transformed) {
            double s = std::sqrt(1 - dir.x * dir.x);
            V4 vec = v4(dir.x, dir.y * s, dir.z * s, 0);
            return length(mvmul(transpose3x3(to_obj), vec)) * radius;
        }
        return radius;
    }
    // Plane.cs:68-74
    if (std::fabs(dot(pnormal, dir)) == 1) return 0;
    return kInf;
}

// ------------------------------------------------------------------- AABB ----
AABB aabb_make(V4 mn, V4 mx)
{
    // AABB ctor (AABB.cs:50-64): Center = (Min + Size/2).WithDefault(0)
    AABB b;
    b.mn = mn;
    b.mx = mx;
    b.size = mx - mn;
    V4 c = mn + b.size / 2;
    if (std::isnan(c.x)) c.x = 0;
    if (std::isnan(c.y)) c.y = 0;
    if (std::isnan(c.z)) c.z = 0;
    if (std::isnan(c.w)) c.w = 0;
    b.ctr = c;
    return b;
}
bool aabb_equals(const AABB& a, const AABB& b) { return eq3(a.mn, b.mn) && eq3(a.mx, b.mx); } // AABB.cs:232-241
double aabb_sa(const AABB& a) // AABB.cs:204-207
{
    return ((a.size.x * a.size.y) + (a.size.y * a.size.z) + (a.size.z * a.size.x)) * 2;
}

// AABB.IntersectAVX (AABB.cs:107-142).
bool aabb_intersect(const AABB& b, const Ray& r, double& near_, double& far_)
{
    const double o[4] = {r.o.x, r.o.y, r.o.z, r.o.w};
    const double d[4] = {r.d.x, r.d.y, r.d.z, r.d.w};
    const double mn[4] = {b.mn.x, b.mn.y, b.mn.z, b.mn.w};
    const double mx[4] = {b.mx.x, b.mx.y, b.mx.z, b.mx.w};
    double n[4], f[4];
    for (int i = 0; i < 4; i++) {
        bool mask = (d[i] == 0) && (o[i] >= mn[i]) && (o[i] <= mx[i]);
        double lo = mask ? -kInf : mn[i], hi = mask ? kInf : mx[i];
        bool neg = std::signbit(d[i]); // BlendVariable selects on the sign bit
        double lom = neg ? hi : lo, him = neg ? lo : hi;
        double inv = 1.0 / d[i];
        n[i] = (lom - o[i]) * inv;
        f[i] = (him - o[i]) * inv;
    }
    double nn = sse_max(sse_max(n[0], n[2]), sse_max(n[1], n[3]));
    double ff = sse_min(sse_min(f[0], f[2]), sse_min(f[1], f[3]));
    if ((nn > ff) | (ff < 0)) {
        near_ = far_ = kNaN;
        return false;
    }
    near_ = nn;
    far_ = ff;
    return true;
}

// ------------------------------------------------------------ intersection ----
static V4 tri_normal(const Prim& p, double u, double v, bool inside)
{
    // Triangle.GetNormal (Triangle.cs:209-224)
    if (p.has_normals) {
        V4 nrm = normalize(p.vn[0] * u + p.vn[1] * v + p.vn[2] * (u + v));
        if (inside) return nrm - p.normal * (2 * dot(nrm, p.normal) / dot(p.normal, p.normal));
        return nrm;
    }
    if (inside) return p.normal * -1;
    return p.normal;
}

// Triangle.RayTraceAVXFaster (Triangle.cs:77-146).
static int tri_trace(const Prim& p, const Ray& r, Hit out[2])
{
    V4 off = r.o - p.vp[0];
    V4 s1 = cross_fma(off, p.e01);
    V4 s2 = cross_fma(r.d, p.e02);
    double uu = hsum(off * s2), vv = hsum(r.d * s1), tt = hsum(p.e02 * s1), det = hsum(p.e01 * s2);
    double inv = 1.0 / det;
    double invz = (inv == inv) ? inv : 0.0; // NaN -> +0 (And with the ordered mask)
    double u = uu * invz, v = vv * invz, t = tt * invz;
    bool rej = (u < 0) | (v < 0);
    if (p.mirror)
        rej |= (u > 1) | (v > 1);
    else
        rej |= ((u + v) > 1);
    rej |= (t < 0);
    if (rej) return 0;
    bool inside = invz < 0;
    V4 pos{std::fma(p.e01.x, u, std::fma(p.e02.x, v, p.vp[0].x)), std::fma(p.e01.y, u, std::fma(p.e02.y, v, p.vp[0].y)),
           std::fma(p.e01.z, u, std::fma(p.e02.z, v, p.vp[0].z)), std::fma(p.e01.w, u, std::fma(p.e02.w, v, p.vp[0].w))};
    out[0].prim = p.id;
    out[0].pos = pos;
    out[0].dist = t;
    out[0].normal = tri_normal(p, u, v, inside);
    out[0].inside = inside;
    return 1;
}

static inline V4 fma4(double s, V4 d, V4 o)
{
    return {std::fma(s, d.x, o.x), std::fma(s, d.y, o.y), std::fma(s, d.z, o.z), std::fma(s, d.w, o.w)};
}

// Sphere.RayTraceAVX (Sphere.cs:50-155).
static int sphere_trace(const Prim& p, const Ray& r, Hit out[2])
{
    V4 oo = r.o, od = r.d;
    const V4 wo = r.o, wd = r.d;
    if (p.transformed) {
        oo = mvmul(p.to_world, r.o);
        od = normalize(mvmul(p.to_world, r.d));
    }
    V4 off = oo - p.center;
    double b = -2 * dot_simd(off, od);
    double c = dot_simd(off, off) - p.radius_sqr;
    double radix = std::sqrt((b * b) - (4 * c));
    double dfar = (b + radix) / 2, dclose = (b - radix) / 2;
    V4 pfar = fma4(dfar, od, oo), pclose = fma4(dclose, od, oo);
    V4 nfar = (pfar - p.center) / p.radius, nclose = (pclose - p.center) / p.radius;
    if (p.transformed) {
        pfar = mvmul(p.to_obj, pfar);
        pclose = mvmul(p.to_obj, pclose);
        nfar = normalize(mvmul(p.to_normal, nfar));
        dfar = dot_simd(wd, pfar - wo);
        nclose = normalize(mvmul(p.to_normal, nclose));
        dclose = dot_simd(wd, pclose - wo);
    }
    nfar = -nfar;
    if (!(dfar >= 0)) return 0;
    if (!(dclose >= 0)) {
        out[0] = Hit{p.id, pfar, dfar, nfar, true};
        return 1;
    }
    out[0] = Hit{p.id, pclose, dclose, nclose, false};
    out[1] = Hit{p.id, pfar, dfar, nfar, true};
    return 2;
}

// Util.NearlyEqual (Util.cs:41-51), NearEnough = 1e-24 (:18).
static bool nearly_equal(double a, double b, double delta)
{
    const double min_normal = 4.9406564584124654e-324 * 1e7; // double.Epsilon * 1e7
    if (delta == 0) return true;
    delta = std::fabs(delta);
    return delta <= min_normal || delta / net_max(a, b) < 1e-24;
}

// Plane.DoRayTrace (Plane.cs:36-66).
static int plane_trace(const Prim& p, const Ray& r, Hit out[2])
{
    double ray_dist = dot(r.o, p.pnormal);
    double denom = dot(r.d, p.pnormal);
    if (nearly_equal(denom, 0, denom - 0) && nearly_equal(p.origin_dist, ray_dist, p.origin_dist - ray_dist)) {
        out[0] = Hit{p.id, r.o, 0, p.pnormal, true};
        return 1;
    }
    if (denom == 0) return 0;
    double dist = (p.origin_dist - ray_dist) / denom;
    if (dist >= -1e-24) {
        V4 hp = ray_point(r, dist);
        V4 hn = p.pnormal;
        bool inside = false;
        if (dot(p.pnormal, r.d) > 0) {
            hn = -hn;
            inside = true;
        }
        out[0] = Hit{p.id, hp, length(hp - r.o), hn, inside};
        return 1;
    }
    return 0;
}

int prim_dotrace(const Prim& p, const Ray& r, Hit out[2])
{
    switch (p.kind) {
    case kTri: return tri_trace(p, r, out);
    case kSphere: return sphere_trace(p, r, out);
    default: return plane_trace(p, r, out);
    }
}

// Hit operator== (Hit.cs:44-59)
static bool hit_eq(const Hit& a, const Hit& b)
{
    return a.prim == b.prim && eq3(a.pos, b.pos) && a.dist == b.dist && eq3(a.normal, b.normal) && a.inside == b.inside;
}

// Util.RayHitMatches (Util.cs:179-192) with Vec4D.NearlyEquals (Vec4D.cs:439-442).
static bool ray_hit_matches(const Ray& r, const Hit& a, const Hit* b)
{
    if (b == nullptr) return false; // a is never null here
    if (hit_eq(a, *b)) return true;
    if (a.prim != b->prim) return false;
    if (!nearly_equal(sqlen(a.pos), sqlen(b->pos), sqlen(a.pos - b->pos))) return false;
    if (dot(r.d, b->normal) > 0) return a.inside != b->inside;
    return a.inside == b->inside;
}

// Primitive.RayTrace (Primitive.cs:46-75).
Hit prim_raytrace(const Prim& p, const Ray& r, const Hit* skip)
{
    Hit hits[2];
    int n = prim_dotrace(p, r, hits);
    for (int i = 0; i < n; i++) {
        Hit h = hits[i];
        if (p.invert) h.inside = !h.inside; // Hit.Inverted (Hit.cs:39-42)
        if (h.inside && !p.two_sided) continue;
        if (!ray_hit_matches(r, h, skip)) return h;
    }
    return Hit{};
}

// ------------------------------------------------------------------ Camera ----
void Camera::init_render(int w, int h)
{
    // Camera.InitRender (Camera.cs:54-63); note it overwrites `up`.
    up = init_up;
    position = init_pos;
    look_at = init_look_at;
    w2 = w / 2.0;
    h2 = h / 2.0;
    look = normalize(look_at - position);
    side = normalize(cross(look, -up));
    up_r = normalize(cross(look, side));
    side = -side;
    if (kind == 0) { // FrustumCamera.InitRender (FrustumCamera.cs:24-31)
        double ty = std::tan(fov_y / 2);
        tan_x = ty * (w / (double)h);
        tan_y = -ty;
    } else { // OrthoCamera.InitRender (OrthoCamera.cs:22-31)
        double cw = 1 / w2;
        double ch = (1 / h2) * (h / (double)w);
        h_mult = cw * size_mult;
        v_mult = -ch * size_mult;
    }
}

Ray Camera::get_ray(double x, double y) const
{
    if (kind == 0) { // FrustumCamera.GetRay (FrustumCamera.cs:33-41)
        double ox = tan_x * ((x - w2) / w2);
        double oy = tan_y * ((y - h2) / h2);
        V4 dir = look + (side * ox) + (up_r * oy);
        return ray_directional(position, dir);
    }
    // OrthoCamera.GetRay (OrthoCamera.cs:33-38)
    V4 start = position + (side * ((x - w2) * h_mult)) + (up_r * ((y - h2) * v_mult));
    return ray_directional(start, look);
}

} // namespace orc
