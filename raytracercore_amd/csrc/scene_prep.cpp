// scene_prep.cpp -- derived primitive data, reference bounds and cameras (host, fp64).
#include <cmath>
#include <cstring>

#include "host_scene.h"

namespace rtc {

Box box_make(Vec4d mn, Vec4d mx)
{
    // AABB(Vec4D, Vec4D) (AABB.cs:50-64): Center = (Min + Size / 2).WithDefault(0)
    Box b;
    b.mn = mn;
    b.mx = mx;
    b.size = sub(mx, mn);
    Vec4d c = add(mn, divs(b.size, 2));
    if (c.x != c.x) c.x = 0;
    if (c.y != c.y) c.y = 0;
    if (c.z != c.z) c.z = 0;
    if (c.w != c.w) c.w = 0;
    b.ctr = c;
    return b;
}

Box box_combine(const Box& a, const Box& b)
{
    Vec4d mn{net_min(a.mn.x, b.mn.x), net_min(a.mn.y, b.mn.y), net_min(a.mn.z, b.mn.z), net_min(a.mn.w, b.mn.w)};
    Vec4d mx{net_max(a.mx.x, b.mx.x), net_max(a.mx.y, b.mx.y), net_max(a.mx.z, b.mx.z), net_max(a.mx.w, b.mx.w)};
    return box_make(mn, mx);
}

bool box_equals(const Box& a, const Box& b) { return eq3(a.mn, b.mn) && eq3(a.mx, b.mx); }

double box_sa(const Box& b) { return ((b.size.x * b.size.y) + (b.size.y * b.size.z) + (b.size.z * b.size.x)) * 2; }

static Vec4d from(const rt_vec4d& v) { return Vec4d{v.x, v.y, v.z, v.w}; }

// IBoundedObject.GetCenter (Triangle.cs:226-229, Sphere.cs:212-218, Plane.cs:24-27)
static Vec4d prim_center(const HostPrim& p)
{
    switch (p.kind) {
    case RT_PRIM_TRIANGLE: return divs(add(add(p.v[0], p.v[1]), p.v[2]), 3);
    case RT_PRIM_SPHERE: return (p.flags & F_TRANSFORMED) ? mat_vec(p.to_obj, p.center) : p.center;
    default: return add(v4d(0, 0, 0, 1), scale(p.pn, p.pd));
    }
}

// IBoundedObject.GetMaxCenterDistance (Triangle.cs:231-263, Sphere.cs:220-232, Plane.cs:68-74)
static double prim_extent(const HostPrim& p, Vec4d dir)
{
    if (p.kind == RT_PRIM_TRIANGLE) {
        Vec4d c = prim_center(p);
        Vec4d a = sub(p.v[0], c), b = sub(p.v[1], c), d = sub(p.v[2], c), e{0, 0, 0, 0};
        if (p.flags & F_MIRROR) e = sub(add(add(p.v[0], p.e01), p.e02), c);
        bool zero = eq3(dir, v4d(0, 0, 0, 0));
        auto f = [&](Vec4d v) { return zero ? length_s(v) : dot_s(v, dir); };
        double dist = 0;
        dist = net_max(f(a), dist);
        dist = net_max(f(b), dist);
        dist = net_max(f(d), dist);
        if (!eq3(e, v4d(0, 0, 0, 0))) dist = net_max(f(e), dist);
        return dist;
    }
    if (p.kind == RT_PRIM_SPHERE) {
        if (p.flags & F_TRANSFORMED) {
            double s = sqrt(1 - dir.x * dir.x);
            Vec4d v = v4d(dir.x, dir.y * s, dir.z * s, 0);
            // MatrixToObject.Transpose3x3() * v
            const double* m = p.to_obj;
            double t[16] = {m[0], m[4], m[8], 0, m[1], m[5], m[9], 0, m[2], m[6], m[10], 0, 0, 0, 0, 1};
            return length_s(mat_vec(t, v)) * p.radius;
        }
        return p.radius;
    }
    if (fabs(dot_s(p.pn, dir)) == 1) return 0;
    return __builtin_huge_val();
}

std::vector<HostPrim> prepare_prims(const rt_prim* in, int n)
{
    std::vector<HostPrim> out(n);
    parallel_for(n, [&](int i) {
        const rt_prim& a = in[i];
        HostPrim& p = out[i];
        p.kind = a.kind;
        p.flags = (uint32_t)a.kind;
        if (a.flags & RT_FLAG_MIRROR) p.flags |= F_MIRROR;
        if (a.flags & RT_FLAG_TWOSIDED) p.flags |= F_TWOSIDED;
        if (a.flags & RT_FLAG_INVERT) p.flags |= F_INVERT;
        if (a.flags & RT_FLAG_HASNORMALS) p.flags |= F_HASNORMALS;
        if (a.flags & RT_FLAG_TRANSFORMED) p.flags |= F_TRANSFORMED;
        p.emission = a.emission;
        p.diffuse = a.diffuse;
        p.specular = a.specular;
        p.refraction = a.refraction;
        p.shininess = a.shininess;
        p.ior = a.refractive_index;
        std::memcpy(p.to_obj, a.to_obj, sizeof p.to_obj);
        std::memcpy(p.to_world, a.to_world, sizeof p.to_world);
        std::memcpy(p.to_normal, a.to_normal, sizeof p.to_normal);
        if (a.kind == RT_PRIM_TRIANGLE) {
            for (int k = 0; k < 3; k++) {
                p.v[k] = from(a.p[k]);
                p.vn[k] = from(a.n[k]);
            }
            // Triangle.Recalculate (Triangle.cs:54-66); HasNormals triangles keep Normal = 0
            p.e01 = sub(p.v[1], p.v[0]);
            p.e02 = sub(p.v[2], p.v[0]);
            p.n = (p.flags & F_HASNORMALS) ? v4d(0, 0, 0, 0) : normalize_v(cross_s(p.e01, p.e02));
        } else if (a.kind == RT_PRIM_SPHERE) {
            p.center = from(a.p[0]);
            p.radius = a.radius;
            p.radius_sqr = a.radius * a.radius;
        } else {
            p.pn = from(a.p[0]);
            p.pd = a.radius;
        }
        p.center_pt = prim_center(p);
        Vec4d lo = v4d(prim_extent(p, v4d(-1, 0, 0, 0)), prim_extent(p, v4d(0, -1, 0, 0)), prim_extent(p, v4d(0, 0, -1, 0)), 0);
        Vec4d hi = v4d(prim_extent(p, v4d(1, 0, 0, 0)), prim_extent(p, v4d(0, 1, 0, 0)), prim_extent(p, v4d(0, 0, 1, 0)), 0);
        p.box = box_make(sub(p.center_pt, lo), add(p.center_pt, hi));
    });
    return out;
}

void camera_init(const rt_camera& c, int w, int h, CameraD& d, CameraF& f)
{
    // Camera.InitRender (Camera.cs:54-63)
    Vec4d pos = from(c.position), look_at = from(c.look_at), up = from(c.up);
    double w2 = w / 2.0, h2 = h / 2.0;
    Vec4d look = normalize_v(sub(look_at, pos));
    Vec4d side = normalize_v(cross_s(look, neg(up)));
    Vec4d up2 = normalize_v(cross_s(look, side));
    side = neg(side);
    std::memset(&d, 0, sizeof d);
    d.kind = c.kind;
    d.position = pos;
    d.look = look;
    d.side = side;
    d.up = up2;
    d.w2 = w2;
    d.h2 = h2;
    if (c.kind == RT_CAMERA_FRUSTUM) { // FrustumCamera.InitRender (FrustumCamera.cs:24-31)
        double ty = tan(c.fov_y / 2);
        d.tan_x = ty * (w / (double)h);
        d.tan_y = -ty;
    } else { // OrthoCamera.InitRender (OrthoCamera.cs:22-31)
        double cw = 1 / w2;
        double ch = (1 / h2) * (h / (double)w);
        d.h_mult = cw * c.size_mult;
        d.v_mult = -ch * c.size_mult;
    }
    d.image_plane = c.image_plane;
    d.dof = c.dof_amount;
    d.focal_length = c.focal_length;

    auto f4 = [](Vec4d v) { return make_float4((float)v.x, (float)v.y, (float)v.z, (float)v.w); };
    std::memset(&f, 0, sizeof f);
    f.kind = c.kind;
    f.position = f4(d.position);
    f.look = f4(d.look);
    f.side = f4(d.side);
    f.up = f4(d.up);
    f.w2 = (float)w2;
    f.h2 = (float)h2;
    f.tan_x = (float)d.tan_x;
    f.tan_y = (float)d.tan_y;
    f.tan_x_per_px = (float)(d.tan_x / w2);
    f.tan_y_per_px = (float)(d.tan_y / h2);
    f.h_mult = (float)d.h_mult;
    f.v_mult = (float)d.v_mult;
    f.image_plane = (float)d.image_plane;
    f.dof = (float)d.dof;
    f.focal_length = (float)d.focal_length;
}

} // namespace rtc
