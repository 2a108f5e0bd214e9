// oracle.cpp -- CPU oracle: bounce loop, camera rays, sample accumulation, tile scheduler
// and the C API.  TEST INFRASTRUCTURE (see oracle.h).
#include "oracle.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>

#include "../include/rtcore_rng.h"
#include "oracle_scene.h"

using namespace orc;

struct orc_scene {
    Scene sc;
};

namespace {

// Vec4D.CreateHorizontal / CreateHorizon (Vec4D.cs:33-58).
V4 create_horizon(V4 pole, double z, double theta)
{
    V4 c = cross(pole, v4(0, 0, 1, 0));
    V4 cr = eq3(c, v4(0, 0, 0, 0)) ? v4(1, 0, 0, 0) : normalize(c);
    return mvmul(m_rotate(theta, pole), (pole * z) + (cr * std::sqrt(1 - z * z)));
}

struct Sampler {
    rt_rng rng;
    double next() { return rt_rng_next_double(&rng); }
};

// System.Random of .NET Core 3.1 (the BCL the reference targets, RaytracerCore.csproj:5; not
// vendored): Knuth's subtractive generator as the BCL implements it, including its second
// index starting at 21 (so X[n] = X[n-55] - X[n-34] mod int.MaxValue), NextDouble =
// InternalSample() / int.MaxValue.  Diagnostic only: the shared keyed stream
// (include/rtcore_rng.h) is the normative one; this one lets the oracle draw the way one
// reference worker thread does (Raytracer.cs:48, one Random per worker, consumed in pixel order).
struct NetRandom {
    int32_t seed_array[56];
    int inext = 0, inextp = 21;
    explicit NetRandom(int32_t seed)
    {
        const int32_t MBIG = 0x7fffffff, MSEED = 161803398;
        int32_t subtraction = (seed == INT32_MIN) ? MBIG : (seed < 0 ? -seed : seed);
        int32_t mj = MSEED - subtraction, mk = 1;
        std::memset(seed_array, 0, sizeof(seed_array));
        seed_array[55] = mj;
        int ii = 0;
        for (int i = 1; i < 55; i++) {
            if ((ii += 21) >= 55) ii -= 55;
            seed_array[ii] = mk;
            mk = mj - mk;
            if (mk < 0) mk += MBIG;
            mj = seed_array[ii];
        }
        for (int k = 1; k < 5; k++)
            for (int i = 1; i < 56; i++) {
                int n = i + 30;
                if (n >= 55) n -= 55;
                seed_array[i] -= seed_array[1 + n];
                if (seed_array[i] < 0) seed_array[i] += MBIG;
            }
    }
    double next()
    {
        const int32_t MBIG = 0x7fffffff;
        if (++inext >= 56) inext = 1;
        if (++inextp >= 56) inextp = 1;
        int32_t r = seed_array[inext] - seed_array[inextp];
        if (r == MBIG) r--;
        if (r < 0) r += MBIG;
        seed_array[inext] = r;
        return r * (1.0 / MBIG);
    }
};

// Raytracer.RandomShine (Raytracer.cs:51-56).
template <class S>
V4 random_shine(S& rs, V4 dir, double shininess)
{
    double z = shininess == kInf ? 1 : std::pow(rs.next(), 1 / shininess);
    double theta = rs.next() * kPi * 2;
    return create_horizon(dir, z, theta);
}

// Raytracer.GetColor(Ray, ref DebugRay[]) (Raytracer.cs:65-246).  Returns the colour;
// `rays` counts Scene.RayTrace calls.
template <class S>
Col get_color(const Scene& sc, Ray ray, S& rs, int& rays, std::vector<Leaf>& scratch, int32_t* trace = nullptr)
{
    // trace (diagnostic, may be null): per bounce i, trace[2i] = primitive hit (-1 miss),
    // trace[2i+1] = event (1 diffuse, 2 specular, 3 specular fail, 4 transmitted, 5 emission, 0 other)
    Hit prev, hit;
    bool have_prev = false;
    Col tint = col(1);
    for (int i = 0; i <= sc.recursion; i++) {
        if (i % 3 == 0) ray = ray_directional(ray.o, ray.d);
        hit = sc.raytrace(ray, have_prev ? &prev : nullptr, scratch);
        rays++;
        if (trace) trace[2 * i] = hit.prim;
        if (hit.prim < 0) {
            if (i == 0) return col(-1);
            return sc.ambient;
        }
        const Prim& pr = sc.prims[hit.prim];
        if (sc.debug_geom) return pr.specular() + pr.diffuse + pr.emission;
        if (i >= sc.recursion) break;
        Ray out{v4(0, 0, 0, 0), v4(0, 0, 0, 0)};
        bool have_out = false;
        V4 rough = random_shine(rs, hit.normal, pr.shininess);
        double diff_lum = lum(pr.diffuse), spec_lum = lum(pr.specular()), refr_lum = lum(pr.refraction()),
               emis_lum = lum(pr.emission);
        double cs = -dot(rough, ray.d);
        double cos_out = 0, ior_ratio = 0;
        if (((refr_lum > 0) | (spec_lum > 0)) && pr.refractive_index != 0 && cs >= 0) {
            double ior_in, ior_out;
            if (hit.inside) {
                ior_in = pr.refractive_index;
                ior_out = sc.air_ior;
            } else {
                ior_in = sc.air_ior;
                ior_out = pr.refractive_index;
            }
            ior_ratio = ior_in / ior_out;
            double sin_out = ior_ratio * std::sqrt(1 - (cs * cs));
            if (sin_out >= 1) {
                refr_lum = 0;
            } else {
                cos_out = std::sqrt(1 - (sin_out * sin_out));
                double rs_ = ((ior_out * cs) - (ior_in * cos_out)) / ((ior_out * cs) + (ior_in * cos_out));
                double rp = ((ior_in * cs) - (ior_out * cos_out)) / ((ior_in * cs) + (ior_out * cos_out));
                double ratio = ((rs_ * rs_) + (rp * rp)) / 2;
                spec_lum *= ratio;
                refr_lum *= 1 - ratio;
            }
        } else {
            refr_lum = 0;
        }
        double total = diff_lum + spec_lum + refr_lum + emis_lum;
        if (total <= 0) break;
        Col new_tint = col(0);
        double ray_rand = rs.next() * total;
        if (refr_lum != 0 && (ray_rand -= refr_lum) <= 0) {
            V4 od = (rough * -cos_out) + ((ray.d + (rough * cs)) * ior_ratio);
            out = Ray{hit.pos, od};
            have_out = true;
            new_tint = pr.refraction();
            if (hit.inside) new_tint = col(1);
            if (trace) trace[2 * i + 1] = 4;
        } else if (spec_lum != 0 && (ray_rand -= spec_lum) <= 0) {
            V4 od = ray.d + (rough * (cs * 2)); // Raytracer.Reflection (:58-61)
            if (dot(od, hit.normal) > 0) {
                out = Ray{hit.pos, od};
                have_out = true;
                new_tint = pr.specular();
                if (trace) trace[2 * i + 1] = 2;
            } else if (trace) {
                trace[2 * i + 1] = 3;
            }
        } else if (diff_lum != 0 && (ray_rand -= diff_lum) <= 0) {
            double z = (2 * std::acos(rs.next())) / kPi;
            double theta = rs.next() * kPi * 2;
            out = Ray{hit.pos, create_horizon(hit.normal, z, theta)};
            have_out = true;
            new_tint = pr.diffuse;
            if (trace) trace[2 * i + 1] = 1;
        } else {
            if (trace) trace[2 * i + 1] = 5;
            break; // emission
        }
        // `outRay == Ray.Zero` (Raytracer.cs:231): origin and direction both zero (XYZ)
        if (!have_out || (eq3(out.o, v4(0, 0, 0, 0)) && eq3(out.d, v4(0, 0, 0, 0)))) break;
        prev = hit;
        have_prev = true;
        ray = out;
        new_tint = new_tint * net_max(total, 1);
        tint = tint * new_tint;
    }
    return tint * sc.prims[hit.prim].emission;
}

// Raytracer.GetCameraRay (Raytracer.cs:262-282).
template <class S>
Ray camera_ray(const Camera& cam, S& rs, int x, int y)
{
    double dof = cam.dof_amount;
    double sx = x + rs.next();
    double sy = y + rs.next();
    Ray r = cam.get_ray(sx, sy);
    r = Ray{ray_point(r, cam.image_plane), r.d};
    if (dof != 0) {
        V4 focus = ray_point(r, cam.focal_length - cam.image_plane);
        double dist = std::sqrt(rs.next()) * dof;
        double angle = rs.next() * kPi * 2;
        double ox = std::cos(angle) * dist;
        double oy = std::sin(angle) * dist;
        r = cam.get_ray(sx + ox, sy + oy);
        r = Ray{ray_point(r, cam.image_plane), r.d};
        r = Ray{r.o, normalize(focus - r.o)}; // PointingTowards -> FromTo
    }
    return r;
}

bool sample(const Scene& sc, int x, int y, uint64_t seed, uint64_t s, Col& c, int& rays, std::vector<Leaf>& scratch)
{
    Sampler rs{rt_rng_init(seed, (uint64_t)y * (uint64_t)sc.width + (uint64_t)x, s)};
    const Camera& cam = sc.cameras[sc.current_camera];
    Ray r = camera_ray(cam, rs, x, y);
    c = get_color(sc, r, rs, rays, scratch);
    return ceq(c, col(-1)); // FullRaytracer.cs:334-337
}

void init_camera(Scene& sc)
{
    if (!sc.cameras.empty()) sc.cameras[sc.current_camera].init_render(sc.width, sc.height);
}

} // namespace

static V4 from_abi(const rt_vec4d& v) { return v4(v.x, v.y, v.z, v.w); }
static rt_vec4d to_abi(V4 v) { return rt_vec4d{v.x, v.y, v.z, v.w}; }
static Col from_abi(const rt_color& c) { return Col{c.r, c.g, c.b}; }
static rt_color to_abi(Col c) { return rt_color{c.r, c.g, c.b}; }

extern "C" {

orc_scene* orc_load_text(const char* text, char* err, int32_t errcap)
{
    orc_scene* s = new orc_scene();
    std::string e;
    if (!load_scene_text(text ? text : "", s->sc, e)) {
        if (err && errcap > 0) {
            std::strncpy(err, e.c_str(), (size_t)errcap - 1);
            err[errcap - 1] = 0;
        }
        delete s;
        return nullptr;
    }
    s->sc.prepare();
    init_camera(s->sc);
    return s;
}


orc_scene* orc_from_prims(const rt_scene_params* params, const rt_prim* prims, int32_t n, const rt_camera* cameras,
                          int32_t n_cameras)
{
    if (!params || (n > 0 && !prims) || n < 0) return nullptr;
    orc_scene* s = new orc_scene();
    Scene& sc = s->sc;
    sc.width = params->width;
    sc.height = params->height;
    sc.recursion = params->recursion;
    sc.debug_geom = params->debug_geom != 0;
    sc.air_ior = params->air_ior;
    sc.ambient = from_abi(params->ambient);
    for (int i = 0; i < n; i++) {
        const rt_prim& a = prims[i];
        Prim p;
        p.kind = a.kind;
        p.id = i;
        p.two_sided = (a.flags & RT_FLAG_TWOSIDED) != 0;
        p.invert = (a.flags & RT_FLAG_INVERT) != 0;
        p.emission = from_abi(a.emission);
        p.diffuse = from_abi(a.diffuse);
        p.specular_raw = from_abi(a.specular);
        p.refraction_raw = from_abi(a.refraction);
        p.shininess = a.shininess;
        p.refractive_index = a.refractive_index;
        if (a.kind == kTri) {
            p.mirror = (a.flags & RT_FLAG_MIRROR) != 0;
            p.has_normals = (a.flags & RT_FLAG_HASNORMALS) != 0;
            for (int k = 0; k < 3; k++) {
                p.vp[k] = from_abi(a.p[k]);
                p.vn[k] = from_abi(a.n[k]);
            }
            p.normal = v4(0, 0, 0, 0);
            p.recalc_triangle();
        } else if (a.kind == kSphere) {
            p.center = from_abi(a.p[0]);
            p.radius = a.radius;
            p.radius_sqr = a.radius * a.radius;
            p.transformed = (a.flags & RT_FLAG_TRANSFORMED) != 0;
            std::memcpy(p.to_obj.d, a.to_obj, sizeof(double) * 16);
            std::memcpy(p.to_world.d, a.to_world, sizeof(double) * 16);
            std::memcpy(p.to_normal.d, a.to_normal, sizeof(double) * 16);
        } else {
            p.pnormal = from_abi(a.p[0]);
            p.origin_dist = a.radius;
        }
        sc.prims.push_back(p);
    }
    for (int i = 0; i < n_cameras; i++) {
        const rt_camera& c = cameras[i];
        Camera cam;
        cam.kind = c.kind;
        cam.init_pos = cam.position = from_abi(c.position);
        cam.init_look_at = cam.look_at = from_abi(c.look_at);
        cam.init_up = cam.up = from_abi(c.up);
        cam.fov_y = c.fov_y;
        cam.size_mult = c.size_mult;
        cam.image_plane = c.image_plane;
        cam.dof_amount = c.dof_amount;
        cam.focal_length = c.focal_length;
        sc.cameras.push_back(cam);
    }
    sc.prepare();
    init_camera(sc);
    return s;
}

void orc_destroy(orc_scene* s) { delete s; }
int32_t orc_num_prims(const orc_scene* s) { return s ? (int32_t)s->sc.prims.size() : -1; }
int32_t orc_num_cameras(const orc_scene* s) { return s ? (int32_t)s->sc.cameras.size() : -1; }

int32_t orc_export(const orc_scene* s, rt_scene_params* params, rt_prim* prims, rt_camera* cameras)
{
    if (!s) return -1;
    const Scene& sc = s->sc;
    if (params) {
        params->width = sc.width;
        params->height = sc.height;
        params->recursion = sc.recursion;
        params->debug_geom = sc.debug_geom ? 1 : 0;
        params->air_ior = sc.air_ior;
        params->ambient = to_abi(sc.ambient);
    }
    if (prims) {
        for (size_t i = 0; i < sc.prims.size(); i++) {
            const Prim& p = sc.prims[i];
            rt_prim a;
            std::memset(&a, 0, sizeof(a));
            a.kind = p.kind;
            a.flags = (p.two_sided ? RT_FLAG_TWOSIDED : 0) | (p.invert ? RT_FLAG_INVERT : 0);
            a.emission = to_abi(p.emission);
            a.diffuse = to_abi(p.diffuse);
            a.specular = to_abi(p.specular_raw);
            a.refraction = to_abi(p.refraction_raw);
            a.shininess = p.shininess;
            a.refractive_index = p.refractive_index;
            std::memcpy(a.to_obj, p.to_obj.d, sizeof(double) * 16);
            std::memcpy(a.to_world, p.to_world.d, sizeof(double) * 16);
            std::memcpy(a.to_normal, p.to_normal.d, sizeof(double) * 16);
            if (p.kind == kTri) {
                a.flags |= (p.mirror ? RT_FLAG_MIRROR : 0) | (p.has_normals ? RT_FLAG_HASNORMALS : 0);
                for (int k = 0; k < 3; k++) {
                    a.p[k] = to_abi(p.vp[k]);
                    a.n[k] = to_abi(p.vn[k]);
                }
            } else if (p.kind == kSphere) {
                a.flags |= p.transformed ? RT_FLAG_TRANSFORMED : 0;
                a.p[0] = to_abi(p.center);
                a.radius = p.radius;
                std::memcpy(a.to_obj, p.to_obj.d, sizeof(double) * 16);
                std::memcpy(a.to_world, p.to_world.d, sizeof(double) * 16);
                std::memcpy(a.to_normal, p.to_normal.d, sizeof(double) * 16);
            } else {
                a.p[0] = to_abi(p.pnormal);
                a.radius = p.origin_dist;
            }
            prims[i] = a;
        }
    }
    if (cameras) {
        for (size_t i = 0; i < sc.cameras.size(); i++) {
            const Camera& c = sc.cameras[i];
            rt_camera a;
            std::memset(&a, 0, sizeof(a));
            a.kind = c.kind;
            a.position = to_abi(c.init_pos);
            a.look_at = to_abi(c.init_look_at);
            a.up = to_abi(c.init_up);
            a.fov_y = c.fov_y;
            a.size_mult = c.size_mult;
            a.image_plane = c.image_plane;
            a.dof_amount = c.dof_amount;
            a.focal_length = c.focal_length;
            cameras[i] = a;
        }
    }
    return (int32_t)sc.prims.size();
}

int32_t orc_background(const orc_scene* s, rt_color* rgb, double* alpha)
{
    if (!s) return -1;
    if (rgb) *rgb = to_abi(s->sc.background);
    if (alpha) *alpha = s->sc.background_alpha;
    return 0;
}

int32_t orc_set_size(orc_scene* s, int32_t w, int32_t h)
{
    if (!s || w <= 0 || h <= 0) return -1;
    s->sc.width = w;
    s->sc.height = h;
    init_camera(s->sc);
    return 0;
}

int32_t orc_select_camera(orc_scene* s, int32_t index)
{
    if (!s || index < 0 || index >= (int32_t)s->sc.cameras.size()) return -1;
    s->sc.current_camera = index;
    init_camera(s->sc);
    return 0;
}

static void bvh_walk(const BNode* n, int depth, int& count, int& maxd, std::vector<int32_t>* order,
                     std::vector<double>* boxes)
{
    count++;
    maxd = std::max(maxd, depth);
    if (boxes) {
        const AABB& b = n->vol;
        double v[8] = {b.mn.x, b.mn.y, b.mn.z, b.mn.w, b.mx.x, b.mx.y, b.mx.z, b.mx.w};
        boxes->insert(boxes->end(), v, v + 8);
    }
    if (n->leaf) {
        if (order) order->push_back(n->prim);
        return;
    }
    bvh_walk(n->left, depth + 1, count, maxd, order, boxes);
    bvh_walk(n->right, depth + 1, count, maxd, order, boxes);
}

int32_t orc_bvh_info(const orc_scene* s, int32_t* nodes, int32_t* depth)
{
    if (!s) return -1;
    int c = 0, d = 0;
    if (s->sc.root) bvh_walk(s->sc.root, 0, c, d, nullptr, nullptr);
    if (nodes) *nodes = c;
    if (depth) *depth = d;
    return 0;
}

int32_t orc_bvh_leaf_order(const orc_scene* s, int32_t* prim_ids)
{
    if (!s) return -1;
    int c = 0, d = 0;
    std::vector<int32_t> order;
    if (s->sc.root) bvh_walk(s->sc.root, 0, c, d, &order, nullptr);
    if (prim_ids) std::copy(order.begin(), order.end(), prim_ids);
    return (int32_t)order.size();
}

int32_t orc_bvh_boxes(const orc_scene* s, double* out)
{
    if (!s) return -1;
    int c = 0, d = 0;
    std::vector<double> boxes;
    if (s->sc.root) bvh_walk(s->sc.root, 0, c, d, nullptr, &boxes);
    if (out) std::copy(boxes.begin(), boxes.end(), out);
    return c;
}

int32_t orc_primary_ids(const orc_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t* ids)
{
    if (!s || !ids || w < 0 || h < 0 || s->sc.cameras.empty()) return -1;
    const Scene& sc = s->sc;
    const Camera& cam = sc.cameras[sc.current_camera];
    std::vector<Leaf> scratch;
    for (int x = 0; x < w; x++)
        for (int y = 0; y < h; y++) {
            // DebugRaycaster.RenderDebug: camera.GetRay(x, y).Offset(camera.imagePlane) (:241)
            Ray r = cam.get_ray(x0 + x, y0 + y);
            r = Ray{ray_point(r, cam.image_plane), r.d};
            Hit hit = sc.raytrace(r, nullptr, scratch);
            ids[x * h + y] = hit.prim;
        }
    return 0;
}

// BVH<T>.GetIntersectionCount (BVH.cs:352-363): nodes whose own volume the ray meets.
static int32_t bvh_count(const BNode* n, const Ray& r)
{
    double nr, fr;
    aabb_intersect(n->vol, r, nr, fr);
    if (!(fr >= 0)) return 0;
    if (n->leaf) return 1;
    return 1 + bvh_count(n->left, r) + bvh_count(n->right, r);
}

int32_t orc_bvh_counts(const orc_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t* counts)
{
    if (!s || !counts || w < 0 || h < 0 || s->sc.cameras.empty()) return -1;
    const Scene& sc = s->sc;
    const Camera& cam = sc.cameras[sc.current_camera];
    for (int x = 0; x < w; x++)
        for (int y = 0; y < h; y++) {
            Ray r = cam.get_ray(x0 + x, y0 + y); // DebugRaycaster.cs:241
            r = Ray{ray_point(r, cam.image_plane), r.d};
            counts[x * h + y] = sc.root ? bvh_count(sc.root, r) : 0;
        }
    return 0;
}

int32_t orc_raytrace(const orc_scene* s, const double o[4], const double d[4], double* dist)
{
    if (!s) return -2;
    std::vector<Leaf> scratch;
    Ray r{v4(o[0], o[1], o[2], o[3]), v4(d[0], d[1], d[2], d[3])};
    Hit h = s->sc.raytrace(r, nullptr, scratch);
    if (dist) *dist = h.dist;
    return h.prim;
}

int32_t orc_sample(const orc_scene* s, int32_t x, int32_t y, uint64_t seed, uint64_t smp, rt_color* color, int32_t* rays)
{
    if (!s || s->sc.cameras.empty()) return -1;
    std::vector<Leaf> scratch;
    Col c;
    int nr = 0;
    bool miss = sample(s->sc, x, y, seed, smp, c, nr, scratch);
    if (color) *color = to_abi(c);
    if (rays) *rays = nr;
    return miss ? 1 : 0;
}

int32_t orc_render_tile(const orc_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t spp, uint64_t seed,
                        uint64_t sample_base, rt_color* sum, uint32_t* samples, uint32_t* misses, uint64_t* rays)
{
    if (!s || s->sc.cameras.empty() || w < 0 || h < 0 || spp < 0) return -1;
    std::vector<Leaf> scratch;
    uint64_t nrays = 0;
    for (int x = 0; x < w; x++)
        for (int y = 0; y < h; y++) {
            size_t i = (size_t)x * h + y;
            Col acc = from_abi(sum[i]);
            for (int k = 0; k < spp; k++) {
                Col c;
                int nr = 0;
                bool miss = sample(s->sc, x0 + x, y0 + y, seed, sample_base + k, c, nr, scratch);
                nrays += nr;
                if (miss) {
                    misses[i]++;
                } else {
                    acc = acc + c;
                    samples[i]++;
                }
            }
            sum[i] = to_abi(acc);
        }
    if (rays) *rays += nrays;
    return 0;
}

// Diagnostic: one reference worker's draw order.  One System.Random(seed) stream; `spp` passes,
// each over the tile row by row (Raytracer.Render, Raytracer.cs:302-320).
// Diagnostic: one sample with its path (see get_color's `trace`, 2 * (recursion + 1) ints, -2 filled).
int32_t orc_sample_trace(const orc_scene* s, int32_t x, int32_t y, uint64_t seed, uint64_t smp, rt_color* color,
                         int32_t* trace)
{
    if (!s || s->sc.cameras.empty() || !trace) return -1;
    const Scene& sc = s->sc;
    std::vector<Leaf> scratch;
    for (int i = 0; i < 2 * (sc.recursion + 1); i++) trace[i] = -2;
    Sampler rs{rt_rng_init(seed, (uint64_t)y * (uint64_t)sc.width + (uint64_t)x, smp)};
    Ray r = camera_ray(sc.cameras[sc.current_camera], rs, x, y);
    int nr = 0;
    Col c = get_color(sc, r, rs, nr, scratch, trace);
    if (color) *color = to_abi(c);
    return ceq(c, col(-1)) ? 1 : 0;
}

int32_t orc_render_tile_netrandom(const orc_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t spp,
                                  int32_t seed, rt_color* sum, uint32_t* samples, uint32_t* misses, uint64_t* rays)
{
    if (!s || s->sc.cameras.empty() || w < 0 || h < 0 || spp < 0) return -1;
    const Scene& sc = s->sc;
    const Camera& cam = sc.cameras[sc.current_camera];
    std::vector<Leaf> scratch;
    NetRandom rs(seed);
    uint64_t nrays = 0;
    for (int k = 0; k < spp; k++)
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) {
                size_t i = (size_t)x * h + y;
                int nr = 0;
                Ray r = camera_ray(cam, rs, x0 + x, y0 + y);
                Col c = get_color(sc, r, rs, nr, scratch);
                nrays += nr;
                if (ceq(c, col(-1))) {
                    misses[i]++;
                } else {
                    sum[i].r += c.r;
                    sum[i].g += c.g;
                    sum[i].b += c.b;
                    samples[i]++;
                }
            }
    if (rays) *rays += nrays;
    return 0;
}

int32_t orc_render_frame(const orc_scene* s, int32_t spp, uint64_t seed, int32_t threads, rt_color* sum,
                         uint32_t* samples, uint32_t* misses, uint64_t* rays, double* seconds, int32_t* threads_used)
{
    if (!s || s->sc.cameras.empty() || spp < 0) return -1;
    const Scene& sc = s->sc;
    int T = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    // FullRaytracer tile grid (FullRaytracer.cs:71-72,271-286)
    int tiles_y = (int)std::floor(std::sqrt((double)T));
    int tiles_x = T / tiles_y;
    int W = sc.width, H = sc.height;
    struct Tile {
        int l, t, r, b;
    };
    std::vector<Tile> tiles(tiles_x * tiles_y);
    for (int x = 0; x < tiles_x; x++) {
        int left = x * W / tiles_x, right = (x + 1) * W / tiles_x;
        for (int y = 0; y < tiles_y; y++) {
            int top = y * H / tiles_y, bottom = (y + 1) * H / tiles_y;
            tiles[y * tiles_x + x] = Tile{left, top, right, bottom};
        }
    }
    const int64_t total_passes = (int64_t)spp * (int64_t)tiles.size();
    std::atomic<int64_t> next{0};
    std::atomic<uint64_t> total_rays{0};
    std::vector<std::mutex> locks(tiles.size());
    auto worker = [&]() {
        std::vector<Leaf> scratch;
        std::vector<Col> buf;
        std::vector<uint8_t> miss;
        while (true) {
            int64_t n = next.fetch_add(1); // GetWorkingTile: round-robin (FullRaytracer.cs:219-229)
            if (n >= total_passes) break;
            int ti = (int)(n % (int64_t)tiles.size());
            uint64_t pass = (uint64_t)(n / (int64_t)tiles.size());
            const Tile& t = tiles[ti];
            int tw = t.r - t.l, th = t.b - t.t;
            buf.assign((size_t)tw * th, col(0));
            miss.assign((size_t)tw * th, 0);
            uint64_t nr_tile = 0;
            for (int y = 0; y < th; y++) // Raytracer.Render pixel loop (Raytracer.cs:309-320)
                for (int x = 0; x < tw; x++) {
                    Col c;
                    int nr = 0;
                    miss[(size_t)x * th + y] = sample(sc, t.l + x, t.t + y, seed, pass, c, nr, scratch);
                    buf[(size_t)x * th + y] = c;
                    nr_tile += nr;
                }
            total_rays += nr_tile;
            std::lock_guard<std::mutex> g(locks[ti]); // FullRaytracer.cs:326-344 merge
            for (int x = 0; x < tw; x++)
                for (int y = 0; y < th; y++) {
                    size_t i = (size_t)(t.l + x) * H + (t.t + y);
                    size_t j = (size_t)x * th + y;
                    if (miss[j]) {
                        misses[i]++;
                    } else {
                        sum[i].r += buf[j].r;
                        sum[i].g += buf[j].g;
                        sum[i].b += buf[j].b;
                        samples[i]++;
                    }
                }
        }
    };
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int i = 0; i < T; i++) pool.emplace_back(worker);
    for (auto& th : pool) th.join();
    auto t1 = std::chrono::steady_clock::now();
    if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
    if (rays) *rays += total_rays.load();
    if (threads_used) *threads_used = T;
    return 0;
}

// SampleSet.GetOutput / GetColorCode (SampleSet.cs:50-113), Util.Clamp SSE form (Util.cs:126-144).
static double clamp01(double v) { return sse_min(sse_max(v, 0.0), 1.0); }
int32_t orc_sample_output(rt_color sum, uint32_t samples, uint32_t misses, rt_color back, double back_alpha,
                          double exposure)
{
    auto code = [](double r, double g, double b, double a) {
        return (int32_t)(((uint32_t)(int32_t)(clamp01(a) * 255) << 24) | ((uint32_t)(int32_t)(clamp01(r) * 255) << 16) |
                         ((uint32_t)(int32_t)(clamp01(g) * 255) << 8) | ((uint32_t)(int32_t)(clamp01(b) * 255)));
    };
    if (samples == 0) return code(back.r * exposure, back.g * exposure, back.b * exposure, back_alpha);
    double total = (double)samples + (double)misses;
    double mult = exposure / samples;
    double r = sum.r * mult, g = sum.g * mult, b = sum.b * mult, a = 1;
    double back_alpha_amt = misses / total;
    double back_amt = back_alpha_amt * back_alpha;
    r += (back.r - r) * back_amt;
    g += (back.g - g) * back_amt;
    b += (back.b - b) * back_amt;
    a += (back_alpha - a) * back_alpha_amt;
    const double gamma = 1 / 2.2;
    return code(std::pow(r, gamma), std::pow(g, gamma), std::pow(b, gamma), a);
}

int32_t orc_rng_draws(uint64_t seed, uint64_t pixel, uint64_t sample, int32_t n, double* out)
{
    rt_rng r = rt_rng_init(seed, pixel, sample);
    for (int32_t k = 0; k < n; k++) out[k] = rt_rng_next_double(&r);
    return 0;
}

double orc_fresnel(double cs, double ior_in, double ior_out)
{
    double ratio_ = ior_in / ior_out;
    double sin_out = ratio_ * std::sqrt(1 - (cs * cs));
    if (sin_out >= 1) return 1;
    double cos_out = std::sqrt(1 - (sin_out * sin_out));
    double rs_ = ((ior_out * cs) - (ior_in * cos_out)) / ((ior_out * cs) + (ior_in * cos_out));
    double rp = ((ior_in * cs) - (ior_out * cos_out)) / ((ior_in * cs) + (ior_out * cos_out));
    return ((rs_ * rs_) + (rp * rp)) / 2;
}

} // extern "C"
