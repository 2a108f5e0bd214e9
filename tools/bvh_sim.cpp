// bvh_sim.cpp -- host simulation of closest-hit traversal counts for wide-BVH layouts (a design
// tool, not product code): for a scene file, the binned-SAH BVH2 of the library collapsed greedily
// (largest-area child opened first) into 4-wide and 8-wide trees, and camera rays plus two diffuse
// bounces traced through each with ordered, best-t-culled traversal.  Reports node visits and
// primitive tests per ray segment for
//   4-wide, children sorted by entry distance (the wide kernel's order);
//   8-wide, children sorted by entry distance;
//   8-wide, children in octant slot order (Ylitie, Karras & Laine 2017: slot s holds the child that
//          comes first for rays of direction octant s; a ray of octant o takes the hit children in
//          order of slot ^ o, no sorting).
// Boxes are the exact fp32 child boxes (no quantisation) in all three, so the figures compare the
// tree shapes and orders only.  Primitives are tested in fp64 (Moller-Trumbore, Mirror
// parallelograms), spheres by the quadratic.
// build: make -C raytracercore_amd/csrc bvh_sim;  run: raytracercore_amd/csrc/_obj/bvh_sim SCENE [W H step [spec_frac [bounces]]]
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>
#include <vector>

#include "host_scene.h"

using namespace rtc;

namespace {

struct Box3 {
    float lo[3], hi[3];
};
struct WNode {
    std::vector<Box3> box;
    std::vector<int> ref; // >= 0 wide node index, < 0 BVH2 leaf code
};
int ref_of(const NodeF& n, bool r)
{
    int v;
    std::memcpy(&v, r ? &n.rmin.w : &n.lmin.w, 4);
    return v;
}
Box3 box_of(const NodeF& n, bool r)
{
    const float4 lo = r ? n.rmin : n.lmin, hi = r ? n.rmax : n.lmax;
    return Box3{{lo.x, lo.y, lo.z}, {hi.x, hi.y, hi.z}};
}
float area(const Box3& b)
{
    const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    return 2 * (dx * dy + dy * dz + dz * dx);
}

// greedy collapse of the BVH2 into `width`-wide nodes; octant: assign children to slots
struct Wide {
    std::vector<WNode> nodes;
    int root = 0;
    int width = 4;
    bool octant = false;
    const std::vector<NodeF>* n2 = nullptr;
    int emit(int i)
    {
        std::vector<std::pair<Box3, int>> ch{{box_of((*n2)[i], false), ref_of((*n2)[i], false)},
                                             {box_of((*n2)[i], true), ref_of((*n2)[i], true)}};
        while ((int)ch.size() < width) {
            int best = -1;
            float ba = -1;
            for (int k = 0; k < (int)ch.size(); k++)
                if (ch[k].second >= 0 && area(ch[k].first) > ba) {
                    ba = area(ch[k].first);
                    best = k;
                }
            if (best < 0) break;
            const NodeF& m = (*n2)[ch[best].second];
            ch[best] = {box_of(m, false), ref_of(m, false)};
            ch.insert(ch.begin() + best + 1, {box_of(m, true), ref_of(m, true)});
        }
        const int me = (int)nodes.size();
        nodes.push_back({});
        std::vector<std::pair<Box3, int>> slots;
        if (octant && width == 8) { // Ylitie et al. 2017 section 3.2: greedy assignment by cost
            float pc[3];
            Box3 u = ch[0].first;
            for (auto& c : ch)
                for (int a = 0; a < 3; a++) {
                    u.lo[a] = std::min(u.lo[a], c.first.lo[a]);
                    u.hi[a] = std::max(u.hi[a], c.first.hi[a]);
                }
            for (int a = 0; a < 3; a++) pc[a] = 0.5f * (u.lo[a] + u.hi[a]);
            std::vector<std::array<float, 8>> cost(ch.size());
            for (size_t c = 0; c < ch.size(); c++)
                for (int s = 0; s < 8; s++) {
                    float d = 0;
                    for (int a = 0; a < 3; a++) {
                        const float cc = 0.5f * (ch[c].first.lo[a] + ch[c].first.hi[a]) - pc[a];
                        d += ((s >> a) & 1) ? -cc : cc;
                    }
                    cost[c][s] = d;
                }
            slots.assign(8, {Box3{{1, 1, 1}, {0, 0, 0}}, INT32_MIN});
            std::vector<char> used_c(ch.size(), 0), used_s(8, 0);
            for (size_t k = 0; k < ch.size(); k++) {
                float bc = INFINITY;
                int bi = -1, bs = -1;
                for (size_t c = 0; c < ch.size(); c++)
                    if (!used_c[c])
                        for (int s = 0; s < 8; s++)
                            if (!used_s[s] && cost[c][s] < bc) {
                                bc = cost[c][s];
                                bi = (int)c;
                                bs = s;
                            }
                used_c[bi] = used_s[bs] = 1;
                slots[bs] = ch[bi];
            }
        } else {
            slots = ch;
        }
        for (auto& sl : slots) {
            if (sl.second == INT32_MIN) {
                nodes[me].box.push_back(sl.first);
                nodes[me].ref.push_back(INT32_MIN);
                continue;
            }
            const int r = sl.second >= 0 ? emit(sl.second) : sl.second;
            nodes[me].box.push_back(sl.first);
            nodes[me].ref.push_back(r);
        }
        return me;
    }
};

struct Ray {
    double o[3], d[3];
};
struct Stats {
    double nodes = 0, prims = 0, rays = 0;
};

bool hit_prim(const HostPrim& p, const Ray& r, double& t)
{
    if (p.kind == RT_PRIM_TRIANGLE) {
        const double e1[3] = {p.e01.x, p.e01.y, p.e01.z}, e2[3] = {p.e02.x, p.e02.y, p.e02.z};
        const double s[3] = {r.o[0] - p.v[0].x, r.o[1] - p.v[0].y, r.o[2] - p.v[0].z};
        const double pv[3] = {r.d[1] * e2[2] - r.d[2] * e2[1], r.d[2] * e2[0] - r.d[0] * e2[2], r.d[0] * e2[1] - r.d[1] * e2[0]};
        const double det = e1[0] * pv[0] + e1[1] * pv[1] + e1[2] * pv[2];
        if (det == 0) return false;
        const double inv = 1 / det;
        const double u = (s[0] * pv[0] + s[1] * pv[1] + s[2] * pv[2]) * inv;
        const double q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
        const double v = (r.d[0] * q[0] + r.d[1] * q[1] + r.d[2] * q[2]) * inv;
        const double tt = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * inv;
        if (u < 0 || v < 0 || tt < 1e-7) return false;
        if ((p.flags & F_MIRROR) ? (u > 1 || v > 1) : (u + v > 1)) return false;
        // Primitive.RayTrace culling (Primitive.cs:56-64): Inside (1/det < 0) flipped by Invert,
        // dropped unless TwoSided
        const bool inside = (inv < 0) != ((p.flags & F_INVERT) != 0);
        if (inside && !(p.flags & F_TWOSIDED)) return false;
        t = tt;
        return true;
    }
    if (p.kind == RT_PRIM_SPHERE) {
        const double oc[3] = {r.o[0] - p.center.x, r.o[1] - p.center.y, r.o[2] - p.center.z};
        const double b = oc[0] * r.d[0] + oc[1] * r.d[1] + oc[2] * r.d[2];
        const double c = oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2] - p.radius_sqr;
        const double disc = b * b - c;
        if (disc < 0) return false;
        const double sq = std::sqrt(disc);
        t = -b - sq > 1e-7 ? -b - sq : -b + sq;
        return t > 1e-7;
    }
    return false;
}

bool slab(const Box3& b, const Ray& r, const double inv[3], double tmax, double& tn)
{
    double t0 = 0, t1 = tmax;
    for (int a = 0; a < 3; a++) {
        double l = (b.lo[a] - r.o[a]) * inv[a], h = (b.hi[a] - r.o[a]) * inv[a];
        if (l > h) std::swap(l, h);
        t0 = std::max(t0, l);
        t1 = std::min(t1, h);
    }
    tn = t0;
    return t0 <= t1;
}

// mode 0: children sorted by entry distance; 1: octant slot order (slot ^ o)
int trace(const Wide& W, const SahBvh& b2, const std::vector<HostPrim>& H, const Ray& r, int mode, double& t_best,
          Stats& st, int best_in = -1, double t_in = INFINITY)
{
    const double inv[3] = {1 / r.d[0], 1 / r.d[1], 1 / r.d[2]};
    const int oct = (r.d[0] < 0 ? 1 : 0) | (r.d[1] < 0 ? 2 : 0) | (r.d[2] < 0 ? 4 : 0);
    int best = best_in;
    t_best = t_in;
    std::vector<int> stack{W.root};
    while (!stack.empty()) {
        const int ref = stack.back();
        stack.pop_back();
        if (ref < 0) {
            const int code = ~ref, first = code >> 3, cnt = (code & 7) + 1;
            for (int k = first; k < first + cnt; k++) {
                st.prims++;
                double t;
                if (hit_prim(H[b2.order[k]], r, t) && t < t_best) {
                    t_best = t;
                    best = b2.order[k];
                }
            }
            continue;
        }
        st.nodes++;
        const WNode& n = W.nodes[ref];
        std::vector<std::pair<double, int>> hits;
        for (int s = 0; s < (int)n.ref.size(); s++) {
            if (n.ref[s] == INT32_MIN) continue;
            double tn;
            if (slab(n.box[s], r, inv, t_best, tn)) hits.push_back({mode == 0 ? tn : (double)(s ^ oct), n.ref[s]});
        }
        std::sort(hits.begin(), hits.end());
        for (int k = (int)hits.size() - 1; k >= 0; k--) stack.push_back(hits[k].second);
    }
    return best;
}

} // namespace

int main(int argc, char** argv)
{
    if (argc < 2) {
        std::fprintf(stderr, "usage: bvh_sim SCENE [W H step [spec_frac [bounces]]]\n");
        return 2;
    }
    std::ifstream f(argv[1]);
    std::stringstream ss;
    ss << f.rdbuf();
    ParsedScene ps;
    std::string err;
    if (!parse_scene_text(ss.str().c_str(), ps, err)) {
        std::fprintf(stderr, "parse: %s\n", err.c_str());
        return 1;
    }
    const int W = argc > 3 ? atoi(argv[2]) : 1920, Hh = argc > 3 ? atoi(argv[3]) : 1080;
    const int step = argc > 4 ? atoi(argv[4]) : 8;
    // optional: the fraction of bounces that reflect as a mirror instead of diffusely, and the
    // number of bounces after the camera ray (defaults 0 and 2: camera rays and two diffuse bounces)
    const double spec_frac = argc > 5 ? atof(argv[5]) : 0.0;
    const int n_bounces = argc > 6 ? atoi(argv[6]) : 2;
    const std::vector<HostPrim> H = prepare_prims(ps.prims.data(), (int)ps.prims.size());
    const SahBvh b2 = build_sah_bvh(H, H.size() > 256 ? 3 : 2);
    // round 5: the axis-aligned rectangles (the room's and the light box's faces: box records in the
    // brute-force kernels) taken out of the tree and tested first, their hit the traversal's
    // initial best
    std::vector<HostPrim> Hin, Hrect;
    for (const HostPrim& p : H) ((p.kind == RT_PRIM_TRIANGLE && (p.flags & F_MIRROR)) ? Hrect : Hin).push_back(p);
    const SahBvh b2in = build_sah_bvh(Hin, Hin.size() > 256 ? 3 : 2);
    Wide w4in;
    w4in.n2 = &b2in.nodes;
    w4in.width = 4;
    w4in.root = w4in.emit(0);
    Stats s4in;
    double rect_tests = 0;
    Wide w4, w8s, w8o;
    w4.n2 = w8s.n2 = w8o.n2 = &b2.nodes;
    w4.width = 4;
    w8s.width = w8o.width = 8;
    w8o.octant = true;
    w4.root = w4.emit(0);
    w8s.root = w8s.emit(0);
    w8o.root = w8o.emit(0);
    std::printf("prims %zu  bvh2 nodes %zu  wide4 nodes %zu  wide8 nodes %zu\n", H.size(), b2.nodes.size(), w4.nodes.size(),
                w8s.nodes.size());
    CameraD cd;
    CameraF cf;
    camera_init(ps.cameras[0], W, Hh, cd, cf);
    std::mt19937 rng(7);
    std::uniform_real_distribution<double> U(0, 1);
    Stats s4, s8s, s8o;
    for (int y = step / 2; y < Hh; y += step)
        for (int x = step / 2; x < W; x += step) {
            Ray r;
            const double ox = cd.tan_x * (x - cd.w2) / cd.w2, oy = cd.tan_y * (y - cd.h2) / cd.h2;
            double d[3] = {cd.look.x + cd.side.x * ox + cd.up.x * oy, cd.look.y + cd.side.y * ox + cd.up.y * oy,
                           cd.look.z + cd.side.z * ox + cd.up.z * oy};
            const double l = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
            for (int a = 0; a < 3; a++) r.d[a] = d[a] / l;
            r.o[0] = cd.position.x;
            r.o[1] = cd.position.y;
            r.o[2] = cd.position.z;
            for (int bounce = 0; bounce <= n_bounces; bounce++) {
                double t4, t8, t8o;
                const int h4 = trace(w4, b2, H, r, 0, t4, s4);
                {
                    int bi = -1;
                    double bt = INFINITY;
                    for (size_t k = 0; k < Hrect.size(); k++) {
                        double t;
                        rect_tests++;
                        if (hit_prim(Hrect[k], r, t) && t < bt) {
                            bt = t;
                            bi = (int)k;
                        }
                    }
                    double tin;
                    trace(w4in, b2in, Hin, r, 0, tin, s4in, bi, bt);
                    s4in.rays++;
                }
                trace(w8s, b2, H, r, 0, t8, s8s);
                trace(w8o, b2, H, r, 1, t8o, s8o);
                s4.rays++;
                s8s.rays++;
                s8o.rays++;
                if (h4 < 0) break;
                const HostPrim& p = H[h4];
                double n[3];
                if (p.kind == RT_PRIM_SPHERE) {
                    for (int a = 0; a < 3; a++) n[a] = r.o[a] + t4 * r.d[a] - (&p.center.x)[a];
                } else {
                    n[0] = p.n.x;
                    n[1] = p.n.y;
                    n[2] = p.n.z;
                }
                double nl = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
                for (int a = 0; a < 3; a++) n[a] /= nl;
                if (n[0] * r.d[0] + n[1] * r.d[1] + n[2] * r.d[2] > 0)
                    for (int a = 0; a < 3; a++) n[a] = -n[a];
                double p0[3];
                for (int a = 0; a < 3; a++) p0[a] = r.o[a] + t4 * r.d[a] + 1e-6 * n[a];
                if (spec_frac > 0 && U(rng) < spec_frac) { // mirror reflection about n
                    const double dn = r.d[0] * n[0] + r.d[1] * n[1] + r.d[2] * n[2];
                    for (int a = 0; a < 3; a++) {
                        r.o[a] = p0[a];
                        r.d[a] -= 2 * dn * n[a];
                    }
                    continue;
                }
                // cosine-weighted direction about n
                const double u1 = U(rng), u2 = U(rng), rr = std::sqrt(u1), ph = 2 * M_PI * u2;
                double tx[3] = {std::fabs(n[0]) < 0.9 ? 1.0 : 0.0, std::fabs(n[0]) < 0.9 ? 0.0 : 1.0, 0};
                double b1[3] = {n[1] * tx[2] - n[2] * tx[1], n[2] * tx[0] - n[0] * tx[2], n[0] * tx[1] - n[1] * tx[0]};
                const double bl = std::sqrt(b1[0] * b1[0] + b1[1] * b1[1] + b1[2] * b1[2]);
                for (int a = 0; a < 3; a++) b1[a] /= bl;
                const double b2v[3] = {n[1] * b1[2] - n[2] * b1[1], n[2] * b1[0] - n[0] * b1[2], n[0] * b1[1] - n[1] * b1[0]};
                const double zz = std::sqrt(std::max(0.0, 1 - u1));
                for (int a = 0; a < 3; a++) {
                    r.o[a] = p0[a];
                    r.d[a] = b1[a] * rr * std::cos(ph) + b2v[a] * rr * std::sin(ph) + n[a] * zz;
                }
            }
        }
    auto rep = [](const char* name, const Stats& s) {
        std::printf("%-26s node visits / ray %6.2f   primitive tests / ray %6.2f   (%.0f rays)\n", name, s.nodes / s.rays,
                    s.prims / s.rays, s.rays);
    };
    rep("4-wide, distance-sorted", s4);
    rep("4-wide, rects out + first", s4in);
    std::printf("  rectangles out of the tree: %zu, tested per ray segment: %.2f\n", Hrect.size(), rect_tests / s4in.rays);
    rep("8-wide, distance-sorted", s8s);
    rep("8-wide, octant order", s8o);
    return 0;
}
