// host_scene.h -- host-side preparation of a scene for the MI355X kernels.
#pragma once
#include <algorithm>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "rt_refmath.h"

namespace rtc {

// Runs task(i) for every i in [0, n) on the process's persistent host worker pool (host_pool.cpp:
// up to 16 threads, OMP_NUM_THREADS where set, the caller included) and returns when all are done.
void host_run(size_t n, const std::function<void(size_t)>& task);
int host_threads();

// fn(i) for i in [0, n) on the host pool (at least 4096 items per thread); fn must only write state
// of its own index.
template <class F>
void parallel_for(int n, F&& fn)
{
    const int T = std::min(host_threads(), (n + 4095) / 4096);
    if (T <= 1) {
        for (int i = 0; i < n; i++) fn(i);
        return;
    }
    const int per = (n + T - 1) / T;
    host_run((size_t)T, [&](size_t t) {
        const int a = (int)t * per, b = std::min(n, a + per);
        for (int i = a; i < b; i++) fn(i);
    });
}

// fn(a, b) over contiguous ranges covering [0, n) on the host pool, each range at least min_items
// long (streaming passes over large arrays).
template <class F>
void parallel_ranges(size_t n, size_t min_items, F&& fn)
{
    const size_t T = std::max<size_t>(1, std::min<size_t>((size_t)host_threads(), n / std::max<size_t>(1, min_items)));
    if (T <= 1) {
        fn((size_t)0, n);
        return;
    }
    const size_t per = (n + T - 1) / T;
    host_run(T, [&](size_t t) { fn(std::min(n, t * per), std::min(n, (t + 1) * per)); });
}

// Axis-aligned box in the reference's fp64 representation (Acceleration/AABB.cs:44-64).
struct Box {
    Vec4d mn, mx, size, ctr;
};
Box box_make(Vec4d mn, Vec4d mx);
Box box_combine(const Box& a, const Box& b); // AABB.Combine (AABB.cs:38-43)
bool box_equals(const Box& a, const Box& b); // AABB.Equals (AABB.cs:232-241)
double box_sa(const Box& b);                 // AABB.GetSurfaceArea (AABB.cs:204-207)

// A primitive with the reference's derived fields (fp64).
struct HostPrim {
    int kind = 0;
    uint32_t flags = 0; // rtc::F_* | kind
    // triangle (Triangle.cs:22-29, Recalculate :54-66)
    Vec4d v[3], vn[3], e01, e02, n;
    // sphere (Sphere.cs:12-21)
    Vec4d center;
    double radius = 0, radius_sqr = 0;
    double to_obj[16], to_world[16], to_normal[16];
    // plane (Plane.cs:13-14)
    Vec4d pn;
    double pd = 0;
    // material (raw backing fields)
    rt_color emission, diffuse, specular, refraction;
    double shininess = 100, ior = 0;
    // bounds (AABB.CreateFromBounded, AABB.cs:22-36) and IBoundedObject center
    Box box;
    Vec4d center_pt;
};

std::vector<HostPrim> prepare_prims(const rt_prim* prims, int n);

// The reference's agglomerative BVH, flattened depth-first (pre-order, left first).
struct RefBvh {
    std::vector<RefNode> nodes;
    int depth = 0;
};
RefBvh build_ref_bvh(const std::vector<HostPrim>& prims);

// One node of the whole binned-SAH tree (down to single primitives): the input of the SAH-optimal
// wide collapse.  Primitives [first, first + count) of SahBvh::order lie below it.
struct SahFullNode {
    float lo[3], hi[3];
    int left, right; // node indices, -1 for a single-primitive leaf
    int first, count;
};

// Binned-SAH BVH2 for the fp32 path kernel (planes are excluded and tested separately).
struct SahBvh {
    std::vector<NodeF> nodes;
    std::vector<int> order; // primitive IDs in leaf order
    int root = 0;           // child reference of the root
    int depth = 0;
    std::vector<SahFullNode> full; // with build_sah_bvh(..., full = true): the tree below the leaves too
    int full_root = 0;
};
// skip: primitives (by index) left out of the tree, besides the planes
SahBvh build_sah_bvh(const std::vector<HostPrim>& prims, int max_leaf, bool full = false,
                     const std::vector<char>* skip = nullptr);
// fp32 box of a primitive for the fast-path BVHs: the fp64 bounds padded by 2^-20 relative and
// rounded outward (used by the host and the GPU builder alike)
void sah_prim_box(const HostPrim& p, float lo[3], float hi[3]);

struct Bvh4 {
    std::vector<Node4Q> nodes;
    int root = 0;       // child reference of the root (wide-node index or leaf code)
    int stack_need = 0; // deepest traversal stack any ray can need
    int depth = 0;
};
// Wide collapse.  Greedy (no costs given, or no full tree): each wide node opens its largest-area
// internal child until it has four children, over the BVH2's own leaves.  SAH-optimal (costs
// given and SahBvh::full built): a dynamic program over the whole tree chooses the wide nodes and
// the leaves (of at most max_leaf primitives) with the least surface-area cost, c_node per wide-node
// visit and c_prim per primitive test (after Ylitie, Karras and Laine 2017, for 4-wide nodes).
struct WideCosts {
    float c_node = 1.0f, c_prim = 0.5f;
    int max_leaf = 3;
};
Bvh4 build_bvh4(const SahBvh& bvh2, const WideCosts* sah = nullptr);

// Camera.InitRender restated for both precisions.
void camera_init(const rt_camera& cam, int width, int height, CameraD& d, CameraF& f);

// Scene text loader (SceneLoader.cs:112-440).
struct ParsedScene {
    rt_scene_params params;
    std::vector<rt_prim> prims;
    std::vector<rt_camera> cameras;
    rt_color background;
    double background_alpha = 0;
};
bool parse_scene_text(const char* text, ParsedScene& out, std::string& err);

// Thread-local error message used by rt_last_error().
void set_error(const std::string& msg);

} // namespace rtc
