// rtcore_api.hip -- the C ABI (include/rtcore.h): scene upload, renders, multi-GPU frame.
//
// Replaces the body of the reference's render worker loop (Raytracer.Render,
// Raytracer.cs:294-330) behind FullRaytracer's GetWorkingTile / OnTileFinished contract
// (FullRaytracer.cs:210-229); see INTEGRATION.md for the C# P/Invoke side.
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <unordered_map>
#include <thread>
#include <vector>

#include "../../include/rtcore_rng.h"
#include "bvh_gpu.h"
#include "host_scene.h"
#include "rt_jit.h"
#include "rt_kernels.h"

using namespace rtc;

namespace rtc {
static thread_local std::string g_error;
void set_error(const std::string& msg) { g_error = msg; }
} // namespace rtc

#define HIP_TRY(expr)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) {                                                                         \
            set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                               \
            return e_ == hipErrorOutOfMemory ? RT_ERR_OOM : RT_ERR_HIP;                                 \
        }                                                                                               \
    } while (0)

namespace {

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    ~DevBuf() { release(); }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    hipError_t reserve(size_t count)
    {
        if (count <= n) return hipSuccess;
        release();
        hipError_t e = hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) n = count;
        return e;
    }
    void adopt(T* q, size_t count) // take ownership of a hipMalloc'd array
    {
        release();
        p = q;
        n = q ? count : 0;
    }
    hipError_t upload(const std::vector<T>& v)
    {
        hipError_t e = reserve(v.size());
        if (e != hipSuccess || v.empty()) return e;
        return hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
    }
};

// Pinned host staging (hipHostMalloc) for the host-buffer entry points: device -> host copies at
// DMA rate into it, then a multi-threaded pass into the caller's (pageable) arrays.
template <class T>
struct HostBuf {
    T* p = nullptr;
    size_t n = 0;
    ~HostBuf() { release(); }
    void release()
    {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
    hipError_t reserve(size_t count)
    {
        if (count <= n) return hipSuccess;
        release();
        hipError_t e = hipHostMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = count;
        return e;
    }
};

float4 f4(Vec4d v, float w) { return make_float4((float)v.x, (float)v.y, (float)v.z, w); }
float as_f(int v)
{
    float f;
    std::memcpy(&f, &v, 4);
    return f;
}
float as_f(uint32_t v)
{
    float f;
    std::memcpy(&f, &v, 4);
    return f;
}
double luminance(rt_color c) { return 0.299 * c.r + 0.587 * c.g + 0.114 * c.b; } // DoubleColor.cs:76-79
uint32_t p_flags_with_axis(uint32_t flags, int axis) { return flags | ((uint32_t)(axis + 1) << F_AXIS_SHIFT); }
// A slot tested as an axis-aligned rectangle on plane `axis`: its flags name the axis, and its
// shading row c (brute-force kernels) the one-hot axis whose hit coordinate is the plane's.
void set_rect_axis(PrimF& f, uint32_t flags, int axis)
{
    const uint32_t fl = p_flags_with_axis(flags, axis);
    std::memcpy(&f.b.w, &fl, 4);
    f.c = make_float4(axis == 0 ? 1.0f : 0.0f, axis == 1 ? 1.0f : 0.0f, axis == 2 ? 1.0f : 0.0f, 0.0f);
}

} // namespace

struct rt_scene {
    int device = 0;
    int n_cu = 256;
    rt_scene_params params{};
    std::vector<HostPrim> host;
    int traversal = RT_TRAVERSAL_AUTO, resolved = RT_TRAVERSAL_BRUTE;
    int variant = 0;
    int blocks_per_cu = 1;
    RefBvh ref;
    bool ref_built = false;
    SahBvh sah;   // host-built trees (empty when the GPU builder made them)
    Bvh4 bvh4;
    struct {
        int builder = RT_BVH_BUILDER_HOST; // the one that ran
        int n_nodes2 = 0, n_nodes4 = 0, root2 = 0, root4 = 0, depth2 = 0, stack4 = 0, rounds = 0;
        int leaves4 = 0, compact4 = 0; // leaf references of the wide tree, compact ones (kLeafCompact)
        float gpu_ms = 0.0f;
    } bvh;
    DevBuf<int32_t> order_d;      // GPU builder: primitive IDs in leaf order, planes appended
    // Outer records (host builder, large scenes): the axis-aligned rectangles left out of the tree
    // and tested as one brute-force group (world rects and closed boxes) when a query ends
    std::vector<char> bvh_outer;  // per primitive: 1 = outside the tree (empty: none)
    DevBuf<RectRec> rects_bvh;
    DevBuf<FrameRec> frames_bvh;  // the group's BoxRecs
    DevBuf<GroupRec> groups_bvh;
    double ms_prepare = 0, ms_bvh = 0, ms_upload = 0;
    struct { // the flat brute-force order's decomposition (build statistics)
        int rects = 0, boxes = 0, frames = 0, frame_boxes = 0, frame_rects = 0, tris = 0, sphs = 0;
        int group_max = 0; // primitives per group of the grouped order
    } layout;
    DevScene dev{};
    DevBuf<PrimF> prims_bf, prims_bvh;
    DevBuf<TestRec> tests_bf, tests_bvh;
    DevBuf<float4> rows_bvh; // tests_bvh without the meta rows (compact leaves)
    DevBuf<RectRec> rects_bf;
    DevBuf<FrameRec> frames_bf;
    DevBuf<GroupRec> groups_bf;
    DevBuf<PrimF> prims_gr;
    DevBuf<TestRec> tests_gr;
    DevBuf<RectRec> rects_gr;
    DevBuf<FrameRec> frames_gr;
    DevBuf<GroupRec> groups_gr;
    std::vector<GroupRec> groups_gr_host; // in build order; uploaded nearest-first per camera
    // host copies of the brute-force records (the scene-specialised kernels, rt_jit.h)
    struct BruteHost {
        std::vector<GroupRec> groups; // the grouped order: in the current camera's upload order
        std::vector<RectRec> rects;
        std::vector<FrameRec> frames;
        std::vector<TestRec> tests;
    } flat_h, grouped_h;
    std::vector<XformF> xf_h;
    unsigned jit_gen = 0; // bumped by every camera change (and with it the grouped order's group order)
    struct {
        int variant = -1;          // the variant and group order the function was built for
        unsigned gen = 0;
        hipFunction_t fn = nullptr;
        int blocks_per_cu = 0;
        int status = 0;            // 1 built, 0 not used (off, or a BVH / staged-less variant), -1 failed
        double compile_ms = 0;
        bool from_cache = false;
        std::string error;
        std::string header;        // the generated scene header fn was built from
    } jit;
    double grouped_measured = 0; // calibrated brute-force cost ratio flat / grouped (AUTO picks grouped above 1.25)
    DevBuf<NodeF> nodes;
    DevBuf<Node4Q> nodes4;
    DevBuf<Node4Q> hot4;        // top of the wide tree, breadth-first, staged in LDS by the wide kernel
    DevBuf<XformF> xf;
    DevBuf<MatF> mats;
    DevBuf<float4> vnormals;
    DevBuf<PrimD> prims_d;
    DevBuf<XformD> xf_d;
    DevBuf<RefNode> ref_nodes;
    // work buffers
    DevBuf<unsigned int> counter;
    DevBuf<rt_key2> pkeys;       // pixel-key table of the brute-force kernels (PathParams::pkeys)
    bool pkeys_valid = false;
    uint64_t pkeys_seed = 0;
    DevBuf<int> stack_ovf;
    DevBuf<unsigned long long> rays;
    DevBuf<float4> partial;
    DevBuf<double> sum, colors;
    DevBuf<float> colors32;        // rt_render_tile_1spp: one pass as fp32 rgb in the caller's order
    HostBuf<unsigned char> stage;  // host-buffer entry points (rt_render_tile, rt_render_tile_1spp)
    HostBuf<unsigned long long> rays_h;
    static constexpr int kCopyChunks = 8; // chunked device -> host copies (copy_consume)
    std::array<hipEvent_t, kCopyChunks> copy_ev{};
    // rt_render_tile: band k's records are copied on copy_stream once band_ev[k] (recorded on the
    // scene's stream after the band's layout kernel) has fired, so band k + 1 renders meanwhile
    hipStream_t copy_stream = nullptr;
    std::array<hipEvent_t, kCopyChunks> band_ev{};
    DevBuf<uint32_t> samples, misses;
    DevBuf<int32_t> ids;
    bool stats_on = false;      // launch the instrumented kernel (rt_scene_set_stats)
    float4* ray_log = nullptr;  // rt_debug_ray_log (instrumented BVH launches)
    unsigned int* ray_log_n = nullptr;
    unsigned int ray_log_cap = 0;
    int stats_blocks_per_cu = 1;
    DevBuf<unsigned long long> stats_buf;
    CameraD camd{};
    CameraF camf{};
    DevBuf<CameraF> camf_d;     // the path kernels read the camera from device memory (not kernel arguments)
    // ... and their launch parameters, from a ring of device slots filled from pinned host slots.
    // A slot is rewritten kParamRing launches later; its event (recorded after the slot's upload)
    // is waited on first, so a caller queueing more launches than that without a sync still
    // hands every launch its own parameters.
    static constexpr int kParamRing = 256;
    DevBuf<PathParams> params_d;
    PathParams* params_h = nullptr;
    std::array<hipEvent_t, kParamRing> slot_ev{};
    unsigned params_next = 0;
    bool has_camera = false;
    bool flat_overflow = false; // the flat brute-force order exceeds GroupRec's counts (BruteOrder::overflow)
    hipStream_t stream = nullptr;
    // Timing of the path kernels: the i-th launch records the event pair i % kTimeRing, so a caller
    // can queue up to that many launches before it reads their durations (rt_kernel_times).
    static constexpr int kTimeRing = 64;
    std::array<hipEvent_t, kTimeRing> t_start{}, t_end{};
    uint64_t launches = 0;
    // Launches share per-scene scratch (partials, work counter, stack overflow area).  The end of
    // the last render operation is recorded here; an operation on a different stream waits for it.
    hipEvent_t done_ev = nullptr;
    hipStream_t last_stream = nullptr;
    bool any_op = false;
    uint64_t device_bytes = 0;

    ~rt_scene()
    {
        if (jit.fn) jit_release(device, jit.fn); // (the stream is synchronised by rt_scene_destroy)
        if (params_h) (void)hipHostFree(params_h);
        for (hipEvent_t e : slot_ev)
            if (e) (void)hipEventDestroy(e);
        if (done_ev) (void)hipEventDestroy(done_ev);
        for (hipEvent_t e : copy_ev)
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : band_ev)
            if (e) (void)hipEventDestroy(e);
        if (copy_stream) {
            (void)hipStreamSynchronize(copy_stream);
            (void)hipStreamDestroy(copy_stream);
        }
        for (int i = 0; i < kTimeRing; i++) {
            if (t_start[i]) (void)hipEventDestroy(t_start[i]);
            if (t_end[i]) (void)hipEventDestroy(t_end[i]);
        }
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace {

PrimF make_primf(const std::vector<HostPrim>& H, const std::vector<int>& xf_index, int i)
{
    {
        const HostPrim& p = H[i];
        PrimF f;
        std::memset(&f, 0, sizeof f);
        if (p.kind == RT_PRIM_TRIANGLE) {
            f.a = f4(p.v[0], as_f(i));
            f.b = f4(p.e01, as_f(p.flags));
            f.c = make_float4(0.0f, 0.0f, 0.0f, 0.0f); // the shading row (see set_rect_axis)
            f.d = f4(p.n, 0.0f);
        } else if (p.kind == RT_PRIM_SPHERE) {
            f.a = f4(p.center, as_f(i));
            f.b = make_float4((float)p.radius, (float)(1.0 / p.radius), as_f(xf_index[i]), as_f(p.flags));
            if (!(p.flags & F_TRANSFORMED)) { // brute-force shading: normal = p / r - centre / r
                const double ir = 1.0 / p.radius;
                f.c = make_float4(0.0f, 0.0f, 0.0f, (float)ir);
                f.d = make_float4((float)(-p.center.x * ir), (float)(-p.center.y * ir), (float)(-p.center.z * ir), 0.0f);
            }
        } else {
            f.a = f4(p.pn, as_f(i));
            f.b = make_float4((float)p.pd, 0.0f, 0.0f, as_f(p.flags));
            f.d = f4(p.pn, 0.0f); // face normal where the shading step reads it for every flat kind
        }
        return f;
    }
}
TestRec make_testrec(const std::vector<HostPrim>& H, const std::vector<int>& xf_index, int i)
{
    {
        const HostPrim& p = H[i];
        TestRec t;
        std::memset(&t, 0, sizeof t);
        t.meta = make_float4(as_f(i), as_f(p.flags), 0.0f, 0.0f);
        if (p.kind == RT_PRIM_TRIANGLE) {
            // inverse of A = [e01 e02 n] (columns) with n = e01 x e02: rows (e02 x n, n x e01, n) / |n|^2
            const Vec4d e1 = p.e01, e2 = p.e02, nn = cross_s(p.e01, p.e02);
            const double D = dot_s(e1, cross_s(e2, nn));
            const Vec4d rows[3] = {cross_s(e2, nn), cross_s(nn, e1), nn};
            float4* out[3] = {&t.r0, &t.r1, &t.r2};
            for (int k = 0; k < 3; k++) {
                const Vec4d r = divs(rows[k], D);
                *out[k] = make_float4((float)r.x, (float)r.y, (float)r.z,
                                      (float)(-(r.x * p.v[0].x + r.y * p.v[0].y + r.z * p.v[0].z)));
            }
        } else if (p.kind == RT_PRIM_SPHERE) {
            t.r0 = f4(p.center, (float)p.radius);
            t.r1 = make_float4((float)p.radius_sqr, as_f(xf_index[i]), 0.0f, 0.0f);
        } else {
            t.r0 = f4(p.pn, (float)p.pd);
        }
        return t;
    }
}

// The brute-force slot orders of a scene (flat and grouped), built on the host only: world
// rectangles, closed and open boxes, frames, triangles, spheres and planes.
struct BruteLayout {
    int rects = 0, boxes = 0, frames = 0, frame_boxes = 0, frame_rects = 0, tris = 0, sphs = 0;
};
struct BruteOrder {
    std::vector<PrimF> prims;
    std::vector<TestRec> tests;
    std::vector<RectRec> rects;
    std::vector<FrameRec> frames; // FrameRecs and BoxRecs
    std::vector<GroupRec> groups;
    int nr[3] = {0, 0, 0}, nt = 0, ns = 0;
    // a group with more triangles or spheres than GroupRec::n_tri_sph holds (16 and 15 bits): the
    // brute-force kernels cannot run the order (rt_scene_set_traversal refuses them)
    bool overflow = false;
    int tris0 = 0, sphs0 = 0; // triangles and spheres of the first group (the flat order's only one)
};
struct BruteOrders {
    BruteOrder flat, grouped;
    BruteOrder outer; // the BVH's outer records: one group, slots numbered from 0 (planes appended)
    int nr[3] = {0, 0, 0}, nt = 0, ns = 0, np = 0;
    int group_max = 0; // primitives per group of the grouped order (kGroupMax at creation)
    BruteLayout layout;
};
// An axis-aligned rectangle: a Mirror parallelogram with both edges on coordinate axes; returns
// the axis of its plane, or -1.
int rect_axis_of(const HostPrim& p)
{
    if (p.kind != RT_PRIM_TRIANGLE || !(p.flags & F_MIRROR) || (p.flags & F_HASNORMALS)) return -1;
    const double e1[3] = {p.e01.x, p.e01.y, p.e01.z}, e2[3] = {p.e02.x, p.e02.y, p.e02.z};
    for (int k = 0; k < 3; k++) {
        const int a = (k + 1) % 3, b = (k + 2) % 3;
        if (e1[k] != 0 || e2[k] != 0) continue;
        const bool e1a = e1[a] != 0 && e1[b] == 0, e1b = e1[b] != 0 && e1[a] == 0;
        const bool e2a = e2[a] != 0 && e2[b] == 0, e2b = e2[b] != 0 && e2[a] == 0;
        if ((e1a && e2b) || (e1b && e2a)) return k;
    }
    return -1;
}

// outer: the primitives the BVH leaves out (rt_scene::bvh_outer, may be empty); they get an order
// of their own (BruteOrders::outer), one group of world rects and closed boxes.
BruteOrders make_brute_orders(const std::vector<HostPrim>& H, const std::vector<int>& xf_index, const SahBvh& sah,
                              const std::vector<char>& outer = {})
{
    BruteOrders out;
    const int n = (int)H.size();
    auto primf = [&](int i) { return make_primf(H, xf_index, i); };
    auto testrec = [&](int i) { return make_testrec(H, xf_index, i); };
    auto rect_axis = [&](int i) { return rect_axis_of(H[i]); };
    auto rectrec = [&](int i, int k) {
        const HostPrim& p = H[i];
        const double v0[3] = {p.v[0].x, p.v[0].y, p.v[0].z}, e1[3] = {p.e01.x, p.e01.y, p.e01.z},
                     e2[3] = {p.e02.x, p.e02.y, p.e02.z}, nn[3] = {p.n.x, p.n.y, p.n.z};
        const int a1 = k == 0 ? 1 : 0, a2 = k == 2 ? 1 : 2; // the other two axes in x, y, z order
        RectRec r;
        r.c = (float)v0[k];
        const double c1[4] = {v0[a1], v0[a1] + e1[a1], v0[a1] + e2[a1], v0[a1] + e1[a1] + e2[a1]};
        const double c2[4] = {v0[a2], v0[a2] + e1[a2], v0[a2] + e2[a2], v0[a2] + e1[a2] + e2[a2]};
        // fp32 extents rounded outward, stored as mid-point +- half-width
        const double lo1 = std::min(std::min(c1[0], c1[1]), std::min(c1[2], c1[3]));
        const double hi1 = std::max(std::max(c1[0], c1[1]), std::max(c1[2], c1[3]));
        const double lo2 = std::min(std::min(c2[0], c2[1]), std::min(c2[2], c2[3]));
        const double hi2 = std::max(std::max(c2[0], c2[1]), std::max(c2[2], c2[3]));
        r.m1 = (float)(0.5 * (lo1 + hi1));
        r.h1 = (float)(0.5 * (hi1 - lo1));
        r.m2 = (float)(0.5 * (lo2 + hi2));
        r.h2 = (float)(0.5 * (hi2 - lo2));
        // gin = N[k] * d[k] > 0; one-sided keeps gin == Invert (Primitive.cs:56-61): with
        // q = +-sign(N[k]) that is q * d[k] <= 0 (d[k] = 0 never hits: t is inf or NaN)
        const float ns = nn[k] > 0 ? 1.0f : -1.0f;
        r.cull = (p.flags & F_TWOSIDED) ? 0.0f : ((p.flags & F_INVERT) ? -ns : ns);
        r.id = i;
        r.sg = 0; // set once the slot is known
        return r;
    };
    std::vector<int> kind_of(n);
    for (int i = 0; i < n; i++) {
        const int ax = rect_axis(i);
        kind_of[i] = ax >= 0 ? ax : (H[i].kind == RT_PRIM_TRIANGLE ? 3 : H[i].kind == RT_PRIM_SPHERE ? 4 : 5);
    }
    // Frames: the general Mirror parallelograms of a group whose edges run along the three edge
    // directions of one affine frame (a transformed cube's faces) become rectangles in that frame
    // (FrameRec); a frame is used when it collects at least two faces.
    struct FrameB {
        Vec4d b[3];
        bool b2_set = false; // b[2] came from an edge (else it is the first face's normal)
        Vec4d org;
        std::vector<int> face[3]; // faces on local plane k (edges along the other two axes)
    };
    auto parallel = [](const Vec4d& a, const Vec4d& b) {
        const Vec4d c = cross_s(a, b);
        const double aa = dot_s(a, a), bb = dot_s(b, b);
        return aa > 0 && bb > 0 && dot_s(c, c) <= 1e-18 * aa * bb;
    };
    // The box and frame finders pair rectangles by search (quadratic in the group's rectangles).
    // They only make the brute-force orders cheaper to test, and a group with more than
    // kFindMax candidates belongs to a scene the BVH kernels render (AUTO takes brute force up to 48
    // primitives), so such a group keeps its rectangles as they are: scene creation stays linear
    // (8,000 single axis-aligned rectangles took 0.7 s, 100,000 would take minutes).
    constexpr size_t kFindMax = 4096;
    auto find_frames = [&](const std::vector<int>& ids) {
        std::vector<FrameB> fr;
        size_t cand = 0;
        for (int i : ids) cand += kind_of[i] == 3 && (H[i].flags & F_MIRROR) && !(H[i].flags & F_HASNORMALS);
        if (cand > kFindMax) return fr;
        for (int i : ids) {
            const HostPrim& p = H[i];
            if (kind_of[i] != 3 || !(p.flags & F_MIRROR) || (p.flags & F_HASNORMALS)) continue;
            bool placed = false;
            for (auto& F : fr) {
                int k1 = -1, k2 = -1;
                for (int k = 0; k < 3; k++) {
                    if (k1 < 0 && parallel(p.e01, F.b[k])) k1 = k;
                    if (k2 < 0 && parallel(p.e02, F.b[k])) k2 = k;
                }
                if (!F.b2_set && F.face[0].empty() && F.face[1].empty()) { // third axis still open
                    if (k1 >= 0 && k1 != 2 && k2 < 0) {
                        F.b[2] = p.e02;
                        k2 = 2;
                    } else if (k2 >= 0 && k2 != 2 && k1 < 0) {
                        F.b[2] = p.e01;
                        k1 = 2;
                    }
                    if (k1 == 2 || k2 == 2) F.b2_set = true;
                }
                if (k1 >= 0 && k2 >= 0 && k1 != k2) {
                    F.face[3 - k1 - k2].push_back(i);
                    placed = true;
                    break;
                }
            }
            if (!placed) {
                FrameB F;
                F.b[0] = p.e01;
                F.b[1] = p.e02;
                F.b[2] = cross_s(p.e01, p.e02);
                F.org = p.v[0];
                F.face[2].push_back(i);
                fr.push_back(F);
            }
        }
        std::vector<FrameB> keep;
        for (auto& F : fr)
            if (F.face[0].size() + F.face[1].size() + F.face[2].size() >= 2) keep.push_back(F);
        return keep;
    };
    // local rows (world -> frame) of F: the inverse of [b0 b1 b2] applied to p - org
    auto frame_rows = [&](const FrameB& F, double M[3][4]) {
        const Vec4d c0 = cross_s(F.b[1], F.b[2]), c1 = cross_s(F.b[2], F.b[0]), c2 = cross_s(F.b[0], F.b[1]);
        const double det = dot_s(F.b[0], c0);
        const Vec4d rows[3] = {c0, c1, c2};
        for (int k = 0; k < 3; k++) {
            M[k][0] = rows[k].x / det;
            M[k][1] = rows[k].y / det;
            M[k][2] = rows[k].z / det;
            M[k][3] = -(M[k][0] * F.org.x + M[k][1] * F.org.y + M[k][2] * F.org.z);
        }
    };
    // Rectangle geometry in double (world axes, or a frame's local axes): plane coordinate c on
    // axis k, extents on the other two axes in increasing axis order, and sign(N . axis k).
    struct RectG {
        int i, k;
        double c, lo1, hi1, lo2, hi2;
        double ns;
    };
    auto rect_geom = [&](int i, int k, const double (*M)[4], const FrameB* F) {
        const HostPrim& p = H[i];
        auto loc = [&](double x, double y, double z, int a) {
            if (!M) return a == 0 ? x : a == 1 ? y : z;
            return M[a][0] * x + M[a][1] * y + M[a][2] * z + M[a][3];
        };
        const Vec4d v0 = p.v[0], e1 = p.e01, e2 = p.e02;
        const double cx[4] = {v0.x, v0.x + e1.x, v0.x + e2.x, v0.x + e1.x + e2.x};
        const double cy[4] = {v0.y, v0.y + e1.y, v0.y + e2.y, v0.y + e1.y + e2.y};
        const double cz[4] = {v0.z, v0.z + e1.z, v0.z + e2.z, v0.z + e1.z + e2.z};
        const int a1 = k == 0 ? 1 : 0, a2 = k == 2 ? 1 : 2;
        RectG g{i, k, 0, 1e300, -1e300, 1e300, -1e300, 0};
        for (int j = 0; j < 4; j++) {
            g.c += 0.25 * loc(cx[j], cy[j], cz[j], k);
            const double q1 = loc(cx[j], cy[j], cz[j], a1), q2 = loc(cx[j], cy[j], cz[j], a2);
            g.lo1 = std::min(g.lo1, q1);
            g.hi1 = std::max(g.hi1, q1);
            g.lo2 = std::min(g.lo2, q2);
            g.hi2 = std::max(g.hi2, q2);
        }
        if (!M) g.c = k == 0 ? v0.x : k == 1 ? v0.y : v0.z; // world rects sit exactly on v0's plane
        const double nk = F ? dot_s(p.n, F->b[k]) : (k == 0 ? p.n.x : k == 1 ? p.n.y : p.n.z);
        g.ns = nk > 0 ? 1.0 : -1.0;
        return g;
    };
    auto frame_rect = [&](const RectG& g) {
        const HostPrim& p = H[g.i];
        RectRec r;
        r.c = (float)g.c;
        r.m1 = (float)(0.5 * (g.lo1 + g.hi1));
        r.m2 = (float)(0.5 * (g.lo2 + g.hi2));
        // half-widths padded by 2^-21 relative: the fp32 frame rows move the shared edges of
        // neighbouring faces by about an ulp, and a padded edge is met by both faces (closest wins)
        r.h1 = (float)(0.5 * (g.hi1 - g.lo1) + (std::fabs(0.5 * (g.lo1 + g.hi1)) + 0.5 * (g.hi1 - g.lo1)) * 4.76837158203125e-07);
        r.h2 = (float)(0.5 * (g.hi2 - g.lo2) + (std::fabs(0.5 * (g.lo2 + g.hi2)) + 0.5 * (g.hi2 - g.lo2)) * 4.76837158203125e-07);
        // gin = N . d > 0 = sign(N . b_k) * d_local[k] > 0; the culling factor as for world rects
        r.cull = (p.flags & F_TWOSIDED) ? 0.0f : ((p.flags & F_INVERT) ? -(float)g.ns : (float)g.ns);
        r.id = g.i;
        r.sg = 0;
        return r;
    };
    // Boxes: rectangles on the faces of one axis-aligned box -- a pair on some axis with equal
    // extents, and the other faces on the planes and extents of the box they span (within 1e-9
    // relative), at least five of the six, with primitive IDs within 16 of each other.  Face
    // lists are in face order f = 2 axis + side, -1 for a missing face (an open box: the ray may
    // enter through the opening, and its exit face is still the other candidate).
    struct BoxFit {
        std::array<int, 6> f;
        double lo[3], hi[3];
    };
    auto find_boxes = [&](const std::vector<RectG>& rg, std::vector<char>& used) {
        std::vector<BoxFit> boxes;
        auto eq = [](double a, double b, double sc) { return std::fabs(a - b) <= 1e-9 * sc; };
        for (int pa = 0; pa < 3; pa++)
            for (size_t A = 0; A < rg.size(); A++) {
                if (used[A] || rg[A].k != pa) continue;
                for (size_t B = 0; B < rg.size(); B++) {
                    if (B == A || used[B] || used[A] || rg[B].k != pa) continue;
                    const RectG &ga = rg[A], &gb = rg[B];
                    // the pair's axis pa and its two in-plane axes (increasing order)
                    const int q1 = pa == 0 ? 1 : 0, q2 = pa == 2 ? 1 : 2;
                    double lo[3], hi[3];
                    lo[pa] = std::min(ga.c, gb.c);
                    hi[pa] = std::max(ga.c, gb.c);
                    lo[q1] = ga.lo1;
                    hi[q1] = ga.hi1;
                    lo[q2] = ga.lo2;
                    hi[q2] = ga.hi2;
                    double sc = 0;
                    for (int k = 0; k < 3; k++) sc = std::max({sc, std::fabs(lo[k]), std::fabs(hi[k]), hi[k] - lo[k]});
                    bool flat = false;
                    for (int k = 0; k < 3; k++) flat |= !(hi[k] - lo[k] > 1e-9 * sc);
                    if (flat || !eq(gb.lo1, ga.lo1, sc) || !eq(gb.hi1, ga.hi1, sc) || !eq(gb.lo2, ga.lo2, sc) ||
                        !eq(gb.hi2, ga.hi2, sc))
                        continue;
                    BoxFit fit;
                    fit.f.fill(-1);
                    fit.f[2 * pa] = ga.c < gb.c ? (int)A : (int)B;
                    fit.f[2 * pa + 1] = ga.c < gb.c ? (int)B : (int)A;
                    int found = 2;
                    for (int k = 0; k < 3; k++) {
                        fit.lo[k] = lo[k];
                        fit.hi[k] = hi[k];
                        if (k == pa) continue;
                        const int a1 = k == 0 ? 1 : 0, a2 = k == 2 ? 1 : 2;
                        for (int side = 0; side < 2; side++) {
                            const double c = side ? hi[k] : lo[k];
                            for (size_t j = 0; j < rg.size(); j++)
                                if (!used[j] && rg[j].k == k && eq(rg[j].c, c, sc) && eq(rg[j].lo1, lo[a1], sc) &&
                                    eq(rg[j].hi1, hi[a1], sc) && eq(rg[j].lo2, lo[a2], sc) && eq(rg[j].hi2, hi[a2], sc)) {
                                    fit.f[2 * k + side] = (int)j;
                                    found++;
                                    break;
                                }
                        }
                    }
                    if (found < 5) continue;
                    int idmin = 1 << 30, idmax = -1;
                    for (int j : fit.f)
                        if (j >= 0) {
                            idmin = std::min(idmin, rg[j].i);
                            idmax = std::max(idmax, rg[j].i);
                        }
                    if (idmax - idmin >= 16) continue;
                    for (int j : fit.f)
                        if (j >= 0) used[j] = 1;
                    boxes.push_back(fit);
                }
            }
        return boxes;
    };
    auto box_rec = [&](const std::vector<RectG>& rg, const BoxFit& fit, int slot0) {
        BoxRec B;
        std::memset(&B, 0, sizeof B);
        int id0 = 1 << 30;
        for (int j : fit.f)
            if (j >= 0) id0 = std::min(id0, rg[j].i);
        uint32_t perm = 0, keep = 0;
        for (int fi = 0; fi < 6; fi++) {
            if (fit.f[fi] < 0) continue; // missing face: keeps nothing
            const RectG& g = rg[fit.f[fi]];
            const uint32_t fl = H[g.i].flags;
            perm |= (uint32_t)(g.i - id0) << (4 * fi);
            // entering through the lower plane moves along +axis: Inside (N . d > 0) iff sign(N_k) > 0
            const bool gin_entry = (fi & 1) == 0 ? g.ns > 0 : g.ns < 0;
            const bool two = (fl & F_TWOSIDED) != 0, inv = (fl & F_INVERT) != 0;
            if (two || gin_entry == inv) keep |= 1u << fi;
            if (two || !gin_entry == inv) keep |= 1u << (8 + fi);
        }
        // the planes: a face's own (fp32) coordinate where it exists (hit points are snapped to it)
        float pl[6];
        for (int fi = 0; fi < 6; fi++)
            pl[fi] = (float)(fit.f[fi] >= 0 ? rg[fit.f[fi]].c : ((fi & 1) ? fit.hi[fi >> 1] : fit.lo[fi >> 1]));
        B.lo = make_float4(pl[0], pl[2], pl[4], as_f(id0));
        B.hi = make_float4(pl[1], pl[3], pl[5], as_f(perm));
        B.keep = keep;
        B.sg0 = slot0 << 1;
        return B;
    };
    // the six slots of a box, face order; a missing face gets a placeholder slot (never hit)
    auto box_face_prim = [&](const std::vector<RectG>& rg, const BoxFit& fit, int fi) {
        const int j = fit.f[fi] >= 0 ? fit.f[fi] : fit.f[fi ^ 1] >= 0 ? fit.f[fi ^ 1] : fit.f[(fi + 2) % 6];
        return rg[j].i;
    };
    // Brute-force slot orders: groups of primitives, each [x-rects | y-rects | z-rects | world
    // box faces | frame rects and frame box faces | triangles | spheres], then the planes.  The
    // flat order is one group of everything; the grouped order cuts the SAH BVH into subtrees of
    // at most kGroupMax primitives.
    auto fbox = [&](const std::vector<int>& ids, float lo[3], float hi[3]) {
        for (int k = 0; k < 3; k++) {
            lo[k] = __builtin_huge_valf();
            hi[k] = -__builtin_huge_valf();
        }
        for (int i : ids) {
            const double l[3] = {H[i].box.mn.x, H[i].box.mn.y, H[i].box.mn.z};
            const double u[3] = {H[i].box.mx.x, H[i].box.mx.y, H[i].box.mx.z};
            for (int k = 0; k < 3; k++) {
                const double pad = (std::fabs(l[k]) + std::fabs(u[k])) * 9.5367431640625e-07 + 1e-30;
                lo[k] = std::min(lo[k], std::nextafter((float)(l[k] - pad), -__builtin_huge_valf()));
                hi[k] = std::max(hi[k], std::nextafter((float)(u[k] + pad), __builtin_huge_valf()));
            }
        }
    };
    const bool use_boxes = !getenv("RTCORE_NO_BOXES"); // A/B switch for measurements
    // skips[k] > 0: groups[k] lists a subtree's primitives for a super record (its box only) that
    // holds the skips[k] records after it
    auto build_order = [&](const std::vector<std::vector<int>>& groups, const std::vector<int>& skips) {
        BruteOrder o;
        for (size_t gi = 0; gi < groups.size(); gi++) {
            const auto& g = groups[gi];
            GroupRec G;
            std::memset(&G, 0, sizeof G);
            float lo[3], hi[3];
            fbox(g, lo, hi);
            if (skips[gi] > 0) {
                G.lo = make_float4(lo[0], lo[1], lo[2], as_f((int)o.rects.size()));
                G.hi = make_float4(hi[0], hi[1], hi[2], as_f((int)o.prims.size()));
                G.frame_first = (int)o.frames.size();
                G.skip = skips[gi];
                o.groups.push_back(G);
                continue;
            }
            const int rect_first = (int)o.rects.size();
            int cnt[5] = {0, 0, 0, 0, 0};
            auto push_slot = [&](int i, PrimF f) {
                o.prims.push_back(f);
                o.tests.push_back(testrec(i));
            };
            // world rects: closed boxes first, the rest as single rects
            std::vector<RectG> wr;
            for (int i : g)
                if (kind_of[i] < 3) wr.push_back(rect_geom(i, kind_of[i], nullptr, nullptr));
            std::vector<char> wused(wr.size(), 0);
            const auto wboxes = use_boxes && wr.size() <= kFindMax ? find_boxes(wr, wused) : std::vector<BoxFit>{};
            for (int kind = 0; kind < 3; kind++)
                for (size_t j = 0; j < wr.size(); j++) {
                    if (wused[j] || wr[j].k != kind) continue;
                    const int i = wr[j].i;
                    PrimF f = primf(i);
                    set_rect_axis(f, H[i].flags, kind);
                    o.rects.push_back(rectrec(i, kind));
                    o.rects.back().sg = (int)o.prims.size() << 1;
                    o.nr[kind]++;
                    cnt[kind]++;
                    push_slot(i, f);
                }
            // frames (their rects after the world rects), then the world boxes, in one array
            const std::vector<FrameB> frames = find_frames(g);
            std::vector<char> in_frame(n, 0);
            for (const auto& F : frames)
                for (int k = 0; k < 3; k++)
                    for (int i : F.face[k]) in_frame[i] = 1;
            G.frame_first = (int)o.frames.size();
            G.n_frames = (int16_t)frames.size();
            G.n_boxes = (int16_t)wboxes.size();
            // the counts are int16 in the record: more would wrap and drop geometry silently
            if (frames.size() > INT16_MAX || wboxes.size() > INT16_MAX ||
                frames.size() + wboxes.size() > INT16_MAX)
                o.overflow = true;
            std::vector<BoxRec> frame_boxes;
            const int frame_box_first = G.frame_first + (int)frames.size() + (int)wboxes.size();
            for (const auto& F : frames) {
                double M[3][4];
                frame_rows(F, M);
                FrameRec R;
                std::memset(&R, 0, sizeof R);
                float4* rows[3] = {&R.r0, &R.r1, &R.r2};
                for (int k = 0; k < 3; k++)
                    *rows[k] = make_float4((float)M[k][0], (float)M[k][1], (float)M[k][2], (float)M[k][3]);
                std::vector<RectG> fr;
                for (int k = 0; k < 3; k++)
                    for (int i : F.face[k]) fr.push_back(rect_geom(i, k, M, &F));
                std::vector<char> fused(fr.size(), 0);
                auto fb = use_boxes ? find_boxes(fr, fused) : std::vector<BoxFit>{};
                for (size_t bi = 1; bi < fb.size(); bi++) // one box per frame; further ones stay rects
                    for (int fi = 0; fi < 6; fi++)
                        if (fb[bi].f[fi] >= 0) fused[fb[bi].f[fi]] = 0;
                fb.resize(std::min<size_t>(fb.size(), 1));
                R.rect_first = (int)o.rects.size();
                for (int k = 0; k < 3; k++) {
                    R.n_rect[k] = 0;
                    for (size_t j = 0; j < fr.size(); j++) {
                        if (fused[j] || fr[j].k != k) continue;
                        const int i = fr[j].i;
                        o.rects.push_back(frame_rect(fr[j]));
                        o.rects.back().sg = (int)o.prims.size() << 1;
                        PrimF f = primf(i);
                        const uint32_t fl = H[i].flags | F_FRAME_RECT;
                        std::memcpy(&f.b.w, &fl, 4);
                        push_slot(i, f);
                        R.n_rect[k]++;
                        G.n_flat_extra++;
                        o.nt++;
                    }
                }
                R.box = -1;
                if (!fb.empty()) { // at most one closed box per frame is tested as a box
                    R.box = (int16_t)(frame_box_first + (int)frame_boxes.size());
                    frame_boxes.push_back(box_rec(fr, fb[0], (int)o.prims.size()));
                    for (int fi = 0; fi < 6; fi++) {
                        const int i = box_face_prim(fr, fb[0], fi);
                        PrimF f = primf(i);
                        const uint32_t fl = H[i].flags | F_FRAME_RECT;
                        std::memcpy(&f.b.w, &fl, 4);
                        push_slot(i, f);
                        G.n_flat_extra += fb[0].f[fi] >= 0;
                        o.nt++;
                    }
                }
                o.frames.push_back(R);
            }
            for (const auto& f6 : wboxes) {
                BoxRec B = box_rec(wr, f6, (int)o.prims.size());
                for (int fi = 0; fi < 6; fi++) {
                    const int i = box_face_prim(wr, f6, fi), kind = fi >> 1;
                    PrimF f = primf(i);
                    set_rect_axis(f, H[i].flags, kind);
                    push_slot(i, f);
                    G.n_flat_extra += f6.f[fi] >= 0;
                    o.nr[kind]++;
                }
                FrameRec R;
                std::memcpy(&R, &B, sizeof R);
                o.frames.push_back(R);
            }
            for (const auto& B : frame_boxes) {
                FrameRec R;
                std::memcpy(&R, &B, sizeof R);
                o.frames.push_back(R);
            }
            const int tri_slot = (int)o.prims.size();
            for (int kind = 3; kind < 5; kind++)
                for (int i : g) {
                    if (kind_of[i] != kind || (kind == 3 && in_frame[i])) continue;
                    (kind == 3 ? o.nt : o.ns)++;
                    cnt[kind]++;
                    push_slot(i, primf(i));
                }
            G.lo = make_float4(lo[0], lo[1], lo[2], as_f(rect_first));
            G.hi = make_float4(hi[0], hi[1], hi[2], as_f(tri_slot));
            for (int k = 0; k < 3; k++) G.n_rect[k] = cnt[k];
            G.n_tri_sph = cnt[3] | (cnt[4] << 16);
            if (cnt[3] > 0xFFFF || cnt[4] > 0x7FFF) o.overflow = true;
            if (gi == 0) {
                o.tris0 = cnt[3];
                o.sphs0 = cnt[4];
            }
            o.groups.push_back(G);
        }
        for (int i = 0; i < n; i++) // planes follow
            if (kind_of[i] == 5) {
                o.prims.push_back(primf(i));
                o.tests.push_back(testrec(i));
            }
        o.tests.push_back(TestRec{}); // spare records: loops may load one past a range
        o.rects.push_back(RectRec{});
        o.frames.push_back(FrameRec{});
        return o;
    };
    std::vector<int> all;
    for (int i = 0; i < n; i++)
        if (kind_of[i] != 5) all.push_back(i);
    BruteOrder flat = build_order({all}, {0});
    if (!outer.empty()) {
        std::vector<int> ids;
        for (int i = 0; i < n; i++)
            if (outer[i]) ids.push_back(i);
        out.outer = build_order({ids}, {0});
    }
    int nr[3] = {flat.nr[0], flat.nr[1], flat.nr[2]}, nt = flat.nt, ns = flat.ns, np = 0;
    if (!flat.groups.empty()) {
        const GroupRec& G = flat.groups[0];
        out.layout.rects = G.n_rect[0] + G.n_rect[1] + G.n_rect[2];
        out.layout.boxes = G.n_boxes;
        out.layout.frames = G.n_frames;
        out.layout.frame_boxes = 0;
        out.layout.frame_rects = 0;
        for (int f = 0; f < G.n_frames; f++) {
            const FrameRec& F = flat.frames[G.frame_first + f];
            out.layout.frame_boxes += F.box >= 0;
            out.layout.frame_rects += F.n_rect[0] + F.n_rect[1] + F.n_rect[2];
        }
        out.layout.tris = flat.tris0;
        out.layout.sphs = flat.sphs0;
    }
    for (int i = 0; i < n; i++) np += kind_of[i] == 5;
    // groups: subtrees of the SAH BVH with at most kGroupMax primitives (small scenes only)
    // generic kernel, die.txt 1080p grouped: 2 -> 50.1 ms, 3 -> 47.6, 4 -> 46.4, 6 -> 48.4, 8 -> 48.4, 16 -> 50.7;
    // scene-specialised build (literal operands make primitive tests cheaper than group tests):
    // 2 -> 32.8, 3 -> 30.6, 4 -> 30.2-30.4, 5 -> 28.9, 6 -> 29.1, 7 -> 28.3, 8 -> 28.3, 10 -> 30.2, 16 -> 30.9
    // The size is fixed here, at scene creation, by the process-wide rt_set_jit state then: a
    // later rt_set_jit(0) leaves the generic grouped kernel on groups of 8 (correct, tuned for the
    // specialised build); build statistic 18 (group_max) records the size chosen.
    int kGroupMax = jit_enabled() ? 8 : 4;
    if (const char* e = getenv("RTCORE_GROUP_MAX")) kGroupMax = std::max(1, atoi(e)); // tuning
    out.group_max = kGroupMax;
    // Super records: a subtree (below the root) that the cut makes into at least kSuperMin groups
    // also gets a record of its own box in front of them, so that a wave that misses it skips them
    // all (die.txt: the die's five groups behind one box; background rays then test two boxes
    // instead of six: 6.0 -> 4.69 box tests per ray, C3 26.81 -> 25.64 ms in the same call,
    // profiles/r04/ab_group_super_boxes.log).  RTCORE_GROUP_SUPER sets kSuperMin (0: none).
    int kSuperMin = 3;
    if (const char* e = getenv("RTCORE_GROUP_SUPER")) kSuperMin = std::max(0, atoi(e));
    std::vector<std::vector<int>> cut;
    std::vector<int> skips;
    // Box-aware cut (RTCORE_GROUP_BOXES=1, off): the world rectangles that make closed boxes (the
    // box finder on the whole scene) go to the first group that holds any of them, all together,
    // so that the group's box finder makes them one slab test instead of rectangles spread over
    // several groups (die.txt's cube: 4 + 1 + 1 faces in three groups).  Measured slower on
    // die.txt (C3 26.81 -> 28.73 ms; with super records 25.64 -> 27.56): the group that takes
    // the cube spans the whole die, so nearly every ray that meets the die tests its pips too
    // (sphere tests per ray 4.61 -> 6.18).
    bool group_boxes = false;
    if (const char* e = getenv("RTCORE_GROUP_BOXES")) group_boxes = atoi(e) != 0;
    std::vector<int> box_of(n, -1);
    std::vector<std::vector<int>> box_faces;
    if (group_boxes && use_boxes) {
        std::vector<RectG> wr;
        for (int i : all)
            if (kind_of[i] < 3) wr.push_back(rect_geom(i, kind_of[i], nullptr, nullptr));
        std::vector<char> used(wr.size(), 0);
        for (const BoxFit& f6 : find_boxes(wr, used)) {
            box_faces.emplace_back();
            for (int j : f6.f)
                if (j >= 0) {
                    box_of[wr[j].i] = (int)box_faces.size() - 1;
                    box_faces.back().push_back(wr[j].i);
                }
        }
    }
    std::vector<char> box_done(box_faces.size(), 0);
    auto take_boxes = [&](const std::vector<int>& sub) { // a group's primitives, boxes whole
        std::vector<int> g;
        for (int i : sub) {
            const int b = box_of[i];
            if (b < 0) {
                g.push_back(i);
            } else if (!box_done[b]) {
                box_done[b] = 1;
                g.insert(g.end(), box_faces[b].begin(), box_faces[b].end());
            }
        }
        return g;
    };
    if ((int)all.size() <= 4096 && !sah.order.empty()) {
        std::function<void(int, std::vector<int>&)> leaves = [&](int ref, std::vector<int>& out) {
            if (ref < 0) {
                const int code = ~ref, first = code >> 3, c = (code & 7) + 1;
                for (int k = first; k < first + c; k++) out.push_back(sah.order[k]);
                return;
            }
            int l, r;
            std::memcpy(&l, &sah.nodes[ref].lmin.w, 4);
            std::memcpy(&r, &sah.nodes[ref].rmin.w, 4);
            leaves(l, out);
            leaves(r, out);
        };
        std::function<int(int)> n_cut = [&](int ref) { // groups the cut makes of a subtree
            std::vector<int> sub;
            leaves(ref, sub);
            if ((int)sub.size() <= kGroupMax || ref < 0) return 1;
            int l, r;
            std::memcpy(&l, &sah.nodes[ref].lmin.w, 4);
            std::memcpy(&r, &sah.nodes[ref].rmin.w, 4);
            return n_cut(l) + n_cut(r);
        };
        std::function<void(int, bool)> split = [&](int ref, bool in_super) {
            std::vector<int> sub;
            leaves(ref, sub);
            if ((int)sub.size() <= kGroupMax || ref < 0) {
                std::vector<int> g = take_boxes(sub);
                if (!g.empty()) {
                    cut.push_back(std::move(g));
                    skips.push_back(0);
                }
                return;
            }
            int l, r;
            std::memcpy(&l, &sah.nodes[ref].lmin.w, 4);
            std::memcpy(&r, &sah.nodes[ref].rmin.w, 4);
            const size_t at = cut.size();
            // one level: a super record inside another mostly repeats its box (die.txt: the die
            // and the die minus a face's pips)
            const bool super = kSuperMin > 0 && !in_super && ref != sah.root && n_cut(ref) >= kSuperMin;
            if (super) {
                cut.push_back(sub);
                skips.push_back(0);
            }
            split(l, in_super || super);
            split(r, in_super || super);
            if (super) {
                skips[at] = (int)(cut.size() - at - 1);
                // its box: the primitives of the groups it holds (a box taken whole may reach
                // outside the subtree); a super record holding fewer than two groups is dropped
                cut[at].clear();
                for (size_t k = at + 1; k < cut.size(); k++) cut[at].insert(cut[at].end(), cut[k].begin(), cut[k].end());
                if (skips[at] < 2) {
                    cut.erase(cut.begin() + (long)at);
                    skips.erase(skips.begin() + (long)at);
                }
            }
        };
        split(sah.root, false);
    }
    BruteOrder grouped = cut.empty() ? BruteOrder{} : build_order(cut, skips);
    out.flat = std::move(flat);
    out.grouped = std::move(grouped);
    for (int k = 0; k < 3; k++) out.nr[k] = nr[k];
    out.nt = nt;
    out.ns = ns;
    out.np = np;
    return out;
}

// Materials, deduplicated: one MatF per distinct record, PrimF.d.w its index.  A 1M-triangle
// mesh of one material then shades from a table of a few records (cache-resident) instead of
// gathering 80 B per hit from an 80 MB per-primitive array.
struct MatTable {
    std::vector<MatF> mats;
    std::vector<int32_t> mat_of; // per primitive ID
};
MatTable make_materials(const std::vector<HostPrim>& H, double air_ior)
{
    MatTable t;
    const int n = (int)H.size();
    t.mat_of.resize(n);
    std::unordered_map<std::string, int32_t> mat_index;
    for (int i = 0; i < n; i++) {
        const HostPrim& p = H[i];
        const bool refl = p.shininess > 0; // Primitive.IsReflective (Primitive.cs:107-129)
        rt_color spec = refl ? p.specular : rt_color{0, 0, 0};
        rt_color refr = refl ? p.refraction : rt_color{0, 0, 0};
        MatF m;
        std::memset(&m, 0, sizeof m);
        m.emission = make_float4((float)p.emission.r, (float)p.emission.g, (float)p.emission.b, (float)luminance(p.emission));
        m.diffuse = make_float4((float)p.diffuse.r, (float)p.diffuse.g, (float)p.diffuse.b, (float)luminance(p.diffuse));
        m.specular = make_float4((float)spec.r, (float)spec.g, (float)spec.b, (float)luminance(spec));
        m.refraction = make_float4((float)refr.r, (float)refr.g, (float)refr.b, (float)luminance(refr));
        m.shininess = (float)p.shininess;
        m.ior = (float)p.ior;
        m.flags = p.flags;
        m.inv_shininess = (float)(1.0 / p.shininess);
        // Raytracer.cs:127-133: ratio = iorIn / iorOut, air outside, swapped when the hit is Inside
        m.eta_enter = p.ior != 0 ? (float)(air_ior / p.ior) : 0.0f;
        m.eta_exit = p.ior != 0 ? (float)(p.ior / air_ior) : 0.0f;
        m.pad[0] = m.pad[1] = 0.0f;
        const std::string key(reinterpret_cast<const char*>(&m), sizeof m);
        auto it = mat_index.find(key);
        if (it == mat_index.end()) {
            it = mat_index.emplace(key, (int32_t)t.mats.size()).first;
            t.mats.push_back(m);
        }
        t.mat_of[i] = it->second;
    }
    return t;
}

// The grouped order's records sorted by the distance from the camera to their boxes (stable), as
// a tree: a super record keeps the records it holds (its skip) right behind it, sorted among
// themselves the same way.
std::vector<GroupRec> groups_nearest_first(const std::vector<GroupRec>& g, const CameraD& cam)
{
    const double px = cam.position.x, py = cam.position.y, pz = cam.position.z;
    auto dist2 = [&](const GroupRec& G) {
        // distance from the camera to the group's box (0 inside)
        const double dx = std::max({0.0, (double)G.lo.x - px, px - (double)G.hi.x});
        const double dy = std::max({0.0, (double)G.lo.y - py, py - (double)G.hi.y});
        const double dz = std::max({0.0, (double)G.lo.z - pz, pz - (double)G.hi.z});
        return dx * dx + dy * dy + dz * dz;
    };
    std::vector<GroupRec> out;
    std::function<void(size_t, size_t)> emit = [&](size_t a, size_t b) { // the sibling subtrees in [a, b)
        std::vector<std::pair<size_t, size_t>> sib;
        for (size_t i = a; i < b; i += 1 + (size_t)std::max(0, g[i].skip))
            sib.push_back({i, std::min(b, i + 1 + (size_t)std::max(0, g[i].skip))});
        std::stable_sort(sib.begin(), sib.end(), [&](const auto& x, const auto& y) { return dist2(g[x.first]) < dist2(g[y.first]); });
        for (const auto& [i, e] : sib) {
            out.push_back(g[i]);
            emit(i + 1, e);
        }
    };
    emit(0, g.size());
    return out;
}

// The fp32 transform rows of a transformed sphere (XformF).
XformF make_xformf(const HostPrim& p)
{
    XformF F;
    const double c[3] = {p.center.x, p.center.y, p.center.z};
    for (int r = 0; r < 3; r++) {
        F.to_world[r] = make_float4((float)p.to_world[4 * r], (float)p.to_world[4 * r + 1], (float)p.to_world[4 * r + 2],
                                    (float)p.to_world[4 * r + 3]);
        // normal(p) = N3 * (W * p + w - c) / r: one affine map of the world hit point
        double row[4] = {0, 0, 0, 0};
        for (int k = 0; k < 3; k++) {
            const double nk = p.to_normal[4 * r + k] / p.radius;
            for (int j = 0; j < 3; j++) row[j] += nk * p.to_world[4 * k + j];
            row[3] += nk * (p.to_world[4 * k + 3] - c[k]);
        }
        F.normal[r] = make_float4((float)row[0], (float)row[1], (float)row[2], (float)row[3]);
    }
    return F;
}

// What the scene's primitives and materials use at all (FACT_*, rt_internal.h).
uint32_t scene_facts(const std::vector<HostPrim>& H)
{
    uint32_t facts = 0;
    for (const HostPrim& p : H) {
        if (std::isinf(p.shininess) && p.shininess > 0) facts |= FACT_INF_SHININESS;
        if ((float)p.ior != 0.0f) facts |= FACT_IOR;
        if (p.flags & F_TRANSFORMED) facts |= FACT_XF;
        if (p.flags & F_HASNORMALS) facts |= FACT_VN;
        if (p.kind == RT_PRIM_SPHERE) facts |= FACT_SPHERE;
    }
    return facts;
}

int upload_scene(rt_scene* s)
{
    const auto& H = s->host;
    const int n = (int)H.size();
    // --- exact fp64 set
    std::vector<PrimD> pd(n);
    std::vector<XformD> xd;
    std::vector<float4> vn((size_t)std::max(1, n) * 3, make_float4(0, 0, 0, 0));
    std::vector<XformF> xf;
    std::vector<int> xf_index(n, -1);
    for (int i = 0; i < n; i++) {
        const HostPrim& p = H[i];
        PrimD& d = pd[i];
        std::memset(&d, 0, sizeof d);
        d.flags = p.flags;
        d.xf = -1;
        if (p.kind == RT_PRIM_TRIANGLE) {
            d.a = p.v[0];
            d.b = p.e01;
            d.c = p.e02;
            d.d = p.n;
            for (int k = 0; k < 3; k++) {
                d.vn[k] = p.vn[k];
                vn[3 * i + k] = f4(p.vn[k], 0.0f);
            }
        } else if (p.kind == RT_PRIM_SPHERE) {
            d.a = p.center;
            d.b = v4d(p.radius, p.radius_sqr, 0, 0);
            if (p.flags & F_TRANSFORMED) {
                d.xf = (int)xd.size();
                xf_index[i] = (int)xf.size();
                XformD X;
                std::memcpy(X.to_world, p.to_world, sizeof X.to_world);
                std::memcpy(X.to_obj, p.to_obj, sizeof X.to_obj);
                std::memcpy(X.to_normal, p.to_normal, sizeof X.to_normal);
                xd.push_back(X);
                xf.push_back(make_xformf(p));
            }
        } else {
            d.a = p.pn;
            d.b = v4d(p.pd, 0, 0, 0);
        }
    }
    // --- fast fp32 set
    auto primf = [&](int i) { return make_primf(H, xf_index, i); };
    auto testrec = [&](int i) { return make_testrec(H, xf_index, i); };
    BruteOrders orders = make_brute_orders(H, xf_index, s->sah, s->bvh_outer);
    BruteOrder& flat = orders.flat;
    BruteOrder& grouped = orders.grouped;
    s->flat_overflow = flat.overflow;
    int nr[3] = {orders.nr[0], orders.nr[1], orders.nr[2]}, nt = orders.nt, ns = orders.ns, np = orders.np;
    {
        const BruteLayout& L = orders.layout;
        s->layout.rects = L.rects;
        s->layout.group_max = orders.group_max;
        s->layout.boxes = L.boxes;
        s->layout.frames = L.frames;
        s->layout.frame_boxes = L.frame_boxes;
        s->layout.frame_rects = L.frame_rects;
        s->layout.tris = L.tris;
        s->layout.sphs = L.sphs;
    }
    // Materials, deduplicated (make_materials), and the scene facts
    const MatTable mt = make_materials(H, s->params.air_ior);
    const std::vector<MatF>& mats = mt.mats;
    const std::vector<int32_t>& mat_of = mt.mat_of;
    uint32_t facts = scene_facts(H);
    if (getenv("RTCORE_NO_FACTS")) facts = FACT_ALL; // A/B: every shading feature compiled in
    auto set_mats = [&](std::vector<PrimF>& v) { // PrimF.d.w = the material of the record's ID
        for (PrimF& f : v) {
            int32_t id;
            std::memcpy(&id, &f.a.w, 4);
            f.d.w = as_f(mat_of[id]);
        }
    };
    set_mats(flat.prims);
    set_mats(grouped.prims);
    // The BVH order: the tree's slots (host: s->sah.order; GPU: gathered on the device), then the
    // outer records' slots (their records renumbered past the tree), then the planes -- the tail,
    // built here for both builders.
    std::vector<PrimF> bv;
    std::vector<TestRec> tbv;
    const int n_tree = s->bvh.builder == RT_BVH_BUILDER_GPU
                           ? (s->order_d.n > 0 ? (int)s->order_d.n - np - 1 : 0)
                           : (int)s->sah.order.size();
    {
        BruteOrder& ob = orders.outer;
        if (!ob.groups.empty()) {
            const int n_slots = (int)ob.prims.size() - np;
            bv.insert(bv.end(), ob.prims.begin(), ob.prims.begin() + n_slots);
            tbv.insert(tbv.end(), ob.tests.begin(), ob.tests.begin() + n_slots);
            for (RectRec& r : ob.rects) r.sg += n_tree << 1;
            const GroupRec& G = ob.groups[0];
            for (int j = G.frame_first + G.n_frames; j < G.frame_first + G.n_frames + G.n_boxes; j++) {
                BoxRec B;
                std::memcpy(&B, &ob.frames[j], sizeof B);
                B.sg0 += n_tree << 1;
                std::memcpy(&ob.frames[j], &B, sizeof B);
            }
        }
        for (int i = 0; i < n; i++) // planes follow the BVH's primitives in both orders
            if (H[i].kind == RT_PRIM_PLANE) {
                bv.push_back(primf(i));
                tbv.push_back(testrec(i));
            }
    }
    const size_t n_bvh_records = (size_t)n_tree + bv.size();
    set_mats(bv);
    if (s->bvh.builder == RT_BVH_BUILDER_GPU) {
        // the tree's records in ID order, gathered on the device into the GPU builder's leaf order
        std::vector<PrimF> pid(n);
        std::vector<TestRec> tid(n);
        parallel_for(n, [&](int i) {
            pid[i] = primf(i);
            tid[i] = testrec(i);
        });
        DevBuf<PrimF> pid_d;
        DevBuf<TestRec> tid_d;
        set_mats(pid);
        HIP_TRY(pid_d.upload(pid));
        HIP_TRY(tid_d.upload(tid));
        HIP_TRY(s->prims_bvh.reserve(n_bvh_records));
        HIP_TRY(s->tests_bvh.reserve(n_bvh_records + kTestSpares));
        HIP_TRY(gather_bvh_records(s->order_d.p, n_tree, pid_d.p, tid_d.p, s->prims_bvh.p, s->tests_bvh.p, s->stream));
        if (!bv.empty()) {
            HIP_TRY(hipMemcpyAsync(s->prims_bvh.p + n_tree, bv.data(), bv.size() * sizeof(PrimF), hipMemcpyHostToDevice,
                                   s->stream));
            HIP_TRY(hipMemcpyAsync(s->tests_bvh.p + n_tree, tbv.data(), tbv.size() * sizeof(TestRec),
                                   hipMemcpyHostToDevice, s->stream));
        }
        // spare records: the BVH leaf step loads up to kTestSpares past a leaf
        HIP_TRY(hipMemsetAsync(s->tests_bvh.p + n_bvh_records, 0, kTestSpares * sizeof(TestRec), s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
        s->order_d.release();
    } else {
        std::vector<PrimF> tree(n_tree);
        std::vector<TestRec> ttree(n_tree);
        parallel_for(n_tree, [&](int k) {
            tree[k] = primf(s->sah.order[k]);
            ttree[k] = testrec(s->sah.order[k]);
        });
        set_mats(tree);
        bv.insert(bv.begin(), tree.begin(), tree.end());
        tbv.insert(tbv.begin(), ttree.begin(), ttree.end());
    }
    HIP_TRY(s->prims_d.upload(pd));
    HIP_TRY(s->xf_d.upload(xd));
    HIP_TRY(s->prims_bf.upload(flat.prims));
    HIP_TRY(s->tests_bf.upload(flat.tests));
    HIP_TRY(s->rects_bf.upload(flat.rects));
    HIP_TRY(s->frames_bf.upload(flat.frames));
    HIP_TRY(s->groups_bf.upload(flat.groups));
    HIP_TRY(s->prims_gr.upload(grouped.prims));
    HIP_TRY(s->tests_gr.upload(grouped.tests));
    HIP_TRY(s->rects_gr.upload(grouped.rects));
    HIP_TRY(s->frames_gr.upload(grouped.frames));
    HIP_TRY(s->groups_gr.upload(grouped.groups));
    s->groups_gr_host = grouped.groups;
    s->flat_h = {flat.groups, flat.rects, flat.frames, flat.tests};
    s->grouped_h = {grouped.groups, grouped.rects, grouped.frames, grouped.tests};
    s->xf_h = xf;
    if (s->bvh.builder != RT_BVH_BUILDER_GPU) {
        HIP_TRY(s->prims_bvh.upload(bv));
        tbv.resize(tbv.size() + kTestSpares, TestRec{}); // spare records: the BVH leaf step loads past a leaf
        HIP_TRY(s->tests_bvh.upload(tbv));
        HIP_TRY(s->nodes.upload(s->sah.nodes));
        HIP_TRY(s->nodes4.upload(s->bvh4.nodes));
    }
    if (!orders.outer.groups.empty()) {
        HIP_TRY(s->rects_bvh.upload(orders.outer.rects));
        HIP_TRY(s->frames_bvh.upload(orders.outer.frames));
        HIP_TRY(s->groups_bvh.upload(orders.outer.groups));
    }
    HIP_TRY(s->xf.upload(xf));
    HIP_TRY(s->mats.upload(mats));
    HIP_TRY(s->vnormals.upload(vn));
    s->device_bytes = pd.size() * sizeof(PrimD) + xd.size() * sizeof(XformD) +
                      (flat.prims.size() + grouped.prims.size() + n_bvh_records) * sizeof(PrimF) +
                      (flat.tests.size() + grouped.tests.size() + n_bvh_records + 1) * sizeof(TestRec) +
                      (size_t)s->bvh.n_nodes2 * sizeof(NodeF) + (size_t)s->bvh.n_nodes4 * sizeof(Node4Q) +
                      xf.size() * sizeof(XformF) + mats.size() * sizeof(MatF) + vn.size() * sizeof(float4);

    // Compact leaves: the BVH order's 48-B rows, and every leaf whose primitives share their kind and
    // test flags referenced as a compact leaf (RTCORE_COMPACT_LEAVES=0 keeps them generic, for A/B)
    {
        const char* e = getenv("RTCORE_COMPACT_LEAVES");
        const bool rewrite = !(e && e[0] == '0');
        const size_t n_rec = n_bvh_records + kTestSpares;
        HIP_TRY(s->rows_bvh.reserve(3 * n_rec));
        HIP_TRY(compact_leaves(s->tests_bvh.p, (int)n_rec, s->rows_bvh.p, s->nodes.p, s->bvh.n_nodes2, s->nodes4.p,
                               s->bvh.n_nodes4, rewrite, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
    }
    // Hot table: the first kHot wide nodes in breadth-first order from the root, their references
    // to each other rewritten to RT_HOT_BIT | hot index (the global tree is unchanged).
    std::vector<Node4Q> hot;
    int root4_hot = s->bvh.root4;
    {
        std::vector<Node4Q> all4((size_t)s->bvh.n_nodes4);
        if (!all4.empty())
            HIP_TRY(hipMemcpy(all4.data(), s->nodes4.p, all4.size() * sizeof(Node4Q), hipMemcpyDeviceToHost));
        s->bvh.leaves4 = s->bvh.compact4 = 0; // build statistics: the wide tree's leaves, compact ones
        for (const Node4Q& nd : all4)
            for (float f : {nd.c.z, nd.c.w, nd.d.x, nd.d.y}) {
                int32_t c;
                std::memcpy(&c, &f, 4);
                if (c < 0 && c != RT_NODE4_EMPTY) {
                    s->bvh.leaves4++;
                    s->bvh.compact4 += ((~c) & kLeafCompact) != 0;
                }
            }
        int k_hot = 64; // with the 16-entry LDS stack: 7 blocks x (16 + 4) KB per CU
        if (const char* e = getenv("RTCORE_HOT_NODES")) k_hot = std::max(0, std::min(1024, atoi(e)));
        if (k_hot > 0 && s->bvh.root4 >= 0 && s->bvh.n_nodes4 > 0) {
            std::vector<int> order{s->bvh.root4};
            std::unordered_map<int, int> slot_of{{s->bvh.root4, 0}};
            for (size_t q = 0; q < order.size() && (int)order.size() < k_hot; q++) {
                const Node4Q& nd = all4[order[q]];
                int32_t ch[4];
                std::memcpy(&ch[0], &nd.c.z, 4);
                std::memcpy(&ch[1], &nd.c.w, 4);
                std::memcpy(&ch[2], &nd.d.x, 4);
                std::memcpy(&ch[3], &nd.d.y, 4);
                for (int c : ch)
                    if (c >= 0 && (int)order.size() < k_hot && !slot_of.count(c)) {
                        slot_of[c] = (int)order.size();
                        order.push_back(c);
                    }
            }
            for (int g : order) {
                Node4Q nd = all4[g];
                float* refs[4] = {&nd.c.z, &nd.c.w, &nd.d.x, &nd.d.y};
                for (float* r : refs) {
                    int32_t c;
                    std::memcpy(&c, r, 4);
                    auto it = c >= 0 ? slot_of.find(c) : slot_of.end();
                    if (it != slot_of.end()) {
                        c = RT_HOT_BIT | it->second;
                        std::memcpy(r, &c, 4);
                    }
                }
                hot.push_back(nd);
            }
            root4_hot = RT_HOT_BIT | 0;
        }
    }
    HIP_TRY(s->hot4.upload(hot));

    DevScene& d = s->dev;
    d.hot4 = s->hot4.p;
    d.n_hot4 = (int)hot.size();
    d.root4_hot = root4_hot;
    d.tests_bf = s->tests_bf.p;
    d.tests_bvh = s->tests_bvh.p;
    d.rows_bvh = s->rows_bvh.p;
    d.rects_bf = s->rects_bf.p;
    d.frames_bf = s->frames_bf.p;
    d.prims_bf = s->prims_bf.p;
    d.groups_bf = s->groups_bf.p;
    d.tests_gr = s->tests_gr.p;
    d.rects_gr = s->rects_gr.p;
    d.frames_gr = s->frames_gr.p;
    d.prims_gr = s->prims_gr.p;
    d.groups_gr = s->groups_gr.p;
    d.n_groups_gr = (int)grouped.groups.size();
    // slots before the planes, per order (open boxes add placeholder slots to the brute orders)
    d.pln0_bf = (int)flat.prims.size() - np;
    d.pln0_gr = grouped.prims.empty() ? 0 : (int)grouped.prims.size() - np;
    d.pln0_bvh = (int)n_bvh_records - np;
    d.rects_bvh = s->rects_bvh.p;
    d.frames_bvh = s->frames_bvh.p;
    d.groups_bvh = s->groups_bvh.p;
    d.n_outer = orders.outer.groups.empty() ? 0 : 1;
    for (int k = 0; k < 3; k++) d.n_rect[k] = nr[k];
    d.n_tri = nt;
    d.n_sph = ns;
    d.n_pln = np;
    d.prims_bvh = s->prims_bvh.p;
    d.nodes = s->nodes.p;
    d.n_nodes = s->bvh.n_nodes2;
    d.root = s->bvh.root2;
    d.nodes4 = s->nodes4.p;
    d.n_nodes4 = s->bvh.n_nodes4;
    d.root4 = s->bvh.root4;
    d.xf = s->xf.p;
    d.mats = s->mats.p;
    d.vnormals = s->vnormals.p;
    d.n_mats = (int)mats.size();
    d.n_xf = (int)xf.size();
    d.facts = facts;
    d.n_vn = 0;
    for (const HostPrim& p : H) d.n_vn += (p.kind == RT_PRIM_TRIANGLE && (p.flags & F_HASNORMALS)) ? 1 : 0;
    d.prims_d = s->prims_d.p;
    d.xf_d = s->xf_d.p;
    d.ref_nodes = nullptr; // built on first use (ensure_ref_bvh)
    d.n_ref_nodes = 0;
    d.width = s->params.width;
    d.height = s->params.height;
    d.recursion = s->params.recursion;
    d.debug_geom = s->params.debug_geom;
    d.air_ior = (float)s->params.air_ior;
    const rt_color& a = s->params.ambient;
    d.ambient = make_float3((float)a.r, (float)a.g, (float)a.b);
    d.ambient_miss = (a.r == -1 && a.g == -1 && a.b == -1) ? 1 : 0; // AmbientRGB == Placeholder
    return RT_OK;
}

// The reference agglomerative BVH (BVH.cs:12-236) serves only the exact debug passes; it is built
// and uploaded on first use, so a render-only scene does not pay for it (5.8 s for 1 M triangles).
int ensure_ref_bvh(rt_scene* s)
{
    if (s->ref_built) return RT_OK;
    s->ref = build_ref_bvh(s->host);
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(s->ref_nodes.upload(s->ref.nodes));
    s->dev.ref_nodes = s->ref_nodes.p;
    s->dev.n_ref_nodes = (int)s->ref.nodes.size();
    s->device_bytes += s->ref.nodes.size() * sizeof(RefNode);
    s->ref_built = true;
    return RT_OK;
}

int resolve_traversal(rt_scene* s)
{
    int t = s->traversal;
    if (t == RT_TRAVERSAL_AUTO) {
        const int n_bvh = s->dev.pln0_bvh; // primitives other than planes
        t = n_bvh <= 48 ? RT_TRAVERSAL_BRUTE : RT_TRAVERSAL_BVH;
    }
    if (s->traversal == RT_TRAVERSAL_AUTO && t == RT_TRAVERSAL_BRUTE && s->grouped_measured > 1.25)
        t = RT_TRAVERSAL_GROUPED;
    if (t == RT_TRAVERSAL_GROUPED && s->dev.n_groups_gr == 0) t = RT_TRAVERSAL_BRUTE; // too big to group
    if (t == RT_TRAVERSAL_BRUTE && s->flat_overflow) {
        set_error("brute-force traversal: more than 65535 triangles or 32767 spheres in the flat order");
        return RT_ERR_ARG;
    }
    // kernel: 0 brute force, 1 grouped brute force, 2 BVH2 (24 + kStackOverflow stack entries),
    // 3 wide BVH (RT_WIDE_STACK + kStackOverflow)
    int kernel = t == RT_TRAVERSAL_GROUPED ? 1 : 0;
    if (t == RT_TRAVERSAL_BVH2) {
        if (s->bvh.depth2 >= 24 + kStackOverflow) {
            set_error("BVH2 deeper than the kernel's traversal stack");
            return RT_ERR_ARG;
        }
        kernel = 2;
    } else if (t == RT_TRAVERSAL_BVH) {
        if (s->bvh.stack4 > path_wide_stack() + kStackOverflow) {
            set_error("wide BVH needs a deeper traversal stack than the kernel's");
            return RT_ERR_ARG;
        }
        kernel = 3;
    }
    s->resolved = t;
    // Stage the shading records in LDS when that costs no occupancy (RTCORE_PATH_LDS=0/1 forces
    // the choice for A/B measurements).
    const size_t lds = path_lds_bytes(s->dev);
    const int plain = path_variant(kernel, false), staged = path_variant(kernel, true);
    const int occ_plain = path_blocks_per_cu(plain, path_dyn_lds(s->dev, plain), false, s->dev.n_vn > 0);
    const int occ_staged = lds <= 64 * 1024 ? path_blocks_per_cu(staged, path_dyn_lds(s->dev, staged), false, s->dev.n_vn > 0) : 0;
    // The scene-specialised build (rt_set_jit) is a build of the staged brute-force variant, and its
    // occupancy is its own: with it on, a brute-force order stays staged whenever the records fit.
    bool use_lds = occ_staged >= occ_plain || (kernel <= 1 && occ_staged > 0 && jit_enabled());
    if (const char* e = getenv("RTCORE_PATH_LDS")) use_lds = e[0] == '1' && occ_staged > 0;
    s->variant = use_lds ? staged : plain;
    s->blocks_per_cu = use_lds ? occ_staged : occ_plain;
    if (s->stats_on) s->stats_blocks_per_cu = path_blocks_per_cu(s->variant, path_dyn_lds(s->dev, s->variant), true, s->dev.n_vn > 0);
    return RT_OK;
}

PathParams make_params(rt_scene* s, int x0, int y0, int w, int h, int spp, uint64_t seed, uint64_t base,
                       double chunk_npix = 0.0);
int run_path(rt_scene* s, PathParams& p, unsigned long long* d_rays, hipStream_t stream, bool timed = true);
int prepare_jit(rt_scene* s);
int end_op(rt_scene* s, hipStream_t stream);

// AUTO on a small scene: flat or grouped brute force?  Whether a group can be skipped depends on
// how coherent a wave's rays are, which the camera decides, so each camera is calibrated once:
// the grouped kernel's instrumented variant renders a fixed 64x64 tile at 2 spp and counts the
// primitive tests it actually made.  The choice is a function of scene, camera and that fixed
// sample only (no timing), so it is the same on every run.
int calibrate_grouping(rt_scene* s)
{
    s->grouped_measured = 0;
    if (s->traversal != RT_TRAVERSAL_AUTO || s->dev.n_groups_gr < 2) return RT_OK;
    const int n_bvh = s->dev.pln0_bvh; // primitives other than planes
    if (n_bvh > 48) return RT_OK;
    const int w = std::min(64, s->params.width), h = std::min(64, s->params.height);
    const int x0 = (s->params.width - w) / 2, y0 = (s->params.height - h) / 2;
    const int saved_variant = s->variant, saved_blocks = s->blocks_per_cu;
    const int variant = path_variant(1, false);
    s->variant = variant;
    s->blocks_per_cu = path_blocks_per_cu(variant, 0, true, s->dev.n_vn > 0);
    HIP_TRY(s->stats_buf.reserve(RT_STATS_COUNT));
    HIP_TRY(s->sum.reserve((size_t)3 * w * h));
    HIP_TRY(s->samples.reserve((size_t)w * h));
    HIP_TRY(s->misses.reserve((size_t)w * h));
    HIP_TRY(hipMemsetAsync(s->stats_buf.p, 0, RT_STATS_COUNT * sizeof(unsigned long long), s->stream));
    HIP_TRY(hipMemsetAsync(s->rays.p, 0, sizeof(unsigned long long), s->stream));
    const bool was_on = s->stats_on;
    const int was_blocks = s->stats_blocks_per_cu;
    s->stats_on = true;
    s->stats_blocks_per_cu = s->blocks_per_cu;
    PathParams p = make_params(s, x0, y0, w, h, 2, 0x5EEDull, 0);
    p.pool = 64; // one chunk per pool: the counts must not depend on the pool size
    int rc = run_path(s, p, s->rays.p, s->stream, false); // an internal probe: not in rt_kernel_times
    if (rc == RT_OK) rc = end_op(s, s->stream);
    s->stats_on = was_on;
    s->stats_blocks_per_cu = was_blocks;
    s->variant = saved_variant;
    s->blocks_per_cu = saved_blocks;
    if (rc != RT_OK) return rc;
    unsigned long long st[RT_STATS_COUNT], rays = 0;
    HIP_TRY(hipMemcpyAsync(st, s->stats_buf.p, sizeof st, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipMemcpyAsync(&rays, s->rays.p, sizeof rays, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    HIP_TRY(hipMemsetAsync(s->stats_buf.p, 0, RT_STATS_COUNT * sizeof(unsigned long long), s->stream));
    if (rays == 0) return RT_OK;
    // relative costs of a rect/triangle test, a sphere test and a group box test (instruction counts)
    const double flat = 20.0 * (n_bvh - s->dev.n_sph) + 30.0 * s->dev.n_sph;
    const double grouped = (15.0 * st[0] + 20.0 * st[1] + 30.0 * st[2]) / (double)rays; // st[0]: box tests made
    s->grouped_measured = flat / std::max(grouped, 1e-9);
    return resolve_traversal(s);
}

// chunk_npix (default w * h): the pixel count the chunks per pixel are chosen for.  A column band of a
// tile passes the whole tile's, so that every pixel's samples fall into the same chunks (and its
// fp64 sum into the same order) as in one launch over the tile.
PathParams make_params(rt_scene* s, int x0, int y0, int w, int h, int spp, uint64_t seed, uint64_t base,
                       double chunk_npix)
{
    PathParams p{};
    p.x0 = x0;
    p.y0 = y0;
    p.w = w;
    p.h = h;
    p.band = 0;
    p.spp = spp;
    // a few chunks per pixel keep the tail of a launch short while each lane still amortises
    // its item fetch over many samples (RTCORE_PATH_CHUNKS overrides the count, for tuning).
    // A launch over fewer pixels than a 1080p frame takes proportionally more chunks per pixel
    // (up to 8 x the base count: 192 for the brute-force kernels, 512 for the BVH kernels; the
    // partial buffer is 16 B x chunks x padded pixels), so that a band set of 1/N of the frame at N x the samples (bench.py on N GPUs)
    // gets items as short as one GPU's whole-frame launch, and with them the same launch tail.
    // The BVH kernels take twice as many (C4 at 64 spp: one sample per item; 16 / 32 / 64 chunks
    // 58.7 / 55.0-55.2 / 53.7 ms): their items start in batched shading phases, so a short item
    // costs little, and the tail of a launch of long, divergent BVH paths shrinks.
    // Brute-force kernels: 24 chunks (round 6, after the xorshift stream; same call, two rounds,
    // profiles/r06/chunk_sweep3.log, ms per step): C2 16 / 20 / 24 / 28 / 32 chunks 17.12 / 16.86 /
    // 16.84-16.86 / 16.85-16.87 / 16.98; C3 22.16-22.29 / 21.49-21.50 / 21.42-21.43 / 21.43-21.46 /
    // 21.86-21.93.  Fewer, longer items (and fewer partials to fold) until the launch tail grows;
    // 24 chunks leave 8 of the 32 power-of-two chunk slots empty, items the refill skips.
    const int base_chunks = (s->variant >> 1) >= 2 ? 64 : 24;
    int chunks = base_chunks;
    const double npix = chunk_npix > 0.0 ? chunk_npix : (double)w * (double)h;
    if (npix > 0 && npix < 2073600.0)
        chunks = (int)std::min(8.0 * base_chunks, base_chunks * std::ceil(2073600.0 / npix));
    // A larger frame has more items, so a relatively shorter tail: fewer, longer items then save
    // item switches and partials (die.txt 4K x 512 spp: 8 / 16 / 32 / 64 chunks -> 55.2 / 55.6 /
    // 56.6-57.0 / 57.0 ms kernel, 55.8 / 56.3-56.5 / 57.8-58.1 / 59.0 ms per step).
    else if (npix > 2073600.0)
        chunks = (int)std::max(base_chunks / 4.0, std::ceil(base_chunks * 2073600.0 / npix));
    if (const char* e = getenv("RTCORE_PATH_CHUNKS")) chunks = std::max(1, atoi(e));
    p.chunk = std::max(1, std::min(64, (spp + chunks - 1) / chunks));
    const int used = (spp + p.chunk - 1) / p.chunk;
    p.log2_chunks = 0;
    while ((1 << p.log2_chunks) < used) p.log2_chunks++;
    p.n_chunks = 1 << p.log2_chunks; // work items: ((block << log2_chunks) + chunk) * 64 + pixel
    p.blocks_x = (w + 7) / 8;
    p.n_pad = p.blocks_x * ((h + 7) / 8) * 64;
    p.inv_blocks_x = 1.0f / (float)p.blocks_x;
    // Item decode by multiply-high (one v_mul_hi_u32) instead of the fp32-reciprocal divmod: exact
    // for every block index x when x * (M * blocks_x - 2^32) < 2^32, M = ceil(2^32 / blocks_x).
    p.magic_bx = 0;
    if (p.blocks_x > 1 && !getenv("RTCORE_NO_MAGIC_DIV")) { // (the env variable: A/B of the decode)
        const uint64_t M = ((1ull << 32) + (uint64_t)p.blocks_x - 1) / (uint64_t)p.blocks_x;
        const uint64_t err = M * (uint64_t)p.blocks_x - (1ull << 32);
        const uint64_t max_blk = (uint64_t)(p.n_pad / 64);
        if (M < (1ull << 32) && max_blk * err < (1ull << 32)) p.magic_bx = (unsigned)M;
    }
    // One device-scope atomic hands a wave p.pool items.  64 per atomic made the dispenser a
    // bottleneck (measured, 1080p: die.txt grouped 50.9 -> 47.0 ms with 256, 48.2 with 128 or 512;
    // bounce.txt flat 33.4 -> 33.0 ms with 128, 33.6 with 256; mesh BVH 82.2 -> 80.3 with 256).
    // With the XCD-local dispensers (8 words instead of one) smaller pools pay again (round 3, pool
    // multiples 1 / 2 / 4 / 8): flat brute force C2 19.54-19.57 / 19.63-19.69 / 20.05 ms, the BVH
    // kernels C4 44.54-44.57 / 44.25-44.28 / 45.0-45.2 / 46.8 ms; grouped C3 27.81 / - / 27.58-27.64.
    const int kernel = s->variant >> 1;
    // Round 6, with the 24-chunk items (longer items, so fewer per atomic; profiles/r06/pool_sweep2.log):
    // grouped C3 pool multiples 2 / 4 / 8: 19.93 / 20.36-20.38 / 21.51-21.57 ms; flat C2 1 / 2: 16.27-16.28 /
    // 16.42-16.49 ms.
    int pool_mul = kernel == 0 ? 1 : 2;
    if (const char* e = getenv("RTCORE_POOL_MUL")) pool_mul = std::max(1, std::min(64, atoi(e)));
    p.pool = 64;
    while (p.pool < 64 * pool_mul && p.pool < 64 * p.n_chunks) p.pool *= 2;
    // BVH kernels: the shading phase runs once 28 lanes wait; a leaf step once 12 lanes are blocked
    // on a pending leaf.  Round 5, C4 with the walls as outer records (profiles/r05/c4_outer_sweep.log):
    // refill 24 / 28 / 32 at spec 16: 44.0 / 43.6 / 43.6 ms; spec 12 / 16 / 20 at refill 24: 43.8 /
    // 44.0 / 44.5; refill 28 + spec 12 (+ leaves of <= 2): 43.2 (43.0).  Earlier tree (round 2):
    // refill 8 / 16 / 20 / 24 / 28 / 32: 71.8 / 64.3 / 63.2 / 62.1-62.6 / 62.9 / 63.6 ms.
    p.refill = 28;
    if (const char* e = getenv("RTCORE_BVH_REFILL")) p.refill = std::max(1, std::min(64, atoi(e)));
    p.spec = 12;
    if (const char* e = getenv("RTCORE_BVH_SPEC")) p.spec = std::max(1, std::min(64, atoi(e)));
    // XCD-local item ranges: the 8x8 blocks cut into kMaxSplit runs of consecutive blocks (horizontal
    // strips of the tile), each dealt first to the workgroups of one XCD, so that one XCD's waves work
    // on neighbouring pixels and their closest-hit queries share that XCD's L2.  A single range hands
    // the whole frame out in order to all XCDs at once: every L2 then holds the nodes of the same
    // band.  RTCORE_XCD_SPLIT=0 turns it off (A/B).
    p.n_split = 1;
    const int n_blocks = p.n_pad / 64;
    int want = kMaxSplit;
    if (const char* e = getenv("RTCORE_XCD_SPLIT")) want = atoi(e) > 0 ? kMaxSplit : 1;
    if (want > 1 && n_blocks >= 4 * kMaxSplit) p.n_split = kMaxSplit;
    for (int g = 0; g <= p.n_split; g++)
        p.split_start[g] = (unsigned)((int64_t)n_blocks * g / p.n_split) * (unsigned)(p.n_chunks * 64);
    p.seed = seed;
    p.seed_key = rt_rng_seed_key(seed);
    p.sample_base = base;
    return p;
}

// Band-set launch: tile row r is frame row ((r / band) * stride + offset) * band + r % band; the
// kernel divides by a shift for power-of-two bands, else by the fp32 reciprocal.
void set_band(PathParams& p, int band, int stride, int offset)
{
    p.band = band;
    p.band_stride = stride;
    p.band_offset = offset;
    p.band_log2 = -1;
    for (int k = 0; k < 31; k++)
        if (band == (1 << k)) p.band_log2 = k;
    p.inv_band = 1.0f / (float)band;
}

int check_tile(rt_scene* s, int x0, int y0, int w, int h)
{
    if (!s) {
        set_error("null scene");
        return RT_ERR_ARG;
    }
    if (!s->has_camera) {
        set_error("no camera set (rt_scene_set_camera)");
        return RT_ERR_STATE;
    }
    if (w <= 0 || h <= 0 || x0 < 0 || y0 < 0 || x0 + w > s->params.width || y0 + h > s->params.height) {
        set_error("tile outside the frame");
        return RT_ERR_ARG;
    }
    return RT_OK;
}

// The scene-specialised kernel (rt_jit.h) of the current brute-force variant, built on first use
// and again after a group-order change.  Returns 1 when it is to be launched, 0 to launch the
// generic kernel: JIT off, the instrumented kernel, a BVH or unstaged variant, or a failed build
// (the generic kernel computes the same; the failure is kept in s->jit.error).
int prepare_jit(rt_scene* s)
{
    // Both brute-force orders (RTCORE_JIT_GROUPED=0 leaves the grouped one generic).  The grouped
    // order's group loop is unrolled by pragma: left to the compiler's heuristics it stayed a loop
    // over constant memory and ran slower than the generic kernel (die.txt 36.6 -> 37.9 ms);
    // unrolled, die.txt C3 36.6 -> 30.9 ms.
    const char* eg = getenv("RTCORE_JIT_GROUPED");
    const bool grouped_ok = !(eg && eg[0] == '0');
    const bool eligible = jit_enabled() && !s->stats_on &&
                          (s->variant == path_variant(0, true) || (grouped_ok && s->variant == path_variant(1, true)));
    if (!eligible) {
        s->jit.status = 0;
        return 0;
    }
    const bool grouped = s->variant == path_variant(1, true);
    const unsigned gen = s->jit_gen;
    if (s->jit.variant == s->variant && s->jit.gen == gen) { // built (or failed) already
        s->jit.status = s->jit.fn ? 1 : (s->jit.error.empty() ? 0 : -1);
        return s->jit.fn ? 1 : 0;
    }
    PathParams lp{};
    fill_launch(s->dev, s->variant, lp);
    const auto& B = grouped ? s->grouped_h : s->flat_h;
    // The grouped order's build carries the camera (its group order is per camera anyway); the flat
    // order's only the camera's kind and depth-of-field switch, so moving the camera among cameras
    // of one kind (MainWindow.cs:262-269 restarts the render with another scene camera) reuses the
    // build: the same header, no hiprtc build and no cache lookup.
    static const bool cam_in = getenv("RTCORE_JIT_CAMERA") && getenv("RTCORE_JIT_CAMERA")[0] == '1'; // A/B: round 3's form
    const std::string header =
        jit_scene_header(lp.scene, s->camf, grouped || cam_in, B.groups, B.rects, B.frames, B.tests, s->xf_h);
    if (s->jit.variant == s->variant && s->jit.fn && header == s->jit.header) {
        s->jit.gen = gen;
        s->jit.status = 1;
        s->jit.compile_ms = 0;
        s->jit.from_cache = true;
        return 1;
    }
    s->jit.error.clear();
    s->jit.variant = s->variant;
    s->jit.gen = gen;
    s->jit.header = header;
    if (s->jit.fn) jit_release(s->device, s->jit.fn); // launches still queued keep it: eviction syncs the device
    s->jit.fn = nullptr;
    if (const char* dump = getenv("RTCORE_JIT_DUMP")) { // inspection: the generated header of the last build
        if (FILE* f = fopen(dump, "w")) {
            fwrite(header.data(), 1, header.size(), f);
            fclose(f);
        }
    }
    JitKernel k;
    std::string err;
    if (!jit_kernel(s->device, header, grouped, k, err)) {
        s->jit.status = -1;
        s->jit.error = err;
        return 0;
    }
    int n = 0;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&n, k.fn, 256, path_dyn_lds(s->dev, s->variant)) !=
            hipSuccess ||
        n < 1) {
        jit_release(s->device, k.fn); // the reference jit_kernel took: the module stays evictable
        (void)hipGetLastError();
        s->jit.status = -1;
        s->jit.error = "occupancy query of the scene-specialised kernel failed";
        return 0;
    }
    s->jit.fn = k.fn;
    s->jit.blocks_per_cu = n;
    s->jit.status = 1;
    s->jit.compile_ms = k.compile_ms;
    s->jit.from_cache = k.from_cache;
    return 1;
}

// Launch the path kernel for p (work buffers sized here), timing it with the scene's events.
int run_path(rt_scene* s, PathParams& p, unsigned long long* d_rays, hipStream_t stream, bool timed)
{
    const size_t need = (size_t)p.n_chunks * (size_t)p.n_pad;
    if (need > 0xF0000000ull) { // 32-bit work-item counter (plus the pools' overshoot)
        set_error("tile x spp too large for one launch; split the tile");
        return RT_ERR_ARG;
    }
    HIP_TRY(s->partial.reserve(need));
    HIP_TRY(s->counter.reserve(kMaxSplit * kSplitStride));
    p.partial = s->partial.p;
    p.counter = s->counter.p;
    p.rays = d_rays;
    p.stats = s->stats_on ? s->stats_buf.p : nullptr;
    // rt_debug_ray_log arms the next instrumented BVH launch only, so a buffer the caller frees
    // afterwards is never written
    p.ray_log = (s->stats_on && s->variant >= 4) ? s->ray_log : nullptr;
    p.ray_log_n = s->ray_log_n;
    p.ray_log_cap = s->ray_log_cap;
    if (p.ray_log) s->ray_log = nullptr;
    // order after the previous operation when it ran on another stream (shared scratch)
    if (s->any_op && stream != s->last_stream) HIP_TRY(hipStreamWaitEvent(stream, s->done_ev, 0));
    HIP_TRY(hipMemsetAsync(p.counter, 0, sizeof(unsigned int) * kSplitStride * p.n_split, stream));
    int grid = s->n_cu * (s->stats_on ? s->stats_blocks_per_cu : s->blocks_per_cu);
    p.stack_ovf = nullptr;
    if (s->variant >= 4) { // BVH kernels: the stacks' global overflow area
        HIP_TRY(s->stack_ovf.reserve((size_t)grid * 256 * kStackOverflow));
        p.stack_ovf = s->stack_ovf.p;
    }
    const int jit = prepare_jit(s);
    int jit_grid = jit ? s->n_cu * s->jit.blocks_per_cu : 0;
    // A small brute-force launch runs fewer blocks per CU.  Its time is a lane's serial chain of
    // samples (each a few dependent iterations), and an iteration takes as long as the waves sharing
    // a SIMD make it: with ~2 samples per lane (bounce.txt 256x256 x 16 spp on 8 blocks per CU) the
    // launch is all tail.  So the grid gives each lane at least kSamplesPerLane samples, up to the
    // occupancy the kernel allows.  Measured on that launch (profiles/r06/probe_grid.log, kernel ms):
    // 8 / 6 / 4 / 3 / 2 blocks per CU 0.205 / 0.191 / 0.165 / 0.156-0.161 / 0.163-0.164; the 1080p x 256
    // spp launch (1,157 samples per lane) stays at the full 8 (16.72-16.75 ms; 6: 17.11).  Which lane
    // renders an item never changes what it computes.  RTCORE_GRID_BPC caps it (tuning).
    if ((s->variant >> 1) < 2 && !s->stats_on) {
        constexpr double kSamplesPerLane = 6.0;
        const double samples = (double)p.w * (double)p.h * (double)p.spp;
        int cap = (int)std::ceil(samples / ((double)s->n_cu * 256.0 * kSamplesPerLane));
        if (const char* e = getenv("RTCORE_GRID_BPC")) cap = atoi(e);
        cap = std::max(1, cap);
        if (jit) jit_grid = s->n_cu * std::min(s->jit.blocks_per_cu, cap);
        else grid = s->n_cu * std::min(s->blocks_per_cu, cap);
    }
    const int tslot = (int)(s->launches % rt_scene::kTimeRing);
    if (timed) HIP_TRY(hipEventRecord(s->t_start[tslot], stream));
    if (!s->params_h) {
        HIP_TRY(hipHostMalloc(&s->params_h, sizeof(PathParams) * rt_scene::kParamRing, hipHostMallocDefault));
        HIP_TRY(s->params_d.reserve(rt_scene::kParamRing));
    }
    fill_launch(s->dev, s->variant, p);
    // The brute-force kernels read each item's pixel key (two lowbias32 rounds of the seed key and
    // the frame pixel index, rtcore_rng.h) from a per-scene table, built here once per seed (a
    // ~10-us kernel on the launch stream): the same keys, without hashing in the loop.
    // RTCORE_PIXEL_KEYS=0 hashes per item (A/B).
    p.pkeys = nullptr;
    static const bool pkeys_on = !(getenv("RTCORE_PIXEL_KEYS") && getenv("RTCORE_PIXEL_KEYS")[0] == '0');
    if ((s->variant >> 1) < 2 && !s->stats_on && pkeys_on) {
        if (!s->pkeys_valid || s->pkeys_seed != p.seed) {
            HIP_TRY(s->pkeys.reserve((size_t)s->params.width * (size_t)s->params.height));
            HIP_TRY(launch_pixel_keys(p.seed_key, s->params.width, s->params.height, s->pkeys.p, stream));
            s->pkeys_valid = true;
            s->pkeys_seed = p.seed;
        }
        p.pkeys = s->pkeys.p;
    }
    const unsigned slot = s->params_next++ % rt_scene::kParamRing;
    hipEvent_t& sev = s->slot_ev[slot];
    if (sev) HIP_TRY(hipEventSynchronize(sev)); // the slot's previous upload has been read
    else HIP_TRY(hipEventCreateWithFlags(&sev, hipEventDisableTiming));
    s->params_h[slot] = p;
    HIP_TRY(hipMemcpyAsync(s->params_d.p + slot, s->params_h + slot, sizeof(PathParams), hipMemcpyHostToDevice, stream));
    HIP_TRY(hipEventRecord(sev, stream));
    if (jit) {
        const CameraF* ca = s->camf_d.p;
        const PathParams* pa = s->params_d.p + slot;
        void* args[] = {&ca, &pa};
        HIP_TRY(hipModuleLaunchKernel(s->jit.fn, jit_grid, 1, 1, 256, 1, 1,
                                      (unsigned)path_dyn_lds(s->dev, s->variant), stream, args, nullptr));
    } else {
        HIP_TRY(launch_path(s->dev, s->camf_d.p, s->params_d.p + slot, s->variant, grid, stream, s->stats_on));
    }
    if (timed) {
        HIP_TRY(hipEventRecord(s->t_end[tslot], stream));
        s->launches++;
    }
    return RT_OK;
}

// Marks the end of a render operation (path kernel + the kernel that consumed its partials).
int end_op(rt_scene* s, hipStream_t stream)
{
    HIP_TRY(hipEventRecord(s->done_ev, stream));
    s->last_stream = stream;
    s->any_op = true;
    return RT_OK;
}

// The host-buffer entry points' device -> host step.  queue_copy queues records [a, b) of d_src (after
// the work already on the scene's stream) into the same offsets of pinned staging, in k chunks whose
// arrivals are recorded by events; consume_copies then runs consume(stage, a, b) on the host pool
// for each chunk's items as soon as that chunk has landed, so the host pass over one chunk overlaps
// the DMA of the next (and whatever device work was queued after it).  Staging must be reserved
// for every queued record first.
struct CopyPlan {
    size_t a[rt_scene::kCopyChunks], b[rt_scene::kCopyChunks];
    int n = 0;
};

int queue_copy(rt_scene* s, CopyPlan& plan, const void* d_src, size_t a, size_t b, size_t rec_bytes, int k,
               hipStream_t stream)
{
    k = std::max(1, std::min(k, rt_scene::kCopyChunks - plan.n));
    const size_t per = (b - a + k - 1) / k;
    for (int c = 0; c < k; c++) {
        const size_t ca = std::min(b, a + c * per), cb = std::min(b, a + (c + 1) * per);
        hipEvent_t& ev = s->copy_ev[plan.n];
        if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        if (cb > ca)
            HIP_TRY(hipMemcpyAsync(s->stage.p + ca * rec_bytes, static_cast<const unsigned char*>(d_src) + ca * rec_bytes,
                                   (cb - ca) * rec_bytes, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipEventRecord(ev, stream));
        plan.a[plan.n] = ca;
        plan.b[plan.n] = cb;
        plan.n++;
    }
    return RT_OK;
}

int consume_copies(rt_scene* s, const CopyPlan& plan, const std::function<void(const unsigned char*, size_t, size_t)>& consume)
{
    // chunks x S slices, handed out in order: the first tasks wait for the first chunk.  A slice
    // holds at least kMinItems records, so a small tile (a few thousand pixels) is consumed on the
    // calling thread instead of waking the pool for a few hundred records per thread.
    constexpr size_t kMinItems = 65536;
    size_t longest = 0;
    for (int k = 0; k < plan.n; k++) longest = std::max(longest, plan.b[k] - plan.a[k]);
    const size_t S = std::max<size_t>(1, std::min<size_t>((size_t)host_threads(), longest / kMinItems));
    std::atomic<int> failed{0};
    host_run((size_t)plan.n * S, [&](size_t t) {
        const size_t k = t / S, j = t % S;
        const size_t a0 = plan.a[k], b0 = plan.b[k];
        const size_t sl = (b0 - a0 + S - 1) / S;
        const size_t a = std::min(b0, a0 + j * sl), b = std::min(b0, a + sl);
        if (hipEventSynchronize(s->copy_ev[k]) != hipSuccess) {
            failed = 1;
            return;
        }
        if (b > a) consume(s->stage.p, a, b);
    });
    if (failed) {
        set_error("device -> host copy failed");
        return RT_ERR_HIP;
    }
    return RT_OK;
}

// n_items records of rec_bytes from d_src in up to kCopyChunks chunks of at least 1 MB.
int copy_consume(rt_scene* s, const void* d_src, size_t n_items, size_t rec_bytes,
                 const std::function<void(const unsigned char*, size_t, size_t)>& consume)
{
    const size_t bytes = n_items * rec_bytes;
    HIP_TRY(s->stage.reserve(bytes));
    CopyPlan plan;
    const int K = (int)std::max<size_t>(1, std::min<size_t>(rt_scene::kCopyChunks, bytes >> 20));
    int rc = queue_copy(s, plan, d_src, 0, n_items, rec_bytes, K, s->stream);
    if (rc != RT_OK) return rc;
    return consume_copies(s, plan, consume);
}

} // namespace

extern "C" {

namespace {
std::atomic<int> g_builder{RT_BVH_BUILDER_AUTO};
// AUTO builds on the GPU from this many BVH primitives.  Below it the host's binned-SAH tree is
// worth its build time: on the 1 M-triangle mesh (C4) the PLOC tree costs 15 % more node visits
// and 8 % of the render rate, against 0.4 s of build time saved.
constexpr int kGpuBuildMin = 1 << 22;

// Which axis-aligned rectangles become outer records.  Only large ones pay: a wall whose box
// overlaps the whole scene sits near the root of any tree, while a small cube face is cheap inside
// it and would cost every query a test outside it (test_outer is linear in the group).  So a
// rectangle qualifies when its area is at least 1/kOuterAreaDiv of the scene box's largest face,
// and at most kOuterMax of them (largest first) are taken.  C4: the room's six walls and the
// light box's five faces (the smallest, 0.75 x 0.1, is 1/213 of the 4 x 4 face).  None, or all
// of the BVH primitives, leaves the tree as it is.
constexpr int kOuterMax = 64;
constexpr double kOuterAreaDiv = 1024.0;

void select_outer(const std::vector<HostPrim>& H, std::vector<char>& out)
{
    out.clear();
    const int n = (int)H.size();
    float slo[3] = {INFINITY, INFINITY, INFINITY}, shi[3] = {-INFINITY, -INFINITY, -INFINITY};
    int nb = 0;
    std::vector<std::pair<double, int>> cand;
    for (int i = 0; i < n; i++) {
        if (H[i].kind == RT_PRIM_PLANE) continue;
        nb++;
        float lo[3], hi[3];
        sah_prim_box(H[i], lo, hi);
        for (int k = 0; k < 3; k++) {
            slo[k] = std::min(slo[k], lo[k]);
            shi[k] = std::max(shi[k], hi[k]);
        }
        const int k = rect_axis_of(H[i]);
        if (k < 0) continue;
        const double a = (double)(hi[(k + 1) % 3] - lo[(k + 1) % 3]) * (double)(hi[(k + 2) % 3] - lo[(k + 2) % 3]);
        cand.push_back({a, i});
    }
    double face = 0.0;
    for (int k = 0; k < 3; k++)
        face = std::max(face, (double)(shi[(k + 1) % 3] - slo[(k + 1) % 3]) * (double)(shi[(k + 2) % 3] - slo[(k + 2) % 3]));
    // largest first, then by ID (a stable choice at the cap)
    std::sort(cand.begin(), cand.end(), [](const auto& a, const auto& b) { return a.first != b.first ? a.first > b.first : a.second < b.second; });
    std::vector<char> m(n, 0);
    int k = 0;
    for (const auto& c : cand) {
        if (k == kOuterMax || !(c.first * kOuterAreaDiv >= face)) break;
        m[c.second] = 1;
        k++;
    }
    if (k > 0 && k < nb) out = std::move(m);
}

int builder_for(int n_bvh)
{
    int b = g_builder.load();
    if (b == RT_BVH_BUILDER_AUTO)
        if (const char* e = getenv("RTCORE_BVH_BUILDER")) // for A/B measurements
            b = std::strcmp(e, "gpu") == 0 ? RT_BVH_BUILDER_GPU : std::strcmp(e, "host") == 0 ? RT_BVH_BUILDER_HOST : b;
    if (b == RT_BVH_BUILDER_AUTO) b = n_bvh >= kGpuBuildMin ? RT_BVH_BUILDER_GPU : RT_BVH_BUILDER_HOST;
    return n_bvh > 0 ? b : RT_BVH_BUILDER_HOST;
}

// The fast-path BVH2 and its wide collapse, by the host (binned SAH, bvh_sah.cpp) or the GPU
// (PLOC, bvh_gpu.hip).  Planes are never in the BVH.
int build_bvhs(rt_scene* s)
{
    const auto& H = s->host;
    const int n = (int)H.size();
    std::vector<int32_t> ids;
    for (int i = 0; i < n; i++)
        if (H[i].kind != RT_PRIM_PLANE) ids.push_back(i);
    const int nb = (int)ids.size();
    if (nb + kTestSpares >= kLeafGenericMaxSlots) { // leaf codes (rt_internal.h) address 2^27 slots
        set_error("rt_scene_create: more than 2^27 - " + std::to_string(kTestSpares) + " BVH primitives");
        return RT_ERR_ARG;
    }
    s->bvh.builder = builder_for(nb);
    // Outer records: in a large scene (nb > 4096: no grouped brute-force order, which would cut
    // this tree) the axis-aligned rectangles -- a room's walls, a light box -- stay out of the
    // tree and are tested as one group of rects and closed boxes when a query ends.  Their
    // large boxes overlap the whole scene near the root (tools/bvh_sim.cpp on C4's mesh: node
    // visits per query 8.75 -> 7.88, primitive tests 5.33 -> 2.46; measured: C4 46.5 -> 44.0 ms,
    // nodes 9.16 -> 8.34 and leaf tests 5.75 -> 2.88 per ray segment).  RTCORE_BVH_OUTER=0: off.
    bool outer_on = nb > 4096;
    if (const char* e = getenv("RTCORE_BVH_OUTER")) outer_on = outer_on && atoi(e) != 0;
    s->bvh_outer.clear();
    if (outer_on) select_outer(H, s->bvh_outer);
    // leaves of <= 3 primitives, <= 2 with outer records (C4, round 2: leaves of <= 2, 3, 4, 6, 8 ->
    // 70.6, 70.5, 72.2, 76.1, 80.2 ms; round 5 with outer records: 2 / 3 / 4 -> 43.8 / 44.0 / 47.2)
    int max_leaf = n > 256 && s->bvh_outer.empty() ? 3 : 2;
    if (const char* e = getenv("RTCORE_MAX_LEAF")) max_leaf = std::max(1, std::min(8, atoi(e))); // tuning
    if (s->bvh.builder == RT_BVH_BUILDER_HOST) {
        // the wide tree: greedy collapse of the BVH2 (default), or the SAH-optimal collapse of the
        // whole SAH tree (RTCORE_WIDE_COLLAPSE=1; RTCORE_WIDE_CNODE / _CPRIM / _LEAF set its costs)
        WideCosts wc;
        bool sah_collapse = false; // measured slower on C4
        if (const char* e = getenv("RTCORE_WIDE_COLLAPSE")) sah_collapse = atoi(e) != 0;
        if (const char* e = getenv("RTCORE_WIDE_CNODE")) wc.c_node = (float)atof(e);
        if (const char* e = getenv("RTCORE_WIDE_CPRIM")) wc.c_prim = (float)atof(e);
        if (const char* e = getenv("RTCORE_WIDE_LEAF")) wc.max_leaf = std::max(1, std::min(8, atoi(e)));
        s->sah = build_sah_bvh(H, max_leaf, sah_collapse, s->bvh_outer.empty() ? nullptr : &s->bvh_outer);
        s->bvh4 = build_bvh4(s->sah, sah_collapse ? &wc : nullptr);
        s->sah.full.clear(); // only the collapse reads the whole tree
        s->sah.full.shrink_to_fit();
        s->bvh.n_nodes2 = (int)s->sah.nodes.size();
        s->bvh.root2 = s->sah.root;
        s->bvh.depth2 = s->sah.depth;
        s->bvh.n_nodes4 = (int)s->bvh4.nodes.size();
        s->bvh.root4 = s->bvh4.root;
        s->bvh.stack4 = s->bvh4.stack_need;
        return RT_OK;
    }
    const int n_planes = n - nb;
    if (!s->bvh_outer.empty()) // the outer records stay out of the GPU builder's tree too
        ids.erase(std::remove_if(ids.begin(), ids.end(), [&](int32_t i) { return s->bvh_outer[i] != 0; }), ids.end());
    const int n_tree = (int)ids.size();
    std::vector<float4> lo(n_tree), hi(n_tree);
    parallel_for(n_tree, [&](int k) {
        float l[3], h[3];
        sah_prim_box(H[ids[k]], l, h);
        lo[k] = make_float4(l[0], l[1], l[2], 0.0f);
        hi[k] = make_float4(h[0], h[1], h[2], 0.0f);
    });
    GpuBvh g;
    HIP_TRY(build_bvh_gpu(lo.data(), hi.data(), ids.data(), n_tree, max_leaf, n_planes + 1, s->stream, g));
    s->nodes.adopt(g.nodes, g.n_nodes);
    s->nodes4.adopt(g.nodes4, g.n_nodes4);
    s->order_d.adopt(g.order, (size_t)n_tree + n_planes + 1);
    s->bvh.n_nodes2 = g.n_nodes;
    s->bvh.root2 = g.root;
    s->bvh.depth2 = g.depth;
    s->bvh.n_nodes4 = g.n_nodes4;
    s->bvh.root4 = g.root4;
    s->bvh.stack4 = g.stack_need;
    s->bvh.rounds = g.rounds;
    s->bvh.gpu_ms = g.ms;
    return RT_OK;
}
} // namespace

int rt_set_bvh_builder(int32_t builder)
{
    if (builder < RT_BVH_BUILDER_AUTO || builder > RT_BVH_BUILDER_GPU) {
        set_error("rt_set_bvh_builder: bad argument");
        return RT_ERR_ARG;
    }
    g_builder.store(builder);
    return RT_OK;
}

int rt_debug_brute_layout(const rt_prim* prims, int32_t n_prims, int32_t* out, int32_t n_out)
{
    if (n_prims < 0 || (n_prims > 0 && !prims) || !out || n_out < 0) {
        set_error("rt_debug_brute_layout: bad argument");
        return RT_ERR_ARG;
    }
    for (int i = 0; i < n_prims; i++)
        if (prims[i].kind < 0 || prims[i].kind > 2) {
            set_error("rt_debug_brute_layout: unknown primitive kind at index " + std::to_string(i));
            return RT_ERR_ARG;
        }
    const std::vector<HostPrim> H = prepare_prims(prims, n_prims);
    const int n = (int)H.size();
    std::vector<int> xf_index(n, -1);
    int nb = 0, nx = 0;
    for (int i = 0; i < n; i++) {
        nb += H[i].kind != RT_PRIM_PLANE;
        if (H[i].kind == RT_PRIM_SPHERE && (H[i].flags & F_TRANSFORMED)) xf_index[i] = nx++;
    }
    SahBvh sah; // the grouping cuts the host SAH tree, as rt_scene_create does for small scenes
    if (nb > 0 && builder_for(nb) == RT_BVH_BUILDER_HOST) sah = build_sah_bvh(H, n > 256 ? 4 : 2);
    const BruteOrders o = make_brute_orders(H, xf_index, sah);
    const BruteLayout& L = o.layout;
    const int32_t v[RT_LAYOUT_COUNT] = {L.rects, L.boxes, L.frames, L.frame_boxes, L.frame_rects, L.tris, L.sphs,
                                        o.np, o.grouped.groups.empty() ? 0 : (int32_t)o.grouped.groups.size(),
                                        (int32_t)o.grouped.prims.size() - o.np};
    for (int i = 0; i < n_out && i < RT_LAYOUT_COUNT; i++) out[i] = v[i];
    return RT_OK;
}

// Experiment support: the flat brute-force order's records as 32-bit words (groups | rects |
// frames | tests); counts = {groups, rects, frames, tests}.  Host code only.
int rt_debug_flat_records(const rt_prim* prims, int32_t n_prims, uint32_t* out, int64_t cap_words, int32_t* counts)
{
    if (n_prims < 0 || (n_prims > 0 && !prims) || !out || !counts) {
        set_error("rt_debug_flat_records: bad argument");
        return RT_ERR_ARG;
    }
    const std::vector<HostPrim> H = prepare_prims(prims, n_prims);
    const int n = (int)H.size();
    std::vector<int> xf_index(n, -1);
    int nb = 0, nx = 0;
    for (int i = 0; i < n; i++) {
        nb += H[i].kind != RT_PRIM_PLANE;
        if (H[i].kind == RT_PRIM_SPHERE && (H[i].flags & F_TRANSFORMED)) xf_index[i] = nx++;
    }
    SahBvh sah;
    if (nb > 0 && builder_for(nb) == RT_BVH_BUILDER_HOST) sah = build_sah_bvh(H, n > 256 ? 4 : 2);
    const BruteOrders o = make_brute_orders(H, xf_index, sah);
    const BruteOrder& f = o.flat;
    size_t w = 0;
    auto put = [&](const void* p, size_t bytes) {
        const size_t k = bytes / 4;
        if ((int64_t)(w + k) <= cap_words) memcpy(out + w, p, bytes);
        w += k;
    };
    put(f.groups.data(), f.groups.size() * sizeof(GroupRec));
    put(f.rects.data(), f.rects.size() * sizeof(RectRec));
    put(f.frames.data(), f.frames.size() * sizeof(FrameRec));
    put(f.tests.data(), f.tests.size() * sizeof(TestRec));
    counts[0] = (int32_t)f.groups.size();
    counts[1] = (int32_t)f.rects.size();
    counts[2] = (int32_t)f.frames.size();
    counts[3] = (int32_t)f.tests.size();
    if ((int64_t)w > cap_words) {
        set_error("rt_debug_flat_records: buffer too small");
        return RT_ERR_ARG;
    }
    return RT_OK;
}

// Experiment support (host only, no device): the generated header of the scene-specialised build
// that rt_scene_create + rt_scene_set_camera would make for these primitives and this camera, so
// that its code can be compiled and read on a machine without a GPU (tools/jit_isa.py).  Returns
// the header's length (copied into buf, NUL-terminated, when it fits in cap).
int rt_debug_jit_header(const rt_scene_params* params, const rt_prim* prims, int32_t n_prims, const rt_camera* camera,
                        int32_t grouped, char* buf, int64_t cap)
{
    if (!params || !camera || n_prims < 0 || (n_prims > 0 && !prims) || (grouped != 0 && grouped != 1)) {
        set_error("rt_debug_jit_header: bad argument");
        return RT_ERR_ARG;
    }
    const std::vector<HostPrim> H = prepare_prims(prims, n_prims);
    const int n = (int)H.size();
    std::vector<int> xf_index(n, -1);
    std::vector<XformF> xf;
    int nb = 0, np = 0, n_vn = 0;
    for (int i = 0; i < n; i++) {
        nb += H[i].kind != RT_PRIM_PLANE;
        np += H[i].kind == RT_PRIM_PLANE;
        n_vn += (H[i].kind == RT_PRIM_TRIANGLE && (H[i].flags & F_HASNORMALS)) ? 1 : 0;
        if (H[i].kind == RT_PRIM_SPHERE && (H[i].flags & F_TRANSFORMED)) {
            xf_index[i] = (int)xf.size();
            xf.push_back(make_xformf(H[i]));
        }
    }
    if (nb > 48) {
        set_error("rt_debug_jit_header: the scene-specialised build serves brute-force scenes (<= 48 primitives)");
        return RT_ERR_ARG;
    }
    const SahBvh sah = nb > 0 ? build_sah_bvh(H, n > 256 ? 3 : 2) : SahBvh{}; // as build_bvhs
    const BruteOrders o = make_brute_orders(H, xf_index, sah);
    const BruteOrder& B = grouped ? o.grouped : o.flat;
    if (grouped && B.groups.empty()) {
        set_error("rt_debug_jit_header: no grouped order for this scene");
        return RT_ERR_ARG;
    }
    PathScene ps; // make_path_scene + fill_launch, from the host records
    std::memset(&ps, 0, sizeof ps);
    for (int k = 0; k < 3; k++) ps.n_rect[k] = o.nr[k];
    ps.n_tri = o.nt;
    ps.n_sph = o.ns;
    ps.n_pln = np;
    ps.n_bvh = (int)B.prims.size() - np;
    ps.n_slots = ps.n_bvh + np;
    ps.n_mats = (int)make_materials(H, params->air_ior).mats.size();
    ps.n_xf = (int)xf.size();
    ps.n_vn = n_vn;
    ps.facts = getenv("RTCORE_NO_FACTS") ? (uint32_t)FACT_ALL : scene_facts(H);
    ps.n_groups = grouped ? (int)B.groups.size() : 1;
    ps.root = nb > 0 ? sah.root : 0;
    ps.width = params->width;
    ps.recursion = params->recursion;
    ps.debug_geom = params->debug_geom;
    const rt_color& a = params->ambient;
    ps.ambient_miss = (a.r == -1 && a.g == -1 && a.b == -1) ? 1 : 0;
    ps.air_ior = (float)params->air_ior;
    ps.ambient_r = (float)a.r;
    ps.ambient_g = (float)a.g;
    ps.ambient_b = (float)a.b;
    CameraD camd;
    CameraF camf;
    camera_init(*camera, params->width, params->height, camd, camf);
    const std::vector<GroupRec> groups =
        (grouped && B.groups.size() > 1 && !getenv("RTCORE_NO_GROUP_SORT")) ? groups_nearest_first(B.groups, camd) : B.groups;
    const std::string h = jit_scene_header(ps, camf, grouped == 1, groups, B.rects, B.frames, B.tests, xf);
    if (buf && cap > (int64_t)h.size()) std::memcpy(buf, h.c_str(), h.size() + 1);
    return (int)h.size();
}

int rt_set_jit(int32_t on)
{
    if (on != 0 && on != 1) {
        set_error("rt_set_jit: on must be 0 or 1");
        return RT_ERR_ARG;
    }
    jit_set_enabled(on == 1);
    return RT_OK;
}

int rt_debug_vn_rehit(const double* v0, const double* e01, const double* e02, int32_t mirror, double u, double v,
                      const float* dir, int32_t* inside, double* t, double* origin)
{
    if (!v0 || !e01 || !e02 || !dir || !inside || !t || !origin) {
        set_error("rt_debug_vn_rehit: bad argument");
        return RT_ERR_ARG;
    }
    int in = 0;
    const int hit = debug_vn_rehit(v0, e01, e02, mirror, u, v, dir, &in, t, origin);
    *inside = in;
    return hit;
}

int rt_debug_ray_log(rt_scene* s, void* d_log, uint32_t cap, void* d_count)
{
    if (!s || (d_log && !d_count)) {
        set_error("rt_debug_ray_log: bad argument");
        return RT_ERR_ARG;
    }
    s->ray_log = static_cast<float4*>(d_log);
    s->ray_log_n = static_cast<unsigned int*>(d_count);
    s->ray_log_cap = d_log ? cap : 0;
    return RT_OK;
}

int rt_debug_trace_rays(rt_scene* s, const void* d_rays, uint32_t n, void* d_hits, int32_t waves, void* d_stats,
                        void* stream, float* ms)
{
    if (!s || !d_rays || !d_hits || !ms || waves < 6 || waves > 8) {
        set_error("rt_debug_trace_rays: bad argument");
        return RT_ERR_ARG;
    }
    if (s->dev.n_pln > 0 || s->bvh.n_nodes4 == 0) {
        set_error("rt_debug_trace_rays: needs a wide BVH and a scene without planes");
        return RT_ERR_STATE;
    }
    // the trace-only kernel starts every query from no hit: the vertex-normal re-hit start of a
    // logged query (Sample.prev <= -2, query_start) is not restated there
    if (s->dev.n_vn > 0) {
        set_error("rt_debug_trace_rays: scenes with vertex-normal triangles are not supported");
        return RT_ERR_STATE;
    }
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    // the work counter and the stack overflow area are the scene's: order after its last render
    if (s->any_op && st != s->last_stream) HIP_TRY(hipStreamWaitEvent(st, s->done_ev, 0));
    const int grid = s->n_cu * trace_rays_blocks_per_cu(waves);
    HIP_TRY(s->stack_ovf.reserve((size_t)grid * 256 * kStackOverflow));
    HIP_TRY(s->counter.reserve(1));
    HIP_TRY(hipMemsetAsync(s->counter.p, 0, sizeof(unsigned int), st));
    TraceRaysParams p{};
    p.rays = static_cast<const float4*>(d_rays);
    p.hits = static_cast<float2*>(d_hits);
    p.n = n;
    p.counter = s->counter.p;
    p.stack_ovf = s->stack_ovf.p;
    p.tests = s->dev.tests_bvh;
    p.rows = s->dev.rows_bvh;
    p.nodes4 = s->dev.nodes4;
    p.xf = s->dev.xf;
    p.root4 = s->dev.root4;
    if (s->dev.n_outer > 0) {
        p.outer = s->dev.groups_bvh;
        p.outer_rects = s->dev.rects_bvh;
        p.outer_boxes = s->dev.frames_bvh;
    }
    p.spec = 16;
    if (const char* e = getenv("RTCORE_BVH_SPEC")) p.spec = std::max(1, std::min(64, atoi(e)));
    p.stats = static_cast<unsigned long long*>(d_stats);
    struct Events { // destroyed on every exit path
        hipEvent_t e0 = nullptr, e1 = nullptr;
        ~Events()
        {
            if (e0) (void)hipEventDestroy(e0);
            if (e1) (void)hipEventDestroy(e1);
        }
    } ev;
    HIP_TRY(hipEventCreate(&ev.e0));
    HIP_TRY(hipEventCreate(&ev.e1));
    HIP_TRY(hipEventRecord(ev.e0, st));
    HIP_TRY(launch_trace_rays(p, waves, grid, st));
    HIP_TRY(hipEventRecord(ev.e1, st));
    const int rc = end_op(s, st);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipEventSynchronize(ev.e1));
    HIP_TRY(hipEventElapsedTime(ms, ev.e0, ev.e1));
    return RT_OK;
}

int rt_debug_jit_compile(const char* arch, int32_t grouped, char* log, int32_t cap)
{
    if (!arch || (grouped != 0 && grouped != 1)) {
        set_error("rt_debug_jit_compile: bad argument");
        return RT_ERR_ARG;
    }
    std::string err;
    const size_t n = jit_compile_check(arch, grouped == 1, err);
    if (log && cap > 0) {
        const size_t k = std::min((size_t)cap - 1, err.size());
        memcpy(log, err.data(), k);
        log[k] = '\0';
    }
    if (n == 0) {
        set_error("rt_debug_jit_compile: " + err);
        return RT_ERR_STATE;
    }
    return (int)std::min(n, (size_t)0x7fffffff);
}

int rt_scene_get_jit_error(const rt_scene* s, char* buf, int32_t cap)
{
    if (!s || !buf || cap <= 0) {
        set_error("rt_scene_get_jit_error: bad argument");
        return RT_ERR_ARG;
    }
    const std::string& e = s->jit.error;
    const size_t n = std::min((size_t)cap - 1, e.size());
    memcpy(buf, e.data(), n);
    buf[n] = '\0';
    return (int)e.size();
}

int rt_scene_get_build_stats(const rt_scene* s, double* out, int32_t n)
{
    if (!s || !out || n < 0) {
        set_error("rt_scene_get_build_stats: bad argument");
        return RT_ERR_ARG;
    }
    const auto& L = s->layout;
    const double v[RT_BUILD_STATS_COUNT] = {s->ms_prepare, s->ms_bvh, s->ms_upload, (double)s->bvh.gpu_ms,
                                           (double)s->bvh.rounds, (double)s->bvh.n_nodes4, (double)s->bvh.stack4,
                                           (double)L.rects, (double)L.boxes, (double)L.frames, (double)L.frame_boxes,
                                           (double)L.frame_rects, (double)L.tris, (double)L.sphs,
                                           (double)s->dev.n_hot4, (double)s->jit.status, s->jit.compile_ms,
                                           s->jit.from_cache ? 1.0 : 0.0, (double)L.group_max,
                                           (double)s->bvh.leaves4, (double)s->bvh.compact4,
                                           (double)std::count(s->bvh_outer.begin(), s->bvh_outer.end(), 1)};
    for (int i = 0; i < n && i < RT_BUILD_STATS_COUNT; i++) out[i] = v[i];
    return RT_OK;
}

// Structural check of the device-resident fast-path BVHs (either builder): every child box of
// the BVH2 and every dequantised child box of the wide tree contains the boxes of all primitives
// below it, every non-plane primitive sits in exactly one leaf of each tree, and the depth and
// stack figures the kernels were sized by are not exceeded.
int rt_scene_check_bvh(rt_scene* s)
{
    if (!s) {
        set_error("rt_scene_check_bvh: bad argument");
        return RT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(s->device));
    const auto& H = s->host;
    const int n = (int)H.size();
    // nb: the slots the tree's leaves address (outer records, when present, follow them)
    auto outside = [&](int i) { return H[i].kind == RT_PRIM_PLANE || (!s->bvh_outer.empty() && s->bvh_outer[i]); };
    int nb = 0;
    for (int i = 0; i < n; i++) nb += !outside(i);
    std::vector<NodeF> n2(s->bvh.n_nodes2);
    std::vector<Node4Q> n4(s->bvh.n_nodes4);
    std::vector<PrimF> recs(nb);
    if (!n2.empty()) HIP_TRY(hipMemcpy(n2.data(), s->nodes.p, n2.size() * sizeof(NodeF), hipMemcpyDeviceToHost));
    if (!n4.empty()) HIP_TRY(hipMemcpy(n4.data(), s->nodes4.p, n4.size() * sizeof(Node4Q), hipMemcpyDeviceToHost));
    if (nb > 0) HIP_TRY(hipMemcpy(recs.data(), s->prims_bvh.p, nb * sizeof(PrimF), hipMemcpyDeviceToHost));
    std::vector<int> id(nb);
    for (int k = 0; k < nb; k++) std::memcpy(&id[k], &recs[k].a.w, 4);
    struct B {
        double lo[3], hi[3];
    };
    auto empty = [] {
        B b;
        for (int a = 0; a < 3; a++) {
            b.lo[a] = __builtin_huge_val();
            b.hi[a] = -__builtin_huge_val();
        }
        return b;
    };
    auto grow = [](B& b, const B& c) {
        for (int a = 0; a < 3; a++) {
            b.lo[a] = std::min(b.lo[a], c.lo[a]);
            b.hi[a] = std::max(b.hi[a], c.hi[a]);
        }
    };
    std::vector<B> pbox(n);
    for (int i = 0; i < n; i++)
        if (H[i].kind != RT_PRIM_PLANE) {
            float l[3], h[3];
            sah_prim_box(H[i], l, h);
            for (int a = 0; a < 3; a++) {
                pbox[i].lo[a] = l[a];
                pbox[i].hi[a] = h[a];
            }
        }
    std::string err;
    std::vector<int> seen(n, 0);
    const uint32_t test_mask = KIND_MASK | F_MIRROR | F_TWOSIDED | F_INVERT | F_TRANSFORMED;
    auto leaf = [&](int ref, B& u) {
        int first, cnt;
        leaf_range(ref, first, cnt);
        const bool compact = ((~ref) & kLeafCompact) != 0;
        const uint32_t lfl = leaf_flags(((uint32_t)(~ref) >> 25) & 31u);
        if (first < 0 || first + cnt > nb) {
            err = "leaf range out of bounds";
            return;
        }
        if (compact && first + cnt > kLeafCompactMaxFirst) {
            err = "compact leaf beyond the slots its code can address";
            return;
        }
        for (int k = first; k < first + cnt; k++) {
            const int p = id[k];
            if (p < 0 || p >= n || outside(p)) {
                err = "leaf record with a bad primitive ID";
                return;
            }
            // a compact leaf's flags are what its primitives' own records say
            if (compact && (H[p].flags & test_mask) != lfl) {
                err = "compact leaf flags differ from primitive " + std::to_string(p);
                return;
            }
            seen[p]++;
            grow(u, pbox[p]);
        }
    };
    auto contains = [](const B& outer, const B& inner) {
        for (int a = 0; a < 3; a++)
            if (!(outer.lo[a] <= inner.lo[a] && outer.hi[a] >= inner.hi[a])) return false;
        return true;
    };
    // BVH2
    int max_depth = 0;
    std::function<B(int, int)> walk2 = [&](int ref, int depth) -> B {
        B u = empty();
        max_depth = std::max(max_depth, depth);
        if (!err.empty()) return u;
        if (ref < 0) {
            leaf(ref, u);
            return u;
        }
        if (ref >= (int)n2.size()) {
            err = "BVH2 child index out of range";
            return u;
        }
        const NodeF& q = n2[ref];
        for (int side = 0; side < 2; side++) {
            const float4 lo = side ? q.rmin : q.lmin, hi = side ? q.rmax : q.lmax;
            int c;
            std::memcpy(&c, &lo.w, 4);
            const B sub = walk2(c, depth + 1);
            const B box{{lo.x, lo.y, lo.z}, {hi.x, hi.y, hi.z}};
            if (err.empty() && !contains(box, sub)) err = "BVH2 child box misses a primitive below it";
            grow(u, sub);
        }
        return u;
    };
    if (nb > 0) walk2(s->bvh.root2, 0);
    for (int i = 0; i < n && err.empty(); i++)
        if (seen[i] != (outside(i) ? 0 : 1))
            err = "BVH2: primitive " + std::to_string(i) + " referenced " + std::to_string(seen[i]) + " times";
    if (err.empty() && max_depth > s->bvh.depth2) err = "BVH2 deeper than its recorded depth";
    // wide tree
    std::fill(seen.begin(), seen.end(), 0);
    int max_stack = 0;
    std::function<B(int, int)> walk4 = [&](int ref, int pushes) -> B {
        B u = empty();
        if (!err.empty()) return u;
        if (ref < 0) {
            leaf(ref, u);
            return u;
        }
        if (ref >= (int)n4.size()) {
            err = "wide child index out of range";
            return u;
        }
        const Node4Q& q = n4[ref];
        uint32_t ex, ql[3], qh[3];
        int refs[4], nc;
        std::memcpy(&ex, &q.a.w, 4);
        std::memcpy(&ql[0], &q.b.x, 4);
        std::memcpy(&qh[0], &q.b.y, 4);
        std::memcpy(&ql[1], &q.b.z, 4);
        std::memcpy(&qh[1], &q.b.w, 4);
        std::memcpy(&ql[2], &q.c.x, 4);
        std::memcpy(&qh[2], &q.c.y, 4);
        std::memcpy(&refs[0], &q.c.z, 4);
        std::memcpy(&refs[1], &q.c.w, 4);
        std::memcpy(&refs[2], &q.d.x, 4);
        std::memcpy(&refs[3], &q.d.y, 4);
        std::memcpy(&nc, &q.d.z, 4);
        if (nc < 1 || nc > 4) {
            err = "wide node with a bad child count";
            return u;
        }
        max_stack = std::max(max_stack, pushes + nc - 1);
        const double org[3] = {q.a.x, q.a.y, q.a.z};
        for (int k = 0; k < nc; k++) {
            const B sub = walk4(refs[k], pushes + nc - 1);
            B box;
            for (int a = 0; a < 3; a++) {
                const double sc = std::ldexp(1.0, (int)((ex >> (8 * a)) & 255u) - 128);
                box.lo[a] = org[a] + ((ql[a] >> (8 * k)) & 255u) * sc;
                box.hi[a] = org[a] + ((qh[a] >> (8 * k)) & 255u) * sc;
            }
            if (err.empty() && !contains(box, sub)) err = "wide child box misses a primitive below it";
            grow(u, sub);
        }
        return u;
    };
    if (err.empty() && nb > 0) walk4(s->bvh.root4, 0);
    for (int i = 0; i < n && err.empty(); i++)
        if (seen[i] != (outside(i) ? 0 : 1))
            err = "wide tree: primitive " + std::to_string(i) + " referenced " + std::to_string(seen[i]) + " times";
    if (err.empty() && max_stack > s->bvh.stack4) err = "wide tree needs more stack than recorded";
    if (!err.empty()) {
        set_error("rt_scene_check_bvh: " + err);
        return RT_ERR_STATE;
    }
    return RT_OK;
}

int rt_abi_version(void) { return RTCORE_ABI_VERSION; }

int rt_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rt_last_error(char* buf, int32_t cap)
{
    if (buf && cap > 0) {
        std::strncpy(buf, g_error.c_str(), (size_t)cap - 1);
        buf[cap - 1] = 0;
    }
    return (int)g_error.size();
}

int rt_scene_create(const rt_scene_params* params, const rt_prim* prims, int32_t n_prims, int32_t device,
                    rt_scene** out_scene)
{
    if (!params || !out_scene || n_prims < 0 || (n_prims > 0 && !prims)) {
        set_error("rt_scene_create: bad argument");
        return RT_ERR_ARG;
    }
    *out_scene = nullptr;
    if (params->width <= 0 || params->height <= 0) {
        set_error("rt_scene_create: width and height must be positive");
        return RT_ERR_ARG;
    }
    if (params->width > 65535 || params->height > 65535) { // the BVH kernels pack a pixel's x, y in 16 bits each
        set_error("rt_scene_create: width and height must be at most 65535");
        return RT_ERR_ARG;
    }
    for (int i = 0; i < n_prims; i++)
        if (prims[i].kind < 0 || prims[i].kind > 2) {
            set_error("rt_scene_create: unknown primitive kind at index " + std::to_string(i));
            return RT_ERR_ARG;
        }
    int ndev = rt_device_count();
    if (ndev <= 0) {
        set_error("rt_scene_create: no HIP device");
        return RT_ERR_NODEVICE;
    }
    if (device < 0 || device >= ndev) {
        set_error("rt_scene_create: device index out of range");
        return RT_ERR_ARG;
    }
    std::unique_ptr<rt_scene> s(new rt_scene());
    s->device = device;
    s->params = *params;
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    s->n_cu = prop.multiProcessorCount;
    HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    for (int i = 0; i < rt_scene::kTimeRing; i++) {
        HIP_TRY(hipEventCreate(&s->t_start[i]));
        HIP_TRY(hipEventCreate(&s->t_end[i]));
    }
    HIP_TRY(hipEventCreateWithFlags(&s->done_ev, hipEventDisableTiming));
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::duration d) { return std::chrono::duration<double, std::milli>(d).count(); };
    const auto t0 = clk::now();
    s->host = prepare_prims(prims, n_prims);
    const auto t1 = clk::now();
    int rc = build_bvhs(s.get());
    if (rc != RT_OK) return rc;
    const auto t2 = clk::now();
    rc = upload_scene(s.get());
    if (rc != RT_OK) return rc;
    s->ms_prepare = ms(t1 - t0);
    s->ms_bvh = ms(t2 - t1);
    s->ms_upload = ms(clk::now() - t2);
    rc = resolve_traversal(s.get());
    if (rc != RT_OK) return rc;
    HIP_TRY(s->rays.reserve(1));
    *out_scene = s.release();
    return RT_OK;
}

int rt_scene_set_camera(rt_scene* s, const rt_camera* cam)
{
    if (!s || !cam || (cam->kind != RT_CAMERA_FRUSTUM && cam->kind != RT_CAMERA_ORTHO)) {
        set_error("rt_scene_set_camera: bad argument");
        return RT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(s->device));
    camera_init(*cam, s->params.width, s->params.height, s->camd, s->camf);
    // launches of the previous camera may still be in flight on any stream
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(s->camf_d.reserve(1));
    HIP_TRY(hipMemcpy(s->camf_d.p, &s->camf, sizeof(CameraF), hipMemcpyHostToDevice));
    // The grouped order's groups nearest to the camera first: camera rays find their closest hit
    // early and skip the primitives of groups behind it (each group owns its own ranges, so only
    // the GroupRec order changes).  Deterministic for a given scene and camera.
    if (s->groups_gr_host.size() > 1 && !getenv("RTCORE_NO_GROUP_SORT")) {
        const std::vector<GroupRec> g = groups_nearest_first(s->groups_gr_host, s->camd);
        HIP_TRY(hipMemcpy(s->groups_gr.p, g.data(), g.size() * sizeof(GroupRec), hipMemcpyHostToDevice));
        s->grouped_h.groups = g; // the order the scene-specialised grouped kernel is built with
    }
    s->has_camera = true;
    s->jit_gen++; // the scene-specialised kernel carries the camera (and the group order)
    const int rc = calibrate_grouping(s);
    if (rc == RT_OK) (void)prepare_jit(s); // build the scene-specialised kernel now, not in a launch
    return rc;
}

int rt_scene_set_traversal(rt_scene* s, int32_t traversal)
{
    if (!s || traversal < RT_TRAVERSAL_AUTO || traversal > RT_TRAVERSAL_GROUPED) {
        set_error("rt_scene_set_traversal: bad argument");
        return RT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(s->device));
    const int before = s->traversal;
    s->traversal = traversal;
    const int rc = (traversal == RT_TRAVERSAL_AUTO && s->has_camera) ? calibrate_grouping(s) : resolve_traversal(s);
    if (rc != RT_OK) {
        s->traversal = before; // a refused mode leaves the scene as it was
        return rc;
    }
    if (s->has_camera) (void)prepare_jit(s);
    return rc;
}

int rt_scene_get_info(const rt_scene* s, rt_scene_info* info)
{
    if (!s || !info) {
        set_error("rt_scene_get_info: bad argument");
        return RT_ERR_ARG;
    }
    std::memset(info, 0, sizeof *info);
    info->n_prims = (int32_t)s->host.size();
    info->ref_bvh_nodes = (int32_t)s->ref.nodes.size();
    info->ref_bvh_depth = s->ref.depth;
    info->sah_bvh_nodes = s->bvh.n_nodes2;
    info->sah_bvh_depth = s->bvh.depth2;
    info->bvh_builder = s->bvh.builder;
    info->traversal = s->resolved;
    info->device = s->device;
    info->device_bytes = s->device_bytes;
    return RT_OK;
}

void rt_scene_destroy(rt_scene* s)
{
    if (!s) return;
    (void)hipSetDevice(s->device);
    (void)hipStreamSynchronize(s->stream);
    delete s;
}

int rt_render_device(rt_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t spp, uint64_t seed,
                     uint64_t sample_base, double* d_sum, uint32_t* d_samples, uint32_t* d_misses,
                     unsigned long long* d_rays, void* stream)
{
    int rc = check_tile(s, x0, y0, w, h);
    if (rc != RT_OK) return rc;
    if (spp <= 0 || !d_sum || !d_samples || !d_misses || !d_rays) {
        set_error("rt_render_device: bad argument");
        return RT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    PathParams p = make_params(s, x0, y0, w, h, spp, seed, sample_base);
    rc = run_path(s, p, d_rays, st);
    if (rc != RT_OK) return rc;
    HIP_TRY(launch_accumulate(p, d_sum, d_samples, d_misses, st));
    return end_op(s, st);
}

int rt_kernel_times(rt_scene* s, int32_t n, float* ms)
{
    if (!s || !ms || n < 1 || n > rt_scene::kTimeRing || (uint64_t)n > s->launches) {
        set_error("rt_kernel_times: bad argument (n must be 1.." + std::to_string(rt_scene::kTimeRing) +
                  " and at most the launches so far)");
        return RT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(s->device));
    for (int i = 0; i < n; i++) { // oldest first
        const int slot = (int)((s->launches - (uint64_t)n + (uint64_t)i) % rt_scene::kTimeRing);
        HIP_TRY(hipEventSynchronize(s->t_end[slot]));
        HIP_TRY(hipEventElapsedTime(ms + i, s->t_start[slot], s->t_end[slot]));
    }
    return RT_OK;
}

int rt_last_kernel_ms(rt_scene* s, float* ms)
{
    if (!s || !ms) {
        set_error("rt_last_kernel_ms: bad argument");
        return RT_ERR_ARG;
    }
    if (s->launches == 0) {
        set_error("rt_last_kernel_ms: no path kernel launched on this scene yet");
        return RT_ERR_ARG;
    }
    return rt_kernel_times(s, 1, ms);
}

int rt_scene_set_stats(rt_scene* s, int32_t enable)
{
    if (!s) {
        set_error("rt_scene_set_stats: null scene");
        return RT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(s->device));
    if (enable) {
        HIP_TRY(s->stats_buf.reserve(RT_STATS_COUNT));
        HIP_TRY(hipMemset(s->stats_buf.p, 0, RT_STATS_COUNT * sizeof(unsigned long long)));
        s->stats_blocks_per_cu = path_blocks_per_cu(s->variant, path_dyn_lds(s->dev, s->variant), true, s->dev.n_vn > 0);
    }
    s->stats_on = enable != 0;
    return RT_OK;
}

int rt_scene_get_stats(rt_scene* s, uint64_t* out, int32_t n)
{
    if (!s || !out || n < 0) {
        set_error("rt_scene_get_stats: bad argument");
        return RT_ERR_ARG;
    }
    if (!s->stats_buf.p) {
        set_error("rt_scene_get_stats: statistics were never enabled");
        return RT_ERR_STATE;
    }
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long v[RT_STATS_COUNT];
    HIP_TRY(hipMemcpy(v, s->stats_buf.p, sizeof v, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(s->stats_buf.p, 0, sizeof v));
    for (int k = 0; k < n && k < RT_STATS_COUNT; k++) out[k] = v[k];
    return RT_OK;
}

int rt_render_tile(rt_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t spp, uint64_t seed,
                   uint64_t sample_base, rt_color* sum_rgb, uint32_t* samples, uint32_t* misses, uint64_t* rays_out)
{
    int rc = check_tile(s, x0, y0, w, h);
    if (rc != RT_OK) return rc;
    if (spp < 0 || !sum_rgb || !samples || !misses) {
        set_error("rt_render_tile: bad argument");
        return RT_ERR_ARG;
    }
    if (spp == 0) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    // A previous call that failed between its first queued copy and its consume step may have left
    // band copies in flight on copy_stream, reading colors into stage: both are about to be
    // reserved (maybe reallocated), so wait for them first (normally the stream is already idle).
    if (s->copy_stream) HIP_TRY(hipStreamSynchronize(s->copy_stream));
    const size_t npix = (size_t)w * h;
    HIP_TRY(s->sum.reserve(3 * npix));
    HIP_TRY(s->samples.reserve(npix));
    HIP_TRY(s->misses.reserve(npix));
    HIP_TRY(s->colors.reserve(4 * npix)); // the caller's layout: one 32-B TileRec per pixel, x*h + y
    HIP_TRY(s->stage.reserve(npix * sizeof(TileRec)));
    HIP_TRY(s->rays_h.reserve(1));
    HIP_TRY(hipMemsetAsync(s->sum.p, 0, 3 * npix * sizeof(double), s->stream));
    HIP_TRY(hipMemsetAsync(s->samples.p, 0, npix * sizeof(uint32_t), s->stream));
    HIP_TRY(hipMemsetAsync(s->misses.p, 0, npix * sizeof(uint32_t), s->stream));
    HIP_TRY(hipMemsetAsync(s->rays.p, 0, sizeof(unsigned long long), s->stream));
    TileRec* d_rec = reinterpret_cast<TileRec*>(s->colors.p);
    // A large call renders in column bands, each a launch of its own whose records are copied (on
    // copy_stream) and added into the caller's arrays (the band's columns are one contiguous range
    // of x*h + y) while the next band renders: only the last band's copy and add are not hidden
    // behind the kernel.  Every band launch takes the whole tile's chunks per pixel, so the sums are
    // those of one launch bit for bit.  bounce.txt 1080p, ms per call into the caller's arrays
    // with 1 / 2 / 4 bands (tools/host_path_timing.py, profiles/r04/host_path_bands.log): 16 spp
    // 4.17 / 3.89 / 3.54, 64 spp 8.13 / 7.88 / 7.21, 256 spp 22.05 / 20.95 / 20.86; after the
    // round's kernel gains (profiles/r04/host_path_timing.log, 1 / 4 bands) 16 spp 4.33 / 4.00, 64 spp
    // 7.99 / 7.49, 256 spp 19.86 / 20.04: a long call gains less from the overlap than its band
    // launches' tails cost, so from 2.5e8 samples per call it is one launch again.
    // RTCORE_TILE_BANDS overrides the count (1 = one launch).
    const double work = (double)npix * spp;
    int nb = work >= 2.5e8 ? 1 : work >= 1.6e7 ? 4 : work >= 4e6 ? 2 : 1;
    if (const char* e = getenv("RTCORE_TILE_BANDS")) nb = std::max(1, std::min(4, atoi(e)));
    nb = std::max(1, std::min(nb, w / 64));
    if (!s->copy_stream) HIP_TRY(hipStreamCreateWithFlags(&s->copy_stream, hipStreamNonBlocking));
    const int per_band_chunks = nb == 1 ? (int)std::max<size_t>(1, std::min<size_t>(rt_scene::kCopyChunks,
                                                                                  (npix * sizeof(TileRec)) >> 20))
                                        : rt_scene::kCopyChunks / nb;
    CopyPlan plan;
    for (int k = 0; k < nb; k++) {
        const int a = nb == 1 ? 0 : (int)((int64_t)w * k / nb) & ~7, b = k + 1 == nb ? w : (int)((int64_t)w * (k + 1) / nb) & ~7;
        const int wb = b - a;
        const size_t off = (size_t)a * h;
        PathParams p = make_params(s, x0 + a, y0, wb, h, spp, seed, sample_base, (double)npix);
        rc = run_path(s, p, s->rays.p, s->stream);
        if (rc != RT_OK) return rc;
        HIP_TRY(launch_accumulate(p, s->sum.p + 3 * off, s->samples.p + off, s->misses.p + off, s->stream));
        HIP_TRY(launch_tile_host_layout(wb, h, s->sum.p + 3 * off, s->samples.p + off, s->misses.p + off, d_rec + off,
                                        s->stream));
        if (!s->band_ev[k]) HIP_TRY(hipEventCreateWithFlags(&s->band_ev[k], hipEventDisableTiming));
        HIP_TRY(hipEventRecord(s->band_ev[k], s->stream));
        HIP_TRY(hipStreamWaitEvent(s->copy_stream, s->band_ev[k], 0));
        if (k + 1 == nb) // (before the last chunks, so it has landed when they have)
            HIP_TRY(hipMemcpyAsync(s->rays_h.p, s->rays.p, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                   s->copy_stream));
        rc = queue_copy(s, plan, d_rec, off, off + (size_t)wb * h, sizeof(TileRec), per_band_chunks, s->copy_stream);
        if (rc != RT_OK) return rc;
    }
    rc = end_op(s, s->stream);
    if (rc != RT_OK) return rc;
    rc = consume_copies(s, plan, [&](const unsigned char* st, size_t a, size_t b) {
        const TileRec* r = reinterpret_cast<const TileRec*>(st);
        for (size_t o = a; o < b; o++) {
            sum_rgb[o].r += r[o].r;
            sum_rgb[o].g += r[o].g;
            sum_rgb[o].b += r[o].b;
            samples[o] += r[o].samples;
            misses[o] += r[o].misses;
        }
    });
    if (rc != RT_OK) return rc;
    if (rays_out) *rays_out += s->rays_h.p[0]; // copied before the last band's chunks, on the copy stream
    return RT_OK;
}

int rt_render_tile_1spp(rt_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, uint64_t seed,
                        uint64_t sample_index, rt_color* out)
{
    int rc = check_tile(s, x0, y0, w, h);
    if (rc != RT_OK) return rc;
    if (!out) {
        set_error("rt_render_tile_1spp: bad argument");
        return RT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(s->device));
    const size_t npix = (size_t)w * h;
    HIP_TRY(s->colors32.reserve(3 * npix));
    HIP_TRY(hipMemsetAsync(s->rays.p, 0, sizeof(unsigned long long), s->stream));
    PathParams p = make_params(s, x0, y0, w, h, 1, seed, sample_index);
    rc = run_path(s, p, s->rays.p, s->stream);
    if (rc != RT_OK) return rc;
    // the pass as fp32 in the caller's order (the kernel's sample values are fp32: widened exactly
    // on the host), 12 B per pixel over PCIe instead of 24, in chunks widened as they land
    HIP_TRY(launch_colors_1spp(p, s->colors32.p, s->stream));
    rc = end_op(s, s->stream);
    if (rc != RT_OK) return rc;
    return copy_consume(s, s->colors32.p, npix, 3 * sizeof(float), [&](const unsigned char* st, size_t a, size_t b) {
        const float* f = reinterpret_cast<const float*>(st);
        for (size_t o = a; o < b; o++) out[o] = rt_color{(double)f[3 * o], (double)f[3 * o + 1], (double)f[3 * o + 2]};
    });
}

} // extern "C"

namespace {

// The exact fp64 debug passes (DebugRaycaster.cs:170-212): mode 0 primary hit IDs, mode 1
// reference-BVH node counts.  Device output is row-major over the tile.
int debug_pass_device(rt_scene* s, int mode, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t* d_out,
                      hipStream_t stream, const char* name)
{
    int rc = check_tile(s, x0, y0, w, h);
    if (rc != RT_OK) return rc;
    if (!d_out) {
        set_error(std::string(name) + ": bad argument");
        return RT_ERR_ARG;
    }
    rc = ensure_ref_bvh(s);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(launch_primary_ids(s->dev, s->camd, x0, y0, w, h, mode, d_out, stream));
    return RT_OK;
}

// The same into a host buffer in the DoubleColor[w, h]-style x*h + y order.
int debug_pass_host(rt_scene* s, int mode, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t* out, const char* name)
{
    int rc = check_tile(s, x0, y0, w, h);
    if (rc != RT_OK) return rc;
    if (!out) {
        set_error(std::string(name) + ": bad argument");
        return RT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(s->device));
    const size_t npix = (size_t)w * h;
    HIP_TRY(s->ids.reserve(npix));
    rc = debug_pass_device(s, mode, x0, y0, w, h, s->ids.p, s->stream, name);
    if (rc != RT_OK) return rc;
    std::vector<int32_t> tmp(npix);
    HIP_TRY(hipMemcpyAsync(tmp.data(), s->ids.p, npix * sizeof(int32_t), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    std::atomic<bool> overflow{false};
    parallel_ranges((size_t)w, 64, [&](size_t xa, size_t xb) { // column ranges: disjoint output spans
        bool of = false;
        for (int y = 0; y < h; y++)
            for (size_t x = xa; x < xb; x++) {
                const int32_t v = tmp[(size_t)y * w + x];
                of |= v == -2;
                out[x * h + y] = v;
            }
        if (of) overflow = true;
    });
    if (overflow) {
        set_error(std::string(name) + ": the reference BVH is deeper than the exact kernel's traversal stack");
        return RT_ERR_STATE;
    }
    return RT_OK;
}

} // namespace

extern "C" {

int rt_primary_ids_device(rt_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t* d_ids, void* stream)
{
    return debug_pass_device(s, 0, x0, y0, w, h, d_ids, static_cast<hipStream_t>(stream), "rt_primary_ids_device");
}

int rt_primary_ids(rt_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t* ids_out)
{
    return debug_pass_host(s, 0, x0, y0, w, h, ids_out, "rt_primary_ids");
}

int rt_bvh_counts(rt_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t* counts_out)
{
    return debug_pass_host(s, 1, x0, y0, w, h, counts_out, "rt_bvh_counts");
}

} // extern "C"

// ------------------------------------------------------------------ row bands (multi-GPU) ----
// A band set (band, stride, offset) is frame rows {y : (y / band) % stride == offset}: device g of
// n owns set (8, n, g), interleaved for load balance (die.txt's background rows cost one ray per
// sample).  On the device a set is rendered as a tile of band_set_rows() rows, tile row r being
// frame row ((r / band) * stride + offset) * band + r % band (PathParams::band), into planar
// accumulators whose planes are `plane` elements apart -- the slot of rt_frame's gather, sized for
// the tallest set, so a shorter set leaves the end of each plane unused.
struct rt_frame {
    int n = 0, W = 0, H = 0, band = 8; // 8-row bands: any split of 1080 or 2160 rows is within one band of even
    std::vector<int> rows;            // rows of device g's band set
    size_t slot_pix = 0, slot_bytes = 0;
    std::vector<rt_scene*> scenes;
    std::vector<ncclComm_t> comms; // one rank per device (n = 1 too: one code path, a local copy)
    // Two pipeline stages (rt_frame_submit / rt_frame_collect): stage j holds every device's gather
    // slot, device 0's receive buffer (n slots), the pinned host copy of the gathered slots and of
    // the devices' ray counts, and the event that says the host copy has landed.
    static constexpr int kStages = 2;
    struct Stage {
        std::vector<unsigned char*> sendb; // per device: Σr | Σg | Σb fp64, samples, misses u32
        unsigned char* recvb = nullptr;    // device 0
        unsigned char* host = nullptr;     // pinned: n slots, then n ray counts
        hipEvent_t gathered = nullptr;     // device 0's render stream: the gather is complete
        hipEvent_t landed = nullptr;       // device 0's copy stream: the host copy is complete
        std::vector<hipEvent_t> rays_ev;   // per device: its ray count has been copied
    } st[kStages];
    hipStream_t copy_stream = nullptr;     // device 0: host copies, off the render streams
    unsigned long long submitted = 0, collected = 0; // renders queued / merged (at most kStages apart)
    int inject = 0;                        // rt_frame_inject_fault (tests)

    unsigned long long* host_rays(int j) { return reinterpret_cast<unsigned long long*>(st[j].host + slot_bytes * n); }
    ~rt_frame()
    {
        for (ncclComm_t c : comms) (void)ncclCommDestroy(c);
        for (auto& S : st) {
            for (int g = 0; g < (int)S.sendb.size(); g++)
                if (S.sendb[g]) {
                    (void)hipSetDevice(scenes[g]->device);
                    (void)hipFree(S.sendb[g]);
                }
            for (int g = 0; g < (int)S.rays_ev.size(); g++)
                if (S.rays_ev[g]) {
                    (void)hipSetDevice(scenes[g]->device);
                    (void)hipEventDestroy(S.rays_ev[g]);
                }
            if (!scenes.empty() && scenes[0]) (void)hipSetDevice(scenes[0]->device);
            if (S.recvb) (void)hipFree(S.recvb);
            if (S.landed) (void)hipEventDestroy(S.landed);
            if (S.gathered) (void)hipEventDestroy(S.gathered);
            if (S.host) (void)hipHostFree(S.host);
        }
        if (copy_stream) (void)hipStreamDestroy(copy_stream);
        for (rt_scene* s : scenes)
            if (s) rt_scene_destroy(s);
    }
};

namespace {

int band_set_rows(int H, int band, int stride, int offset)
{
    int rows = 0;
    for (int b = offset; b * band < H; b += stride) rows += std::min(band, H - b * band);
    return rows;
}

// Largest band set of the split: the plane stride of a gather slot.
int band_slot_rows(int H, int band, int stride)
{
    int m = 0;
    for (int o = 0; o < stride; o++) m = std::max(m, band_set_rows(H, band, stride, o));
    return m;
}

// Adds one band set's planar accumulators (device layout, planes `plane` apart) into frame buffers
// in the C# [x, y] order (x * H + y).
void scatter_band_set(const unsigned char* slot, size_t plane, int W, int H, int band, int stride, int offset,
                      rt_color* sum_rgb, uint32_t* samples, uint32_t* misses)
{
    const double* hs = reinterpret_cast<const double*>(slot);
    const uint32_t* hn = reinterpret_cast<const uint32_t*>(hs + 3 * plane);
    const uint32_t* hm = hn + plane;
    parallel_ranges((size_t)W, 64, [&](size_t xa, size_t xb) { // column ranges: disjoint output spans
        int tr = 0;
        for (int b = offset; b * band < H; b += stride)
            for (int y = b * band; y < std::min(H, (b + 1) * band); y++, tr++)
                for (size_t x = xa; x < xb; x++) {
                    const size_t i = (size_t)tr * W + x, o = x * H + y;
                    sum_rgb[o].r += hs[i];
                    sum_rgb[o].g += hs[plane + i];
                    sum_rgb[o].b += hs[2 * plane + i];
                    samples[o] += hn[i];
                    misses[o] += hm[i];
                }
    });
}

// Queues one band set's render on stream: path kernel + accumulate into d_slot (added to).
int render_band_set(rt_scene* s, int band, int stride, int offset, int rows, size_t plane, int spp, uint64_t seed,
                    uint64_t sample_base, unsigned char* d_slot, unsigned long long* d_rays, hipStream_t stream)
{
    double* d_sum = reinterpret_cast<double*>(d_slot);
    uint32_t* d_n = reinterpret_cast<uint32_t*>(d_sum + 3 * plane);
    uint32_t* d_m = d_n + plane;
    PathParams p = make_params(s, 0, 0, s->params.width, rows, spp, seed, sample_base);
    set_band(p, band, stride, offset);
    int rc = run_path(s, p, d_rays, stream);
    if (rc != RT_OK) return rc;
    HIP_TRY(launch_accumulate(p, d_sum, d_n, d_m, stream, plane));
    return end_op(s, stream);
}

} // namespace

extern "C" {

int rt_render_bands(rt_scene* s, int32_t band, int32_t band_stride, int32_t band_offset, int32_t spp, uint64_t seed,
                    uint64_t sample_base, rt_color* sum_rgb, uint32_t* samples, uint32_t* misses, uint64_t* rays_out)
{
    if (!s || band <= 0 || band_stride <= 0 || band_offset < 0 || band_offset >= band_stride || spp < 0 || !sum_rgb ||
        !samples || !misses) {
        set_error("rt_render_bands: bad argument");
        return RT_ERR_ARG;
    }
    if (!s->has_camera) {
        set_error("no camera set (rt_scene_set_camera)");
        return RT_ERR_STATE;
    }
    const int W = s->params.width, H = s->params.height;
    const int rows = band_set_rows(H, band, band_stride, band_offset);
    if (rows == 0 || spp == 0) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    const size_t plane = (size_t)band_slot_rows(H, band, band_stride) * W; // rt_frame's slot layout
    const size_t bytes = plane * (3 * sizeof(double) + 2 * sizeof(uint32_t));
    DevBuf<unsigned char> slot;
    HIP_TRY(slot.reserve(bytes));
    HIP_TRY(hipMemsetAsync(slot.p, 0, bytes, s->stream));
    HIP_TRY(hipMemsetAsync(s->rays.p, 0, sizeof(unsigned long long), s->stream));
    int rc = render_band_set(s, band, band_stride, band_offset, rows, plane, spp, seed, sample_base, slot.p, s->rays.p,
                             s->stream);
    if (rc != RT_OK) return rc;
    std::vector<unsigned char> host(bytes);
    unsigned long long hr = 0;
    HIP_TRY(hipMemcpyAsync(host.data(), slot.p, bytes, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipMemcpyAsync(&hr, s->rays.p, sizeof hr, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    scatter_band_set(host.data(), plane, W, H, band, band_stride, band_offset, sum_rgb, samples, misses);
    if (rays_out) *rays_out += hr;
    return RT_OK;
}

int rt_render_bands_device(rt_scene* s, int32_t band, int32_t band_stride, int32_t band_offset, int32_t spp,
                           uint64_t seed, uint64_t sample_base, double* d_sum, uint32_t* d_samples, uint32_t* d_misses,
                           uint64_t plane, unsigned long long* d_rays, void* stream)
{
    if (!s || band <= 0 || band_stride <= 0 || band_offset < 0 || band_offset >= band_stride || spp <= 0 || !d_sum ||
        !d_samples || !d_misses || !d_rays) {
        set_error("rt_render_bands_device: bad argument");
        return RT_ERR_ARG;
    }
    if (!s->has_camera) {
        set_error("no camera set (rt_scene_set_camera)");
        return RT_ERR_STATE;
    }
    const int W = s->params.width, H = s->params.height;
    const int rows = band_set_rows(H, band, band_stride, band_offset);
    if (plane == 0) plane = (uint64_t)band_slot_rows(H, band, band_stride) * W;
    if (plane < (uint64_t)rows * W) {
        set_error("rt_render_bands_device: plane stride smaller than the band set");
        return RT_ERR_ARG;
    }
    if (rows == 0) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    // the slot's sample/miss planes follow the sum planes only in rt_frame; here they are separate
    // buffers, each row-major over the set with the same plane stride as the sums
    double* sum = d_sum;
    uint32_t* n = d_samples;
    uint32_t* m = d_misses;
    PathParams p = make_params(s, 0, 0, W, rows, spp, seed, sample_base);
    set_band(p, band, band_stride, band_offset);
    hipStream_t st = static_cast<hipStream_t>(stream);
    int rc = run_path(s, p, d_rays, st);
    if (rc != RT_OK) return rc;
    HIP_TRY(launch_accumulate(p, sum, n, m, st, (size_t)plane));
    return end_op(s, st);
}

int rt_band_rows(int32_t height, int32_t band, int32_t band_stride, int32_t band_offset)
{
    if (height < 0 || band <= 0 || band_stride <= 0 || band_offset < 0 || band_offset >= band_stride) {
        set_error("rt_band_rows: bad argument");
        return RT_ERR_ARG;
    }
    return band_set_rows(height, band, band_stride, band_offset);
}

int rt_band_slot_rows(int32_t height, int32_t band, int32_t band_stride)
{
    if (height < 0 || band <= 0 || band_stride <= 0) {
        set_error("rt_band_slot_rows: bad argument");
        return RT_ERR_ARG;
    }
    return band_slot_rows(height, band, band_stride);
}

int rt_scatter_band_slot(const void* slot, uint64_t plane, int32_t width, int32_t height, int32_t band,
                         int32_t band_stride, int32_t band_offset, rt_color* sum_rgb, uint32_t* samples,
                         uint32_t* misses)
{
    if (!slot || !sum_rgb || !samples || !misses || width <= 0 || height <= 0 || band <= 0 || band_stride <= 0 ||
        band_offset < 0 || band_offset >= band_stride ||
        plane < (uint64_t)band_set_rows(height, band, band_stride, band_offset) * (uint64_t)width) {
        set_error("rt_scatter_band_slot: bad argument");
        return RT_ERR_ARG;
    }
    scatter_band_set(static_cast<const unsigned char*>(slot), (size_t)plane, width, height, band, band_stride,
                     band_offset, sum_rgb, samples, misses);
    return RT_OK;
}

int rt_frame_create(const rt_scene_params* params, const rt_prim* prims, int32_t n_prims, const rt_camera* camera,
                    int32_t n_gpus, rt_frame** out)
{
    if (!params || !camera || !out || n_gpus <= 0 || params->width <= 0 || params->height <= 0) {
        set_error("rt_frame_create: bad argument");
        return RT_ERR_ARG;
    }
    *out = nullptr;
    if (n_gpus > rt_device_count()) {
        set_error("rt_frame_create: not enough devices");
        return RT_ERR_NODEVICE;
    }
    std::unique_ptr<rt_frame> f(new rt_frame);
    f->n = n_gpus;
    f->W = params->width;
    f->H = params->height;
    for (int g = 0; g < n_gpus; g++) f->rows.push_back(band_set_rows(f->H, f->band, n_gpus, g));
    f->slot_pix = (size_t)band_slot_rows(f->H, f->band, n_gpus) * f->W;
    f->slot_bytes = f->slot_pix * (3 * sizeof(double) + 2 * sizeof(uint32_t));
    f->scenes.assign(n_gpus, nullptr);
    for (auto& S : f->st) {
        S.sendb.assign(n_gpus, nullptr);
        S.rays_ev.assign(n_gpus, nullptr);
    }
    std::vector<int> devs(n_gpus);
    for (int g = 0; g < n_gpus; g++) {
        devs[g] = g;
        int rc = rt_scene_create(params, prims, n_prims, g, &f->scenes[g]);
        if (rc == RT_OK) rc = rt_scene_set_camera(f->scenes[g], camera);
        if (rc != RT_OK) return rc;
        HIP_TRY(hipSetDevice(g));
        for (auto& S : f->st) {
            HIP_TRY(hipMalloc(&S.sendb[g], f->slot_bytes));
            HIP_TRY(hipEventCreateWithFlags(&S.rays_ev[g], hipEventDisableTiming));
        }
    }
    HIP_TRY(hipSetDevice(0));
    HIP_TRY(hipStreamCreateWithFlags(&f->copy_stream, hipStreamNonBlocking));
    for (auto& S : f->st) {
        HIP_TRY(hipMalloc(&S.recvb, f->slot_bytes * n_gpus));
        HIP_TRY(hipHostMalloc(&S.host, f->slot_bytes * n_gpus + sizeof(unsigned long long) * n_gpus,
                              hipHostMallocDefault));
        HIP_TRY(hipEventCreateWithFlags(&S.landed, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&S.gathered, hipEventDisableTiming));
    }
    f->comms.assign(n_gpus, nullptr);
    if (ncclCommInitAll(f->comms.data(), n_gpus, devs.data()) != ncclSuccess) {
        f->comms.clear();
        set_error("rt_frame_create: ncclCommInitAll failed");
        return RT_ERR_NCCL;
    }
    *out = f.release();
    return RT_OK;
}

int rt_frame_set_camera(rt_frame* f, const rt_camera* camera)
{
    if (!f || !camera) {
        set_error("rt_frame_set_camera: bad argument");
        return RT_ERR_ARG;
    }
    for (rt_scene* s : f->scenes) {
        int rc = rt_scene_set_camera(s, camera);
        if (rc != RT_OK) return rc;
    }
    return RT_OK;
}

namespace {

// Drops every queued stage after a failure: waits for the devices' streams, so that no queued
// copy still writes a stage's buffers, and restarts the pipeline empty.
void frame_drain(rt_frame* f)
{
    for (rt_scene* s : f->scenes) {
        (void)hipSetDevice(s->device);
        (void)hipStreamSynchronize(s->stream);
    }
    (void)hipSetDevice(f->scenes[0]->device);
    (void)hipStreamSynchronize(f->copy_stream);
    f->submitted = f->collected = 0;
}

// The gather of stage j: every device's slot onto device 0, one grouped RCCL call.  The group is
// closed on every path (an open group would swallow the next call's gathers).
int frame_gather(rt_frame* f, int j)
{
    if (ncclGroupStart() != ncclSuccess) {
        set_error("rt_frame_render: ncclGroupStart failed");
        return RT_ERR_NCCL;
    }
    int rc = RT_OK;
    for (int g = 0; g < f->n && rc == RT_OK; g++) {
        if (f->inject == 1) { // rt_frame_inject_fault: a failure inside the group, before any gather
            f->inject = 0;
            set_error("rt_frame_render: injected fault inside the gather group");
            rc = RT_ERR_HIP;
            break;
        }
        const hipError_t e = hipSetDevice(f->scenes[g]->device);
        if (e != hipSuccess) {
            set_error(std::string("rt_frame_render: ") + hipGetErrorString(e));
            rc = RT_ERR_HIP;
            break;
        }
        if (ncclGather(f->st[j].sendb[g], g == 0 ? f->st[j].recvb : nullptr, f->slot_bytes, ncclUint8, 0, f->comms[g],
                       f->scenes[g]->stream) != ncclSuccess) {
            set_error("rt_frame_render: ncclGather failed");
            rc = RT_ERR_NCCL;
        }
    }
    if (ncclGroupEnd() != ncclSuccess && rc == RT_OK) {
        set_error("rt_frame_render: ncclGather failed");
        rc = RT_ERR_NCCL;
    }
    return rc;
}

int frame_submit(rt_frame* f, int32_t spp, uint64_t seed, uint64_t sample_base)
{
    const int j = (int)(f->submitted % rt_frame::kStages);
    auto& S = f->st[j];
    rt_scene* s0 = f->scenes[0];
    // every device renders its band set into its slot of stage j, concurrently (asynchronous launches);
    // the stage's previous host copy has been collected (at most kStages in flight), so its buffers
    // are free once device 0's copy stream has passed it, which the render streams wait for
    for (int g = 0; g < f->n; g++) {
        rt_scene* s = f->scenes[g];
        HIP_TRY(hipSetDevice(s->device));
        if (g == 0) HIP_TRY(hipStreamWaitEvent(s->stream, S.landed, 0));
        HIP_TRY(hipMemsetAsync(S.sendb[g], 0, f->slot_bytes, s->stream));
        HIP_TRY(hipMemsetAsync(s->rays.p, 0, sizeof(unsigned long long), s->stream));
        if (f->rows[g] > 0) {
            int rc = render_band_set(s, f->band, f->n, g, f->rows[g], f->slot_pix, spp, seed, sample_base, S.sendb[g],
                                     s->rays.p, s->stream);
            if (rc != RT_OK) return rc;
        }
        // the ray count, before the next stage's render zeroes it (pinned: the copy is asynchronous)
        HIP_TRY(hipMemcpyAsync(f->host_rays(j) + g, s->rays.p, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                               s->stream));
        HIP_TRY(hipEventRecord(S.rays_ev[g], s->stream));
    }
    // the slots meet on device 0 through one RCCL gather over xGMI
    int rc = frame_gather(f, j);
    if (rc != RT_OK) return rc;
    // the host copy on device 0's copy stream, so that the next stage's render does not queue behind it
    HIP_TRY(hipSetDevice(s0->device));
    HIP_TRY(hipEventRecord(S.gathered, s0->stream));
    HIP_TRY(hipStreamWaitEvent(f->copy_stream, S.gathered, 0));
    HIP_TRY(hipMemcpyAsync(S.host, S.recvb, f->slot_bytes * f->n, hipMemcpyDeviceToHost, f->copy_stream));
    HIP_TRY(hipEventRecord(S.landed, f->copy_stream));
    f->submitted++;
    return RT_OK;
}

int frame_collect(rt_frame* f, rt_color* sum_rgb, uint32_t* samples, uint32_t* misses, uint64_t* rays_out)
{
    const int j = (int)(f->collected % rt_frame::kStages);
    auto& S = f->st[j];
    HIP_TRY(hipSetDevice(f->scenes[0]->device));
    HIP_TRY(hipEventSynchronize(S.landed));
    for (int g = 0; g < f->n; g++) {
        HIP_TRY(hipSetDevice(f->scenes[g]->device));
        HIP_TRY(hipEventSynchronize(S.rays_ev[g]));
    }
    for (int g = 0; g < f->n; g++)
        scatter_band_set(S.host + f->slot_bytes * g, f->slot_pix, f->W, f->H, f->band, f->n, g, sum_rgb, samples,
                         misses);
    if (rays_out)
        for (int g = 0; g < f->n; g++) *rays_out += f->host_rays(j)[g];
    f->collected++;
    return RT_OK;
}

} // namespace

int rt_frame_submit(rt_frame* f, int32_t spp, uint64_t seed, uint64_t sample_base)
{
    if (!f || spp <= 0) {
        set_error("rt_frame_submit: bad argument");
        return RT_ERR_ARG;
    }
    if (f->submitted - f->collected >= (unsigned long long)rt_frame::kStages) {
        set_error("rt_frame_submit: two renders in flight; rt_frame_collect the oldest first");
        return RT_ERR_STATE;
    }
    const int rc = frame_submit(f, spp, seed, sample_base);
    if (rc != RT_OK) frame_drain(f);
    return rc;
}

int rt_frame_collect(rt_frame* f, rt_color* sum_rgb, uint32_t* samples, uint32_t* misses, uint64_t* rays_out)
{
    if (!f || !sum_rgb || !samples || !misses) {
        set_error("rt_frame_collect: bad argument");
        return RT_ERR_ARG;
    }
    if (f->collected == f->submitted) {
        set_error("rt_frame_collect: nothing submitted");
        return RT_ERR_STATE;
    }
    const int rc = frame_collect(f, sum_rgb, samples, misses, rays_out);
    if (rc != RT_OK) frame_drain(f);
    return rc;
}

int rt_frame_render(rt_frame* f, int32_t spp, uint64_t seed, uint64_t sample_base, rt_color* sum_rgb,
                    uint32_t* samples, uint32_t* misses, uint64_t* rays_out)
{
    if (!f || spp < 0 || !sum_rgb || !samples || !misses) {
        set_error("rt_frame_render: bad argument");
        return RT_ERR_ARG;
    }
    if (spp == 0) return RT_OK;
    if (f->submitted != f->collected) {
        set_error("rt_frame_render: renders submitted and not collected");
        return RT_ERR_STATE;
    }
    int rc = rt_frame_submit(f, spp, seed, sample_base);
    if (rc == RT_OK) rc = rt_frame_collect(f, sum_rgb, samples, misses, rays_out);
    return rc;
}

int rt_frame_inject_fault(rt_frame* f, int32_t point)
{
    if (!f || point < 0 || point > 1) {
        set_error("rt_frame_inject_fault: bad argument");
        return RT_ERR_ARG;
    }
    f->inject = point;
    return RT_OK;
}

void rt_frame_destroy(rt_frame* f)
{
    if (!f) return;
    for (rt_scene* s : f->scenes)
        if (s) {
            (void)hipSetDevice(s->device);
            (void)hipStreamSynchronize(s->stream);
        }
    if (f->copy_stream) {
        (void)hipSetDevice(f->scenes[0]->device);
        (void)hipStreamSynchronize(f->copy_stream);
    }
    delete f;
}

int rt_render_frame_multi(const rt_scene_params* params, const rt_prim* prims, int32_t n_prims,
                          const rt_camera* camera, int32_t n_gpus, int32_t spp, uint64_t seed, uint64_t sample_base,
                          rt_color* sum_rgb, uint32_t* samples, uint32_t* misses, uint64_t* rays_out)
{
    if (!sum_rgb || !samples || !misses || spp < 0) {
        set_error("rt_render_frame_multi: bad argument");
        return RT_ERR_ARG;
    }
    rt_frame* f = nullptr;
    int rc = rt_frame_create(params, prims, n_prims, camera, n_gpus, &f);
    if (rc == RT_OK) rc = rt_frame_render(f, spp, seed, sample_base, sum_rgb, samples, misses, rays_out);
    rt_frame_destroy(f);
    return rc;
}

int rt_parse_scene(const char* text, rt_scene_params* params, rt_prim* prims, int32_t* n_prims, rt_camera* cameras,
                   int32_t* n_cameras)
{
    if (!text || !n_prims || !n_cameras) {
        set_error("rt_parse_scene: bad argument");
        return RT_ERR_ARG;
    }
    ParsedScene ps;
    std::string err;
    if (!parse_scene_text(text, ps, err)) {
        set_error(err);
        return RT_ERR_PARSE;
    }
    const int cap_p = *n_prims, cap_c = *n_cameras;
    *n_prims = (int32_t)ps.prims.size();
    *n_cameras = (int32_t)ps.cameras.size();
    if (params) *params = ps.params;
    if (prims) {
        if (cap_p < (int)ps.prims.size()) {
            set_error("rt_parse_scene: primitive array too small");
            return RT_ERR_ARG;
        }
        std::copy(ps.prims.begin(), ps.prims.end(), prims);
    }
    if (cameras) {
        if (cap_c < (int)ps.cameras.size()) {
            set_error("rt_parse_scene: camera array too small");
            return RT_ERR_ARG;
        }
        std::copy(ps.cameras.begin(), ps.cameras.end(), cameras);
    }
    return RT_OK;
}

int rt_ref_bvh_export(const rt_prim* prims, int32_t n, int32_t* leaf_order, double* boxes, int32_t* n_nodes,
                      int32_t* depth)
{
    if (n < 0 || (n > 0 && !prims)) {
        set_error("rt_ref_bvh_export: bad argument");
        return RT_ERR_ARG;
    }
    std::vector<HostPrim> host = prepare_prims(prims, n);
    RefBvh ref = build_ref_bvh(host);
    int k = 0;
    for (size_t i = 0; i < ref.nodes.size(); i++) {
        const RefNode& r = ref.nodes[i];
        if (r.prim >= 0 && leaf_order) leaf_order[k++] = r.prim;
        if (boxes) {
            double* b = boxes + 8 * i;
            b[0] = r.mn.x; b[1] = r.mn.y; b[2] = r.mn.z; b[3] = r.mn.w;
            b[4] = r.mx.x; b[5] = r.mx.y; b[6] = r.mx.z; b[7] = r.mx.w;
        }
    }
    if (n_nodes) *n_nodes = (int32_t)ref.nodes.size();
    if (depth) *depth = ref.depth;
    return RT_OK;
}

int rt_tonemap_device(const double* d_sum, const uint32_t* d_samples, const uint32_t* d_misses, int32_t w, int32_t h,
                      rt_color background, double background_alpha, double exposure, int32_t* d_argb, void* stream)
{
    if (!d_sum || !d_samples || !d_misses || !d_argb || w <= 0 || h <= 0) {
        set_error("rt_tonemap_device: bad argument");
        return RT_ERR_ARG;
    }
    HIP_TRY(launch_tonemap(w, h, d_sum, d_samples, d_misses, background, background_alpha, exposure, d_argb,
                           static_cast<hipStream_t>(stream)));
    return RT_OK;
}

int32_t rt_sample_output(rt_color sum, uint32_t n_samples, uint32_t n_misses, rt_color back, double back_alpha,
                         double exposure)
{
    // SampleSet.GetOutput / GetColorCode (SampleSet.cs:50-113) with Util.Clamp's SSE form
    auto clamp01 = [](double v) {
        v = v > 0.0 ? v : 0.0;
        return v < 1.0 ? v : 1.0;
    };
    auto code = [&](double r, double g, double b, double a) {
        return (int32_t)(((uint32_t)(int32_t)(clamp01(a) * 255) << 24) | ((uint32_t)(int32_t)(clamp01(r) * 255) << 16) |
                         ((uint32_t)(int32_t)(clamp01(g) * 255) << 8) | (uint32_t)(int32_t)(clamp01(b) * 255));
    };
    if (n_samples == 0) return code(back.r * exposure, back.g * exposure, back.b * exposure, back_alpha);
    double total = (double)n_samples + (double)n_misses;
    double mult = exposure / n_samples;
    double r = sum.r * mult, g = sum.g * mult, b = sum.b * mult, a = 1;
    double bam = n_misses / total, bk = bam * back_alpha;
    r += (back.r - r) * bk;
    g += (back.g - g) * bk;
    b += (back.b - b) * bk;
    a += (back_alpha - a) * bam;
    const double gamma = 1 / 2.2;
    return code(pow(r, gamma), pow(g, gamma), pow(b, gamma), a);
}

} // extern "C"
