// bvh_check.cpp -- host-side structural checks of the fast-path acceleration structures
// (built by tests/test_host.py through `make -C raytracercore_amd/csrc bvh_check`).
//
// For a scene file: the binned-SAH BVH2 and both 4-wide quantised collapses (greedy, SAH-optimal) must
//   * reference every non-plane primitive exactly once;
//   * have, for every wide node, dequantised child planes (origin + q * 2^e, in exact
//     arithmetic) that contain every primitive box below that child;
//   * never need more traversal-stack entries than the computed stack_need.
// Prints "ok <n_prims> <bvh2 nodes> <wide nodes> <stack_need>" per collapse or the first failure;
// with --ref also builds the reference BVH and the cameras (the host inputs of the exact pass).
// `make bvh_check_asan` builds it with AddressSanitizer and UndefinedBehaviorSanitizer on the host
// sources (tests/test_host.py runs both builds).
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <vector>

#include "host_scene.h"

using namespace rtc;

static int as_i(float f)
{
    int i;
    std::memcpy(&i, &f, 4);
    return i;
}
static unsigned as_u(float f)
{
    unsigned u;
    std::memcpy(&u, &f, 4);
    return u;
}

struct Ctx {
    const std::vector<HostPrim>* H;
    const SahBvh* b2;
    const Bvh4* b4;
    std::vector<int> seen;
    int max_stack = 0;
    bool ok = true;
    char msg[256] = {0};
};

static void leaf_prims(const Ctx& c, int ref, std::vector<int>& out)
{
    const int code = ~ref, first = code >> 3, cnt = (code & 7) + 1;
    for (int k = first; k < first + cnt; k++) out.push_back(c.b2->order[k]);
}

// all primitives below a wide-tree reference
static void below(const Ctx& c, int ref, std::vector<int>& out)
{
    if (ref < 0) {
        leaf_prims(c, ref, out);
        return;
    }
    const Node4Q& q = c.b4->nodes[ref];
    const int nc = as_i(q.d.z);
    const int refs[4] = {as_i(q.c.z), as_i(q.c.w), as_i(q.d.x), as_i(q.d.y)};
    for (int k = 0; k < nc; k++) below(c, refs[k], out);
}

static void visit(Ctx& c, int ref, int pushes)
{
    if (!c.ok) return;
    if (ref < 0) {
        std::vector<int> p;
        leaf_prims(c, ref, p);
        for (int i : p) c.seen[i]++;
        return;
    }
    const Node4Q& q = c.b4->nodes[ref];
    const int nc = as_i(q.d.z);
    c.max_stack = std::max(c.max_stack, pushes + nc - 1);
    const unsigned ex = as_u(q.a.w);
    const double org[3] = {q.a.x, q.a.y, q.a.z};
    const int e[3] = {(int)(ex & 255u) - 128, (int)((ex >> 8) & 255u) - 128, (int)((ex >> 16) & 255u) - 128};
    const unsigned lo[3] = {as_u(q.b.x), as_u(q.b.z), as_u(q.c.x)}, hi[3] = {as_u(q.b.y), as_u(q.b.w), as_u(q.c.y)};
    const int refs[4] = {as_i(q.c.z), as_i(q.c.w), as_i(q.d.x), as_i(q.d.y)};
    for (int k = 0; k < nc; k++) {
        std::vector<int> p;
        below(c, refs[k], p);
        for (int a = 0; a < 3; a++) {
            const double s = std::ldexp(1.0, e[a]);
            const double plo = org[a] + ((lo[a] >> (8 * k)) & 255u) * s;
            const double phi = org[a] + ((hi[a] >> (8 * k)) & 255u) * s;
            for (int i : p) {
                const double bl[3] = {(*c.H)[i].box.mn.x, (*c.H)[i].box.mn.y, (*c.H)[i].box.mn.z};
                const double bh[3] = {(*c.H)[i].box.mx.x, (*c.H)[i].box.mx.y, (*c.H)[i].box.mx.z};
                if (!(plo <= bl[a] && phi >= bh[a])) {
                    c.ok = false;
                    std::snprintf(c.msg, sizeof c.msg, "node %d child %d axis %d: [%.9g, %.9g] misses prim %d [%.9g, %.9g]",
                                  ref, k, a, plo, phi, i, bl[a], bh[a]);
                    return;
                }
            }
        }
        visit(c, refs[k], pushes + nc - 1);
    }
}

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    std::ifstream f(argv[1]);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    ParsedScene ps;
    std::string err;
    if (!parse_scene_text(text.c_str(), ps, err)) {
        std::printf("parse error: %s\n", err.c_str());
        return 1;
    }
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const std::vector<HostPrim> H = prepare_prims(ps.prims.data(), (int)ps.prims.size());
    const auto t1 = clk::now();
    const SahBvh b2 = build_sah_bvh(H, H.size() > 256 ? 4 : 2, true);
    const auto t2 = clk::now();
    // both wide collapses: greedy over the BVH2's leaves, SAH-optimal over the whole tree
    const WideCosts wc;
    for (int mode = 0; mode < 2; mode++) {
        const auto t3 = clk::now();
        const Bvh4 b4 = build_bvh4(b2, mode ? &wc : nullptr);
        const auto t4 = clk::now();
        if (std::getenv("BVH_CHECK_TIME")) {
            auto ms = [](clk::duration d) { return std::chrono::duration<double, std::milli>(d).count(); };
            std::fprintf(stderr, "prepare %.1f ms, sah %.1f ms, %s collapse %.1f ms\n", ms(t1 - t0), ms(t2 - t1),
                         mode ? "sah" : "greedy", ms(t4 - t3));
        }
        Ctx c;
        c.H = &H;
        c.b2 = &b2;
        c.b4 = &b4;
        c.seen.assign(H.size(), 0);
        if (!b4.nodes.empty() || (b4.root < 0 && !b2.order.empty())) visit(c, b4.root, 0);
        if (!c.ok) {
            std::printf("FAIL %s (%s collapse)\n", c.msg, mode ? "sah" : "greedy");
            return 1;
        }
        for (size_t i = 0; i < H.size(); i++) {
            const int want = H[i].kind == RT_PRIM_PLANE ? 0 : 1;
            if (c.seen[i] != want) {
                std::printf("FAIL prim %zu referenced %d times (%s collapse)\n", i, c.seen[i], mode ? "sah" : "greedy");
                return 1;
            }
        }
        if (c.max_stack > b4.stack_need) {
            std::printf("FAIL stack %d > stack_need %d\n", c.max_stack, b4.stack_need);
            return 1;
        }
        std::printf("%s %zu %zu %zu %d\n", mode ? "" : "ok", H.size(), b2.nodes.size(), b4.nodes.size(), b4.stack_need);
    }
    if (argc > 2 && std::strcmp(argv[2], "--ref") == 0) { // the exact pass's inputs too (sanitizer runs)
        const RefBvh r = build_ref_bvh(H);
        for (const rt_camera& cam : ps.cameras) {
            CameraD d;
            CameraF cf;
            camera_init(cam, ps.params.width, ps.params.height, d, cf);
        }
        std::printf("ref %zu %d\n", r.nodes.size(), r.depth);
    }
    return 0;
}
