// abi_host_check.cpp -- the library's host-only C entry points driven from C++, built with
// AddressSanitizer and UndefinedBehaviorSanitizer over the whole library's host code
// (`make -C raytracercore_amd/csrc abi_host_check_asan`; tests/test_host.py runs it).  No device is
// touched: the scene text parser (two-call protocol), the brute-force layout (rectangles, boxes,
// frames, the grouped cut, the finders' caps), the reference BVH export, the scene-specialised
// build's header, the band-set layout and merge, the tonemap of one pixel, and the argument checks.
// usage: abi_host_check SCENE_FILE...   Prints one "ok ..." line per scene.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/rtcore.h"

static int fail(const char* what, int rc)
{
    char buf[512];
    rt_last_error(buf, sizeof buf);
    std::printf("FAIL %s: %d %s\n", what, rc, buf);
    return 1;
}

int main(int argc, char** argv)
{
    for (int a = 1; a < argc; a++) {
        std::ifstream f(argv[a]);
        std::stringstream ss;
        ss << f.rdbuf();
        const std::string text = ss.str();
        rt_scene_params params;
        int32_t n = 0, nc = 0;
        int rc = rt_parse_scene(text.c_str(), &params, nullptr, &n, nullptr, &nc);
        if (rc != 0) return fail("rt_parse_scene (counts)", rc);
        std::vector<rt_prim> prims(n);
        std::vector<rt_camera> cams(nc);
        rc = rt_parse_scene(text.c_str(), &params, prims.data(), &n, cams.data(), &nc);
        if (rc != 0) return fail("rt_parse_scene", rc);
        int32_t layout[RT_LAYOUT_COUNT];
        rc = rt_debug_brute_layout(prims.data(), n, layout, RT_LAYOUT_COUNT);
        if (rc != 0) return fail("rt_debug_brute_layout", rc);
        int32_t nodes = 0, depth = 0;
        if (n > 0 && n <= 50000) {
            std::vector<int32_t> order(n);
            std::vector<double> boxes((size_t)8 * (2 * n - 1));
            rc = rt_ref_bvh_export(prims.data(), n, order.data(), boxes.data(), &nodes, &depth);
            if (rc != 0) return fail("rt_ref_bvh_export", rc);
        }
        int64_t hdr = 0;
        if (nc > 0 && n <= 48) {
            hdr = rt_debug_jit_header(&params, prims.data(), n, &cams[0], 0, nullptr, 0);
            if (hdr < 0) return fail("rt_debug_jit_header (length)", (int)hdr);
            std::vector<char> buf((size_t)hdr + 1);
            if (rt_debug_jit_header(&params, prims.data(), n, &cams[0], 0, buf.data(), (int64_t)buf.size()) != hdr)
                return fail("rt_debug_jit_header", -1);
        }
        // the band-set layout and merge of a frame of this scene's size split 3 ways
        const int W = params.width > 0 ? params.width : 64, H = params.height > 0 ? params.height : 48, stride = 3;
        const int slot_rows = rt_band_slot_rows(H, 8, stride);
        std::vector<rt_color> sum((size_t)W * H);
        std::vector<uint32_t> ns((size_t)W * H), ms((size_t)W * H);
        int rows_total = 0;
        for (int off = 0; off < stride; off++) {
            const int rows = rt_band_rows(H, 8, stride, off);
            rows_total += rows;
            const size_t plane = (size_t)slot_rows * W;
            std::vector<double> slot(4 * plane, 0.0);
            uint32_t* su = reinterpret_cast<uint32_t*>(slot.data() + 3 * plane);
            for (size_t i = 0; i < (size_t)rows * W; i++) {
                slot[i] = 1.0;
                su[i] = 1;
            }
            rc = rt_scatter_band_slot(slot.data(), plane, W, H, 8, stride, off, sum.data(), ns.data(), ms.data());
            if (rc != 0) return fail("rt_scatter_band_slot", rc);
        }
        for (size_t i = 0; i < ns.size(); i++)
            if (ns[i] != 1 || sum[i].r != 1.0) return fail("band sets do not cover the frame once", -1);
        if (rows_total != H) return fail("rt_band_rows", -1);
        const rt_color c{0.5, 0.25, 2.0}, bg{0, 0, 0};
        (void)rt_sample_output(c, 1, 1, bg, 0.0, 1.0);
        // refused arguments
        if (rt_scatter_band_slot(nullptr, 0, W, H, 8, stride, 0, sum.data(), ns.data(), ms.data()) == 0 ||
            rt_debug_brute_layout(prims.data(), -1, layout, 1) == 0 || rt_band_rows(H, 0, 1, 0) >= 0)
            return fail("argument checks", -1);
        std::printf("ok %s prims %d cameras %d rects %d boxes %d frames %d ref nodes %d header %lld\n", argv[a], n, nc,
                    layout[0], layout[1], layout[2], nodes, (long long)hdr);
    }
    return 0;
}
