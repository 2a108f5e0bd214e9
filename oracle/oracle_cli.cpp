// oracle_cli.cpp -- command-line driver of the CPU oracle (TEST INFRASTRUCTURE).
//   oracle_cli SCENE [--size W H] [--camera I] [--spp N] [--seed S] [--threads T]
//              [--ids OUT.bin] [--ppm OUT.ppm] [--exposure E]
// Renders a whole frame FullRaytracer-style and prints a JSON line with samples/s and
// Mrays/s (the reference status line's quantities, FullRaytracer.cs:346-357).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "oracle.h"

int main(int argc, char** argv)
{
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s SCENE [--size W H] [--camera I] [--spp N] [--seed S] [--threads T] "
                             "[--ids OUT] [--ppm OUT]\n", argv[0]);
        return 2;
    }
    std::ifstream f(argv[1]);
    if (!f) {
        std::fprintf(stderr, "cannot open %s\n", argv[1]);
        return 2;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    int w = -1, h = -1, cam = 0, spp = 1, threads = 0;
    unsigned long long seed = 0;
    double exposure = 1.0;
    const char *ids_path = nullptr, *ppm_path = nullptr;
    for (int i = 2; i < argc; i++) {
        std::string a = argv[i];
        if (a == "--size" && i + 2 < argc) {
            w = std::atoi(argv[++i]);
            h = std::atoi(argv[++i]);
        } else if (a == "--camera" && i + 1 < argc) cam = std::atoi(argv[++i]);
        else if (a == "--spp" && i + 1 < argc) spp = std::atoi(argv[++i]);
        else if (a == "--seed" && i + 1 < argc) seed = std::strtoull(argv[++i], nullptr, 10);
        else if (a == "--threads" && i + 1 < argc) threads = std::atoi(argv[++i]);
        else if (a == "--ids" && i + 1 < argc) ids_path = argv[++i];
        else if (a == "--ppm" && i + 1 < argc) ppm_path = argv[++i];
        else if (a == "--exposure" && i + 1 < argc) exposure = std::atof(argv[++i]);
        else {
            std::fprintf(stderr, "bad argument %s\n", a.c_str());
            return 2;
        }
    }
    char err[512];
    orc_scene* s = orc_load_text(ss.str().c_str(), err, sizeof err);
    if (!s) {
        std::fprintf(stderr, "load failed: %s\n", err);
        return 1;
    }
    if (w > 0) orc_set_size(s, w, h);
    if (orc_select_camera(s, cam) != 0) {
        std::fprintf(stderr, "bad camera\n");
        return 1;
    }
    rt_scene_params p;
    orc_export(s, &p, nullptr, nullptr);
    int W = p.width, H = p.height;
    int nodes = 0, depth = 0;
    orc_bvh_info(s, &nodes, &depth);
    if (ids_path) {
        std::vector<int32_t> ids((size_t)W * H);
        orc_primary_ids(s, 0, 0, W, H, ids.data());
        FILE* o = std::fopen(ids_path, "wb");
        std::fwrite(ids.data(), 4, ids.size(), o);
        std::fclose(o);
    }
    std::vector<rt_color> sum((size_t)W * H, rt_color{0, 0, 0});
    std::vector<uint32_t> samples((size_t)W * H, 0), misses((size_t)W * H, 0);
    uint64_t rays = 0;
    double secs = 0;
    int used = 0;
    if (spp > 0) orc_render_frame(s, spp, seed, threads, sum.data(), samples.data(), misses.data(), &rays, &secs, &used);
    double nsamp = (double)W * H * spp;
    std::printf("{\"scene\": \"%s\", \"width\": %d, \"height\": %d, \"spp\": %d, \"prims\": %d, \"bvh_nodes\": %d, "
                "\"bvh_depth\": %d, \"threads\": %d, \"seconds\": %.4f, \"samples_per_s\": %.1f, \"mrays_per_s\": %.3f, "
                "\"rays\": %llu}\n",
                argv[1], W, H, spp, orc_num_prims(s), nodes, depth, used, secs, secs > 0 ? nsamp / secs : 0.0,
                secs > 0 ? rays / secs / 1e6 : 0.0, (unsigned long long)rays);
    if (ppm_path && spp > 0) {
        rt_color back;
        double back_a;
        orc_background(s, &back, &back_a);
        FILE* o = std::fopen(ppm_path, "wb");
        std::fprintf(o, "P6\n%d %d\n255\n", W, H);
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) {
                size_t i = (size_t)x * H + y;
                int32_t c = orc_sample_output(sum[i], samples[i], misses[i], back, back_a, exposure);
                unsigned char px[3] = {(unsigned char)((c >> 16) & 255), (unsigned char)((c >> 8) & 255),
                                       (unsigned char)(c & 255)};
                std::fwrite(px, 1, 3, o);
            }
        std::fclose(o);
    }
    orc_destroy(s);
    return 0;
}
