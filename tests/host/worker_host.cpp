// worker_host.cpp -- a native stand-in for the C# drop-in of INTEGRATION.md §3: the GpuRaytracer
// worker and FullRaytracer's tile hand-out and update loop, driving librtcore_hip.so only through
// include/rtcore.h (no Python, no torch), as the C# host would through P/Invoke.
//
//   FullRaytracer(threads)         FullRaytracer.cs:66-72   TilesY = floor(sqrt(T)), TilesX = T / TilesY
//   Start: tile rectangles         FullRaytracer.cs:271-285 left = x*w/TilesX ... (FromLTRB)
//   GetWorkingTile                 FullRaytracer.cs:219-229 round-robin under a lock
//   spawn one worker per thread    FullRaytracer.cs:297-302 (here: one rt_scene handle per worker)
//   worker pass loop               Raytracer.cs:294-330     tile -> one pass -> OnTileFinished
//   OnTileFinished / update merge  FullRaytracer.cs:210-214, 326-344: AddSample, or AddMiss for a
//                                  DoubleColor.Placeholder (1-spp mode); the bulk merge of
//                                  INTEGRATION.md §3 (Σ, samples, misses added) in bulk mode
//
// Pass arrays are recycled under INTEGRATION.md's ownership rule (worker from take to
// OnTileFinished, update loop until its merge, then back to the worker).  The k-th hand-out of a
// tile renders that tile's samples [k*spp, (k+1)*spp) with one seed, so the merged frame can be
// checked against single-threaded whole-frame renders of the same sample indices:
//   1spp: every tile pass equals the matching window of the whole-frame pass bit for bit (the
//         stream is keyed by (seed, pixel, sample), not by tile or thread), and the merged frame
//         equals the whole-frame passes merged in order -- counts exactly, Σ to 1e-12 (two workers
//         holding the same tile may finish its passes out of order);
//   bulk: counts exactly, Σ to 1e-5 relative (a launch sums a pixel's samples in fp32 chunks
//         whose size follows the launch's shape, so tile and frame group them differently).
// MODE frame is the whole-frame loop of INTEGRATION.md §3 instead: one rt_frame over DEVICES
// devices (band sets, RCCL gather to device 0), passes submitted one ahead of their collect
// (rt_frame_submit / rt_frame_collect) and merged in bulk; checked like bulk (THREADS unused).
// usage: worker_host SCENE W H THREADS PASSES MODE(1spp|bulk|frame) SPP [DEVICES]
// Prints "ok ..." with the rates, or "FAIL ..." and exits non-zero.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rtcore.h"

namespace {

struct Rect {
    int left, top, width, height;
};

struct PassBuffers { // one pass of one tile, laid out x*h + y (C# rectangular arrays)
    std::vector<rt_color> color;     // 1spp: the pass's colours (Placeholder = miss); bulk: Σ
    std::vector<uint32_t> samples, misses;
    void fit(size_t n, bool bulk)
    {
        color.resize(n);
        if (bulk) {
            samples.resize(n);
            misses.resize(n);
        }
    }
};

class Worker;

struct ImageUpdate {
    Rect tile;
    PassBuffers* buf;
    Worker* worker;
    uint64_t rays;
};

std::atomic<bool> g_failed{false};
std::mutex g_print;

void report_failure(const char* what, int rc)
{
    char msg[512] = {0};
    rt_last_error(msg, sizeof msg);
    std::lock_guard<std::mutex> g(g_print);
    std::printf("FAIL %s: %d %s\n", what, rc, msg);
    g_failed = true;
}

// FullRaytracer: tiles, the hand-out, the update queue and the per-pixel SampleSets.
class Owner {
public:
    Owner(int w, int h, int threads, int passes, bool bulk) : w_(w), h_(h), passes_(passes), bulk_(bulk)
    {
        const int tiles_y = (int)std::floor(std::sqrt((double)threads)); // FullRaytracer.cs:70-71
        const int tiles_x = threads / tiles_y;
        tiles_.resize((size_t)tiles_x * tiles_y);
        for (int x = 0; x < tiles_x; x++) { // FullRaytracer.cs:271-285
            const int left = x * w / tiles_x, right = (x + 1) * w / tiles_x;
            for (int y = 0; y < tiles_y; y++) {
                const int top = y * h / tiles_y, bottom = (y + 1) * h / tiles_y;
                tiles_[(size_t)y * tiles_x + x] = Rect{left, top, right - left, bottom - top};
            }
        }
        handed_.assign(tiles_.size(), 0);
        sum_.assign((size_t)w * h, rt_color{0, 0, 0});
        samples_.assign((size_t)w * h, 0);
        misses_.assign((size_t)w * h, 0);
    }
    // GetWorkingTile (FullRaytracer.cs:219-229), plus the tile's pass index; false once every tile
    // has been handed out `passes` times (the stand-in for the UI's Stop)
    bool get_working_tile(Rect& tile, uint64_t& pass)
    {
        std::lock_guard<std::mutex> g(next_tile_lock_);
        if (handed_[next_tile_] >= (uint64_t)passes_) return false;
        tile = tiles_[next_tile_];
        pass = handed_[next_tile_]++;
        next_tile_ = (next_tile_ + 1) % tiles_.size();
        return true;
    }
    void on_tile_finished(const ImageUpdate& u) // FullRaytracer.cs:210-214
    {
        {
            std::lock_guard<std::mutex> g(q_m_);
            updates_.push_back(u);
        }
        q_cv_.notify_one();
    }
    void worker_done()
    {
        {
            std::lock_guard<std::mutex> g(q_m_);
            live_workers_--;
        }
        q_cv_.notify_one();
    }
    void set_workers(int n) { live_workers_ = n; }
    // the update loop (FullRaytracer.cs:305-344): merge every finished pass, hand its arrays back
    void update_loop();
    size_t tile_count() const { return tiles_.size(); }
    const std::vector<rt_color>& sum() const { return sum_; }
    const std::vector<uint32_t>& samples() const { return samples_; }
    const std::vector<uint32_t>& misses() const { return misses_; }
    uint64_t rays() const { return rays_; }
    uint64_t merged_passes() const { return merged_; }

private:
    int w_, h_, passes_;
    bool bulk_;
    std::vector<Rect> tiles_;
    std::vector<uint64_t> handed_;
    size_t next_tile_ = 0;
    std::mutex next_tile_lock_;
    std::deque<ImageUpdate> updates_;
    std::mutex q_m_;
    std::condition_variable q_cv_;
    int live_workers_ = 0;
    std::vector<rt_color> sum_; // SampleSets[x, y] at x * h + y
    std::vector<uint32_t> samples_, misses_;
    uint64_t rays_ = 0, merged_ = 0;
};

// GpuRaytracer: one scene handle, the pass loop, recycled arrays.
class Worker {
public:
    Worker(Owner& owner, const rt_scene_params& params, const std::vector<rt_prim>& prims, const rt_camera& cam,
           int device, uint64_t seed, bool bulk, int spp)
        : owner_(owner), seed_(seed), bulk_(bulk), spp_(spp)
    {
        int rc = rt_scene_create(&params, prims.data(), (int32_t)prims.size(), device, &handle_);
        if (rc == 0) rc = rt_scene_set_camera(handle_, &cam);
        if (rc != 0) report_failure("rt_scene_create / rt_scene_set_camera", rc);
    }
    ~Worker()
    {
        if (handle_) rt_scene_destroy(handle_);
        for (PassBuffers* b : recycled_) delete b;
    }
    void give_back(PassBuffers* b) // the update loop hands a merged pass's arrays back
    {
        std::lock_guard<std::mutex> g(m_);
        recycled_.push_back(b);
    }
    void render() // Raytracer.Render's loop shape (Raytracer.cs:294-330)
    {
        Rect tile{0, 0, 0, 0};
        uint64_t pass = 0;
        while (handle_ && !g_failed && owner_.get_working_tile(tile, pass)) {
            PassBuffers* b = nullptr;
            {
                std::lock_guard<std::mutex> g(m_);
                if (!recycled_.empty()) {
                    b = recycled_.back();
                    recycled_.pop_back();
                }
            }
            if (!b) b = new PassBuffers();
            const size_t n = (size_t)tile.width * tile.height;
            b->fit(n, bulk_);
            uint64_t rays = 0;
            int rc;
            if (bulk_) { // rt_render_tile accumulates: a recycled array is cleared first
                std::fill(b->color.begin(), b->color.end(), rt_color{0, 0, 0});
                std::fill(b->samples.begin(), b->samples.end(), 0u);
                std::fill(b->misses.begin(), b->misses.end(), 0u);
                rc = rt_render_tile(handle_, tile.left, tile.top, tile.width, tile.height, spp_, seed_,
                                    pass * (uint64_t)spp_, b->color.data(), b->samples.data(), b->misses.data(), &rays);
            } else { // every element is overwritten: no clearing
                rc = rt_render_tile_1spp(handle_, tile.left, tile.top, tile.width, tile.height, seed_, pass,
                                         b->color.data());
            }
            if (rc != 0) {
                report_failure(bulk_ ? "rt_render_tile" : "rt_render_tile_1spp", rc);
                delete b;
                break;
            }
            owner_.on_tile_finished(ImageUpdate{tile, b, this, rays});
        }
        owner_.worker_done();
    }

private:
    Owner& owner_;
    rt_scene* handle_ = nullptr;
    uint64_t seed_;
    bool bulk_;
    int spp_;
    std::mutex m_;
    std::vector<PassBuffers*> recycled_;
};

void Owner::update_loop()
{
    for (;;) {
        ImageUpdate u;
        {
            std::unique_lock<std::mutex> g(q_m_);
            q_cv_.wait(g, [this] { return !updates_.empty() || live_workers_ == 0; });
            if (updates_.empty()) return; // every worker stopped and everything is merged
            u = updates_.front();
            updates_.pop_front();
        }
        const Rect& t = u.tile;
        for (int x = 0; x < t.width; x++)
            for (int y = 0; y < t.height; y++) {
                const size_t src = (size_t)x * t.height + y, dst = (size_t)(t.left + x) * h_ + (t.top + y);
                const rt_color c = u.buf->color[src];
                if (bulk_) { // the bulk merge: SampleSet(old.Color + sum, old.Samples + samples, old.Misses + misses)
                    sum_[dst].r += c.r;
                    sum_[dst].g += c.g;
                    sum_[dst].b += c.b;
                    samples_[dst] += u.buf->samples[src];
                    misses_[dst] += u.buf->misses[src];
                } else if (c.r == -1.0 && c.g == -1.0 && c.b == -1.0) { // DoubleColor.Placeholder: AddMiss
                    misses_[dst]++;
                } else { // AddSample (SampleSet.cs:32-36)
                    sum_[dst].r += c.r;
                    sum_[dst].g += c.g;
                    sum_[dst].b += c.b;
                    samples_[dst]++;
                }
            }
        rays_ += u.rays;
        merged_++;
        u.worker->give_back(u.buf);
    }
}

int fail(const char* what, int rc = -1)
{
    report_failure(what, rc);
    return 1;
}

} // namespace

int main(int argc, char** argv)
{
    if (argc < 8) {
        std::printf("usage: worker_host SCENE W H THREADS PASSES MODE(1spp|bulk|frame) SPP [DEVICES]\n");
        return 2;
    }
    const int W = std::atoi(argv[2]), H = std::atoi(argv[3]), T = std::atoi(argv[4]), P = std::atoi(argv[5]);
    const bool frame_mode = std::strcmp(argv[6], "frame") == 0;
    const bool bulk = frame_mode || std::strcmp(argv[6], "bulk") == 0;
    const int spp = bulk ? std::atoi(argv[7]) : 1;
    int devices = rt_device_count();
    if (argc > 8) devices = std::min(devices, std::atoi(argv[8]));
    if (W <= 0 || H <= 0 || T <= 0 || P <= 0 || spp <= 0 || devices <= 0) return fail("arguments / no device");
    std::ifstream f(argv[1]);
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
    if (rc != 0 || nc < 1) return fail("rt_parse_scene", rc);
    params.width = W; // the UI's render size (Scene.Width / Height)
    params.height = H;
    const uint64_t seed = 0x5eed5eedULL;

    const size_t N = (size_t)W * H;
    Owner owner(W, H, T, P, bulk);
    std::vector<rt_color> frame_sum;
    std::vector<uint32_t> frame_samples, frame_misses;
    uint64_t frame_rays = 0;
    double host_s = 0.0;
    if (!frame_mode) {
        // --- the threaded host: T workers, one scene handle each, devices round-robin ---
        std::vector<Worker*> workers;
        for (int i = 0; i < T; i++)
            workers.push_back(new Worker(owner, params, prims, cams[0], i % devices, seed, bulk, spp));
        if (g_failed) return 1;
        owner.set_workers(T);
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> threads;
        for (Worker* w : workers) threads.emplace_back([w] { w->render(); });
        owner.update_loop();
        for (auto& t : threads) t.join();
        host_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (Worker* w : workers) delete w;
        if (g_failed) return 1;
        if (owner.merged_passes() != (uint64_t)P * owner.tile_count()) return fail("not every pass was merged");
    } else {
        // --- the whole-frame loop: submit one pass ahead, collect, merge in bulk ---
        rt_frame* fr = nullptr;
        rc = rt_frame_create(&params, prims.data(), n, &cams[0], devices, &fr);
        if (rc != 0) return fail("rt_frame_create", rc);
        frame_sum.assign(N, rt_color{0, 0, 0});
        frame_samples.assign(N, 0);
        frame_misses.assign(N, 0);
        std::vector<rt_color> s(N);
        std::vector<uint32_t> ns(N), ms(N);
        const auto t0 = std::chrono::steady_clock::now();
        rc = rt_frame_submit(fr, spp, seed, 0);
        for (int k = 0; k < P && rc == 0; k++) {
            if (k + 1 < P) rc = rt_frame_submit(fr, spp, seed, (uint64_t)(k + 1) * spp); // next pass renders...
            if (rc != 0) break;
            std::fill(s.begin(), s.end(), rt_color{0, 0, 0}); // collect adds into its buffers
            std::fill(ns.begin(), ns.end(), 0u);
            std::fill(ms.begin(), ms.end(), 0u);
            uint64_t rays = 0;
            rc = rt_frame_collect(fr, s.data(), ns.data(), ms.data(), &rays); // ...while this one merges
            for (size_t i = 0; rc == 0 && i < N; i++) {
                frame_sum[i].r += s[i].r;
                frame_sum[i].g += s[i].g;
                frame_sum[i].b += s[i].b;
                frame_samples[i] += ns[i];
                frame_misses[i] += ms[i];
            }
            frame_rays += rays;
        }
        host_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        rt_frame_destroy(fr);
        if (rc != 0) return fail("rt_frame_submit / rt_frame_collect", rc);
    }
    const std::vector<rt_color>& got_sum = frame_mode ? frame_sum : owner.sum();
    const std::vector<uint32_t>& got_samples = frame_mode ? frame_samples : owner.samples();
    const std::vector<uint32_t>& got_misses = frame_mode ? frame_misses : owner.misses();
    const uint64_t got_rays = frame_mode ? frame_rays : owner.rays();

    // --- the reference: one handle, whole-frame renders of the same sample indices, merged in order ---
    rt_scene* ref = nullptr;
    rc = rt_scene_create(&params, prims.data(), n, 0, &ref);
    if (rc == 0) rc = rt_scene_set_camera(ref, &cams[0]);
    if (rc != 0) return fail("reference scene", rc);
    std::vector<rt_color> rsum(N, rt_color{0, 0, 0});
    std::vector<uint32_t> rsam(N, 0), rmis(N, 0);
    uint64_t rrays = 0;
    const auto t1 = std::chrono::steady_clock::now();
    std::vector<rt_color> pass(N);
    for (int k = 0; k < P; k++) {
        if (bulk) {
            std::vector<rt_color> s(N, rt_color{0, 0, 0});
            std::vector<uint32_t> ns(N, 0), ms(N, 0);
            uint64_t rays = 0;
            rc = rt_render_tile(ref, 0, 0, W, H, spp, seed, (uint64_t)k * spp, s.data(), ns.data(), ms.data(), &rays);
            if (rc != 0) return fail("reference rt_render_tile", rc);
            for (size_t i = 0; i < N; i++) {
                rsum[i].r += s[i].r;
                rsum[i].g += s[i].g;
                rsum[i].b += s[i].b;
                rsam[i] += ns[i];
                rmis[i] += ms[i];
            }
            rrays += rays;
        } else {
            rc = rt_render_tile_1spp(ref, 0, 0, W, H, seed, (uint64_t)k, pass.data());
            if (rc != 0) return fail("reference rt_render_tile_1spp", rc);
            for (size_t i = 0; i < N; i++) {
                const rt_color c = pass[i];
                if (c.r == -1.0 && c.g == -1.0 && c.b == -1.0) rmis[i]++;
                else {
                    rsum[i].r += c.r;
                    rsum[i].g += c.g;
                    rsum[i].b += c.b;
                    rsam[i]++;
                }
            }
        }
    }
    const double ref_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    if (!bulk) { // tile passes are windows of the frame's pass, bit for bit (pass P - 1 of one tile)
        Owner probe(W, H, T, 1, false);
        Rect t{0, 0, 0, 0};
        uint64_t k0 = 0;
        probe.get_working_tile(t, k0);
        std::vector<rt_color> tile((size_t)t.width * t.height);
        rc = rt_render_tile_1spp(ref, t.left, t.top, t.width, t.height, seed, (uint64_t)(P - 1), tile.data());
        if (rc != 0) return fail("tile window pass", rc);
        for (int x = 0; x < t.width; x++)
            for (int y = 0; y < t.height; y++)
                if (std::memcmp(&tile[(size_t)x * t.height + y], &pass[(size_t)(t.left + x) * H + (t.top + y)],
                                sizeof(rt_color)) != 0)
                    return fail("a tile pass differs from the frame pass's window");
    }
    rt_scene_destroy(ref);

    // --- compare ---
    const double tol = bulk ? 1e-5 : 1e-12;
    uint64_t total_samples = 0, total_misses = 0;
    double worst = 0.0;
    for (size_t i = 0; i < N; i++) {
        if (got_samples[i] != rsam[i] || got_misses[i] != rmis[i]) {
            std::printf("FAIL counts at pixel x=%zu y=%zu: %u/%u against %u/%u\n", i / H, i % H, got_samples[i],
                        got_misses[i], rsam[i], rmis[i]);
            return 1;
        }
        total_samples += rsam[i];
        total_misses += rmis[i];
        const double a[3] = {got_sum[i].r, got_sum[i].g, got_sum[i].b};
        const double b[3] = {rsum[i].r, rsum[i].g, rsum[i].b};
        for (int c = 0; c < 3; c++) {
            if (!std::isfinite(a[c])) return fail("non-finite Σ");
            worst = std::max(worst, std::fabs(a[c] - b[c]) / std::max(1.0, std::fabs(b[c])));
        }
    }
    if (worst > tol) {
        std::printf("FAIL Σ differs from the whole-frame reference: worst relative %.3g > %.3g\n", worst, tol);
        return 1;
    }
    if (total_samples + total_misses != (uint64_t)N * P * spp) return fail("samples + misses != pixels x passes x spp");
    if (bulk && got_rays != rrays) {
        std::printf("FAIL rays %llu against %llu\n", (unsigned long long)got_rays, (unsigned long long)rrays);
        return 1;
    }
    const double msps = (double)N * P * spp / host_s * 1e-6;
    std::printf("ok %s %dx%d threads %d tiles %zu passes %d mode %s spp %d devices %d: samples %llu misses %llu "
                "worst %.3g; workers %.3f s (%.1f M samples/s incl. merge), one handle %.3f s\n",
                argv[1], W, H, T, owner.tile_count(), P, argv[6], spp, devices,
                (unsigned long long)total_samples, (unsigned long long)total_misses, worst, host_s, msps, ref_s);
    return 0;
}
