// host_pool.cpp -- the persistent host worker pool behind parallel_ranges (host_scene.h).
//
// The host-buffer entry points (rt_render_tile, rt_render_tile_1spp, the band scatter) stream tens
// of MB per call between pinned staging and the caller's arrays on up to 16 host threads.  Spawning
// and joining those threads on every call cost ~0.3 ms, a fifth of a 1080p one-pass call; the pool
// keeps them parked on a condition variable instead.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "host_scene.h"

namespace rtc {
namespace {

class Pool {
public:
    explicit Pool(int workers)
    {
        for (int i = 0; i < workers; i++) threads_.emplace_back([this] { loop(); });
    }
    ~Pool()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            quit_ = true;
            gen_++;
        }
        cv_.notify_all();
        for (auto& t : threads_) t.join();
    }
    int size() const { return (int)threads_.size() + 1; }
    // false when another run is in progress (the caller then uses threads of its own)
    bool run(size_t n, const std::function<void(size_t)>& task)
    {
        std::unique_lock<std::mutex> busy(run_m_, std::try_to_lock);
        if (!busy.owns_lock()) return false;
        {
            std::lock_guard<std::mutex> g(m_);
            task_ = &task;
            n_ = n;
            next_.store(0);
            left_ = (int)threads_.size();
            gen_++;
        }
        cv_.notify_all();
        work(task, n); // the calling thread takes tasks too
        std::unique_lock<std::mutex> g(m_);
        done_cv_.wait(g, [this] { return left_ == 0; });
        task_ = nullptr;
        return true;
    }

private:
    void work(const std::function<void(size_t)>& task, size_t n)
    {
        for (size_t i = next_.fetch_add(1); i < n; i = next_.fetch_add(1)) task(i);
    }
    void loop()
    {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(size_t)>* t;
            size_t n;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                if (quit_) return;
                t = task_;
                n = n_;
            }
            work(*t, n);
            std::lock_guard<std::mutex> g(m_);
            if (--left_ == 0) done_cv_.notify_one();
        }
    }
    std::vector<std::thread> threads_;
    std::mutex m_, run_m_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t)>* task_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    int left_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
};

int pool_width()
{
    int w = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    if (const char* e = std::getenv("OMP_NUM_THREADS")) { // the job's CPU share where one is set
        const int k = std::atoi(e);
        if (k > 0) w = std::min(w, k);
    }
    return w;
}

Pool& pool()
{
    static Pool* p = new Pool(pool_width() - 1); // never destroyed: workers may outlive static teardown
    return *p;
}

} // namespace

int host_threads() { return pool().size(); }

void host_run(size_t n, const std::function<void(size_t)>& task)
{
    if (n == 0) return;
    if (n == 1) {
        task(0);
        return;
    }
    if (pool().run(n, task)) return;
    // the pool is busy (another thread's call): threads of our own
    const size_t T = std::min<size_t>(n, (size_t)pool_width());
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    for (size_t t = 1; t < T; t++)
        th.emplace_back([&] {
            for (size_t i = next.fetch_add(1); i < n; i = next.fetch_add(1)) task(i);
        });
    for (size_t i = next.fetch_add(1); i < n; i = next.fetch_add(1)) task(i);
    for (auto& x : th) x.join();
}

} // namespace rtc
