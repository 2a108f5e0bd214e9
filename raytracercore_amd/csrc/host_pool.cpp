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
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <pthread.h>
#include <unistd.h>

#include "host_scene.h"

namespace rtc {
namespace {

// Set on the threads of a pool run (the caller and the workers): a host_run issued from inside a
// task runs inline instead of re-entering the pool (whose run lock the caller already holds).
thread_local bool t_in_pool = false;

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
        std::exception_ptr err;
        t_in_pool = true;
        try {
            work(task, n); // the calling thread takes tasks too
        } catch (...) { // stop handing out tasks, drain the workers, then rethrow with the flag reset
            err = std::current_exception();
            next_.store(n);
        }
        t_in_pool = false;
        {
            std::unique_lock<std::mutex> g(m_);
            done_cv_.wait(g, [this] { return left_ == 0; });
            task_ = nullptr;
        }
        if (err) std::rethrow_exception(err);
        return true;
    }

private:
    void work(const std::function<void(size_t)>& task, size_t n)
    {
        for (size_t i = next_.fetch_add(1); i < n; i = next_.fetch_add(1)) task(i);
    }
    void loop()
    {
        t_in_pool = true;
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

// The pool of this process.  A fork()ed child inherits the pointer but none of the worker threads
// (nor, if the fork came mid-run, a usable lock), so an atfork handler drops it in the child and
// the child's first host_run builds a pool of its own.  Pools are never destroyed: workers may
// outlive static teardown.
std::atomic<Pool*> g_pool{nullptr};

void drop_pool_in_child() { g_pool.store(nullptr); }

Pool& pool()
{
    Pool* p = g_pool.load();
    if (p) return *p;
    static const int registered = pthread_atfork(nullptr, nullptr, drop_pool_in_child);
    (void)registered;
    Pool* fresh = new Pool(pool_width() - 1);
    if (g_pool.compare_exchange_strong(p, fresh)) return *fresh;
    delete fresh; // another thread installed one first
    return *p;
}

} // namespace

int host_threads() { return pool().size(); }

void host_run(size_t n, const std::function<void(size_t)>& task)
{
    if (n == 0) return;
    if (n == 1 || t_in_pool) { // nested inside a pool task: inline
        for (size_t i = 0; i < n; i++) task(i);
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
