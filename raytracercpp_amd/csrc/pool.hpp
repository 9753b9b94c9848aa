// pool.hpp -- a small fixed thread pool for the host builds (octree.cpp, wbvh.cpp):
// std::thread workers, no OpenMP (the library shares its process with torch's runtime).
#pragma once

#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <type_traits>
#include <thread>
#include <vector>

namespace rt {

// Workers wait for a job by spinning on an atomic generation counter for a short while
// (a build issues hundreds of short cooperative passes back to back), then block on a
// condition variable; the caller spins for the workers' completion.
class Pool {
public:
    explicit Pool(int n) : n_(n)
    {
        for (int w = 1; w < n; w++)
            th_.emplace_back([this, w] { loop(w); });
    }
    ~Pool()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_.store(true);
            gen_.fetch_add(1);
        }
        cv_.notify_all();
        for (auto& t : th_)
            t.join();
    }
    int size() const { return n_; }
    // runs f(worker) on every worker (the caller is worker 0) and waits for all
    void run(const std::function<void(int)>& f)
    {
        if (n_ == 1) {
            f(0);
            return;
        }
        job_ = &f;
        pending_.store(n_ - 1, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> g(m_);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        f(0);
        while (pending_.load(std::memory_order_acquire) != 0)
            std::this_thread::yield();
    }

private:
    void loop(int w)
    {
        uint64_t seen = 0;
        for (;;) {
            // spin briefly for the next job, then sleep
            uint64_t g = gen_.load(std::memory_order_acquire);
            for (int k = 0; g == seen && k < 20000; k++) {
                std::this_thread::yield();
                g = gen_.load(std::memory_order_acquire);
            }
            if (g == seen) {
                std::unique_lock<std::mutex> l(m_);
                cv_.wait(l, [&] { return gen_.load(std::memory_order_acquire) != seen; });
                g = gen_.load(std::memory_order_acquire);
            }
            seen = g;
            if (stop_.load())
                return;
            (*job_)(w);
            pending_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_;
    const std::function<void(int)>* job_ = nullptr;
    std::atomic<int> pending_{0};
    std::atomic<uint64_t> gen_{0};
    std::atomic<bool> stop_{false};
};

// dynamic work split: calls body(i) for i in [0, n) in chunks
template <class F>
void parallel_for(Pool& pool, int64_t n, int64_t chunk, F&& body)
{
    std::atomic<int64_t> next{0};
    pool.run([&](int) {
        for (;;) {
            int64_t b = next.fetch_add(chunk);
            if (b >= n)
                return;
            int64_t e = std::min(n, b + chunk);
            for (int64_t i = b; i < e; i++)
                body(i);
        }
    });
}

// Large temporaries released on a detached thread, off the caller's critical path (freeing
// hundreds of MB of build scratch takes milliseconds).
template <class... T>
void free_later(T&&... v)
{
    std::thread([](std::decay_t<T>...) {}, std::move(v)...).detach();
}

inline int build_threads()
{
    if (const char* e = std::getenv("RT_BUILD_THREADS")) {
        int v = std::atoi(e);
        if (v >= 1)
            return v;
    }
    unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hc, 16u));
}

// The calling thread's build pool, created at its first build and kept (joining 16 workers
// after every build cost more than the build's last phase): builds on different threads
// (a renderer's background wide-BVH build, another renderer) each have their own.
inline Pool& build_pool()
{
    thread_local std::unique_ptr<Pool> pool;
    const int nt = build_threads();
    if (!pool || pool->size() != nt)
        pool = std::make_unique<Pool>(nt);
    return *pool;
}

}  // namespace rt
