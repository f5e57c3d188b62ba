// pool.cpp -- see pool.h.
#include "pool.h"

#include <algorithm>
#include <cstdlib>
#include <pthread.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>

namespace sgpu {


int WorkerPool::shared_nice()
{
    // the shared pool's workers yield to the launcher and completer threads
    // (0 measured no different on the box, profiles/r5a ab runs)
    return 10;
}

unsigned WorkerPool::default_threads()
{
    for (const char* var : {"SIAMESE_AMD_THREADS", "OMP_NUM_THREADS"}) {
        const char* v = std::getenv(var);
        if (v && std::atoi(v) > 0)
            return (unsigned)std::min(256, std::atoi(v));
    }
    const unsigned hw = std::thread::hardware_concurrency();
    return std::max(1u, std::min(16u, hw));
}

WorkerPool::WorkerPool(unsigned threads, int nice, const char* name)
{
    for (unsigned i = 1; i < threads; ++i)
        workers_.emplace_back([this, nice, name] {
            pthread_setname_np(pthread_self(), name);
            if (nice != 0)
                (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), nice);
            loop();
        });
}

WorkerPool::~WorkerPool()
{
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_.store(true, std::memory_order_relaxed);
    }
    cv_.notify_all();
    for (std::thread& t : workers_)
        t.join();
}

void WorkerPool::drain()
{
    for (;;) {
        const size_t i = next_.fetch_add(1, std::memory_order_acq_rel);
        if (i >= count_)
            return;
        (*fn_)(i);
    }
}

void WorkerPool::loop()
{
    uint64_t seen = 0;
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(mu_);
            if (gen_.load(std::memory_order_relaxed) == seen && !stop_.load(std::memory_order_relaxed)) {
                ++sleepers_;
                cv_.wait(lk, [&] {
                    return stop_.load(std::memory_order_relaxed) ||
                           gen_.load(std::memory_order_relaxed) != seen;
                });
                --sleepers_;
            }
            if (stop_.load(std::memory_order_relaxed))
                return;
            seen = gen_.load(std::memory_order_relaxed);
            busy_.fetch_add(1, std::memory_order_acq_rel);
        }
        drain();
        if (busy_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
            std::lock_guard<std::mutex> g(mu_);
            doneCv_.notify_all();
        }
    }
}

void WorkerPool::run(size_t count, const std::function<void(size_t)>& fn)
{
    if (count == 0)
        return;
    if (workers_.empty() || count == 1) {
        for (size_t i = 0; i < count; ++i)
            fn(i);
        return;
    }
    bool wake;
    {
        std::lock_guard<std::mutex> g(mu_);
        fn_ = &fn;
        count_ = count;
        next_.store(0, std::memory_order_release);
        gen_.fetch_add(1, std::memory_order_acq_rel);
        wake = sleepers_ > 0;
    }
    if (wake)
        cv_.notify_all();
    drain();
    // every index has been claimed; wait for the workers still finishing one
    // (a spinning wait measured slower on the box's 16-core share: the
    // spinners take cycles from the stepping threads)
    std::unique_lock<std::mutex> lk(mu_);
    doneCv_.wait(lk, [&] { return busy_.load(std::memory_order_acquire) == 0; });
    fn_ = nullptr;
}

} // namespace sgpu
