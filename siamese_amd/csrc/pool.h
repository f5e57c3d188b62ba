// pool.h -- a small fork-join worker pool for the host control plane
// (flush assembly).  run(n, fn) calls fn(i) for i in [0, n) on the pool's
// threads plus the caller and returns when all calls are done.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace sgpu {

class WorkerPool
{
public:
    explicit WorkerPool(unsigned threads);
    ~WorkerPool();
    WorkerPool(const WorkerPool&) = delete;
    WorkerPool& operator=(const WorkerPool&) = delete;

    unsigned size() const { return (unsigned)workers_.size() + 1; }
    void run(size_t count, const std::function<void(size_t)>& fn);

    /// Threads to use by default: SIAMESE_AMD_THREADS, else OMP_NUM_THREADS,
    /// else min(16, hardware threads).
    static unsigned default_threads();

private:
    void loop();
    void drain();

    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_, doneCv_;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t count_ = 0;
    std::atomic<size_t> next_{0};
    std::atomic<unsigned> busy_{0};
    std::atomic<uint64_t> gen_{0};
    unsigned sleepers_ = 0;   // workers blocked on cv_ (mu_)
    std::atomic<bool> stop_{false};
};

} // namespace sgpu
