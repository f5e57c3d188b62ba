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
    /// `nice`: scheduling priority of the worker threads (0 = the caller's);
    /// `name`: their thread name (at most 15 characters; diagnostics).
    explicit WorkerPool(unsigned threads, int nice = 0, const char* name = "sgpu-pool");
    ~WorkerPool();
    WorkerPool(const WorkerPool&) = delete;
    WorkerPool& operator=(const WorkerPool&) = delete;

    unsigned size() const { return (unsigned)workers_.size() + 1; }
    void run(size_t count, const std::function<void(size_t)>& fn);

    /// Threads to use by default: SIAMESE_AMD_THREADS, else OMP_NUM_THREADS,
    /// else min(16, hardware threads).
    static unsigned default_threads();
    /// Priority of the engine's shared stepping pool (Engine::pool):
    /// SIAMESE_AMD_WORKER_NICE, default 10, so its workers yield to the
    /// engine's launcher and completer threads, which sit on the device's
    /// critical path.  Other pools (the launcher's assembly pool, pools an
    /// application creates) keep the caller's priority.
    static int shared_nice();

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
