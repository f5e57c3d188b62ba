// Stress test of the drop-in API's InstanceLock (siamese_amd/csrc/engine.h):
// readers in per-thread slots, a writer that excludes every reader.  Built
// and run by tests/test_instance_lock.py on the CPU.
#include "engine.h"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

int main(int argc, char** argv)
{
    if (argc > 1 && std::string(argv[1]) == "nested") {
        // a second shared acquisition on one thread: SGPU_DEBUG_LOCKS aborts
        static sgpu::InstanceLock lk;
        lk.lock_shared();
        lk.lock_shared();
        std::printf("nested acquisition not caught\n");
        return 0;
    }
    sgpu::InstanceLock lk;
    std::atomic<int> readersIn{0}, writersIn{0};
    std::atomic<long> reads{0}, writes{0}, bad{0};
    std::atomic<bool> stop{false};
    long shared = 0;   // written under the exclusive lock only
    std::vector<std::thread> ts;
    for (int r = 0; r < 5; ++r)
        ts.emplace_back([&] {
            while (!stop.load()) {
                std::shared_lock<sgpu::InstanceLock> g(lk);
                readersIn.fetch_add(1);
                if (writersIn.load() != 0)
                    bad.fetch_add(1);
                const long a = shared;
                for (int k = 0; k < 50; ++k)
                    asm volatile("" ::: "memory");
                if (shared != a)
                    bad.fetch_add(1);
                readersIn.fetch_sub(1);
                reads.fetch_add(1);
            }
        });
    for (int w = 0; w < 2; ++w)
        ts.emplace_back([&] {
            while (!stop.load()) {
                {
                    std::unique_lock<sgpu::InstanceLock> g(lk);
                    if (writersIn.fetch_add(1) != 0 || readersIn.load() != 0)
                        bad.fetch_add(1);
                    ++shared;
                    writersIn.fetch_sub(1);
                }
                writes.fetch_add(1);
                std::this_thread::sleep_for(std::chrono::microseconds(20));
            }
        });
    std::this_thread::sleep_for(std::chrono::milliseconds(700));
    stop.store(true);
    for (std::thread& t : ts)
        t.join();
    std::printf("reads %ld writes %ld shared %ld bad %ld\n", reads.load(), writes.load(), shared, bad.load());
    return (bad.load() == 0 && writes.load() == shared && reads.load() > 0 && writes.load() > 0) ? 0 : 1;
}
