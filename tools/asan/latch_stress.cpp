// Stress test of zk::Latch / zk::HostPool (csrc/host_pool.hpp) under ThreadSanitizer (tests/test_asan.py): many short
// batches whose stack-local Latch goes out of scope as soon as wait() or ready() reports zero, while the pool's
// threads may still be inside count_down() -- the use-after-scope race ADVICE r4 found in the lock-free form.
#include <atomic>
#include <cstdio>

#include "../../encrypt-zkvm_amd/csrc/host_pool.hpp"

int main(int argc, char **argv) {
    const int batches = argc > 1 ? atoi(argv[1]) : 20000;
    std::atomic<long> done{0};
    for (int b = 0; b < batches; b++) {
        const int k = 1 + b % 7;
        zk::Latch latch;  // dies at the end of this iteration
        latch.reset(k);
        for (int t = 0; t < k; t++)
            zk::HostPool::get().submit([&latch, &done] {
                done.fetch_add(1, std::memory_order_relaxed);
                latch.count_down();
            });
        if (b % 2) {
            while (!latch.ready()) {
            }
        } else {
            latch.wait();
        }
    }
    long want = 0;
    for (int b = 0; b < batches; b++) want += 1 + b % 7;
    printf("latch stress: %d batches, %ld tasks (want %ld)\n", batches, done.load(), want);
    return done.load() == want ? 0 : 1;
}
