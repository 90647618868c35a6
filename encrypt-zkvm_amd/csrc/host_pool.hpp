// host_pool.hpp -- a small process-wide pool of host threads for the prover's host-side passes over a trace (packing
// narrow columns for upload, prover.hip).  Tasks are plain closures; a Latch counts a batch down and is waited for
// before the memory the tasks read or write goes away.  The pool is created on first use and lives until the
// process exits (its threads are never joined: a static destructor that joins could hang an exiting process).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>

namespace zk {

// The count is read and written only under mu_, and count_down() notifies while it still holds mu_: a waiter can
// only observe zero after the last count_down() has released the mutex for good, so a Latch that lives on the
// waiter's stack may go out of scope as soon as wait() or ready() reports zero.
class Latch {
public:
    explicit Latch(int count = 0) : left_(count) {}
    void reset(int count) {
        std::lock_guard<std::mutex> lk(mu_);
        left_ = count;
    }
    void count_down() {
        std::lock_guard<std::mutex> lk(mu_);
        if (--left_ == 0) cv_.notify_all();
    }
    bool ready() {
        std::lock_guard<std::mutex> lk(mu_);
        return left_ <= 0;
    }
    void wait() {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return left_ <= 0; });
    }

private:
    int left_;
    std::mutex mu_;
    std::condition_variable cv_;
};

class HostPool {
public:
    // ZK_HOST_THREADS (default 8, at most 64): the box's CPU share is shared by every prover in flight
    static HostPool &get() {
        static HostPool *pool = [] {
            const char *e = getenv("ZK_HOST_THREADS");
            int k = e ? atoi(e) : 8;
            if (k < 1) k = 1;
            if (k > 64) k = 64;
            return new HostPool(k);
        }();
        return *pool;
    }
    void submit(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(std::move(f));
        }
        cv_.notify_one();
    }

private:
    explicit HostPool(int k) {
        for (int i = 0; i < k; i++) std::thread([this] { work(); }).detach();
    }
    void work() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return !q_.empty(); });
                f = std::move(q_.front());
                q_.pop_front();
            }
            f();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
};

}  // namespace zk
