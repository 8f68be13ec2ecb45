// copy_pool.hpp -- a coder's persistent host worker threads for the per-call
// drop-in (hec_encode / hec_decode, ec_capi.cpp): the pageable <-> pinned
// copies of one row's shards run side by side instead of one memcpy after
// another, and each shard's DMA is issued as soon as its copy is done.
// Host code only.  One batch at a time per pool (the coder's host mutex
// serialises its callers).
#pragma once

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace hec {

class CopyPool {
  public:
    CopyPool() = default;
    CopyPool(const CopyPool&) = delete;
    CopyPool& operator=(const CopyPool&) = delete;
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_work_.notify_all();
        for (auto& t : workers_) t.join();
    }

    // Grows the pool to n workers, best effort (a thread that cannot start is
    // skipped); returns the number running.
    int ensure(int n) {
        while (int(workers_.size()) < n) {
            try {
                workers_.emplace_back([this] { loop(); });
            } catch (...) {
                break;
            }
        }
        return int(workers_.size());
    }

    // Runs task(i) for i = 0 .. n-1 on the workers, started in index order.
    // The caller keeps everything task touches alive until wait_all().
    void start(int n, std::function<void(int)> task) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            task_ = std::move(task);
            done_.assign(size_t(n), 0);
            n_ = n;
            next_ = 0;
            ndone_ = 0;
        }
        cv_work_.notify_all();
    }

    void wait(int i) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_done_.wait(lk, [&] { return done_[size_t(i)] != 0; });
    }

    void wait_all() {
        std::unique_lock<std::mutex> lk(mu_);
        cv_done_.wait(lk, [&] { return ndone_ == n_; });
    }

  private:
    void loop() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_work_.wait(lk, [&] { return stop_ || next_ < n_; });
            if (next_ >= n_) return;  // stop_ and nothing left
            const int i = next_++;
            lk.unlock();
            task_(i);  // task_ is not reassigned before every task of the batch is done
            lk.lock();
            done_[size_t(i)] = 1;
            ndone_++;
            cv_done_.notify_all();
        }
    }

    std::mutex mu_;
    std::condition_variable cv_work_, cv_done_;
    std::vector<std::thread> workers_;
    std::function<void(int)> task_;
    std::vector<uint8_t> done_;
    int n_ = 0, next_ = 0, ndone_ = 0;
    bool stop_ = false;
};

// Waits for the pool's batch on scope exit (error paths included): no worker
// may still touch the caller's buffers or the bounce buffer after a return.
struct PoolBatch {
    CopyPool* pool;
    ~PoolBatch() {
        if (pool) pool->wait_all();
    }
};

}  // namespace hec
