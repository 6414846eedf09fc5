// Small fixed pool of host threads for the staging copies of the synchronous
// host-memory entry points (rs_encode / rs_reconst / rs_update / rs_replace).
// One memcpy thread moves ~10-20 GB/s; a 10+4 stripe of 1 MiB vectors is
// 14 MiB of copies per call, so several threads keep the copies under the
// PCIe time.  Size: RSAMD_HOST_THREADS (default 4, 1 = no workers).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace rsamd {

class CopyPool {
public:
    static CopyPool& get() {
        static CopyPool pool(threads_from_env());
        return pool;
    }

    int size() const { return static_cast<int>(workers_.size()) + 1; }

    // fn(i) for every i in [0, n), spread over the pool and the calling
    // thread; returns when all are done.  One job runs at a time.
    void run(size_t n, const std::function<void(size_t)>& fn) {
        if (workers_.empty() || n <= 1) {
            for (size_t i = 0; i < n; ++i) fn(i);
            return;
        }
        std::lock_guard<std::mutex> one(run_mu_);
        run_locked(n, fn);
    }

    // run() if the pool is idle; otherwise fn(i) for every i on the calling
    // thread alone (concurrent callers - device-group workers, several host
    // calls - copy in parallel on their own threads instead of queueing).
    void run_or_inline(size_t n, const std::function<void(size_t)>& fn) {
        std::unique_lock<std::mutex> one(run_mu_, std::try_to_lock);
        if (workers_.empty() || n <= 1 || !one.owns_lock()) {
            for (size_t i = 0; i < n; ++i) fn(i);
            return;
        }
        run_locked(n, fn);
    }

    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : workers_) t.join();
    }

private:
    void run_locked(size_t n, const std::function<void(size_t)>& fn) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &fn;
            n_ = n;
            next_.store(0, std::memory_order_relaxed);
            pending_ = workers_.size();
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
    }

    explicit CopyPool(int threads) {
        for (int i = 1; i < threads; ++i) workers_.emplace_back([this] { loop(); });
    }

    static int threads_from_env() {
        const char* e = std::getenv("RSAMD_HOST_THREADS");
        int n = e ? std::atoi(e) : 4;
        return n < 1 ? 1 : (n > 32 ? 32 : n);
    }

    void work() {
        for (size_t i; (i = next_.fetch_add(1, std::memory_order_relaxed)) < n_;) (*job_)(i);
    }

    void loop() {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            lk.unlock();
            work();
            lk.lock();
            if (--pending_ == 0) done_.notify_one();
        }
    }

    std::vector<std::thread> workers_;
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_;
    const std::function<void(size_t)>* job_ = nullptr;
    size_t n_ = 0, pending_ = 0;
    std::atomic<size_t> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace rsamd
