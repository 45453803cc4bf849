// bsw_pool.h -- the engine's host worker pool (host-buffer staging, packing, scans).
//
// One process-wide pool of workers() threads, created on first use (the process's CPU share
// minus the caller: the cgroup CPU quota when one is set, else the affinity set; 2..32 lanes).  parallel_for(n, fn) runs
// fn(0..n-1), the caller taking part; several callers (upstream calls getScores* from kt_for
// workers) may submit at once -- tasks interleave in one queue and each call waits only for its
// own.  Spawning threads per call instead cost ~30 us each, several ms per 1M-pair call.
#pragma once
#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <sched.h>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace bsw {

class HostPool {
public:
    static int workers()                        // + the calling thread = lanes of host work
    {
        static const int w = [] {
            int n = (int)std::thread::hardware_concurrency();
            if (n <= 0) n = 8;
#ifdef __linux__
            cpu_set_t cs;
            if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = std::min(n, (int)CPU_COUNT(&cs));
            if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
                char q[32] = {0};
                long per = 0;
                if (fscanf(f, "%31s %ld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0)
                    n = std::min(n, (int)((atol(q) + per - 1) / per));
                fclose(f);
            }
#endif
            if (const char *e = getenv("BSW_HOST_THREADS")) n = atoi(e);   // tuning override
            return std::max(2, std::min(n, 32)) - 1;
        }();
        return w;
    }
    static HostPool &get()
    {
        static HostPool p;
        return p;
    }
    // fn(k) for k in [0, n); returns when all have run
    void parallel_for(int n, const std::function<void(int)> &fn)
    {
        if (n <= 1) {
            if (n == 1) fn(0);
            return;
        }
        struct Call { std::mutex mu; std::condition_variable cv; int left; } call;
        call.left = n - 1;
        {
            std::lock_guard<std::mutex> g(mu_);
            for (int k = 1; k < n; ++k)
                q_.push_back([&call, &fn, k] {
                    fn(k);
                    std::lock_guard<std::mutex> g2(call.mu);
                    if (--call.left == 0) call.cv.notify_all();
                });
        }
        cv_.notify_all();
        fn(0);
        // help with queued work (ours or another caller's) rather than sleep
        for (;;) {
            std::function<void()> t;
            {
                std::lock_guard<std::mutex> g(mu_);
                if (q_.empty()) break;
                t = std::move(q_.front());
                q_.pop_front();
            }
            t();
        }
        std::unique_lock<std::mutex> lk(call.mu);
        call.cv.wait(lk, [&] { return call.left == 0; });
    }
    ~HostPool()
    {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }

private:
    HostPool()
    {
        for (int k = 0; k < workers(); ++k)
            th_.emplace_back([this] {
                for (;;) {
                    std::function<void()> t;
                    {
                        std::unique_lock<std::mutex> lk(mu_);
                        cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
                        if (stop_ && q_.empty()) return;
                        t = std::move(q_.front());
                        q_.pop_front();
                    }
                    t();
                }
            });
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    std::vector<std::thread> th_;
    bool stop_ = false;
};

// memcpy split over the pool when large (staging into / out of pinned memory)
inline void par_memcpy(void *dst, const void *src, size_t bytes)
{
    constexpr size_t kPiece = (size_t)2 << 20;
    const int nt = (int)std::min<size_t>(HostPool::workers() + 1, bytes / kPiece);
    if (nt <= 1) { memcpy(dst, src, bytes); return; }
    HostPool::get().parallel_for(nt, [=](int t) {
        const size_t a = bytes * t / nt, b = bytes * (t + 1) / nt;
        memcpy((char *)dst + a, (const char *)src + a, b - a);
    });
}

}  // namespace bsw
