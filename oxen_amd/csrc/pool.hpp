// oxen_amd/csrc/pool.hpp -- the runtime's blocking thread pool (file readers / copiers / writers).
#pragma once
#include <dirent.h>
#include <sched.h>
#include <stdlib.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace oxh {
// A worker of a pool made with private_fds gets a file-descriptor table of its own: it calls
// unshare(CLONE_FILES) and drops every descriptor the copy inherited (stdin/out/err stay), so the
// files it opens and closes never take the table lock the rest of the process takes. On the MI355X
// boxes that lock is the warm small-file floor of one process: 200 000 open + close pairs take
// 0.28 s in one process whatever its thread count and 0.13-0.16 s in 2-4 processes
// (profiles/r02e_open_procs.json); tools/open_probe.cpp UNSHARE=1 measures the same threads with
// private tables. Only for workers that use nothing but the descriptors they open themselves (the
// streaming readers). OXH_SHARED_FDS=1 turns it off.
inline void make_fd_table_private() {
    const char* e = getenv("OXH_SHARED_FDS");
    if (e && atoi(e) != 0) return;
    if (unshare(CLONE_FILES) != 0) return;  // keep sharing: correct, just slower
#ifdef SYS_close_range
    if (syscall(SYS_close_range, 3u, ~0u, 0u) == 0) return;
#endif
    if (DIR* d = opendir("/proc/thread-self/fd")) {  // older kernels: close the copies one by one
        std::vector<int> fds;
        while (dirent* de = readdir(d)) {
            const int fd = atoi(de->d_name);
            if (fd > 2 && fd != dirfd(d)) fds.push_back(fd);
        }
        closedir(d);
        for (int fd : fds) close(fd);
    }
}

// The file engine's thread polls its slots' events in 20 us timed waits while a slot is in flight;
// Linux stretches every such wait by the thread's timer slack, 50 us by default, so a one-file request
// paid 50-70 us oversleeps end to end (tools/latency_probe.py). The engine thread runs with a slack of
// OXH_TIMER_SLACK_NS (default 1000 ns; 0 keeps the kernel's default). The pools' threads (readers that
// wait 2-5 us for a slot, copiers) and callers' threads keep theirs: tighter reader waits would spin
// the 16 readers against each other on a CPU-bound walk.
inline void runtime_thread_timer_slack() {
    static const long ns = [] {
        const char* e = getenv("OXH_TIMER_SLACK_NS");
        return e ? atol(e) : 1000L;
    }();
    if (ns > 0) (void)prctl(PR_SET_TIMERSLACK, (unsigned long)ns, 0, 0, 0);
}

class Pool {
   public:
    explicit Pool(int n, bool private_fds = false) {
        for (int i = 0; i < n; ++i)
            th_.emplace_back([this, private_fds] {
                if (private_fds) make_fd_table_private();
                run();
            });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return (int)th_.size(); }
    // Run fn(t) for t in [0, ntasks) across the pool; blocks until all are done.
    void parallel_for(int ntasks, const std::function<void(int)>& fn) {
        if (ntasks <= 0) return;
        std::atomic<int> next{0}, done{0};
        std::mutex dmu;
        std::condition_variable dcv;
        auto body = [&] {
            for (;;) {
                const int t = next.fetch_add(1);
                if (t >= ntasks) break;
                fn(t);
                if (done.fetch_add(1) + 1 == ntasks) {
                    std::lock_guard<std::mutex> g(dmu);
                    dcv.notify_all();
                }
            }
        };
        const int nw = std::min(ntasks, size());
        {
            std::lock_guard<std::mutex> g(mu_);
            for (int i = 0; i < nw; ++i) q_.push_back(body);
        }
        cv_.notify_all();
        {
            std::unique_lock<std::mutex> lk(dmu);
            dcv.wait(lk, [&] { return done.load() == ntasks; });
        }  // release dmu: the worker that finished the last task may still be about to take it
        // the helpers may still be returning from `body`; wait until none holds a reference
        std::unique_lock<std::mutex> g(mu_);
        idle_cv_.wait(g, [&] { return busy_ == 0 && q_.empty(); });
    }

    // Start fn(t) for t in [0, ntasks) on the pool WITHOUT waiting; wait() on the returned group
    // blocks until all have returned. The caller keeps working meanwhile (the streaming pipeline's
    // coordinator runs on the calling thread while the readers run here).
    struct Group {
        std::mutex mu;
        std::condition_variable cv;
        int left = 0;
        void wait() {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return left == 0; });
        }
    };
    void start(int ntasks, const std::function<void(int)>& fn, Group& grp) {
        {
            std::lock_guard<std::mutex> g(grp.mu);
            grp.left = ntasks;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            for (int t = 0; t < ntasks; ++t)
                q_.push_back([&fn, &grp, t] {
                    fn(t);
                    std::lock_guard<std::mutex> g2(grp.mu);
                    if (--grp.left == 0) grp.cv.notify_all();
                });
        }
        cv_.notify_all();
    }

   private:
    void run() {
        for (;;) {
            std::function<void()> job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (stop_ && q_.empty()) return;
                if (lifo_) {  // OXH_POOL_LIFO=1: last in, first out (the r04 order; for A/Bs)
                    job = std::move(q_.back());
                    q_.pop_back();
                } else {
                    job = std::move(q_.front());  // first in, first out: a caller waiting on its oldest
                    q_.pop_front();               // group (the bounce windows) gets it done first
                }
                ++busy_;
            }
            job();
            {
                std::lock_guard<std::mutex> lk(mu_);
                --busy_;
            }
            idle_cv_.notify_all();
        }
    }
    const bool lifo_ = getenv("OXH_POOL_LIFO") && atoi(getenv("OXH_POOL_LIFO")) != 0;
    std::vector<std::thread> th_;
    std::deque<std::function<void()>> q_;
    std::mutex mu_;
    std::condition_variable cv_, idle_cv_;
    int busy_ = 0;
    bool stop_ = false;
};

}  // namespace oxh
