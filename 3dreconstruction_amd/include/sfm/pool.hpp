// Host worker pool shared by the planner (csrc/ba_plan.cpp) and the header-
// only façade (the BundleAdjuster's walk over the world): up to 15 threads
// started once and parked on a condition variable, so a parallel phase costs
// a wake-up instead of thread creations.  Header-only; each binary that
// includes it has its own pool.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace sfm {

// One caller at a time uses the pool; a concurrent caller (another context
// planning at the same moment) runs its tasks on fresh threads instead.
class PlanPool {
   public:
    static PlanPool& get() {
        static PlanPool p;
        return p;
    }
    static int width() {
        // SFM_PLAN_THREADS: override (1 = serial planning, for profiling)
        static const int w = [] {
            int64_t n = std::min<int64_t>(16, std::thread::hardware_concurrency());
            if (const char* e = std::getenv("SFM_PLAN_THREADS")) n = std::min<int64_t>(16, std::atoi(e));
            return (int)std::max<int64_t>(1, n);
        }();
        return w;
    }
    // fn(t) for t in [0, n): tasks spread over the workers and the caller; an
    // exception of any task is rethrown here once every task has finished
    // A nested call (a task of this pool calling run() again, on a worker or
    // on the calling thread) runs its tasks serially on the thread that makes
    // it: it never touches use_, which that thread may already hold.
    void run(int n, const std::function<void(int)>& fn) {
        if (n <= 1) {
            if (n == 1) fn(0);
            return;
        }
        if (in_task()) {
            for (int t = 0; t < n; ++t) fn(t);
            return;
        }
        std::unique_lock<std::mutex> busy(use_, std::try_to_lock);
        if (!busy.owns_lock() || workers_.empty()) {
            std::exception_ptr err;
            std::mutex em;
            auto call = [&](int t) {
                try { fn(t); } catch (...) { std::lock_guard<std::mutex> g(em); if (!err) err = std::current_exception(); }
            };
            std::vector<std::thread> th;
            for (int t = 1; t < n; ++t) th.emplace_back(call, t);
            call(0);
            for (auto& x : th) x.join();
            if (err) std::rethrow_exception(err);
            return;
        }
        uint32_t g;
        {
            std::lock_guard<std::mutex> lk(m_);
            g = ++gen_;
            job_ = &fn;
            n_tasks_ = n;
            left_ = n;
            err_ = nullptr;
            next_.store((uint64_t)g << 32);
        }
        cv_.notify_all();
        {
            TaskScope scope;
            work(g, &fn, n);
        }
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [&] { return left_ == 0; });
        job_ = nullptr;
        if (err_) std::rethrow_exception(err_);
    }

   private:
    // set while this thread runs tasks of the pool (workers: always)
    static bool& in_task() {
        static thread_local bool f = false;
        return f;
    }
    struct TaskScope {
        bool prev = in_task();
        TaskScope() { in_task() = true; }
        ~TaskScope() { in_task() = prev; }
    };
    PlanPool() {
        for (int t = 1; t < width(); ++t) workers_.emplace_back([this] { loop(); });
    }
    ~PlanPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& x : workers_) x.join();
    }
    // Tasks are claimed from one word holding (generation << 32 | next task):
    // a worker that wakes late for a finished run can never claim (or count)
    // a task of the next one.
    void work(uint32_t g, const std::function<void(int)>* job, int n) {
        int done = 0;
        for (;;) {
            uint64_t v = next_.load();
            int t = -1;
            while ((uint32_t)(v >> 32) == g && (int)(v & 0xffffffffu) < n) {
                if (next_.compare_exchange_weak(v, v + 1)) {
                    t = (int)(v & 0xffffffffu);
                    break;
                }
            }
            if (t < 0) break;
            try {
                (*job)(t);
            } catch (...) {
                std::lock_guard<std::mutex> lk(m_);
                if (!err_) err_ = std::current_exception();
            }
            ++done;
        }
        if (done) {
            std::lock_guard<std::mutex> lk(m_);
            left_ -= done;
            if (left_ == 0) done_.notify_all();
        }
    }
    void loop() {
        in_task() = true;
        uint32_t seen = 0;
        for (;;) {
            uint32_t g;
            const std::function<void(int)>* job;
            int n;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = g = gen_;
                job = job_;
                n = n_tasks_;
            }
            work(g, job, n);
        }
    }
    std::mutex use_, m_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> workers_;
    const std::function<void(int)>* job_ = nullptr;
    std::atomic<uint64_t> next_{0};
    std::exception_ptr err_;
    int n_tasks_ = 0, left_ = 0;
    uint32_t gen_ = 0;
    bool stop_ = false;
};

// fn(k0, k1, t) over nt contiguous ranges of [0, n) on the pool
template <class F>
void pool_ranges(int64_t n, int nt, F&& fn) {
    if (nt <= 1) {
        fn(0, n, 0);
        return;
    }
    PlanPool::get().run(nt, [&](int t) { fn(n * t / nt, n * (t + 1) / nt, t); });
}

}  // namespace sfm
