// Stress test of the planner's host worker pool (csrc/ba_plan.cpp PlanPool):
// back-to-back parallel phases of varying size must each run every task
// exactly once and never deadlock (a worker waking late for a finished phase
// must not claim or count a task of the next one).  Built from the planner
// source itself, with the few library hooks it needs stubbed on malloc.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <vector>

#include "../../3dreconstruction_amd/csrc/ba_plan.cpp"

namespace sfm {
void host_free(void* p) { std::free(p); }
void* host_alloc(size_t n) { return std::malloc(n); }
void set_error(const char* fmt, ...) {
    va_list a;
    va_start(a, fmt);
    std::vfprintf(stderr, fmt, a);
    va_end(a);
}
}  // namespace sfm

int main(int argc, char** argv) {
    using namespace sfm;
    const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
    long bad = 0;
    for (int it = 0; it < iters; ++it) {
        const int64_t n = 4096 + (int64_t)(it * 7919) % 40000;
        std::vector<int> hit(n, 0);
        parallel_ranges(n, [&](int64_t a, int64_t b, int) {
            for (int64_t i = a; i < b; ++i) hit[i]++;
        });
        for (int64_t i = 0; i < n; ++i) bad += hit[i] != 1;
        int seg[5] = {0};
        parallel_segments(5, [&](int g) { seg[g]++; });
        for (int g = 0; g < 5; ++g) bad += seg[g] != 1;
    }
    // an exception in a task reaches the caller after every task has run
    bool caught = false;
    try {
        parallel_segments(6, [&](int g) {
            if (g == 3) throw std::runtime_error("task 3");
        });
    } catch (const std::runtime_error&) {
        caught = true;
    }
    // a task that runs a phase of its own (on a worker or on the caller,
    // which holds the pool): serial on its thread, every inner task once
    std::vector<int> nested(8 * 9, 0);
    PlanPool::get().run(8, [&](int g) {
        PlanPool::get().run(9, [&](int h) { nested[g * 9 + h]++; });
    });
    for (int v : nested) bad += v != 1;
    std::printf("pool: %d phases, %ld bad, exception %s\n", iters, bad, caught ? "caught" : "lost");
    return bad == 0 && caught ? 0 : 1;
}
