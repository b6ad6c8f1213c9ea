#include "sfm/pool.hpp"
#include <chrono>
#include <cstdio>
#include <cmath>
int main() {
    using namespace sfm;
    std::vector<double> out(64);
    for (int rep = 0; rep < 3; ++rep) {
        for (int nt : {1, 2, 4, 8}) {
            auto t0 = std::chrono::steady_clock::now();
            for (int it = 0; it < 200; ++it)
                pool_ranges(8000000, nt, [&](int64_t a, int64_t b, int t) {
                    double s = 0;
                    for (int64_t i = a; i < b; i += 64) s += std::sqrt((double)i);
                    out[t] += s;
                });
            auto t1 = std::chrono::steady_clock::now();
            std::printf("nt %d: %.2f ms\n", nt, std::chrono::duration<double, std::milli>(t1 - t0).count());
        }
    }
}
