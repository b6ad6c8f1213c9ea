// Counter-based RNG for the synthetic generators: SplitMix64 increments with
// the Stafford "mix13" finaliser, one independent stream per entity.
#pragma once
#include <cmath>
#include <cstdint>

namespace sfm::synth {

inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

inline uint64_t entity_seed(uint64_t seed, uint64_t stream, uint64_t id) {
    return mix64(mix64(seed ^ (stream * 0xD1B54A32D192ED03ULL)) + id * 0x9E3779B97F4A7C15ULL);
}

struct Rng {
    uint64_t s;
    bool has_spare = false;
    double spare = 0.0;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() { s += 0x9E3779B97F4A7C15ULL; return mix64(s); }
    double uni() { return (double)(next() >> 11) * 0x1.0p-53; }  // [0, 1)
    double gauss() {  // Box-Muller, polar-free form
        if (has_spare) { has_spare = false; return spare; }
        const double u1 = 1.0 - uni();   // (0, 1]
        const double u2 = uni();
        const double r = std::sqrt(-2.0 * std::log(u1));
        spare = r * std::sin(2.0 * M_PI * u2);
        has_spare = true;
        return r * std::cos(2.0 * M_PI * u2);
    }
};

}  // namespace sfm::synth
