// Geometric filter of putative matches on gfx950:
// GeometricFilter_FMatrix_AC(4.0, 2048), the step sparseBuilder::filter()
// runs after match() (src/sparseBuilder/sparseBuilder.cpp:1179-1186):
// OpenMVG's a-contrario RANSAC (ACRANSAC) over the 7-point fundamental-matrix
// kernel, one independent problem per image pair.
//
// Layout and work split: one 256-thread workgroup per pair.  The sampling
// and the 7-point fit are a short serial chain (lane 0); every model's
// residual pass, the compaction of the residuals under the a-contrario upper
// bound, their (error, index) bitonic sort in LDS and the NFA scan over the
// sorted prefix are spread over the 256 threads.  The pair's normalised
// coordinates (32 B per correspondence) are read from L2 once per model.
// Pairs are independent: a collection fills the chip with workgroups.
//
// The arithmetic is OpenMVG's as restated in oracle/fmat_oracle.cpp (see the
// header there for the two places where libm / Eigen calls are replaced by
// exact-operation restatements): the same operation sequences, no FMA
// contraction (pragma below), so the GPU and the oracle agree bit for bit.
// Sampling consumes std::mt19937(default_seed) -- the raw stream is generated
// once on the host and shared by all pairs, each starting at position 0 as
// ACRANSAC's per-call generator does -- through a restatement of libstdc++'s
// uniform_int_distribution (Lemire's nearly-divisionless method, 64-bit
// product), pinned against std:: by tests/test_fmatrix.py.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <random>
#include <vector>

#include "common.h"

namespace sfm {
namespace {

constexpr int kFT = 256;            // threads per pair
constexpr int kSample = 7;          // SevenPointSolver::MINIMUM_SAMPLES
constexpr int kMaxModels = 3;       // SevenPointSolver::MAX_MODELS
constexpr int kMaxLdsSort = 8192;   // sort buffer in LDS up to this many slots
constexpr int64_t kRngWords = 1 << 18;

// ---- exact-operation math, identical to oracle/fmat_oracle.cpp ---------------
__host__ __device__ double det_log10(double x) {
    int e = 0;
    double m = frexp(x, &e);
    if (m < 0.70710678118654752440) {
        m = m * 2.0;
        e = e - 1;
    }
    const double s = (m - 1.0) / (m + 1.0);
    const double s2 = s * s;
    double p = 1.0 / 23.0;
    p = p * s2 + 1.0 / 21.0;
    p = p * s2 + 1.0 / 19.0;
    p = p * s2 + 1.0 / 17.0;
    p = p * s2 + 1.0 / 15.0;
    p = p * s2 + 1.0 / 13.0;
    p = p * s2 + 1.0 / 11.0;
    p = p * s2 + 1.0 / 9.0;
    p = p * s2 + 1.0 / 7.0;
    p = p * s2 + 1.0 / 5.0;
    p = p * s2 + 1.0 / 3.0;
    p = p * s2 + 1.0;
    const double ln = (double)e * 0.69314718055994530942 + 2.0 * s * p;
    return ln * 0.43429448190325182765;
}

__device__ double det_cbrt(double v) {
    int e = 0;
    double m = frexp(v, &e);
    int r = e % 3;
    if (r < 0) r += 3;
    m = ldexp(m, r);
    e = e - r;
    double y = 1.0;
    for (int it = 0; it < 8; ++it) y = y - (y * y * y - m) / (3.0 * y * y);
    return ldexp(y, e / 3);
}

__device__ __forceinline__ double dep_cubic(double t, double q3, double r2) { return (t * t - q3) * t + r2; }

__device__ double bisect(double lo, double hi, double q3, double r2, bool up) {
    for (int it = 0; it < 200; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (!(mid > lo && mid < hi)) break;
        const double g = dep_cubic(mid, q3, r2);
        if ((g < 0.0) == up) lo = mid;
        else hi = mid;
    }
    return 0.5 * (lo + hi);
}

__device__ int solve_cubic(const double P[4], double roots[3]) {
    if (P[0] == 0.0) return 0;
    const double a = P[2] / P[3], b = P[1] / P[3], c = P[0] / P[3];
    const double q = a * a - 3.0 * b;
    const double r = 2.0 * a * a * a - 9.0 * a * b + 27.0 * c;
    const double Q = q / 9.0;
    const double R = r / 54.0;
    const double Q3 = Q * Q * Q;
    const double R2 = R * R;
    const double CR2 = 729.0 * r * r;
    const double CQ3 = 2916.0 * q * q * q;
    const double a3 = a / 3.0;
    if (R == 0.0 && Q == 0.0) {
        roots[0] = roots[1] = roots[2] = -a3;
        return 3;
    }
    if (CR2 == CQ3) {
        const double sQ = sqrt(Q);
        if (R > 0.0) {
            roots[0] = -2.0 * sQ - a3;
            roots[1] = sQ - a3;
            roots[2] = sQ - a3;
        } else {
            roots[0] = -sQ - a3;
            roots[1] = -sQ - a3;
            roots[2] = 2.0 * sQ - a3;
        }
        return 3;
    }
    if (CR2 < CQ3) {
        const double sQ = sqrt(Q);
        const double q3 = 3.0 * Q, r2 = 2.0 * R;
        roots[0] = bisect(-2.0 * sQ, -sQ, q3, r2, true) - a3;
        roots[1] = bisect(-sQ, sQ, q3, r2, false) - a3;
        roots[2] = bisect(sQ, 2.0 * sQ, q3, r2, true) - a3;
        return 3;
    }
    const double sgnR = R >= 0.0 ? 1.0 : -1.0;
    const double A = -sgnR * det_cbrt(fabs(R) + sqrt(R2 - Q3));
    roots[0] = A + Q / A - a3;
    return 1;
}

// 7-point fundamental matrices (x2' F x1 = 0, row-major), up to 3.  The
// oracle's full-pivot elimination with its column indirection cp[] done as
// physical row / column swaps with static indices only (select chains), so
// the 7 x 9 system stays in registers; every arithmetic operation is the
// oracle's, on the same operands, in the same order.  Run by a whole wave on
// identical data (uniform control flow).
__device__ int seven_point(const double (&x1)[7][2], const double (&x2)[7][2], double (*F)[9], bool store) {
    double A[7][9];
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        A[i][0] = x2[i][0] * x1[i][0];
        A[i][1] = x2[i][0] * x1[i][1];
        A[i][2] = x2[i][0];
        A[i][3] = x2[i][1] * x1[i][0];
        A[i][4] = x2[i][1] * x1[i][1];
        A[i][5] = x2[i][1];
        A[i][6] = x1[i][0];
        A[i][7] = x1[i][1];
        A[i][8] = 1.0;
    }
    int perm[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) perm[c] = c;
#pragma unroll
    for (int t = 0; t < 7; ++t) {
        int br = -1, bc = -1;
        double bv = 0.0;
#pragma unroll
        for (int r = t; r < 7; ++r)
#pragma unroll
            for (int c = t; c < 9; ++c) {
                const double v = fabs(A[r][c]);
                if (v > bv) { bv = v; br = r; bc = c; }
            }
        if (br < 0) return 0;
#pragma unroll
        for (int i = t + 1; i < 7; ++i)
            if (i == br) {
#pragma unroll
                for (int c = 0; c < 9; ++c) {
                    const double tmp = A[t][c];
                    A[t][c] = A[i][c];
                    A[i][c] = tmp;
                }
            }
#pragma unroll
        for (int j = t + 1; j < 9; ++j)
            if (j == bc) {
#pragma unroll
                for (int r = 0; r < 7; ++r) {
                    const double tmp = A[r][t];
                    A[r][t] = A[r][j];
                    A[r][j] = tmp;
                }
                const int tp = perm[t];
                perm[t] = perm[j];
                perm[j] = tp;
            }
        const double p = A[t][t];
#pragma unroll
        for (int r = t + 1; r < 7; ++r) {
            const double f = A[r][t] / p;
#pragma unroll
            for (int c = t; c < 9; ++c) A[r][c] = A[r][c] - f * A[t][c];
        }
    }
    double f1[9], f2[9];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
        double xp[9];
        xp[7] = v == 0 ? 1.0 : 0.0;
        xp[8] = v == 0 ? 0.0 : 1.0;
#pragma unroll
        for (int t = 6; t >= 0; --t) {
            double s = 0.0;
#pragma unroll
            for (int c = t + 1; c < 9; ++c) s = s - A[t][c] * xp[c];
            xp[t] = s / A[t][t];
        }
        double* x = v == 0 ? f1 : f2;
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            double val = 0.0;
#pragma unroll
            for (int c = 0; c < 9; ++c) val = perm[c] == j ? xp[c] : val;
            x[j] = val;
        }
    }
    const double a = f1[0], j = f2[0], b = f1[1], k = f2[1], c = f1[2], l = f2[2], d = f1[3], m = f2[3],
                 e = f1[4], n = f2[4], f = f1[5], o = f2[5], g = f1[6], p = f2[6], h = f1[7], q = f2[7],
                 i = f1[8], r = f2[8];
    const double P[4] = {
        a * e * i + b * f * g + c * d * h - a * f * h - b * d * i - c * e * g,
        a * e * r + a * i * n + b * f * p + b * g * o + c * d * q + c * h * m + d * h * l + e * i * j + f * g * k -
            a * f * q - a * h * o - b * d * r - b * i * m - c * e * p - c * g * n - d * i * k - e * g * l - f * h * j,
        a * n * r + b * o * p + c * m * q + d * l * q + e * j * r + f * k * p + g * k * o + h * l * m + i * j * n -
            a * o * q - b * m * r - c * n * p - d * k * r - e * l * p - f * j * q - g * l * n - h * j * o - i * k * m,
        j * n * r + k * o * p + l * m * q - j * o * q - k * m * r - l * n * p,
    };
    double roots[3];
    const int nr = solve_cubic(P, roots);
    if (store)
        for (int s = 0; s < nr; ++s)
            for (int z = 0; z < 9; ++z) F[s][z] = f1[z] + roots[s] * f2[z];
    return nr;
}

__device__ __forceinline__ double epi_error(const double* F, double x1, double y1, double x2, double y2) {
    const double fx0 = F[0] * x1 + F[1] * y1 + F[2];
    const double fx1 = F[3] * x1 + F[4] * y1 + F[5];
    const double fx2 = F[6] * x1 + F[7] * y1 + F[8];
    const double dist = x2 * fx0 + y2 * fx1 + fx2;
    return (dist * dist) / (fx0 * fx0 + fx1 * fx1);
}

// libstdc++ uniform_int_distribution<uint32_t>(lo, hi) over mt19937 (32-bit
// outputs): Lemire's nearly-divisionless downscaling with a 64-bit product
struct Stream {
    const uint32_t* w;
    int64_t pos, cap;
    bool over = false;
    __device__ uint32_t next() {
        if (pos >= cap) { over = true; return 0u; }
        return w[pos++];
    }
    __device__ uint32_t uniform(uint32_t lo, uint32_t hi) {
        const uint32_t urange = hi - lo;
        if (urange == 0xFFFFFFFFu) return lo + next();
        const uint32_t range = urange + 1u;
        uint64_t product = (uint64_t)next() * (uint64_t)range;
        uint32_t low = (uint32_t)product;
        if (low < range) {
            const uint32_t threshold = (0u - range) % range;
            while (low < threshold && !over) {
                product = (uint64_t)next() * (uint64_t)range;
                low = (uint32_t)product;
            }
        }
        return lo + (uint32_t)(product >> 32);
    }
};

struct FArgs {
    const int64_t* off;       // [n_pairs + 1]
    const double* xn;         // [4 * n] normalised (x1, y1, x2, y2)
    const double* cst;        // [n_pairs][4] logalpha0, maxThreshold, loge0, 0
    const uint32_t* rng;      // raw mt19937(default_seed) stream
    int64_t rng_n;
    double* ltab;             // [n + n_pairs] log10(j), j = 0..n of each pair (scratch)
    float* logc;              // [2 (n + n_pairs)] logc_n | logc_k per pair (scratch)
    uint32_t* vidx;           // [n] vec_index per pair (scratch)
    uint32_t* binl;           // [n] best inliers so far (result)
    unsigned long long* gkey; // sort keys of the pairs whose sort exceeds LDS, packed
    uint32_t* gval;
    const int64_t* goff;      // [n_pairs] slot offset of the pair in gkey / gval, -1: LDS
    double* Fout;             // [n_pairs][9] best model, normalised
    double* stat;             // [n_pairs][4] minNFA, errorMax (normalised), n_inliers, iterations
    int32_t* fail;            // set when a pair exhausts the random stream
    int32_t max_iter;
    int32_t lds_slots;        // sort slots in dynamic LDS
};

__device__ __forceinline__ unsigned long long err_key(double r) {
    // non-negative doubles order as their bit patterns; NaN never reaches the
    // threshold (filtered before)
    return (unsigned long long)__double_as_longlong(r);
}

__global__ __launch_bounds__(kFT) void fmatrix_ac_kernel(FArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int q = blockIdx.x, tid = threadIdx.x;
    const int64_t o0 = a.off[q], n = a.off[q + 1] - o0;
    double* Fo = a.Fout + 9 * (size_t)q;
    double* st = a.stat + 4 * (size_t)q;
    if (n <= kSample) {
        if (tid < 9) Fo[tid] = 0.0;
        if (tid == 0) {
            st[0] = 0.0; st[1] = 0.0; st[2] = 0.0; st[3] = 0.0;
        }
        return;
    }
    const double* X = a.xn + 4 * o0;
    const double logalpha0 = a.cst[4 * q], maxThr = a.cst[4 * q + 1], loge0 = a.cst[4 * q + 2];
    double* L = a.ltab + o0 + q;                 // [n + 1]
    float* logc_n = a.logc + 2 * (o0 + q);       // [n + 1]
    float* logc_k = logc_n + (n + 1);            // [n + 1]
    uint32_t* vidx = a.vidx + o0;
    uint32_t* binl = a.binl + o0;
    const int64_t go = a.goff[q];
    const bool lds_sort = go < 0;
    unsigned long long* keys = lds_sort ? reinterpret_cast<unsigned long long*>(smem) : a.gkey + go;
    uint32_t* vals = lds_sort ? reinterpret_cast<uint32_t*>(smem + 8 * (size_t)a.lds_slots) : a.gval + go;

    __shared__ double s_models[kMaxModels][9], s_bestF[9];
    __shared__ double s_red[kFT / 64];
    __shared__ int s_redk[kFT / 64];
    __shared__ int s_nm, s_m, s_cnt, s_ac, s_upd, s_copy, s_stop;
    __shared__ uint32_t s_sample[kSample];
    __shared__ int64_t s_nIter, s_nIterReserve, s_vsize, s_ninl;
    __shared__ double s_minNFA, s_errorMax;

    // ---- prologue: log10 table, logcombi tables, vec_index --------------------
    for (int64_t j = tid; j <= n; j += kFT) L[j] = j == 0 ? 0.0 : det_log10((double)j);
    for (int64_t j = tid; j < n; j += kFT) vidx[j] = (uint32_t)j;
    __syncthreads();
    for (int64_t k = tid; k <= n; k += kFT) {
        // logcombi(k, n) and logcombi(7, k): OpenMVG's loop, log10 from the table
        double r = 0.0;
        int64_t kk = k;
        if (!(kk >= n || kk <= 0)) {
            if (n - kk < kk) kk = n - kk;
            for (int64_t i = 1; i <= kk; ++i) r = r + (L[n - i + 1] - L[i]);
        }
        logc_n[k] = (float)r;
        double r7 = 0.0;
        int64_t k7 = kSample;
        if (!(k7 >= k || k7 <= 0)) {
            if (k - k7 < k7) k7 = k - k7;
            for (int64_t i = 1; i <= k7; ++i) r7 = r7 + (L[k - i + 1] - L[i]);
        }
        logc_k[k] = (float)r7;
    }
    if (tid == 0) {
        s_ac = 0;
        s_minNFA = __longlong_as_double(0x7FF0000000000000LL);   // +inf
        s_errorMax = __longlong_as_double(0x7FF0000000000000LL);
        s_nIterReserve = a.max_iter / 10;
        s_nIter = a.max_iter - s_nIterReserve;
        s_vsize = n;
        s_ninl = 0;
        s_stop = 0;
    }
    __syncthreads();
    Stream rs{a.rng, 0, a.rng_n};
    int64_t iter = 0;
    for (iter = 0; iter < s_nIter; ++iter) {
        // ---- sampling (lane 0), 7-point fit (wave 0) -------------------------
        if (tid == 0) {
            if (s_ac) {
                for (int i = 0; i < kSample; ++i) {
                    const uint32_t d = rs.uniform((uint32_t)i, (uint32_t)(s_vsize - 1));
                    const uint32_t t = vidx[i];
                    vidx[i] = vidx[d];
                    vidx[d] = t;
                    s_sample[i] = vidx[i];
                }
            } else {
                int ns = 0;
                while (ns < kSample && !rs.over) {
                    const uint32_t sm = rs.uniform(0u, (uint32_t)(n - 1));
                    bool found = false;
                    for (int j = 0; j < ns && !found; ++j) found = s_sample[j] == sm;
                    if (!found) s_sample[ns++] = sm;
                }
            }
            s_stop = rs.over ? 1 : 0;
            if (rs.over) a.fail[0] = 1;
            s_upd = 0;
        }
        __syncthreads();
        if (s_stop) break;
        if (tid < 64) {
            double sx1[kSample][2], sx2[kSample][2];
#pragma unroll
            for (int i = 0; i < kSample; ++i) {
                const double* p = X + 4 * (size_t)s_sample[i];
                sx1[i][0] = p[0]; sx1[i][1] = p[1];
                sx2[i][0] = p[2]; sx2[i][1] = p[3];
            }
            const int nm = seven_point(sx1, sx2, s_models, tid == 0);
            if (tid == 0) s_nm = nm;
        }
        __syncthreads();
        const int nm = s_nm;
        for (int mi = 0; mi < nm; ++mi) {
            const double* F = s_models[mi];
            if (!s_ac) {   // does the model explain > 2.5 * 7 residuals under the bound?
                int c = 0;
                for (int64_t k = tid; k < n; k += kFT) {
                    const double* p = X + 4 * k;
                    c += epi_error(F, p[0], p[1], p[2], p[3]) <= maxThr;
                }
                for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);
                if (tid == 0) s_cnt = 0;
                __syncthreads();
                if ((tid & 63) == 0) atomicAdd(&s_cnt, c);
                __syncthreads();
                if (tid == 0 && (double)s_cnt > 2.5 * kSample) s_ac = 1;
                __syncthreads();
                if (!s_ac) continue;
            }
            // residuals under the bound -> (error, index) keys
            if (tid == 0) s_m = 0;
            __syncthreads();
            for (int64_t k = tid; k < n; k += kFT) {
                const double* p = X + 4 * k;
                const double r = epi_error(F, p[0], p[1], p[2], p[3]);
                if (r <= maxThr) {
                    const int slot = atomicAdd(&s_m, 1);
                    keys[slot] = err_key(r);
                    vals[slot] = (uint32_t)k;
                }
            }
            __syncthreads();
            const int m = s_m;
            int P2 = 1;
            while (P2 < m) P2 <<= 1;
            for (int k = m + tid; k < P2; k += kFT) {
                keys[k] = ~0ull;
                vals[k] = 0xFFFFFFFFu;
            }
            __syncthreads();
            // bitonic sort of (key, val) ascending
            for (int size = 2; size <= P2; size <<= 1) {
                for (int stride = size >> 1; stride > 0; stride >>= 1) {
                    for (int t = tid; t < P2 / 2; t += kFT) {
                        const int lo = 2 * t - (t & (stride - 1));
                        const int hi = lo + stride;
                        const bool asc = (lo & size) == 0;
                        const unsigned long long kl = keys[lo], kh = keys[hi];
                        const uint32_t vl = vals[lo], vh = vals[hi];
                        const bool gt = kl > kh || (kl == kh && vl > vh);
                        if (gt == asc) {
                            keys[lo] = kh; keys[hi] = kl;
                            vals[lo] = vh; vals[hi] = vl;
                        }
                    }
                    __syncthreads();
                }
            }
            // bestNFA over the sorted prefix: k = 8 .. m
            double bn = __longlong_as_double(0x7FF0000000000000LL);
            int bk = kSample;
            for (int k = kSample + 1 + tid; k <= m; k += kFT) {
                const double e = __longlong_as_double((long long)keys[k - 1]);
                const double logalpha = logalpha0 + 0.5 * det_log10(e + 1.1920928955078125e-07);
                const double nfa = loge0 + logalpha * (double)(k - kSample) + (double)logc_n[k] + (double)logc_k[k];
                if (nfa < bn) { bn = nfa; bk = k; }
            }
            for (int d = 32; d >= 1; d >>= 1) {
                const double on = __shfl_xor(bn, d);
                const int ok = __shfl_xor(bk, d);
                if (on < bn || (on == bn && ok < bk)) { bn = on; bk = ok; }
            }
            if ((tid & 63) == 0) { s_red[tid >> 6] = bn; s_redk[tid >> 6] = bk; }
            __syncthreads();
            if (tid == 0) {
                for (int w = 1; w < kFT / 64; ++w)
                    if (s_red[w] < bn || (s_red[w] == bn && s_redk[w] < bk)) { bn = s_red[w]; bk = s_redk[w]; }
                s_copy = 0;
                if (bn < s_minNFA) {
                    s_upd = 1;
                    s_copy = 1;
                    s_minNFA = bn;
                    s_ninl = bk;
                    s_errorMax = __longlong_as_double((long long)keys[bk - 1]);
                    for (int z = 0; z < 9; ++z) s_bestF[z] = F[z];
                }
            }
            __syncthreads();
            if (s_copy)
                for (int64_t k = tid; k < s_ninl; k += kFT) binl[k] = vals[k];
            __syncthreads();
        }
        // focused sampling: draw among the best inliers so far
        if (tid == 0) {
            s_copy = 0;
            if ((s_upd && s_minNFA < 0) || (iter + 1 == s_nIter && s_nIterReserve)) {
                if (s_ninl == 0) {
                    s_nIter++;
                    s_nIterReserve--;
                } else {
                    s_copy = 1;
                    s_vsize = s_ninl;
                    if (s_nIterReserve) {
                        s_nIter = iter + 1 + s_nIterReserve;
                        s_nIterReserve = 0;
                    }
                }
            }
        }
        __syncthreads();
        if (s_copy)
            for (int64_t k = tid; k < s_ninl; k += kFT) vidx[k] = binl[k];
        __syncthreads();
    }
    if (tid == 0) {
        const bool keep = s_minNFA < 0 && s_ninl > 0;
        st[0] = s_minNFA;
        st[1] = s_errorMax;
        st[2] = keep ? (double)s_ninl : 0.0;
        st[3] = (double)iter;
        for (int z = 0; z < 9; ++z) Fo[z] = keep ? s_bestF[z] : 0.0;
    }
}

struct Norm {
    double s, tx, ty;
};

Norm precondition(int w, int h) {
    const double dn = 1.0 / std::sqrt((double)w * (double)h);
    return Norm{dn, (double)(-0.5f * (float)w) * dn, -0.5 * (double)h * dn};
}

// raw mt19937(default_seed) outputs, generated once per process
const std::vector<uint32_t>& rng_stream() {
    static const std::vector<uint32_t> w = [] {
        std::vector<uint32_t> v((size_t)kRngWords);
        std::mt19937 g(std::mt19937::default_seed);
        for (auto& x : v) x = (uint32_t)g();
        return v;
    }();
    return w;
}

}  // namespace
}  // namespace sfm

using namespace sfm;

extern "C" int sfm_fmatrix_ac(sfm_ctx* ctx, int64_t n_pairs, const int64_t* off, const double* xy,
                              const int32_t* wh, const sfm_fmatrix_opts* opts, sfm_fmatrix_result* results,
                              int32_t* inliers) {
    return guarded([&] {
        SFM_REQUIRE(ctx && n_pairs >= 0 && (n_pairs == 0 || (off && wh && results && inliers)), SFM_ERR_INVALID_ARG,
                    "sfm_fmatrix_ac: bad arguments");
        if (n_pairs == 0) return SFM_OK;
        const double precision = opts ? opts->precision : 4.0;
        const int32_t max_iter = opts ? opts->max_iterations : 2048;
        SFM_REQUIRE(precision > 0 && max_iter > 0, SFM_ERR_INVALID_ARG, "sfm_fmatrix_ac: bad options");
        SFM_REQUIRE(off[0] == 0, SFM_ERR_INVALID_ARG, "sfm_fmatrix_ac: off[0] must be 0");
        int64_t max_n = 0;
        for (int64_t q = 0; q < n_pairs; ++q) {
            SFM_REQUIRE(off[q + 1] >= off[q], SFM_ERR_INVALID_ARG, "sfm_fmatrix_ac: off not monotone at %lld",
                        (long long)q);
            SFM_REQUIRE(wh[4 * q] > 0 && wh[4 * q + 1] > 0 && wh[4 * q + 2] > 0 && wh[4 * q + 3] > 0,
                        SFM_ERR_INVALID_ARG, "sfm_fmatrix_ac: pair %lld has a non-positive image size", (long long)q);
            max_n = std::max(max_n, off[q + 1] - off[q]);
        }
        SFM_REQUIRE(max_n < (int64_t)1 << 31, SFM_ERR_UNSUPPORTED, "sfm_fmatrix_ac: pair too large");
        const int64_t n = off[n_pairs];
        SFM_REQUIRE(n == 0 || xy, SFM_ERR_INVALID_ARG, "sfm_fmatrix_ac: null coordinates");
        CtxScope scope_(ctx);
        hipStream_t s = ctx->stream;
        PhaseTimer tm("sfm_fmatrix_ac");
        // normalised coordinates and the a-contrario constants per pair (host:
        // O(n) setup; the O(iterations x n log n) search runs on the device)
        std::vector<double> xn((size_t)std::max<int64_t>(4 * n, 1)), cst(4 * (size_t)n_pairs);
        for (int64_t q = 0; q < n_pairs; ++q) {
            const Norm N1 = precondition(wh[4 * q], wh[4 * q + 1]), N2 = precondition(wh[4 * q + 2], wh[4 * q + 3]);
            for (int64_t k = off[q]; k < off[q + 1]; ++k) {
                xn[4 * k] = N1.s * xy[4 * k] + N1.tx;
                xn[4 * k + 1] = N1.s * xy[4 * k + 1] + N1.ty;
                xn[4 * k + 2] = N2.s * xy[4 * k + 2] + N2.tx;
                xn[4 * k + 3] = N2.s * xy[4 * k + 3] + N2.ty;
            }
            const double w2 = (double)wh[4 * q + 2], h2 = (double)wh[4 * q + 3];
            const double Dg = std::sqrt(w2 * w2 + h2 * h2), Ar = w2 * h2;
            const int64_t np = off[q + 1] - off[q];
            cst[4 * q] = det_log10(2.0 * Dg / Ar / N2.s);
            cst[4 * q + 1] = precision * precision * N2.s * N2.s;
            cst[4 * q + 2] = det_log10((double)kMaxModels * (double)(np > kSample ? np - kSample : 1));
            cst[4 * q + 3] = 0.0;
        }
        tm.mark("normalise");
        DBuf<int64_t> d_off, d_goff;
        DBuf<double> d_xn, d_cst, d_ltab, d_F, d_stat;
        DBuf<float> d_logc;
        DBuf<uint32_t> d_rng, d_vidx, d_binl, d_gval;
        DBuf<unsigned long long> d_gkey;
        DBuf<int32_t> d_fail;
        d_off.alloc(n_pairs + 1);
        d_off.upload(off, n_pairs + 1, s);
        d_xn.alloc(xn.size());
        d_xn.upload(xn.data(), xn.size(), s);
        d_cst.alloc(cst.size());
        d_cst.upload(cst.data(), cst.size(), s);
        const auto& rw = rng_stream();
        d_rng.alloc(rw.size());
        d_rng.upload(rw.data(), rw.size(), s);
        d_ltab.alloc((size_t)(n + n_pairs));
        d_logc.alloc(2 * (size_t)(n + n_pairs));
        d_vidx.alloc((size_t)std::max<int64_t>(n, 1));
        d_binl.alloc((size_t)std::max<int64_t>(n, 1));
        d_F.alloc(9 * (size_t)n_pairs);
        d_stat.alloc(4 * (size_t)n_pairs);
        d_fail.alloc(1);
        d_fail.zero(s);
        // sort buffers per pair: next_pow2(n) slots, in LDS up to kMaxLdsSort;
        // only the pairs above that get global (L2) buffers, packed by prefix
        // sum, so one large pair does not move every pair to global memory
        std::vector<int64_t> goff((size_t)n_pairs, -1);
        int64_t lds_slots = 1, g_slots = 0;
        for (int64_t q = 0; q < n_pairs; ++q) {
            int64_t sl = 1;
            while (sl < off[q + 1] - off[q]) sl <<= 1;
            if (sl <= kMaxLdsSort) {
                lds_slots = std::max(lds_slots, sl);
            } else {
                goff[q] = g_slots;
                g_slots += sl;
            }
        }
        FArgs a{};
        a.off = d_off.p; a.xn = d_xn.p; a.cst = d_cst.p; a.rng = d_rng.p; a.rng_n = (int64_t)rw.size();
        a.ltab = d_ltab.p; a.logc = d_logc.p; a.vidx = d_vidx.p; a.binl = d_binl.p;
        a.Fout = d_F.p; a.stat = d_stat.p; a.fail = d_fail.p; a.max_iter = max_iter;
        d_goff.alloc(goff.size());
        d_goff.upload(goff.data(), goff.size(), s);
        a.goff = d_goff.p;
        a.lds_slots = (int32_t)lds_slots;
        const size_t lds = 12 * (size_t)lds_slots;
        if (g_slots) {   // large pairs: sort buffers in global memory (L2)
            d_gkey.alloc((size_t)g_slots);
            d_gval.alloc((size_t)g_slots);
            a.gkey = d_gkey.p;
            a.gval = d_gval.p;
        }
        set_dyn_lds((const void*)fmatrix_ac_kernel, 12 * kMaxLdsSort);
        SFM_REQUIRE(n_pairs < ((int64_t)1 << 31), SFM_ERR_UNSUPPORTED, "sfm_fmatrix_ac: too many pairs");
        // the kernel alone (sfm_ctx_last_kernel_ms, SFM_CTX_TIME_KERNELS only):
        // the uploads are drained first, or the start event can be stamped
        // while a DMA of the stream is still running (measured: 48 ms by
        // events against rocprofv3's 29)
        const bool timed = ctx->time_kernels;
        hipEvent_t* ev = timed ? ctx_events(ctx) : nullptr;
        if (timed) {
            SFM_HIP(hipStreamSynchronize(s));
            SFM_HIP(hipEventRecord(ev[0], s));
        }
        tm.mark("upload");
        hipLaunchKernelGGL(fmatrix_ac_kernel, dim3((unsigned)n_pairs), dim3(kFT), lds, s, a);
        SFM_HIP(hipGetLastError());
        if (timed) SFM_HIP(hipEventRecord(ev[1], s));
        tm.mark("launch");
        std::vector<double> F(9 * (size_t)n_pairs), stat(4 * (size_t)n_pairs);
        std::vector<uint32_t> binl((size_t)std::max<int64_t>(n, 1));
        int32_t fail = 0;
        SFM_HIP(hipMemcpyAsync(F.data(), d_F.p, F.size() * 8, hipMemcpyDeviceToHost, s));
        SFM_HIP(hipMemcpyAsync(stat.data(), d_stat.p, stat.size() * 8, hipMemcpyDeviceToHost, s));
        if (n) SFM_HIP(hipMemcpyAsync(binl.data(), d_binl.p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        SFM_HIP(hipMemcpyAsync(&fail, d_fail.p, 4, hipMemcpyDeviceToHost, s));
        SFM_HIP(hipStreamSynchronize(s));
        ctx->last_kernel_ms = -1.0;
        if (timed) {
            float ms = 0.f;
            SFM_HIP(hipEventElapsedTime(&ms, ev[0], ev[1]));
            ctx->last_kernel_ms = ms;
        }
        tm.mark("kernel+download");
        SFM_REQUIRE(!fail, SFM_ERR_UNSUPPORTED, "sfm_fmatrix_ac: a pair drew more than %lld random numbers",
                    (long long)kRngWords);
        for (int64_t q = 0; q < n_pairs; ++q) {
            sfm_fmatrix_result& r = results[q];
            std::memset(&r, 0, sizeof r);
            const int64_t np = off[q + 1] - off[q];
            r.iterations = (int32_t)stat[4 * q + 3];
            if (np <= kSample) continue;
            r.min_nfa = stat[4 * q];
            const int64_t ninl = (int64_t)stat[4 * q + 2];
            const Norm N1 = precondition(wh[4 * q], wh[4 * q + 1]), N2 = precondition(wh[4 * q + 2], wh[4 * q + 3]);
            if (ninl == 0) {   // no meaningful model (ACRANSAC clears its inliers)
                r.error_max = stat[4 * q + 1];
                continue;
            }
            // Unnormalize: F = N2' F N1
            const double* Fn = &F[9 * q];
            const double T1[9] = {N1.s, 0, N1.tx, 0, N1.s, N1.ty, 0, 0, 1};
            const double T2[9] = {N2.s, 0, N2.tx, 0, N2.s, N2.ty, 0, 0, 1};
            double FT1[9];
            for (int rr = 0; rr < 3; ++rr)
                for (int c = 0; c < 3; ++c)
                    FT1[3 * rr + c] = Fn[3 * rr] * T1[c] + Fn[3 * rr + 1] * T1[3 + c] + Fn[3 * rr + 2] * T1[6 + c];
            for (int rr = 0; rr < 3; ++rr)
                for (int c = 0; c < 3; ++c)
                    r.F[3 * rr + c] = T2[rr] * FT1[c] + T2[3 + rr] * FT1[3 + c] + T2[6 + rr] * FT1[6 + c];
            r.error_max = std::sqrt(stat[4 * q + 1]) / N2.s;
            // GeometricFilter_FMatrix_AC: keep the pair iff > 2.5 * 7 inliers
            if ((double)ninl > kSample * 2.5) {
                r.n_inliers = (int32_t)ninl;
                for (int64_t k = 0; k < ninl; ++k) inliers[off[q] + k] = (int32_t)binl[off[q] + k];
            }
        }
        return SFM_OK;
    });
}
