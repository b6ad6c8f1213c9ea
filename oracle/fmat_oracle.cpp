// oracle/fmat_oracle.cpp — TEST INFRASTRUCTURE ONLY (see oracle.h): CPU
// restatement of the reference's geometric filter, SURVEY.md §8(f) row 3.
//
// src/sparseBuilder/sparseBuilder.cpp:1179-1186 runs
//   filter_ptr->Robust_model_estimation(GeometricFilter_FMatrix_AC(4.0, 2048), ...)
// over every putative pair.  OpenMVG is un-vendored, so this
// restates its published 2.x code at that call site — PARITY UNPINNED:
//   * GeometricFilter_FMatrix_AC::Robust_estimation: MatchesPairToMat (pixel
//     coordinates: the views carry no distortion at this stage), an
//     ACKernelAdaptor<SevenPointSolver, EpipolarDistanceError, UnnormalizerT,
//     Mat3> with point-to-line a-contrario constants, ACRANSAC(kernel,
//     inliers, 2048, &F, 4.0^2), and "keep the pair iff #inliers > 2.5 * 7";
//   * NormalizePointsFromImageSize / PreconditionerFromImageSize
//     (1/sqrt(w h) scale, image centre to the origin);
//   * ACRANSAC: std::mt19937(default_seed) per call, the rejection sampler
//     UniformSample(7, n) until a model has > 2.5 * 7 residuals under the
//     upper bound (then the a-contrario mode and the partial Fisher-Yates
//     UniformSample(7, &vec_index)), residuals sorted as (error, index)
//     pairs, bestNFA with float logcombi tables, 10 % of the iterations
//     reserved for sampling among the best inliers (vec_index = inliers);
//   * EpipolarDistanceError: (x2' F x1)^2 / |(F x1)_{0,1}|^2.
// Two deliberate, documented restatements of arithmetic OpenMVG takes from
// Eigen / libm (both exact up to rounding, and shared by the GPU kernel so
// the two agree bit for bit):
//   * the 2-D null space of the 7 x 9 epipolar system comes from
//     full-pivot Gaussian elimination (OpenMVG: JacobiSVD's last two right
//     singular vectors); every basis of that space gives the same pencil
//     F1 + a F2 and the same F up to scale, and the residual is scale free;
//   * SolveCubicPolynomial keeps libmv's case split (triple, double, three,
//     one real root) but finds three distinct roots by bisection between
//     the critical points of the depressed cubic instead of acos/cos, and
//     the single root with a Newton cube root instead of pow(., 1/3); log10
//     is a fixed atanh series.  No transcendental libm call remains.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <random>
#include <utility>
#include <vector>

#include "oracle.h"

namespace {

// log10 of x > 0: x = m 2^e, m in [sqrt(1/2), sqrt(2)), ln m = 2 atanh(s),
// s = (m - 1) / (m + 1), |s| <= 0.1716, series to s^23.
double det_log10(double x) {
    int e = 0;
    double m = std::frexp(x, &e);
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

// cube root of v > 0: exponent split by 3, Newton from 1 on the mantissa
double det_cbrt(double v) {
    int e = 0;
    double m = std::frexp(v, &e);
    int r = e % 3;
    if (r < 0) r += 3;
    m = std::ldexp(m, r);
    e = e - r;
    double y = 1.0;
    for (int it = 0; it < 8; ++it) y = y - (y * y * y - m) / (3.0 * y * y);
    return std::ldexp(y, e / 3);
}

// depressed cubic t^3 - 3Q t + 2R
double dep_cubic(double t, double q3, double r2) { return (t * t - q3) * t + r2; }

// root of g in [lo, hi] with g(lo) and g(hi) of opposite signs (rising when
// up), bisection until the midpoint is no longer strictly inside
double bisect(double lo, double hi, double q3, double r2, bool up) {
    for (int it = 0; it < 200; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (!(mid > lo && mid < hi)) break;
        const double g = dep_cubic(mid, q3, r2);
        if ((g < 0.0) == up) lo = mid;
        else hi = mid;
    }
    return 0.5 * (lo + hi);
}

// libmv SolveCubicPolynomial(coeffs) as OpenMVG's seven-point solver calls
// it: coeffs in ascending powers; 0 roots when coeffs[0] == 0
int solve_cubic(const double P[4], double roots[3]) {
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
        const double sQ = std::sqrt(Q);
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
        const double sQ = std::sqrt(Q);
        const double q3 = 3.0 * Q, r2 = 2.0 * R;
        roots[0] = bisect(-2.0 * sQ, -sQ, q3, r2, true) - a3;
        roots[1] = bisect(-sQ, sQ, q3, r2, false) - a3;
        roots[2] = bisect(sQ, 2.0 * sQ, q3, r2, true) - a3;
        return 3;
    }
    const double sgnR = R >= 0.0 ? 1.0 : -1.0;
    const double A = -sgnR * det_cbrt(std::fabs(R) + std::sqrt(R2 - Q3));
    roots[0] = A + Q / A - a3;
    return 1;
}

// Seven-point fundamental matrices of normalised correspondences
// (x1: image I, x2: image J; x2' F x1 = 0, F row-major)
int seven_point(const double (*x1)[2], const double (*x2)[2], double F[3][9]) {
    double A[7][9];
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
    int cp[9] = {0, 1, 2, 3, 4, 5, 6, 7, 8};
    for (int t = 0; t < 7; ++t) {
        int br = -1, bc = -1;
        double bv = 0.0;
        for (int r = t; r < 7; ++r)
            for (int c = t; c < 9; ++c) {
                const double v = std::fabs(A[r][cp[c]]);
                if (v > bv) { bv = v; br = r; bc = c; }
            }
        if (br < 0) return 0;   // rank < 7: degenerate sample
        if (br != t)
            for (int c = 0; c < 9; ++c) std::swap(A[t][c], A[br][c]);
        std::swap(cp[t], cp[bc]);
        const double p = A[t][cp[t]];
        for (int r = t + 1; r < 7; ++r) {
            const double f = A[r][cp[t]] / p;
            for (int c = t; c < 9; ++c) A[r][cp[c]] = A[r][cp[c]] - f * A[t][cp[c]];
        }
    }
    double f1[9], f2[9];
    for (int v = 0; v < 2; ++v) {
        double* x = v == 0 ? f1 : f2;
        x[cp[7]] = v == 0 ? 1.0 : 0.0;
        x[cp[8]] = v == 0 ? 0.0 : 1.0;
        for (int t = 6; t >= 0; --t) {
            double s = 0.0;
            for (int c = t + 1; c < 9; ++c) s = s - A[t][cp[c]] * x[cp[c]];
            x[cp[t]] = s / A[t][cp[t]];
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
    for (int s = 0; s < nr; ++s)
        for (int z = 0; z < 9; ++z) F[s][z] = f1[z] + roots[s] * f2[z];
    return nr;
}

// EpipolarDistanceError, point to line (squared, normalised units)
double epi_error(const double F[9], double x1, double y1, double x2, double y2) {
    const double fx0 = F[0] * x1 + F[1] * y1 + F[2];
    const double fx1 = F[3] * x1 + F[4] * y1 + F[5];
    const double fx2 = F[6] * x1 + F[7] * y1 + F[8];
    const double dist = x2 * fx0 + y2 * fx1 + fx2;
    return (dist * dist) / (fx0 * fx0 + fx1 * fx1);
}

// logcombi(k, n) = log10 C(n, k), OpenMVG's loop
double logcombi(int k, int n) {
    if (k >= n || k <= 0) return 0.0;
    if (n - k < k) k = n - k;
    double r = 0.0;
    for (int i = 1; i <= k; ++i) r = r + (det_log10((double)(n - i + 1)) - det_log10((double)i));
    return r;
}

struct Norm {
    double s, tx, ty;   // x' = s x + tx, y' = s y + ty
};

Norm precondition(int w, int h) {
    const double dn = 1.0 / std::sqrt((double)w * (double)h);
    return Norm{dn, (double)(-0.5f * (float)w) * dn, -0.5 * (double)h * dn};
}

constexpr int kSample = 7, kMaxModels = 3;

void fmatrix_ac_pair(int64_t n, const double* xy, const int32_t* wh, double precision, int32_t max_iter,
                     sfm_fmatrix_result* res, int32_t* inliers_out) {
    std::memset(res, 0, sizeof *res);
    if (n <= kSample) return;
    const Norm N1 = precondition(wh[0], wh[1]), N2 = precondition(wh[2], wh[3]);
    std::vector<double> x1((size_t)n), y1((size_t)n), x2((size_t)n), y2((size_t)n);
    for (int64_t k = 0; k < n; ++k) {
        x1[k] = N1.s * xy[4 * k] + N1.tx;
        y1[k] = N1.s * xy[4 * k + 1] + N1.ty;
        x2[k] = N2.s * xy[4 * k + 2] + N2.tx;
        y2[k] = N2.s * xy[4 * k + 3] + N2.ty;
    }
    // a-contrario constants (point to line): alpha0 = 2 D / A / N2, multError 0.5
    const double w2 = (double)wh[2], h2 = (double)wh[3];
    const double Dg = std::sqrt(w2 * w2 + h2 * h2), Ar = w2 * h2;
    const double logalpha0 = det_log10(2.0 * Dg / Ar / N2.s);
    const double mult = 0.5;
    const double maxThreshold = precision * precision * N2.s * N2.s;
    const double loge0 = det_log10((double)kMaxModels * (double)(n - kSample));
    std::vector<float> logc_n((size_t)n + 1), logc_k((size_t)n + 1);
    for (int64_t k = 0; k <= n; ++k) {
        logc_n[k] = (float)logcombi((int)k, (int)n);
        logc_k[k] = (float)logcombi(kSample, (int)k);
    }
    std::mt19937 rng(std::mt19937::default_seed);
    std::vector<uint32_t> vec_index((size_t)n), vec_inliers, sample(kSample);
    std::iota(vec_index.begin(), vec_index.end(), 0u);
    std::vector<double> resid((size_t)n);
    std::vector<std::pair<double, uint32_t>> er((size_t)n);
    double minNFA = std::numeric_limits<double>::infinity();
    double errorMax = std::numeric_limits<double>::infinity();
    double bestF[9] = {0};
    size_t nIterReserve = (size_t)max_iter / 10;
    size_t nIter = (size_t)max_iter - nIterReserve;
    bool acMode = false;   // precision is finite (4^2)
    size_t iter = 0;
    for (iter = 0; iter < nIter; ++iter) {
        if (acMode) {
            for (int i = 0; i < kSample; ++i) {
                std::uniform_int_distribution<uint32_t> dist((uint32_t)i, (uint32_t)(vec_index.size() - 1));
                std::swap(vec_index[i], vec_index[dist(rng)]);
                sample[i] = vec_index[i];
            }
        } else {
            std::uniform_int_distribution<uint32_t> dist(0, (uint32_t)(n - 1));
            sample.clear();
            while (sample.size() < (size_t)kSample) {
                const uint32_t s = dist(rng);
                bool found = false;
                for (size_t j = 0; j < sample.size() && !found; ++j) found = sample[j] == s;
                if (!found) sample.push_back(s);
            }
        }
        double sx1[kSample][2], sx2[kSample][2];
        for (int i = 0; i < kSample; ++i) {
            sx1[i][0] = x1[sample[i]]; sx1[i][1] = y1[sample[i]];
            sx2[i][0] = x2[sample[i]]; sx2[i][1] = y2[sample[i]];
        }
        double models[kMaxModels][9];
        const int nm = seven_point(sx1, sx2, models);
        bool better = false;
        for (int mi = 0; mi < nm; ++mi) {
            for (int64_t k = 0; k < n; ++k) resid[k] = epi_error(models[mi], x1[k], y1[k], x2[k], y2[k]);
            if (!acMode) {
                unsigned nIn = 0;
                for (int64_t k = 0; k < n; ++k) nIn += resid[k] <= maxThreshold;
                if (nIn > 2.5 * kSample) acMode = true;
            }
            if (!acMode) continue;
            // (error, index) order; non-finite residuals never reach the
            // threshold and sort last (NaN ordered as +inf)
            for (int64_t k = 0; k < n; ++k)
                er[k] = {std::isnan(resid[k]) ? std::numeric_limits<double>::infinity() : resid[k], (uint32_t)k};
            std::sort(er.begin(), er.end());
            double bNFA = std::numeric_limits<double>::infinity();
            int64_t bK = kSample;
            for (int64_t k = kSample + 1; k <= n && er[k - 1].first <= maxThreshold; ++k) {
                const double logalpha = logalpha0 + mult * det_log10(er[k - 1].first + (double)std::numeric_limits<float>::epsilon());
                const double nfa = loge0 + logalpha * (double)(k - kSample) + (double)logc_n[k] + (double)logc_k[k];
                if (nfa < bNFA) { bNFA = nfa; bK = k; }
            }
            if (bNFA < minNFA) {
                better = true;
                minNFA = bNFA;
                vec_inliers.resize((size_t)bK);
                for (int64_t k = 0; k < bK; ++k) vec_inliers[k] = er[k].second;
                errorMax = er[bK - 1].first;
                std::memcpy(bestF, models[mi], sizeof bestF);
            }
        }
        if ((better && minNFA < 0) || (iter + 1 == nIter && nIterReserve)) {
            if (vec_inliers.empty()) {
                nIter++;
                nIterReserve--;
            } else {
                vec_index = vec_inliers;
                if (nIterReserve) {
                    nIter = iter + 1 + nIterReserve;
                    nIterReserve = 0;
                }
            }
        }
    }
    res->iterations = (int32_t)iter;
    if (minNFA >= 0) vec_inliers.clear();
    res->min_nfa = minNFA;
    if (vec_inliers.empty()) {
        res->error_max = errorMax;
        return;
    }
    // Unnormalize: F = N2' F N1 (N = [s 0 tx; 0 s ty; 0 0 1])
    const double T1[9] = {N1.s, 0, N1.tx, 0, N1.s, N1.ty, 0, 0, 1};
    const double T2[9] = {N2.s, 0, N2.tx, 0, N2.s, N2.ty, 0, 0, 1};
    double FT1[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            FT1[3 * r + c] = bestF[3 * r] * T1[c] + bestF[3 * r + 1] * T1[3 + c] + bestF[3 * r + 2] * T1[6 + c];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            res->F[3 * r + c] = T2[r] * FT1[c] + T2[3 + r] * FT1[3 + c] + T2[6 + r] * FT1[6 + c];
    res->error_max = std::sqrt(errorMax) / N2.s;
    // GeometricFilter_FMatrix_AC: the pair keeps its inliers iff > 2.5 * 7
    if ((double)vec_inliers.size() > kSample * 2.5) {
        res->n_inliers = (int32_t)vec_inliers.size();
        for (size_t k = 0; k < vec_inliers.size(); ++k) inliers_out[k] = (int32_t)vec_inliers[k];
    }
}

}  // namespace

extern "C" int orc_fmatrix_ac(int64_t n_pairs, const int64_t* off, const double* xy, const int32_t* wh,
                              const sfm_fmatrix_opts* opts, sfm_fmatrix_result* results, int32_t* inliers,
                              int32_t n_threads) {
    if (n_pairs < 0 || (n_pairs && (!off || !wh || !results || !inliers))) return SFM_ERR_INVALID_ARG;
    const double precision = opts ? opts->precision : 4.0;
    const int32_t max_iter = opts ? opts->max_iterations : 2048;
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads > 0 ? n_threads : 1)
    for (int64_t q = 0; q < n_pairs; ++q)
        fmatrix_ac_pair(off[q + 1] - off[q], xy + 4 * off[q], wh + 4 * q, precision, max_iter, results + q,
                        inliers + off[q]);
    return SFM_OK;
}

extern "C" int orc_uniform_draws(const uint32_t* lo, const uint32_t* hi, int64_t n, uint32_t* out) {
    std::mt19937 rng(std::mt19937::default_seed);
    for (int64_t k = 0; k < n; ++k) out[k] = std::uniform_int_distribution<uint32_t>(lo[k], hi[k])(rng);
    return SFM_OK;
}

extern "C" int orc_det_math(int32_t fn, const double* x, int64_t n, double* out) {
    for (int64_t k = 0; k < n; ++k) out[k] = fn == 0 ? det_log10(x[k]) : det_cbrt(x[k]);
    return SFM_OK;
}

extern "C" int orc_seven_point(const double* x1, const double* x2, double* F, int32_t* n_models) {
    double a[7][2], b[7][2], M[3][9];
    for (int i = 0; i < 7; ++i) {
        a[i][0] = x1[2 * i]; a[i][1] = x1[2 * i + 1];
        b[i][0] = x2[2 * i]; b[i][1] = x2[2 * i + 1];
    }
    *n_models = seven_point(a, b, M);
    for (int s = 0; s < *n_models; ++s)
        for (int z = 0; z < 9; ++z) F[9 * s + z] = M[s][z];
    return SFM_OK;
}
