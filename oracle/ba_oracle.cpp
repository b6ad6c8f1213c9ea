// CPU restatement of the reference bundle adjuster — TEST INFRASTRUCTURE
// ONLY (see oracle.h; parity unpinned: Ceres is absent).
//
// Model (src/adjuster/BundleAdjuster.h; SFM_CAM_SNAVELY: the in-tree
// src/adjuster/SnavelyReprojectionError.h:16-54 instead of ReprojectCost):
//   ReprojectCost :40-65   P = AngleAxisRotatePoint(w, X) + t; x = P0/P2;
//                          y = P1/P2; r = (fx x + cx - u, fy y + cy - v)
//   HuberLoss(4)   :109    rho(s) = s (s <= 16), 2*4*sqrt(s) - 16 otherwise
//   gauge          :105    pose of local_frames_.front()->getImage2() constant
//   RMSE           :137-138 sqrt(cost / num_residuals)
//   options        :167-174 SPARSE_SCHUR, JACOBI, num_threads 1; all other
//                          ceres::Solver::Options at their Ceres 2.2 defaults.
// Minimizer: the Ceres 2.2 TrustRegionMinimizer + LevenbergMarquardtStrategy
// control flow, restated from the published algorithm (ceres-solver 2.2,
// internal/ceres/trust_region_minimizer.cc, levenberg_marquardt_strategy.cc,
// trust_region_step_evaluator.cc, corrector.cc, loss_function.cc,
// schur_eliminator_impl.h, rotation.h):
//   * Jacobi column scaling 1/(1+sqrt(|J_col|^2)) from the loss-corrected
//     Jacobian at iteration 0, applied to every later Jacobian;
//   * LM diagonal clamp(|J_s col|^2, 1e-6, 1e32), D = sqrt(diag/radius),
//     diagonal reused after rejected steps;
//   * step from (J_s'J_s + D'D) y = J_s' f by Schur elimination of the 3-dof
//     point blocks; step = -y; invalid unless model_cost_change > 0;
//   * check order per iteration: parameter tolerance, function tolerance,
//     step quality > min_relative_decrease;
//   * radius /= max(1/3, 1-(2 rho-1)^3) on success, radius /= 2^k on
//     consecutive rejections;
//   * termination tests after every iteration: max_num_iterations (counts
//     rejected iterations), gradient tolerance on |x - (x - g)|_inf,
//     min_trust_region_radius.
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "oracle.h"
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

constexpr double kEps = std::numeric_limits<double>::epsilon();

// Jacobian row layout: intrinsics (up to 6; the model's width iw, zeros past
// it) | extr 6 (w 3, t 3) | X 3.
constexpr int kJR = 15, kJE = 6, kJX = 12;
inline int intr_width(int model) { return model == SFM_CAM_RADIAL3 ? 6 : 4; }

// ---------------------------------------------------------------------------
// Analytic residual + Jacobian (row-major 2 x kJR).
// dP/dw for the Rodrigues branch: -R [X]x (w w' + (R' - I)[w]x) / |w|^2
// (Gallego & Yezzi 2015); small-angle branch of AngleAxisRotatePoint:
// P = X + w x X, dP/dw = -[X]x, dP/dX = I + [w]x.
// ---------------------------------------------------------------------------
bool residual_jacobian(int model, const double* in, const double* e, const double* X, const double* uv,
                       double r[2], double* J) {
    const double* w = e;
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double P[3], dPdw[9], dPdX[9];
    if (th2 > kEps) {
        const double th = std::sqrt(th2), c = std::cos(th), s = std::sin(th), it = 1.0 / th;
        const double u[3] = {w[0] * it, w[1] * it, w[2] * it};
        const double cr[3] = {u[1] * X[2] - u[2] * X[1], u[2] * X[0] - u[0] * X[2],
                              u[0] * X[1] - u[1] * X[0]};
        const double tmp = (u[0] * X[0] + u[1] * X[1] + u[2] * X[2]) * (1.0 - c);
        for (int a = 0; a < 3; ++a) P[a] = X[a] * c + cr[a] * s + u[a] * tmp;
        if (J) {
            double R[9];
            const double oc = 1.0 - c;
            R[0] = c + oc * u[0] * u[0];       R[1] = oc * u[0] * u[1] - s * u[2]; R[2] = oc * u[0] * u[2] + s * u[1];
            R[3] = oc * u[1] * u[0] + s * u[2]; R[4] = c + oc * u[1] * u[1];       R[5] = oc * u[1] * u[2] - s * u[0];
            R[6] = oc * u[2] * u[0] - s * u[1]; R[7] = oc * u[2] * u[1] + s * u[0]; R[8] = c + oc * u[2] * u[2];
            for (int a = 0; a < 9; ++a) dPdX[a] = R[a];
            // M = w w' + (R' - I)[w]x
            const double Wx[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
            double M[9];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double acc = w[i] * w[j];
                    for (int k = 0; k < 3; ++k) acc += (R[k * 3 + i] - (i == k ? 1.0 : 0.0)) * Wx[k * 3 + j];
                    M[i * 3 + j] = acc;
                }
            const double Xx[9] = {0, -X[2], X[1], X[2], 0, -X[0], -X[1], X[0], 0};
            double N[9];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double acc = 0;
                    for (int k = 0; k < 3; ++k) acc += Xx[i * 3 + k] * M[k * 3 + j];
                    N[i * 3 + j] = acc;
                }
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double acc = 0;
                    for (int k = 0; k < 3; ++k) acc += R[i * 3 + k] * N[k * 3 + j];
                    dPdw[i * 3 + j] = -acc / th2;
                }
        }
    } else {
        const double cr[3] = {w[1] * X[2] - w[2] * X[1], w[2] * X[0] - w[0] * X[2],
                              w[0] * X[1] - w[1] * X[0]};
        for (int a = 0; a < 3; ++a) P[a] = X[a] + cr[a];
        if (J) {
            const double I3[9] = {1, -w[2], w[1], w[2], 1, -w[0], -w[1], w[0], 1};
            const double mXx[9] = {0, X[2], -X[1], -X[2], 0, X[0], X[1], -X[0], 0};
            for (int a = 0; a < 9; ++a) { dPdX[a] = I3[a]; dPdw[a] = mXx[a]; }
        }
    }
    P[0] += e[3]; P[1] += e[4]; P[2] += e[5];
    double A[2][3], Ji[2][6] = {{0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0}};
    if (model == SFM_CAM_RADIAL3) {
        // OpenMVG ResidualErrorFunctor_Pinhole_Intrinsic_Radial_K3 (PINHOLE_CAMERA_RADIAL3,
        // sparseBuilder.cpp:1292-1299): x_u = P/P2, r_coeff = 1 + k1 r2 + k2 r4 + k3 r6,
        // r = (ppx + f x_u r_coeff, ppy + f y_u r_coeff) - obs; in = (f, ppx, ppy, k1, k2, k3)
        const double xu = P[0] / P[2], yu = P[1] / P[2];
        const double r2 = xu * xu + yu * yu, r4 = r2 * r2, r6 = r4 * r2;
        const double rc = 1.0 + in[3] * r2 + in[4] * r4 + in[5] * r6;
        r[0] = in[1] + in[0] * (xu * rc) - uv[0];
        r[1] = in[2] + in[0] * (yu * rc) - uv[1];
        if (J) {
            // d(rc)/d(xu, yu) = D (xu, yu), D = 2 (k1 + 2 k2 r2 + 3 k3 r4)
            const double iz = 1.0 / P[2], D = 2.0 * (in[3] + 2.0 * in[4] * r2 + 3.0 * in[5] * r4);
            const double B[2][2] = {{in[0] * (rc + D * xu * xu), in[0] * D * xu * yu},
                                    {in[0] * D * xu * yu, in[0] * (rc + D * yu * yu)}};
            const double pu[2] = {xu, yu};
            for (int row = 0; row < 2; ++row) {
                A[row][0] = iz * B[row][0];
                A[row][1] = iz * B[row][1];
                A[row][2] = -iz * (B[row][0] * xu + B[row][1] * yu);
                Ji[row][0] = pu[row] * rc;
                Ji[row][1] = row == 0 ? 1.0 : 0.0;
                Ji[row][2] = row == 1 ? 1.0 : 0.0;
                Ji[row][3] = in[0] * pu[row] * r2;
                Ji[row][4] = in[0] * pu[row] * r4;
                Ji[row][5] = in[0] * pu[row] * r6;
            }
        }
    } else if (model == SFM_CAM_SNAVELY) {
        // SnavelyReprojectionError.h:31-47: p = -P/P2, d = 1 + r2 (l1 + l2 r2),
        // r = f d p - obs.  dr/dP = f [d I + 2 (l1 + 2 l2 r2) p p'] dp/dP,
        // dp/dP = -1/P2 [1 0 xp; 0 1 yp]
        const double xp = -P[0] / P[2], yp = -P[1] / P[2];
        const double r2 = xp * xp + yp * yp;
        const double d = 1.0 + r2 * (in[1] + in[2] * r2);
        r[0] = in[0] * d * xp - uv[0];
        r[1] = in[0] * d * yp - uv[1];
        if (J) {
            const double iz = 1.0 / P[2], dd2 = 2.0 * (in[1] + 2.0 * in[2] * r2);
            const double B[2][2] = {{in[0] * (d + dd2 * xp * xp), in[0] * dd2 * xp * yp},
                                    {in[0] * dd2 * xp * yp, in[0] * (d + dd2 * yp * yp)}};
            const double p[2] = {xp, yp};
            for (int row = 0; row < 2; ++row) {
                A[row][0] = -iz * B[row][0];
                A[row][1] = -iz * B[row][1];
                A[row][2] = -iz * (B[row][0] * xp + B[row][1] * yp);
                Ji[row][0] = d * p[row];
                Ji[row][1] = in[0] * r2 * p[row];
                Ji[row][2] = in[0] * r2 * r2 * p[row];
                Ji[row][3] = 0.0;
            }
        }
    } else {
        const double x = P[0] / P[2], y = P[1] / P[2];
        r[0] = in[0] * x + in[2] - uv[0];
        r[1] = in[1] * y + in[3] - uv[1];
        if (J) {
            const double iz = 1.0 / P[2];
            const double A0[2][3] = {{in[0] * iz, 0.0, -in[0] * x * iz}, {0.0, in[1] * iz, -in[1] * y * iz}};
            const double J0[2][4] = {{x, 0.0, 1.0, 0.0}, {0.0, y, 0.0, 1.0}};
            std::memcpy(A, A0, sizeof A);
            for (int row = 0; row < 2; ++row)
                for (int k = 0; k < 4; ++k) Ji[row][k] = J0[row][k];
        }
    }
    if (J) {
        for (int row = 0; row < 2; ++row) {
            double* Jr = J + row * kJR;
            for (int k = 0; k < 6; ++k) Jr[k] = Ji[row][k];
            for (int j = 0; j < 3; ++j) {
                double a = 0, b = 0;
                for (int k = 0; k < 3; ++k) { a += A[row][k] * dPdw[k * 3 + j]; b += A[row][k] * dPdX[k * 3 + j]; }
                Jr[kJE + j] = a; Jr[kJE + 3 + j] = A[row][j]; Jr[kJX + j] = b;
            }
        }
    }
    return std::isfinite(r[0]) && std::isfinite(r[1]);
}

// ---------------------------------------------------------------------------
// Forward-mode dual numbers (ceres::Jet<double,N> semantics) for the
// autodiff cross-check.
// ---------------------------------------------------------------------------
struct Jet {
    double a; double v[kJR];
    Jet() : a(0) { std::memset(v, 0, sizeof v); }
    explicit Jet(double x) : a(x) { std::memset(v, 0, sizeof v); }
    Jet(double x, int k) : a(x) { std::memset(v, 0, sizeof v); v[k] = 1.0; }
};
inline Jet operator+(const Jet& f, const Jet& g) { Jet r(f.a + g.a); for (int k = 0; k < kJR; ++k) r.v[k] = f.v[k] + g.v[k]; return r; }
inline Jet operator-(const Jet& f, const Jet& g) { Jet r(f.a - g.a); for (int k = 0; k < kJR; ++k) r.v[k] = f.v[k] - g.v[k]; return r; }
inline Jet operator*(const Jet& f, const Jet& g) { Jet r(f.a * g.a); for (int k = 0; k < kJR; ++k) r.v[k] = f.a * g.v[k] + f.v[k] * g.a; return r; }
inline Jet operator/(const Jet& f, const Jet& g) {
    const double ia = 1.0 / g.a, abyb = f.a * ia;
    Jet r(abyb); for (int k = 0; k < kJR; ++k) r.v[k] = (f.v[k] - abyb * g.v[k]) * ia; return r;
}
inline Jet jsqrt(const Jet& f) { const double t = std::sqrt(f.a), i2 = 1.0 / (2.0 * t); Jet r(t); for (int k = 0; k < kJR; ++k) r.v[k] = f.v[k] * i2; return r; }
inline Jet jcos(const Jet& f) { Jet r(std::cos(f.a)); const double s = -std::sin(f.a); for (int k = 0; k < kJR; ++k) r.v[k] = s * f.v[k]; return r; }
inline Jet jsin(const Jet& f) { Jet r(std::sin(f.a)); const double c = std::cos(f.a); for (int k = 0; k < kJR; ++k) r.v[k] = c * f.v[k]; return r; }

void residual_jet(int model, const Jet* intr, const Jet* extr, const Jet* pt, const double* uv, Jet* res) {
    const Jet* w = extr;
    Jet P[3];
    const Jet theta2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    if (theta2.a > kEps) {
        const Jet theta = jsqrt(theta2), c = jcos(theta), s = jsin(theta), ti = Jet(1.0) / theta;
        const Jet u[3] = {w[0] * ti, w[1] * ti, w[2] * ti};
        const Jet cr[3] = {u[1] * pt[2] - u[2] * pt[1], u[2] * pt[0] - u[0] * pt[2], u[0] * pt[1] - u[1] * pt[0]};
        const Jet tmp = (u[0] * pt[0] + u[1] * pt[1] + u[2] * pt[2]) * (Jet(1.0) - c);
        for (int a = 0; a < 3; ++a) P[a] = pt[a] * c + cr[a] * s + u[a] * tmp;
    } else {
        const Jet cr[3] = {w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2], w[0] * pt[1] - w[1] * pt[0]};
        for (int a = 0; a < 3; ++a) P[a] = pt[a] + cr[a];
    }
    P[0] = P[0] + extr[3]; P[1] = P[1] + extr[4]; P[2] = P[2] + extr[5];
    if (model == SFM_CAM_RADIAL3) {   // ResidualErrorFunctor_Pinhole_Intrinsic_Radial_K3, term by term
        const Jet xu = P[0] / P[2], yu = P[1] / P[2];
        const Jet r2 = xu * xu + yu * yu, r4 = r2 * r2, r6 = r4 * r2;
        const Jet rc = Jet(1.0) + intr[3] * r2 + intr[4] * r4 + intr[5] * r6;
        const Jet xd = xu * rc, yd = yu * rc;
        res[0] = intr[1] + intr[0] * xd - Jet(uv[0]);
        res[1] = intr[2] + intr[0] * yd - Jet(uv[1]);
        return;
    }
    if (model == SFM_CAM_SNAVELY) {   // SnavelyReprojectionError.h:31-47, term by term
        const Jet xp = Jet(0.0) - P[0] / P[2], yp = Jet(0.0) - P[1] / P[2];
        const Jet r2 = xp * xp + yp * yp;
        const Jet dist = Jet(1.0) + r2 * (intr[1] + intr[2] * r2);
        res[0] = intr[0] * dist * xp - Jet(uv[0]);
        res[1] = intr[0] * dist * yp - Jet(uv[1]);
        return;
    }
    const Jet x = P[0] / P[2], y = P[1] / P[2];
    res[0] = intr[0] * x + intr[2] - Jet(uv[0]);
    res[1] = intr[1] * y + intr[3] - Jet(uv[1]);
}

// Huber (ceres::HuberLoss::Evaluate); a <= 0 means no loss.
inline void huber(double a, double s, double rho[2]) {
    if (a > 0 && s > a * a) {
        const double r = std::sqrt(s);
        rho[0] = 2.0 * a * r - a * a;
        rho[1] = std::max(std::numeric_limits<double>::min(), a / r);
    } else {
        rho[0] = s; rho[1] = 1.0;
    }
}

// ---------------------------------------------------------------------------
// Reduced camera system: lower band (cameras) + dense arrow (intrinsics).
// ---------------------------------------------------------------------------
struct BandArrow {
    int64_t nb = 0, na = 0, bw = 0;
    std::vector<double> band, arrow, corner;   // band[i*(bw+1) + (i-j)], arrow[a*nb+j], corner[a*na+b]
    void init(int64_t nb_, int64_t na_, int64_t bw_) {
        nb = nb_; na = na_; bw = bw_;
        band.assign(nb * (bw + 1), 0.0); arrow.assign(na * nb, 0.0); corner.assign(na * na, 0.0);
    }
    void zero() { std::fill(band.begin(), band.end(), 0.0); std::fill(arrow.begin(), arrow.end(), 0.0); std::fill(corner.begin(), corner.end(), 0.0); }
    double& at(int64_t i, int64_t j) {  // requires i >= j
        if (i < nb) return band[i * (bw + 1) + (i - j)];
        if (j < nb) return arrow[(i - nb) * nb + j];
        return corner[(i - nb) * na + (j - nb)];
    }
    size_t size() const { return band.size() + arrow.size() + corner.size(); }
    void pack(double* out) const {
        std::copy(band.begin(), band.end(), out);
        std::copy(arrow.begin(), arrow.end(), out + band.size());
        std::copy(corner.begin(), corner.end(), out + band.size() + arrow.size());
    }
    void unpack(const double* in) {
        std::copy(in, in + band.size(), band.begin());
        std::copy(in + band.size(), in + band.size() + arrow.size(), arrow.begin());
        std::copy(in + band.size() + arrow.size(), in + size(), corner.begin());
    }
    void add(const BandArrow& o) {
        for (size_t k = 0; k < band.size(); ++k) band[k] += o.band[k];
        for (size_t k = 0; k < arrow.size(); ++k) arrow[k] += o.arrow[k];
        for (size_t k = 0; k < corner.size(); ++k) corner[k] += o.corner[k];
    }
    // In-place Cholesky L L' = S.  Returns false if not positive definite.
    bool cholesky() {
        for (int64_t i = 0; i < nb; ++i) {
            for (int64_t j = std::max<int64_t>(0, i - bw); j <= i; ++j) {
                double s = band[i * (bw + 1) + (i - j)];
                for (int64_t k = std::max<int64_t>(0, i - bw); k < j; ++k)
                    s -= band[i * (bw + 1) + (i - k)] * band[j * (bw + 1) + (j - k)];
                if (i == j) {
                    if (!(s > 0.0)) return false;
                    band[i * (bw + 1)] = std::sqrt(s);
                } else {
                    band[i * (bw + 1) + (i - j)] = s / band[j * (bw + 1)];
                }
            }
        }
        for (int64_t a = 0; a < na; ++a) {
            double* La = &arrow[a * nb];
            for (int64_t j = 0; j < nb; ++j) {
                double s = La[j];
                for (int64_t k = std::max<int64_t>(0, j - bw); k < j; ++k) s -= La[k] * band[j * (bw + 1) + (j - k)];
                La[j] = s / band[j * (bw + 1)];
            }
        }
        for (int64_t a = 0; a < na; ++a) {
            for (int64_t b = 0; b <= a; ++b) {
                double s = corner[a * na + b];
                for (int64_t k = 0; k < nb; ++k) s -= arrow[a * nb + k] * arrow[b * nb + k];
                for (int64_t k = 0; k < b; ++k) s -= corner[a * na + k] * corner[b * na + k];
                if (a == b) {
                    if (!(s > 0.0)) return false;
                    corner[a * na + a] = std::sqrt(s);
                } else {
                    corner[a * na + b] = s / corner[b * na + b];
                }
            }
        }
        return true;
    }
    void solve(std::vector<double>& x) const {  // x <- (L L')^{-1} x
        const int64_t n = nb + na;
        for (int64_t i = 0; i < n; ++i) {  // forward
            double s = x[i];
            if (i < nb) {
                for (int64_t k = std::max<int64_t>(0, i - bw); k < i; ++k) s -= band[i * (bw + 1) + (i - k)] * x[k];
                x[i] = s / band[i * (bw + 1)];
            } else {
                const int64_t a = i - nb;
                for (int64_t k = 0; k < nb; ++k) s -= arrow[a * nb + k] * x[k];
                for (int64_t k = 0; k < a; ++k) s -= corner[a * na + k] * x[nb + k];
                x[i] = s / corner[a * na + a];
            }
        }
        for (int64_t i = n - 1; i >= 0; --i) {  // backward
            double s = x[i];
            if (i >= nb) {
                const int64_t a = i - nb;
                for (int64_t b = a + 1; b < na; ++b) s -= corner[b * na + a] * x[nb + b];
                x[i] = s / corner[a * na + a];
            } else {
                for (int64_t k = i + 1; k <= std::min(nb - 1, i + bw); ++k) s -= band[k * (bw + 1) + (k - i)] * x[k];
                for (int64_t b = 0; b < na; ++b) s -= arrow[b * nb + i] * x[nb + b];
                x[i] = s / band[i * (bw + 1)];
            }
        }
    }
};

// 3x3 SPD inverse via Cholesky solve against the identity (Ceres
// InvertPSDMatrix with assume_full_rank_ete).
bool inv3_spd(const double V[9], double Vi[9]) {
    const double l00 = V[0];
    if (!(l00 > 0)) return false;
    const double L00 = std::sqrt(l00), L10 = V[3] / L00, L20 = V[6] / L00;
    const double d1 = V[4] - L10 * L10;
    if (!(d1 > 0)) return false;
    const double L11 = std::sqrt(d1), L21 = (V[7] - L20 * L10) / L11;
    const double d2 = V[8] - L20 * L20 - L21 * L21;
    if (!(d2 > 0)) return false;
    const double L22 = std::sqrt(d2);
    for (int c = 0; c < 3; ++c) {
        double b[3] = {c == 0 ? 1.0 : 0.0, c == 1 ? 1.0 : 0.0, c == 2 ? 1.0 : 0.0};
        const double z0 = b[0] / L00, z1 = (b[1] - L10 * z0) / L11, z2 = (b[2] - L20 * z0 - L21 * z1) / L22;
        const double y2 = z2 / L22, y1 = (z1 - L21 * y2) / L11, y0 = (z0 - L10 * y1 - L20 * y2) / L00;
        Vi[0 * 3 + c] = y0; Vi[1 * 3 + c] = y1; Vi[2 * 3 + c] = y2;
    }
    return true;
}

struct Oracle {
    const sfm_ba_problem& P;
    const sfm_ba_options& O;
    orc_allreduce_fn ar; void* user;
    int nthreads;

    std::vector<int> cam_blk, intr_blk;
    int64_t ncam = 0, nintr = 0, nb = 0, na = 0, nF = 0, bw = 0;
    int iw = 4;                        // intrinsics block width of the model
    std::vector<int64_t> pts;          // shard points (global ids)
    std::vector<int64_t> obs_ptr;      // per shard point: first obs slot in the shard obs arrays
    int64_t n_sobs = 0;

    std::vector<double> extr, intr;    // current full camera tables
    std::vector<double> xF, xE;        // active parameters (F: cams then intr; E: shard points)
    std::vector<double> scaleF, scaleE;
    std::vector<double> f, J;          // per shard obs: corrected residual (2), Jacobian (2 x kJR)
    double x_cost = 0;

    Oracle(const sfm_ba_problem& p, const sfm_ba_options& o, orc_allreduce_fn a, void* u, int t)
        : P(p), O(o), ar(a), user(u), nthreads(t > 0 ? t : 1) {}

    void allreduce(double* b, int64_t n, int op) { if (ar) ar(user, b, n, op); }

    int64_t colF_cam(int img) const { return cam_blk[img] < 0 ? -1 : 6 * (int64_t)cam_blk[img]; }
    int64_t colF_intr(int img) const {
        const int q = intr_blk[P.img_intr[img]];
        return q < 0 ? -1 : nb + iw * (int64_t)q;
    }

    void setup(const double* e, const double* in, const double* X, const int64_t* shard, int64_t nsh) {
        iw = intr_width(P.camera_model);
        cam_blk.assign(P.n_img, -1); intr_blk.assign(P.n_intr, -1);
        std::vector<char> cam_used(P.n_img, 0), intr_used(P.n_intr, 0);
        for (int64_t o = 0; o < P.n_obs; ++o) { cam_used[P.obs_img[o]] = 1; intr_used[P.img_intr[P.obs_img[o]]] = 1; }
        for (int i = 0; i < P.n_img; ++i) if (cam_used[i] && i != P.const_img) cam_blk[i] = (int)ncam++;
        for (int q = 0; q < P.n_intr; ++q) if (intr_used[q]) intr_blk[q] = (int)nintr++;
        nb = 6 * ncam; na = iw * nintr; nF = nb + na;
        int64_t D = 0;
        for (int64_t p = 0; p < P.n_pt; ++p) {
            int lo = INT32_MAX, hi = -1;
            for (int64_t o = P.pt_offsets[p]; o < P.pt_offsets[p + 1]; ++o) {
                const int b = cam_blk[P.obs_img[o]];
                if (b >= 0) { lo = std::min(lo, b); hi = std::max(hi, b); }
            }
            if (hi >= 0) D = std::max<int64_t>(D, hi - lo);
        }
        bw = ncam > 0 ? std::min<int64_t>(nb - 1, 6 * D + 5) : 0;
        if (shard) pts.assign(shard, shard + nsh);
        else { pts.resize(P.n_pt); for (int64_t p = 0; p < P.n_pt; ++p) pts[p] = p; }
        obs_ptr.resize(pts.size() + 1);
        obs_ptr[0] = 0;
        for (size_t k = 0; k < pts.size(); ++k)
            obs_ptr[k + 1] = obs_ptr[k] + (P.pt_offsets[pts[k] + 1] - P.pt_offsets[pts[k]]);
        n_sobs = obs_ptr.back();
        extr.assign(e, e + 6 * (size_t)P.n_img); intr.assign(in, in + iw * (size_t)P.n_intr);
        xF.assign(nF, 0.0);
        for (int i = 0; i < P.n_img; ++i) if (cam_blk[i] >= 0) for (int a = 0; a < 6; ++a) xF[6 * cam_blk[i] + a] = extr[6 * i + a];
        // SNAVELY: the 4th intrinsics double is not a parameter (held at 0, never written back)
        for (int q = 0; q < P.n_intr; ++q)
            if (intr_blk[q] >= 0)
                for (int a = 0; a < iw; ++a)
                    xF[nb + iw * intr_blk[q] + a] = (P.camera_model == SFM_CAM_SNAVELY && a == 3) ? 0.0 : intr[iw * q + a];
        xE.resize(3 * pts.size());
        for (size_t k = 0; k < pts.size(); ++k) for (int a = 0; a < 3; ++a) xE[3 * k + a] = X[3 * pts[k] + a];
        f.assign(2 * n_sobs, 0.0); J.assign(2 * kJR * n_sobs, 0.0);
        scaleF.assign(nF, 1.0); scaleE.assign(xE.size(), 1.0);
    }

    void load_cams(const std::vector<double>& xf) {
        for (int i = 0; i < P.n_img; ++i) if (cam_blk[i] >= 0) for (int a = 0; a < 6; ++a) extr[6 * i + a] = xf[6 * cam_blk[i] + a];
        for (int q = 0; q < P.n_intr; ++q) if (intr_blk[q] >= 0) for (int a = 0; a < iw; ++a) intr[iw * q + a] = xf[nb + iw * intr_blk[q] + a];
    }

    // Evaluate cost (and optionally corrected f/J) at (xf, xe). Returns false
    // if any residual is non-finite (on any rank).
    bool evaluate(const std::vector<double>& xf, const std::vector<double>& xe, double* cost, bool jac) {
        load_cams(xf);
        const int64_t npt = (int64_t)pts.size();
        std::vector<double> part(nthreads, 0.0);
        std::vector<char> bad(nthreads, 0);
#pragma omp parallel for schedule(static) num_threads(nthreads)
        for (int64_t k = 0; k < npt; ++k) {
            int tid = 0;
#ifdef _OPENMP
            tid = omp_get_thread_num();
#endif
            const int64_t p = pts[k];
            for (int64_t o = P.pt_offsets[p], s = obs_ptr[k]; o < P.pt_offsets[p + 1]; ++o, ++s) {
                const int img = P.obs_img[o];
                double r[2], Jl[2 * kJR];
                const bool ok = residual_jacobian(P.camera_model, &intr[iw * (size_t)P.img_intr[img]], &extr[6 * (size_t)img],
                                                  &xe[3 * k], &P.obs_uv[2 * o], r, jac ? Jl : nullptr);
                if (!ok) { bad[tid] = 1; continue; }
                const double sq = r[0] * r[0] + r[1] * r[1];
                double rho[2];
                huber(P.huber_a, sq, rho);
                part[tid] += 0.5 * rho[0];
                if (jac) {
                    const double sr = std::sqrt(rho[1]);
                    f[2 * s] = r[0] * sr; f[2 * s + 1] = r[1] * sr;
                    for (int a = 0; a < 2 * kJR; ++a) J[2 * kJR * s + a] = Jl[a] * sr;
                }
            }
        }
        double buf[2] = {0.0, 0.0};
        for (int t = 0; t < nthreads; ++t) { buf[0] += part[t]; buf[1] = std::max(buf[1], (double)bad[t]); }
        allreduce(buf, 1, 0);
        allreduce(buf + 1, 1, 1);
        *cost = buf[0];
        return buf[1] == 0.0 && std::isfinite(buf[0]);
    }

    // Column squared norms of the (scaled if `scaled`) Jacobian: F global, E local.
    void colnorms(bool scaled, std::vector<double>& cF, std::vector<double>& cE) {
        cF.assign(nF, 0.0); cE.assign(xE.size(), 0.0);
        for (size_t k = 0; k < pts.size(); ++k) {
            const int64_t p = pts[k];
            for (int64_t o = P.pt_offsets[p], s = obs_ptr[k]; o < P.pt_offsets[p + 1]; ++o, ++s) {
                const int img = P.obs_img[o];
                const int64_t ci = colF_intr(img), cc = colF_cam(img);
                for (int row = 0; row < 2; ++row) {
                    const double* Jr = &J[2 * kJR * s + kJR * row];
                    for (int a = 0; a < iw; ++a) { const double v = Jr[a] * (scaled ? scaleF[ci + a] : 1.0); cF[ci + a] += v * v; }
                    if (cc >= 0) for (int a = 0; a < 6; ++a) { const double v = Jr[kJE + a] * (scaled ? scaleF[cc + a] : 1.0); cF[cc + a] += v * v; }
                    for (int a = 0; a < 3; ++a) { const double v = Jr[kJX + a] * (scaled ? scaleE[3 * k + a] : 1.0); cE[3 * k + a] += v * v; }
                }
            }
        }
        allreduce(cF.data(), nF, 0);
    }

    // |x - (x - g)|_inf with g = J' f (unscaled, corrected).
    double gradient_max_norm() {
        std::vector<double> gF(nF, 0.0), gE(xE.size(), 0.0);
        for (size_t k = 0; k < pts.size(); ++k) {
            const int64_t p = pts[k];
            for (int64_t o = P.pt_offsets[p], s = obs_ptr[k]; o < P.pt_offsets[p + 1]; ++o, ++s) {
                const int img = P.obs_img[o];
                const int64_t ci = colF_intr(img), cc = colF_cam(img);
                for (int row = 0; row < 2; ++row) {
                    const double* Jr = &J[2 * kJR * s + kJR * row];
                    const double fr = f[2 * s + row];
                    for (int a = 0; a < iw; ++a) gF[ci + a] += Jr[a] * fr;
                    if (cc >= 0) for (int a = 0; a < 6; ++a) gF[cc + a] += Jr[kJE + a] * fr;
                    for (int a = 0; a < 3; ++a) gE[3 * k + a] += Jr[kJX + a] * fr;
                }
            }
        }
        allreduce(gF.data(), nF, 0);
        double m = 0.0;
        for (int64_t c = 0; c < nF; ++c) m = std::max(m, std::fabs(xF[c] - (xF[c] - gF[c])));
        double mE = 0.0;
        for (size_t c = 0; c < gE.size(); ++c) mE = std::max(mE, std::fabs(xE[c] - (xE[c] - gE[c])));
        allreduce(&mE, 1, 1);
        return std::max(m, mE);
    }

    double sqnorm_x(const std::vector<double>& xf, const std::vector<double>& xe) {
        double sE = 0.0;
        for (double v : xe) sE += v * v;
        allreduce(&sE, 1, 0);
        double s = 0.0;
        for (double v : xf) s += v * v;
        return s + sE;
    }

    // Solve (Js'Js + D'D) y = Js' f by Schur elimination.  Returns false on
    // linear-solver failure.
    bool schur_solve(const std::vector<double>& lmF, const std::vector<double>& lmE,
                     std::vector<double>& yF, std::vector<double>& yE) {
        const int64_t npt = (int64_t)pts.size();
        BandArrow S; S.init(nb, na, bw);
        std::vector<double> rhs(nF, 0.0);
        std::vector<BandArrow> St(nthreads);
        std::vector<std::vector<double>> rt(nthreads);
        std::vector<char> fail(nthreads, 0);
        for (int t = 0; t < nthreads; ++t) { St[t].init(nb, na, bw); rt[t].assign(nF, 0.0); }
#pragma omp parallel for schedule(static) num_threads(nthreads)
        for (int64_t k = 0; k < npt; ++k) {
            int tid = 0;
#ifdef _OPENMP
            tid = omp_get_thread_num();
#endif
            BandArrow& Sl = St[tid];
            std::vector<double>& rl = rt[tid];
            const int64_t p = pts[k];
            const int64_t o0 = P.pt_offsets[p], o1 = P.pt_offsets[p + 1];
            // local F column list of this point
            std::vector<int64_t> cols;
            std::vector<int> c_of(2 * (o1 - o0));
            for (int64_t o = o0; o < o1; ++o) {
                const int img = P.obs_img[o];
                for (int which = 0; which < 2; ++which) {
                    const int64_t g = which == 0 ? colF_intr(img) : colF_cam(img);
                    if (g < 0) { c_of[2 * (o - o0) + which] = -1; continue; }
                    auto it = std::find(cols.begin(), cols.end(), g);
                    if (it == cols.end()) { c_of[2 * (o - o0) + which] = (int)cols.size(); cols.push_back(g); }
                    else c_of[2 * (o - o0) + which] = (int)(it - cols.begin());
                }
            }
            // local dense column index of every F column
            std::vector<int64_t> gcol;  // per local scalar column: global column
            std::vector<int> base(cols.size());
            for (size_t b = 0; b < cols.size(); ++b) {
                base[b] = (int)gcol.size();
                const int w = cols[b] >= nb ? iw : 6;
                for (int a = 0; a < w; ++a) gcol.push_back(cols[b] + a);
            }
            const int nl = (int)gcol.size();
            std::vector<double> Wl(3 * nl, 0.0), Ul(nl * nl, 0.0), bF(nl, 0.0);
            double V[9] = {0}, bE[3] = {0};
            for (int64_t o = o0, s = obs_ptr[k]; o < o1; ++o, ++s) {
                const int img = P.obs_img[o];
                const int64_t ci = colF_intr(img), cc = colF_cam(img);
                // scaled row pieces
                for (int row = 0; row < 2; ++row) {
                    const double* Jr = &J[2 * kJR * s + kJR * row];
                    const double fr = f[2 * s + row];
                    double jx[3], jf[12]; int lf[12]; int nf = 0;
                    for (int a = 0; a < 3; ++a) jx[a] = Jr[kJX + a] * scaleE[3 * k + a];
                    { const int b = c_of[2 * (o - o0)]; for (int a = 0; a < iw; ++a) { jf[nf] = Jr[a] * scaleF[ci + a]; lf[nf++] = base[b] + a; } }
                    if (cc >= 0) { const int b = c_of[2 * (o - o0) + 1]; for (int a = 0; a < 6; ++a) { jf[nf] = Jr[kJE + a] * scaleF[cc + a]; lf[nf++] = base[b] + a; } }
                    for (int a = 0; a < 3; ++a) { bE[a] += jx[a] * fr; for (int c = 0; c < 3; ++c) V[3 * a + c] += jx[a] * jx[c]; }
                    for (int u = 0; u < nf; ++u) {
                        bF[lf[u]] += jf[u] * fr;
                        for (int a = 0; a < 3; ++a) Wl[3 * lf[u] + a] += jf[u] * jx[a];
                        for (int v = 0; v < nf; ++v) Ul[lf[u] * nl + lf[v]] += jf[u] * jf[v];
                    }
                }
            }
            for (int a = 0; a < 3; ++a) V[4 * a] += lmE[3 * k + a] * lmE[3 * k + a];
            double Vi[9];
            if (!inv3_spd(V, Vi)) { fail[tid] = 1; continue; }
            // Y = W Vi ; S_loc = U - Y W' ; r_loc = bF - Y bE
            std::vector<double> Y(3 * nl);
            for (int u = 0; u < nl; ++u)
                for (int a = 0; a < 3; ++a) {
                    double acc = 0; for (int c = 0; c < 3; ++c) acc += Wl[3 * u + c] * Vi[3 * c + a];
                    Y[3 * u + a] = acc;
                }
            for (int u = 0; u < nl; ++u) {
                double acc = bF[u];
                for (int a = 0; a < 3; ++a) acc -= Y[3 * u + a] * bE[a];
                rl[gcol[u]] += acc;
                for (int v = 0; v < nl; ++v) {
                    if (gcol[u] < gcol[v]) continue;
                    double s2 = Ul[u * nl + v];
                    for (int a = 0; a < 3; ++a) s2 -= Y[3 * u + a] * Wl[3 * v + a];
                    Sl.at(gcol[u], gcol[v]) += s2;
                }
            }
        }
        double fl = 0.0;
        for (int t = 0; t < nthreads; ++t) fl = std::max(fl, (double)fail[t]);
        allreduce(&fl, 1, 1);
        if (fl != 0.0) return false;
        for (int t = 0; t < nthreads; ++t) {
            S.add(St[t]);
            for (int64_t c = 0; c < nF; ++c) rhs[c] += rt[t][c];
        }
        if (ar) {
            std::vector<double> buf(S.size() + nF);
            S.pack(buf.data());
            std::copy(rhs.begin(), rhs.end(), buf.begin() + S.size());
            allreduce(buf.data(), (int64_t)buf.size(), 0);
            S.unpack(buf.data());
            std::copy(buf.begin() + S.size(), buf.end(), rhs.begin());
        }
        for (int64_t c = 0; c < nF; ++c) S.at(c, c) += lmF[c] * lmF[c];
        if (!S.cholesky()) return false;
        yF = rhs;
        S.solve(yF);
        // back substitution: yE = Vi (bE - W' yF)
        yE.assign(xE.size(), 0.0);
        for (int64_t k = 0; k < npt; ++k) {
            const int64_t p = pts[k];
            double V[9] = {0}, b[3] = {0};
            for (int64_t o = P.pt_offsets[p], s = obs_ptr[k]; o < P.pt_offsets[p + 1]; ++o, ++s) {
                const int img = P.obs_img[o];
                const int64_t ci = colF_intr(img), cc = colF_cam(img);
                for (int row = 0; row < 2; ++row) {
                    const double* Jr = &J[2 * kJR * s + kJR * row];
                    double jx[3];
                    for (int a = 0; a < 3; ++a) jx[a] = Jr[kJX + a] * scaleE[3 * k + a];
                    double q = 0;  // (J_F y_F) for this row
                    for (int a = 0; a < iw; ++a) q += Jr[a] * scaleF[ci + a] * yF[ci + a];
                    if (cc >= 0) for (int a = 0; a < 6; ++a) q += Jr[kJE + a] * scaleF[cc + a] * yF[cc + a];
                    const double fr = f[2 * s + row];
                    for (int a = 0; a < 3; ++a) {
                        b[a] += jx[a] * fr - jx[a] * q;
                        for (int c = 0; c < 3; ++c) V[3 * a + c] += jx[a] * jx[c];
                    }
                }
            }
            for (int a = 0; a < 3; ++a) V[4 * a] += lmE[3 * k + a] * lmE[3 * k + a];
            double Vi[9];
            if (!inv3_spd(V, Vi)) return false;
            for (int a = 0; a < 3; ++a) yE[3 * k + a] = Vi[3 * a] * b[0] + Vi[3 * a + 1] * b[1] + Vi[3 * a + 2] * b[2];
        }
        return true;
    }

    // model_cost_change = -(J_s step)' (f + J_s step / 2)
    double model_cost_change(const std::vector<double>& sF, const std::vector<double>& sE) {
        double acc = 0.0;
        for (size_t k = 0; k < pts.size(); ++k) {
            const int64_t p = pts[k];
            for (int64_t o = P.pt_offsets[p], s = obs_ptr[k]; o < P.pt_offsets[p + 1]; ++o, ++s) {
                const int img = P.obs_img[o];
                const int64_t ci = colF_intr(img), cc = colF_cam(img);
                for (int row = 0; row < 2; ++row) {
                    const double* Jr = &J[2 * kJR * s + kJR * row];
                    double m = 0;
                    for (int a = 0; a < iw; ++a) m += Jr[a] * scaleF[ci + a] * sF[ci + a];
                    if (cc >= 0) for (int a = 0; a < 6; ++a) m += Jr[kJE + a] * scaleF[cc + a] * sF[cc + a];
                    for (int a = 0; a < 3; ++a) m += Jr[kJX + a] * scaleE[3 * k + a] * sE[3 * k + a];
                    acc += m * (f[2 * s + row] + m / 2.0);
                }
            }
        }
        allreduce(&acc, 1, 0);
        return -acc;
    }
};

}  // namespace

extern "C" int orc_ba_jacobian(int32_t mode, const double* intr, const double* extr, const double* X,
                               const double* uv, double* r, double* J) {
    return orc_ba_jacobian_model(SFM_CAM_PINHOLE, mode, intr, extr, X, uv, r, J);
}

extern "C" int orc_ba_jacobian_model(int32_t model, int32_t mode, const double* intr, const double* extr,
                                     const double* X, const double* uv, double* r, double* J) {
    if (model != SFM_CAM_PINHOLE && model != SFM_CAM_SNAVELY && model != SFM_CAM_RADIAL3) return SFM_ERR_INVALID_ARG;
    // public layout: 2 x (iw + 6 + 3), intrinsics | extr | X
    const int iw = intr_width(model), w = iw + 9;
    double Jf[2 * kJR];
    bool ok;
    if (mode == 0) {
        ok = residual_jacobian(model, intr, extr, X, uv, r, Jf);
    } else {
        Jet in[6], ex[6], pt[3], res[2];
        for (int a = 0; a < iw; ++a) in[a] = Jet(intr[a], a);
        for (int a = 0; a < 6; ++a) ex[a] = Jet(extr[a], kJE + a);
        for (int a = 0; a < 3; ++a) pt[a] = Jet(X[a], kJX + a);
        residual_jet(model, in, ex, pt, uv, res);
        for (int row = 0; row < 2; ++row) {
            r[row] = res[row].a;
            for (int k = 0; k < kJR; ++k) Jf[kJR * row + k] = res[row].v[k];
        }
        ok = std::isfinite(r[0]) && std::isfinite(r[1]);
    }
    for (int row = 0; row < 2; ++row) {
        for (int k = 0; k < iw; ++k) J[w * row + k] = Jf[kJR * row + k];
        for (int k = 0; k < 9; ++k) J[w * row + iw + k] = Jf[kJR * row + kJE + k];
    }
    return ok ? SFM_OK : SFM_ERR_NOT_FINITE;
}

extern "C" int orc_ba_cost(const sfm_ba_problem* P, const double* extr, const double* intr,
                           const double* X, double* cost, double* residuals) {
    if (!P || !cost) return SFM_ERR_INVALID_ARG;
    double c = 0.0;
    for (int64_t p = 0; p < P->n_pt; ++p)
        for (int64_t o = P->pt_offsets[p]; o < P->pt_offsets[p + 1]; ++o) {
            const int img = P->obs_img[o];
            double r[2];
            residual_jacobian(P->camera_model, &intr[intr_width(P->camera_model) * (size_t)P->img_intr[img]], &extr[6 * (size_t)img], &X[3 * p],
                              &P->obs_uv[2 * o], r, nullptr);
            double rho[2];
            huber(P->huber_a, r[0] * r[0] + r[1] * r[1], rho);
            c += 0.5 * rho[0];
            if (residuals) { residuals[2 * o] = r[0]; residuals[2 * o + 1] = r[1]; }
        }
    *cost = c;
    return SFM_OK;
}

extern "C" int orc_ba_solve(const sfm_ba_problem* P, double* extr, double* intr, double* X,
                            const sfm_ba_options* opts, sfm_ba_summary* sum, sfm_ba_iter* trace,
                            int32_t trace_cap, int32_t* trace_n, const int64_t* shard_pts,
                            int64_t n_shard_pts, orc_allreduce_fn allreduce, void* user,
                            int32_t n_threads) {
    if (!P || !extr || !intr || !X || !sum || P->n_img < 0 || P->n_pt < 0) return SFM_ERR_INVALID_ARG;
    if (P->camera_model != SFM_CAM_PINHOLE && P->camera_model != SFM_CAM_SNAVELY && P->camera_model != SFM_CAM_RADIAL3)
        return SFM_ERR_INVALID_ARG;
    sfm_ba_options O;
    if (opts) {
        O = *opts;
    } else {  // Ceres 2.2 defaults (BundleAdjuster.h:167-174 overrides none of these)
        std::memset(&O, 0, sizeof O);
        O.max_num_iterations = 50; O.max_num_consecutive_invalid_steps = 5; O.jacobi_scaling = 1;
        O.function_tolerance = 1e-6; O.gradient_tolerance = 1e-10; O.parameter_tolerance = 1e-8;
        O.initial_trust_region_radius = 1e4; O.max_trust_region_radius = 1e16;
        O.min_trust_region_radius = 1e-32; O.min_relative_decrease = 1e-3;
        O.min_lm_diagonal = 1e-6; O.max_lm_diagonal = 1e32;
    }
    const auto t0 = std::chrono::steady_clock::now();
    Oracle S(*P, O, allreduce, user, n_threads);
    S.setup(extr, intr, X, shard_pts, n_shard_pts);
    std::memset(sum, 0, sizeof *sum);
    sum->num_residuals = 2 * P->n_obs;
    std::vector<sfm_ba_iter> iters;
    auto finish = [&](int term) {
        sum->termination = term;
        sum->usable = term != SFM_TERM_FAILURE;
        sum->iterations = iters.empty() ? 0 : iters.back().iteration;
        sum->final_cost = sum->initial_cost;
        for (const auto& it : iters) if (it.step_is_successful) sum->final_cost = std::min(sum->final_cost, it.cost);
        sum->rmse_initial = sum->num_residuals ? std::sqrt(sum->initial_cost / sum->num_residuals) : 0.0;
        sum->rmse_final = sum->num_residuals ? std::sqrt(sum->final_cost / sum->num_residuals) : 0.0;
        sum->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (trace_n) *trace_n = (int32_t)std::min<size_t>(iters.size(), trace_cap > 0 ? trace_cap : 0);
        for (size_t k = 0; trace && k < iters.size() && (int32_t)k < trace_cap; ++k) trace[k] = iters[k];
        if (sum->usable) {  // BundleAdjuster::updateWorld only on a usable solution
            for (int i = 0; i < P->n_img; ++i) if (S.cam_blk[i] >= 0) for (int a = 0; a < 6; ++a) extr[6 * i + a] = S.xF[6 * S.cam_blk[i] + a];
            for (int q = 0; q < P->n_intr; ++q)
                if (S.intr_blk[q] >= 0)
                    for (int a = 0; a < (P->camera_model == SFM_CAM_SNAVELY ? 3 : S.iw); ++a)
                        intr[S.iw * q + a] = S.xF[S.nb + S.iw * S.intr_blk[q] + a];
            for (size_t k = 0; k < S.pts.size(); ++k) for (int a = 0; a < 3; ++a) X[3 * S.pts[k] + a] = S.xE[3 * k + a];
        }
        return term == SFM_TERM_FAILURE ? SFM_ERR_SOLVER : SFM_OK;
    };

    // ---- iteration zero -------------------------------------------------
    double x_norm = std::sqrt(S.sqnorm_x(S.xF, S.xE));
    if (!S.evaluate(S.xF, S.xE, &S.x_cost, true)) { finish(SFM_TERM_FAILURE); return SFM_ERR_NOT_FINITE; }
    if (O.jacobi_scaling) {
        std::vector<double> cF, cE;
        S.colnorms(false, cF, cE);
        for (int64_t c = 0; c < S.nF; ++c) S.scaleF[c] = 1.0 / (1.0 + std::sqrt(cF[c]));
        for (size_t c = 0; c < cE.size(); ++c) S.scaleE[c] = 1.0 / (1.0 + std::sqrt(cE[c]));
    }
    sum->initial_cost = S.x_cost;
    sfm_ba_iter it{};
    it.iteration = 0; it.step_is_valid = 1; it.step_is_successful = 1;
    it.cost = S.x_cost;
    it.gradient_max_norm = S.gradient_max_norm();
    double radius = O.initial_trust_region_radius, decrease_factor = 2.0;
    bool reuse_diag = false;
    it.trust_region_radius = radius;
    int consecutive_invalid = 0;
    std::vector<double> diagF, diagE, lmF, lmE, yF, yE, cF(S.nF), cE(S.xE.size());
    double model_change = 0.0;

    auto finalize = [&](const sfm_ba_iter& cur) -> int {  // -1: continue
        iters.push_back(cur);
        if (cur.step_is_successful) sum->successful_steps++; else sum->unsuccessful_steps++;
        if (cur.iteration >= O.max_num_iterations) return SFM_TERM_NO_CONVERGENCE;
        if (cur.gradient_max_norm <= O.gradient_tolerance) return SFM_TERM_CONVERGENCE;
        if (radius < O.min_trust_region_radius) return SFM_TERM_CONVERGENCE;
        return -1;
    };
    int term = finalize(it);
    while (term < 0) {
        const sfm_ba_iter prev = iters.back();
        sfm_ba_iter cur{};
        cur.iteration = prev.iteration + 1;
        // ---- ComputeTrustRegionStep (LevenbergMarquardtStrategy) ---------
        if (!reuse_diag) {
            S.colnorms(true, diagF, diagE);
            for (double& v : diagF) v = std::min(std::max(v, O.min_lm_diagonal), O.max_lm_diagonal);
            for (double& v : diagE) v = std::min(std::max(v, O.min_lm_diagonal), O.max_lm_diagonal);
        }
        lmF.resize(S.nF); lmE.resize(diagE.size());
        for (int64_t c = 0; c < S.nF; ++c) lmF[c] = std::sqrt(diagF[c] / radius);
        for (size_t c = 0; c < diagE.size(); ++c) lmE[c] = std::sqrt(diagE[c] / radius);
        bool solved = S.schur_solve(lmF, lmE, yF, yE);
        reuse_diag = true;
        bool finite = solved;
        if (solved) {
            double fl = 0.0;
            for (double v : yF) if (!std::isfinite(v)) fl = 1.0;
            for (double v : yE) if (!std::isfinite(v)) fl = 1.0;
            S.allreduce(&fl, 1, 1);
            finite = fl == 0.0;
        }
        cur.step_is_valid = 0;
        std::vector<double> sF(S.nF), sE(S.xE.size());
        if (finite) {
            for (int64_t c = 0; c < S.nF; ++c) sF[c] = -yF[c];
            for (size_t c = 0; c < sE.size(); ++c) sE[c] = -yE[c];
            model_change = S.model_cost_change(sF, sE);
            cur.model_cost_change = model_change;
            cur.step_is_valid = model_change > 0.0;
        }
        if (!cur.step_is_valid) {
            // HandleInvalidStep
            if (++consecutive_invalid >= O.max_num_consecutive_invalid_steps) { term = SFM_TERM_FAILURE; break; }
            radius = radius / decrease_factor; decrease_factor *= 2.0; reuse_diag = true;  // StepRejected(0)
            cur.cost = S.x_cost;
            cur.gradient_max_norm = prev.gradient_max_norm;
            cur.trust_region_radius = radius;
            term = finalize(cur);
            continue;
        }
        consecutive_invalid = 0;
        // candidate point
        std::vector<double> cxF(S.nF), cxE(S.xE.size());
        for (int64_t c = 0; c < S.nF; ++c) cxF[c] = S.xF[c] + sF[c] * S.scaleF[c];
        for (size_t c = 0; c < cxE.size(); ++c) cxE[c] = S.xE[c] + sE[c] * S.scaleE[c];
        double cand_cost;
        if (!S.evaluate(cxF, cxE, &cand_cost, false)) cand_cost = std::numeric_limits<double>::max();
        // ParameterToleranceReached
        double sn2F = 0.0, sn2E = 0.0;
        for (int64_t c = 0; c < S.nF; ++c) { const double d = S.xF[c] - cxF[c]; sn2F += d * d; }
        for (size_t c = 0; c < cxE.size(); ++c) { const double d = S.xE[c] - cxE[c]; sn2E += d * d; }
        S.allreduce(&sn2E, 1, 0);
        cur.step_norm = std::sqrt(sn2F + sn2E);
        if (cur.step_norm <= O.parameter_tolerance * (x_norm + O.parameter_tolerance)) { term = SFM_TERM_CONVERGENCE; break; }
        // FunctionToleranceReached
        cur.cost_change = S.x_cost - cand_cost;
        if (std::fabs(cur.cost_change) <= O.function_tolerance * S.x_cost) { term = SFM_TERM_CONVERGENCE; break; }
        // IsStepSuccessful (monotonic TrustRegionStepEvaluator)
        cur.relative_decrease = cand_cost >= std::numeric_limits<double>::max()
                                    ? std::numeric_limits<double>::lowest()
                                    : (S.x_cost - cand_cost) / model_change;
        if (cur.relative_decrease > O.min_relative_decrease) {
            S.xF = cxF; S.xE = cxE;
            x_norm = std::sqrt(S.sqnorm_x(S.xF, S.xE));
            if (!S.evaluate(S.xF, S.xE, &S.x_cost, true)) { term = SFM_TERM_FAILURE; break; }
            cur.step_is_successful = 1;
            cur.cost = S.x_cost;
            cur.gradient_max_norm = S.gradient_max_norm();
            const double q = cur.relative_decrease;
            radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * q - 1.0, 3));
            radius = std::min(O.max_trust_region_radius, radius);
            decrease_factor = 2.0; reuse_diag = false;
        } else {
            cur.step_is_successful = 0;
            cur.cost = cand_cost;
            cur.gradient_max_norm = prev.gradient_max_norm;
            radius = radius / decrease_factor; decrease_factor *= 2.0; reuse_diag = true;
        }
        cur.trust_region_radius = radius;
        term = finalize(cur);
    }
    return finish(term);
}
