// Device arithmetic of the LM candidate (x + delta) shared by cand_kernel
// (ba_kernels.hip) and the BCR back substitution, which forms its blocks'
// camera candidates as soon as their y is known (ba_bcr.hip): the per-camera
// precompute and the per-column step, one definition so both give the same
// bits per element.
#pragma once
#include <hip/hip_runtime.h>

#include "ba_types.h"

namespace sfm {
namespace {

constexpr double kCandEps = 2.220446049250313e-16;  // std::numeric_limits<double>::epsilon()

// Rodrigues terms of one camera (extrinsics e = [w | t])
__device__ inline CamPre make_campre(const double* e) {
    CamPre cp;
    const double w[3] = {e[0], e[1], e[2]};
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    cp.t[0] = e[3]; cp.t[1] = e[4]; cp.t[2] = e[5];
    if (th2 > kCandEps) {
        const double th = sqrt(th2), c = cos(th), s = sin(th), it = 1.0 / th, oc = 1.0 - c;
        const double u[3] = {w[0] * it, w[1] * it, w[2] * it};
        cp.c = c; cp.s = s; cp.omc = oc; cp.small = 0.0;
        for (int a = 0; a < 3; ++a) cp.u[a] = u[a];
        double* R = cp.R;
        R[0] = c + oc * u[0] * u[0];        R[1] = oc * u[0] * u[1] - s * u[2]; R[2] = oc * u[0] * u[2] + s * u[1];
        R[3] = oc * u[1] * u[0] + s * u[2]; R[4] = c + oc * u[1] * u[1];        R[5] = oc * u[1] * u[2] - s * u[0];
        R[6] = oc * u[2] * u[0] - s * u[1]; R[7] = oc * u[2] * u[1] + s * u[0]; R[8] = c + oc * u[2] * u[2];
        const double Wx[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                double acc = w[a] * w[b];
                for (int k = 0; k < 3; ++k) acc += (R[k * 3 + a] - (a == k ? 1.0 : 0.0)) * Wx[k * 3 + b];
                cp.Ar[a * 3 + b] = acc / th2;
            }
    } else {
        cp.c = 1.0; cp.s = 0.0; cp.omc = 0.0; cp.small = 1.0;
        for (int a = 0; a < 3; ++a) cp.u[a] = w[a];
        const double Rs[9] = {1, -w[2], w[1], w[2], 1, -w[0], -w[1], w[0], 1};
        for (int a = 0; a < 9; ++a) {
            cp.R[a] = Rs[a];
            cp.Ar[a] = (a % 4 == 0) ? 1.0 : 0.0;
        }
    }
    return cp;
}

// one active F column: the candidate x - y scale (Ceres' x + delta in the
// unscaled frame), with this column's terms of |x|^2, |delta|^2 and max |g|
struct CandAcc {
    double x2 = 0.0, d2 = 0.0, gm = 0.0;
};
__device__ __forceinline__ double cand_col(double x, double y, double sf, double bf, CandAcc& a) {
    const double cand = x + (-y) * sf;
    const double d = x - cand;
    a.x2 += x * x;
    a.d2 += d * d;
    const double g = bf / sf;
    a.gm = fmax(a.gm, fabs(x - (x - g)));
    return cand;
}

}  // namespace
}  // namespace sfm
