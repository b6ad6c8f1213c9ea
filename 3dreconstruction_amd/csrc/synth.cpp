// Deterministic synthetic inputs: BA scenes and RootSIFT-like
// descriptor collections.  Pure host code, counter-based RNG (SplitMix64
// finaliser per entity + Box-Muller), so every entity's draws are independent
// of generation order and identical on every host with the same libm.
//
// Reference defaults used here: fx=fy=2905.88 (src/main.cpp:124, :59 K),
// cx=1416, cy=1064 (src/main.cpp:59); RootSIFT uchar conversion
// 512*sqrt(d/sum d) (src/nonFree/sift/SIFT_describer.hpp:31-45).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>

#include "../../include/sfmcore.h"
#include "synth_rng.h"

namespace {

using sfm::synth::Rng;
using sfm::synth::entity_seed;

void mat_to_angle_axis(const double R[9], double w[3]) {
    // rotation matrix -> quaternion (Shepperd) -> angle-axis
    const double tr = R[0] + R[4] + R[8];
    double q[4];  // w, x, y, z
    if (tr >= 0) {
        double t = std::sqrt(tr + 1.0);
        q[0] = 0.5 * t; t = 0.5 / t;
        q[1] = (R[7] - R[5]) * t; q[2] = (R[2] - R[6]) * t; q[3] = (R[3] - R[1]) * t;
    } else {
        int i = 0;
        if (R[4] > R[0]) i = 1;
        if (R[8] > R[i * 4]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double t = std::sqrt(R[i * 4] - R[j * 4] - R[k * 4] + 1.0);
        q[i + 1] = 0.5 * t; t = 0.5 / t;
        q[0] = (R[k * 3 + j] - R[j * 3 + k]) * t;
        q[j + 1] = (R[j * 3 + i] + R[i * 3 + j]) * t;
        q[k + 1] = (R[k * 3 + i] + R[i * 3 + k]) * t;
    }
    if (q[0] < 0) for (double& v : q) v = -v;
    const double sn = std::sqrt(q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (sn < 1e-300) { w[0] = 2 * q[1]; w[1] = 2 * q[2]; w[2] = 2 * q[3]; return; }
    const double theta = 2.0 * std::atan2(sn, q[0]);
    for (int a = 0; a < 3; ++a) w[a] = q[a + 1] * theta / sn;
}

void rotate(const double w[3], const double X[3], double out[3]) {
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    if (th2 > 2.220446049250313e-16) {
        const double th = std::sqrt(th2), c = std::cos(th), s = std::sin(th);
        const double u[3] = {w[0] / th, w[1] / th, w[2] / th};
        const double cr[3] = {u[1] * X[2] - u[2] * X[1], u[2] * X[0] - u[0] * X[2],
                              u[0] * X[1] - u[1] * X[0]};
        const double tmp = (u[0] * X[0] + u[1] * X[1] + u[2] * X[2]) * (1.0 - c);
        for (int a = 0; a < 3; ++a) out[a] = X[a] * c + cr[a] * s + u[a] * tmp;
    } else {
        const double cr[3] = {w[1] * X[2] - w[2] * X[1], w[2] * X[0] - w[0] * X[2],
                              w[0] * X[1] - w[1] * X[0]};
        for (int a = 0; a < 3; ++a) out[a] = X[a] + cr[a];
    }
}

void project(int model, const double* intr, const double* extr, const double* X, double uv[2]) {
    double P[3];
    rotate(extr, X, P);
    P[0] += extr[3]; P[1] += extr[4]; P[2] += extr[5];
    if (model == SFM_CAM_SNAVELY) {   // SnavelyReprojectionError.h:27-47
        const double xp = -P[0] / P[2], yp = -P[1] / P[2];
        const double r2 = xp * xp + yp * yp;
        const double d = 1.0 + r2 * (intr[1] + intr[2] * r2);
        uv[0] = intr[0] * d * xp;
        uv[1] = intr[0] * d * yp;
        return;
    }
    if (model == SFM_CAM_RADIAL3) {   // OpenMVG Pinhole_Intrinsic_Radial_K3 (f, ppx, ppy, k1, k2, k3)
        const double x = P[0] / P[2], y = P[1] / P[2];
        const double r2 = x * x + y * y;
        const double c = 1.0 + intr[3] * r2 + intr[4] * r2 * r2 + intr[5] * r2 * r2 * r2;
        uv[0] = intr[1] + intr[0] * (x * c);
        uv[1] = intr[2] + intr[0] * (y * c);
        return;
    }
    uv[0] = intr[0] * (P[0] / P[2]) + intr[2];
    uv[1] = intr[1] * (P[1] / P[2]) + intr[3];
}

// doubles per intrinsics block (as sfm_ba_intr_width; this file also builds
// into the oracle library, which has no planner)
int synth_intr_width(int model) {
    return model == SFM_CAM_RADIAL3 ? 6 : (model == SFM_CAM_PINHOLE || model == SFM_CAM_SNAVELY) ? 4 : 0;
}

enum : uint64_t { kStreamCam = 1, kStreamPt = 2, kStreamIntr = 3, kStreamLm = 4,
                  kStreamUniq = 5, kStreamFrame = 6 };

}  // namespace

extern "C" int sfm_synth_ba(const sfm_synth_ba_config* cfg, int64_t* pt_offsets,
                            int32_t* obs_img, double* obs_uv, int32_t* img_intr,
                            double* extr, double* intr, double* X, double* gt_extr,
                            double* gt_intr, double* gt_X, int64_t* n_obs_out) {
    if (!cfg || cfg->n_cam < 1 || cfg->n_pt < 0 || cfg->k < 1 || cfg->k > cfg->n_cam ||
        cfg->n_intr < 1 || cfg->n_intr > cfg->n_cam || synth_intr_width(cfg->camera_model) == 0)
        return SFM_ERR_INVALID_ARG;
    const int model = cfg->camera_model, iw = synth_intr_width(model);
    const int64_t n_obs = cfg->n_pt * cfg->k;
    if (n_obs_out) *n_obs_out = n_obs;
    if (!pt_offsets) return SFM_OK;  // size query

    const int nc = cfg->n_cam, k = cfg->k;
    const uint64_t seed = cfg->seed;
    std::vector<double> ge(6 * (size_t)nc), gi((size_t)iw * cfg->n_intr);
    for (int q = 0; q < cfg->n_intr; ++q) {
        Rng r(entity_seed(seed, kStreamIntr, q));
        const double df = q == 0 ? 0.0 : 40.0 * (r.uni() - 0.5);
        if (model == SFM_CAM_SNAVELY) {   // BAL-like: f, l1, l2 (principal point at 0)
            gi[4 * q + 0] = 1000.0 + df; gi[4 * q + 1] = -0.08;
            gi[4 * q + 2] = 0.02;         gi[4 * q + 3] = 0.0;
            continue;
        }
        if (model == SFM_CAM_RADIAL3) {
            double* g = &gi[6 * (size_t)q];
            g[0] = 2905.88 + df; g[1] = 1416.0; g[2] = 1064.0;
            g[3] = -0.05;        g[4] = 0.01;   g[5] = -0.002;
            continue;
        }
        gi[4 * q + 0] = 2905.88 + df; gi[4 * q + 1] = 2905.88 + df;
        gi[4 * q + 2] = 1416.0;       gi[4 * q + 3] = 1064.0;
    }
    for (int c = 0; c < nc; ++c) {
        Rng r(entity_seed(seed, kStreamCam, c));
        const double phi = 2.0 * M_PI * c / nc;
        const double C[3] = {10.0 * std::cos(phi), 1.0 * std::sin(3.0 * phi), 10.0 * std::sin(phi)};
        const double tgt[3] = {0.1 * r.gauss(), 0.1 * r.gauss(), 0.1 * r.gauss()};
        double z[3] = {tgt[0] - C[0], tgt[1] - C[1], tgt[2] - C[2]};
        double zn = std::sqrt(z[0] * z[0] + z[1] * z[1] + z[2] * z[2]);
        for (double& v : z) v /= zn;
        const double up[3] = {0.0, 1.0, 0.0};
        double x[3] = {z[1] * up[2] - z[2] * up[1], z[2] * up[0] - z[0] * up[2],
                       z[0] * up[1] - z[1] * up[0]};
        double xn = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
        for (double& v : x) v /= xn;
        const double y[3] = {z[1] * x[2] - z[2] * x[1], z[2] * x[0] - z[0] * x[2],
                             z[0] * x[1] - z[1] * x[0]};
        const double R[9] = {x[0], x[1], x[2], y[0], y[1], y[2], z[0], z[1], z[2]};
        double* e = &ge[6 * (size_t)c];
        mat_to_angle_axis(R, e);
        for (int a = 0; a < 3; ++a)
            e[3 + a] = -(R[3 * a + 0] * C[0] + R[3 * a + 1] * C[1] + R[3 * a + 2] * C[2]);
    }
    for (int c = 0; c < nc; ++c) img_intr[c] = c % cfg->n_intr;

    // points, visibility, observations
    pt_offsets[0] = 0;
    std::vector<int> cams(k);
    for (int64_t p = 0; p < cfg->n_pt; ++p) {
        Rng r(entity_seed(seed, kStreamPt, (uint64_t)p));
        double Xg[3] = {4.0 * r.uni() - 2.0, 4.0 * r.uni() - 2.0, 4.0 * r.uni() - 2.0};
        if (cfg->vis_mode == 0) {
            const int64_t c0 = cfg->n_pt > 0 ? (p * (int64_t)(nc - k + 1)) / cfg->n_pt : 0;
            for (int a = 0; a < k; ++a) cams[a] = (int)c0 + a;
        } else if (cfg->vis_mode == 2) {
            // closed orbit: k consecutive cameras modulo n_cam (the last
            // images see the first images' points)
            const int64_t c0 = cfg->n_pt > 0 ? (p * (int64_t)nc) / cfg->n_pt : 0;
            for (int a = 0; a < k; ++a) cams[a] = (int)((c0 + a) % nc);
            std::sort(cams.begin(), cams.end());
        } else {
            int got = 0;
            while (got < k) {
                int c = (int)(r.next() % (uint64_t)nc);
                bool dup = false;
                for (int a = 0; a < got; ++a) dup |= cams[a] == c;
                if (!dup) cams[got++] = c;
            }
            std::sort(cams.begin(), cams.end());
        }
        const int64_t o0 = p * k;
        for (int a = 0; a < k; ++a) {
            const int c = cams[a];
            double uv[2];
            project(model, &gi[(size_t)iw * img_intr[c]], &ge[6 * (size_t)c], Xg, uv);
            uv[0] += cfg->noise_px * r.gauss();
            uv[1] += cfg->noise_px * r.gauss();
            if (r.uni() < cfg->outlier_frac) {
                for (int d = 0; d < 2; ++d) {
                    const double mag = 20.0 + 40.0 * r.uni();
                    uv[d] += (r.uni() < 0.5 ? -mag : mag);
                }
            }
            obs_img[o0 + a] = c;
            obs_uv[2 * (o0 + a)] = uv[0];
            obs_uv[2 * (o0 + a) + 1] = uv[1];
        }
        pt_offsets[p + 1] = o0 + k;
        for (int a = 0; a < 3; ++a) {
            if (gt_X) gt_X[3 * p + a] = Xg[a];
            X[3 * p + a] = Xg[a] + cfg->perturb_X * r.gauss();
        }
    }
    for (int c = 0; c < nc; ++c) {
        Rng r(entity_seed(seed ^ 0xA5A5ULL, kStreamCam, c));
        for (int a = 0; a < 6; ++a) {
            const double g = ge[6 * (size_t)c + a];
            if (gt_extr) gt_extr[6 * (size_t)c + a] = g;
            const double s = a < 3 ? cfg->perturb_rot : cfg->perturb_t;
            extr[6 * (size_t)c + a] = (c == cfg->const_img) ? g : g + s * r.gauss();
        }
    }
    for (int q = 0; q < cfg->n_intr; ++q) {
        Rng r(entity_seed(seed ^ 0xA5A5ULL, kStreamIntr, q));
        for (int a = 0; a < iw; ++a) {
            const double g = gi[(size_t)iw * q + a];
            if (gt_intr) gt_intr[(size_t)iw * q + a] = g;
            if (model == SFM_CAM_RADIAL3)   // f by perturb_f, k1..k3 by a small relative amount
                intr[6 * (size_t)q + a] = a == 0 ? g + cfg->perturb_f * r.gauss()
                                        : a >= 3 ? g * (1.0 + 0.02 * r.gauss())
                                                 : g;
            else if (model == SFM_CAM_SNAVELY)   // f by perturb_f, l1 / l2 by a proportional small amount
                intr[4 * (size_t)q + a] = a == 0 ? g + cfg->perturb_f * r.gauss()
                                        : a < 3  ? g + 2e-3 * cfg->perturb_f / 5.0 * r.gauss() / (a == 1 ? 1.0 : 4.0)
                                                 : g;
            else
                intr[4 * (size_t)q + a] = a < 2 ? g + cfg->perturb_f * r.gauss() : g;
        }
    }
    return SFM_OK;
}

namespace {
// RootSIFT-like 128-D uchar descriptor: exponential bin masses with ~11%
// empty bins, then 512*sqrt(x/sum x) truncated to uchar (SIFT_describer.hpp:38-40).
void rootsift_like(Rng& r, uint8_t* out) {
    float x[128];
    float sum = 0.f;
    for (int d = 0; d < 128; ++d) {
        const double u = r.uni();
        x[d] = u < 0.11 ? 0.f : (float)(-std::log(1.0 - r.uni()) * (0.2 + u));
        sum += x[d];
    }
    if (sum <= 0.f) sum = 1.f;
    for (int d = 0; d < 128; ++d) {
        float v = 512.f * std::sqrt(x[d] / sum);
        out[d] = (uint8_t)std::min(255.f, v);
    }
}
}  // namespace

extern "C" int sfm_synth_descriptors(int32_t n_img, int32_t n_kp, uint64_t seed, uint8_t* desc) {
    if (n_img < 0 || n_kp < 0 || (!desc && n_img * (int64_t)n_kp > 0)) return SFM_ERR_INVALID_ARG;
    const int64_t step = std::max<int64_t>(1, n_kp / 4);   // landmark window advance per frame
    const int64_t win = std::max<int64_t>(1, 4 * (int64_t)n_kp);
    for (int32_t f = 0; f < n_img; ++f) {
        Rng fr(entity_seed(seed, kStreamFrame, (uint64_t)f));
        for (int32_t s = 0; s < n_kp; ++s) {
            uint8_t* out = desc + ((int64_t)f * n_kp + s) * 128;
            if (fr.uni() < 0.5) {
                const uint64_t lm = (uint64_t)(f * step) + (fr.next() % (uint64_t)win);
                Rng lr(entity_seed(seed, kStreamLm, lm));
                rootsift_like(lr, out);
                for (int d = 0; d < 128; ++d) {
                    if (fr.uni() < 0.3) {
                        int v = (int)out[d] + (int)(fr.next() % 7) - 3;
                        out[d] = (uint8_t)std::min(255, std::max(0, v));
                    }
                }
            } else {
                Rng ur(entity_seed(seed, kStreamUniq, ((uint64_t)f << 32) | (uint32_t)s));
                rootsift_like(ur, out);
            }
        }
    }
    return SFM_OK;
}

extern "C" int sfm_exhaustive_pairs(int32_t n_img, int32_t* pairs) {
    if (n_img < 0 || (!pairs && n_img > 1)) return SFM_ERR_INVALID_ARG;
    int64_t q = 0;
    for (int32_t i = 0; i < n_img; ++i)
        for (int32_t j = i + 1; j < n_img; ++j) { pairs[2 * q] = i; pairs[2 * q + 1] = j; ++q; }
    return SFM_OK;
}

// ---------------------------------------------------------------------------
// C5: closed-orbit image sequence for the SequentialActuator loop
// (src/main.cpp:99-108).  See include/sfmcore.h sfm_synth_orbit_image.
// ---------------------------------------------------------------------------
namespace {

enum : uint64_t { kStreamOrbLm = 11, kStreamOrbDesc = 12, kStreamOrbObs = 13, kStreamOrbClutter = 14,
                  kStreamOrbPrior = 15 };

// ground-truth Tcw of orbit camera c: centre on the circle of radius 10 in
// the XZ plane, looking at the origin, image y axis along world y
void orbit_pose(int c, int n, double R[9], double t[3]) {
    const double phi = 2.0 * M_PI * c / n;
    const double C[3] = {10.0 * std::cos(phi), 0.0, 10.0 * std::sin(phi)};
    const double z[3] = {-C[0] / 10.0, 0.0, -C[2] / 10.0};
    const double up[3] = {0.0, 1.0, 0.0};
    double x[3] = {z[1] * up[2] - z[2] * up[1], z[2] * up[0] - z[0] * up[2], z[0] * up[1] - z[1] * up[0]};
    const double xn = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
    for (double& v : x) v /= xn;
    const double y[3] = {z[1] * x[2] - z[2] * x[1], z[2] * x[0] - z[0] * x[2], z[0] * x[1] - z[1] * x[0]};
    const double Rm[9] = {x[0], x[1], x[2], y[0], y[1], y[2], z[0], z[1], z[2]};
    for (int a = 0; a < 9; ++a) R[a] = Rm[a];
    for (int a = 0; a < 3; ++a) t[a] = -(R[3 * a] * C[0] + R[3 * a + 1] * C[1] + R[3 * a + 2] * C[2]);
}

struct OrbitLandmark {
    double X[3];     // ground truth, orbit frame
    double psi, h;   // facing direction, half-arc of the cameras that see it
};

OrbitLandmark orbit_landmark(const sfm_synth_orbit_config* cfg, int64_t l) {
    Rng r(entity_seed(cfg->seed, kStreamOrbLm, (uint64_t)l));
    OrbitLandmark L;
    for (double& v : L.X) v = 4.0 * r.uni() - 2.0;
    L.psi = 2.0 * M_PI * r.uni();
    const double dphi = 2.0 * M_PI / cfg->n_img;
    L.h = dphi * std::max(0.0, cfg->track_mean - 1.0) * 0.5 * (0.5 + r.uni());
    return L;
}

}  // namespace

extern "C" int sfm_synth_orbit_image(const sfm_synth_orbit_config* cfg, int32_t img, int32_t* n_kp,
                                     double* kp_xy, uint8_t* desc, double* pose_prior, int64_t* landmark,
                                     double* gt_X) {
    if (!cfg || !n_kp || cfg->n_img < 2 || img < 0 || img >= cfg->n_img || cfg->n_landmarks < 0 ||
        cfg->n_clutter < 0 || cfg->desc_noise_dims < 0 || cfg->desc_noise_amp < 0)
        return SFM_ERR_INVALID_ARG;
    const double fx = 2905.88, fy = 2905.88, cx = 1416.0, cy = 1064.0;   // src/main.cpp:59,124
    const int n = cfg->n_img;
    double R0[9], t0[3], Rc[9], tc[3];
    orbit_pose(0, n, R0, t0);
    orbit_pose(img, n, Rc, tc);
    const double phi = 2.0 * M_PI * img / n;
    // items: (shuffle key, landmark id or -1 - clutter slot)
    std::vector<std::pair<uint64_t, int64_t>> items;
    for (int64_t l = 0; l < cfg->n_landmarks; ++l) {
        const OrbitLandmark L = orbit_landmark(cfg, l);
        if (std::fabs(std::remainder(phi - L.psi, 2.0 * M_PI)) > L.h) continue;
        Rng r(entity_seed(cfg->seed, kStreamOrbObs, (uint64_t)l * (uint64_t)n + (uint64_t)img));
        if (r.uni() >= cfg->detect_prob) continue;
        items.push_back({r.next(), l});
    }
    for (int32_t s = 0; s < cfg->n_clutter; ++s) {
        Rng r(entity_seed(cfg->seed, kStreamOrbClutter, ((uint64_t)img << 32) | (uint32_t)s));
        items.push_back({r.next(), -1 - (int64_t)s});
    }
    std::sort(items.begin(), items.end());
    *n_kp = (int32_t)items.size();
    if (gt_X)
        for (int64_t l = 0; l < cfg->n_landmarks; ++l) {
            const OrbitLandmark L = orbit_landmark(cfg, l);
            for (int a = 0; a < 3; ++a)
                gt_X[3 * l + a] = R0[3 * a] * L.X[0] + R0[3 * a + 1] * L.X[1] + R0[3 * a + 2] * L.X[2] + t0[a];
        }
    if (pose_prior) {
        // Tcw relative to image 0: R = Rc R0^T, t = tc - R t0
        double R[9], w[3], t[3];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c)
                R[3 * r + c] = Rc[3 * r] * R0[3 * c] + Rc[3 * r + 1] * R0[3 * c + 1] + Rc[3 * r + 2] * R0[3 * c + 2];
        for (int a = 0; a < 3; ++a) t[a] = tc[a] - (R[3 * a] * t0[0] + R[3 * a + 1] * t0[1] + R[3 * a + 2] * t0[2]);
        mat_to_angle_axis(R, w);
        if (img == 0) { w[0] = w[1] = w[2] = 0.0; t[0] = t[1] = t[2] = 0.0; }
        Rng r(entity_seed(cfg->seed, kStreamOrbPrior, (uint64_t)img));
        for (int a = 0; a < 3; ++a) {
            pose_prior[a] = w[a] + (img ? cfg->prior_rot * r.gauss() : 0.0);
            pose_prior[3 + a] = t[a] + (img ? cfg->prior_t * r.gauss() : 0.0);
        }
    }
    if (!kp_xy && !desc && !landmark) return SFM_OK;
    for (size_t k = 0; k < items.size(); ++k) {
        const int64_t id = items[k].second;
        double uv[2];
        uint8_t d[128];
        if (id >= 0) {
            const OrbitLandmark L = orbit_landmark(cfg, id);
            double P[3];
            for (int a = 0; a < 3; ++a)
                P[a] = Rc[3 * a] * L.X[0] + Rc[3 * a + 1] * L.X[1] + Rc[3 * a + 2] * L.X[2] + tc[a];
            Rng r(entity_seed(cfg->seed, kStreamOrbObs, (uint64_t)id * (uint64_t)n + (uint64_t)img));
            r.uni(); r.next();   // the draws the visibility test made
            uv[0] = fx * P[0] / P[2] + cx + cfg->noise_px * r.gauss();
            uv[1] = fy * P[1] / P[2] + cy + cfg->noise_px * r.gauss();
            Rng dr(entity_seed(cfg->seed, kStreamOrbDesc, (uint64_t)id));
            rootsift_like(dr, d);
            for (int q = 0; q < cfg->desc_noise_dims; ++q) {
                const int dim = (int)(r.next() % 128);
                const int v = (int)d[dim] + (int)(r.next() % (uint64_t)(2 * cfg->desc_noise_amp + 1)) -
                              cfg->desc_noise_amp;
                d[dim] = (uint8_t)std::min(255, std::max(0, v));
            }
        } else {
            Rng r(entity_seed(cfg->seed, kStreamOrbClutter, ((uint64_t)img << 32) | (uint32_t)(-1 - id)));
            r.next();
            uv[0] = 2832.0 * r.uni();
            uv[1] = 2128.0 * r.uni();
            rootsift_like(r, d);
        }
        if (kp_xy) { kp_xy[2 * k] = uv[0]; kp_xy[2 * k + 1] = uv[1]; }
        if (desc) std::memcpy(desc + 128 * k, d, 128);
        if (landmark) landmark[k] = id >= 0 ? id : -1;
    }
    return SFM_OK;
}
