// SequentialActuator (src/actuator/SequentialActuator.h:16-236): the legacy
// incremental pipeline that calls the hot path — init(img0, img1), then
// addSingleImage(img) per image, each followed by bundleAdjustment() with a
// fresh BundleAdjuster (:226-229) — as driven by src/main.cpp:99-108
// (BASELINE.json config C5).
//
// What is the reference's and what is a stand-in:
//   * LocalFrame mutual matching + 4*min filter, GlobalFrame world-point
//     matching + 3*min filter, savePointCloudToWorld's track building
//     (:25-72), the gauge / lazy zero pose / write-back of BundleAdjuster and
//     the loop order are the reference's.
//   * The OpenCV geometry (findEssentialMat + recoverPose :110-127,
//     solvePnPRansac :177-181, findEssentialMat's inlier mask :196-198) is out
//     of scope.  Its outputs are replaced by: the pose
//     of each new image = the caller's pose prior (what the geometric solver
//     would return; the synthetic sequence supplies ground truth + noise),
//     the essential-matrix inlier mask = Sampson distance w.r.t. the
//     essential matrix of the two current poses <= epipolar_px (OpenCV's
//     RANSAC error measure and pixel threshold convention), plus recoverPose's
//     cheirality / distance test in init, and the PnP inlier count = global
//     matches reprojecting within pnp_reproj_px (solvePnPRansac's 8.0).
//   * triangulatePoints (:217-219) is linear DLT (smallest eigenvector of
//     AᵀA) on normalised coordinates, as OpenCV's, in double.
// Keypoint -> world point bookkeeping and the image / world-point order are
// deterministic (index order) where the reference iterates unordered maps.
//
// BasicSequentialActuator<Backend>: Backend supplies the matcher
// (knnMatch shape, frames.hpp) and a fresh bundle adjuster per call.  The
// product (sfm.hpp) binds the GPU; the loop oracle binds the CPU restatement.
#pragma once
#include <algorithm>
#include <array>
#include <chrono>
#include <unordered_map>
#include <cmath>
#include <cstdint>
#include <memory>
#include <vector>

#include "../../../include/sfmcore.h"
#include "adjuster.hpp"
#include "frames.hpp"
#include "world.hpp"

namespace sfm {

namespace geom {

// ceres::AngleAxisRotatePoint (both branches), as ReprojectCost uses it
inline void aa_rotate(const double w[3], const double X[3], double out[3]) {
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    if (th2 > 2.220446049250313e-16) {
        const double th = std::sqrt(th2), c = std::cos(th), s = std::sin(th);
        const double u[3] = {w[0] / th, w[1] / th, w[2] / th};
        const double cr[3] = {u[1] * X[2] - u[2] * X[1], u[2] * X[0] - u[0] * X[2], u[0] * X[1] - u[1] * X[0]};
        const double tmp = (u[0] * X[0] + u[1] * X[1] + u[2] * X[2]) * (1.0 - c);
        for (int a = 0; a < 3; ++a) out[a] = X[a] * c + cr[a] * s + u[a] * tmp;
    } else {
        const double cr[3] = {w[1] * X[2] - w[2] * X[1], w[2] * X[0] - w[0] * X[2], w[0] * X[1] - w[1] * X[0]};
        for (int a = 0; a < 3; ++a) out[a] = X[a] + cr[a];
    }
}

// Tcw as a 3x4 row-major [R | t]
inline void pose_matrix(const std::array<double, 6>& p, double P[12]) {
    double R[9];
    rot::aa_to_matrix(p.data(), R);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) P[4 * r + c] = R[3 * r + c];
        P[4 * r + 3] = p[3 + r];
    }
}

// camera-frame point of X under pose p
inline void to_camera(const std::array<double, 6>& p, const double X[3], double Pc[3]) {
    aa_rotate(p.data(), X, Pc);
    for (int a = 0; a < 3; ++a) Pc[a] += p[3 + a];
}

// pixel reprojection error of X (ReprojectCost's projection, no distortion)
inline double reproj_error(const Camera& cam, const std::array<double, 6>& p, const double X[3], const Point2d& kp) {
    double Pc[3];
    to_camera(p, X, Pc);
    const double u = cam.fx * (Pc[0] / Pc[2]) + cam.cx, v = cam.fy * (Pc[1] / Pc[2]) + cam.cy;
    return std::sqrt((u - kp.x) * (u - kp.x) + (v - kp.y) * (v - kp.y));
}

// Camera::pixel2normal
inline void normalise(const Camera& cam, const Point2d& kp, double n[2]) {
    n[0] = (kp.x - cam.cx) / cam.fx;
    n[1] = (kp.y - cam.cy) / cam.fy;
}

// E = [t]x R of the relative pose from camera 1 to camera 2
inline void essential(const std::array<double, 6>& p1, const std::array<double, 6>& p2, double E[9]) {
    double R1[9], R2[9], R[9], t[3];
    rot::aa_to_matrix(p1.data(), R1);
    rot::aa_to_matrix(p2.data(), R2);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += R2[3 * r + k] * R1[3 * c + k];   // R2 R1^T
            R[3 * r + c] = s;
        }
    for (int r = 0; r < 3; ++r)
        t[r] = p2[3 + r] - (R[3 * r] * p1[3] + R[3 * r + 1] * p1[4] + R[3 * r + 2] * p1[5]);
    const double tx[9] = {0, -t[2], t[1], t[2], 0, -t[0], -t[1], t[0], 0};
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            E[3 * r + c] = tx[3 * r] * R[c] + tx[3 * r + 1] * R[3 + c] + tx[3 * r + 2] * R[6 + c];
}

// squared Sampson distance of x2^T E x1 = 0 (OpenCV's essential-matrix
// RANSAC error, normalised coordinates)
inline double sampson2(const double E[9], const double n1[2], const double n2[2]) {
    const double x1[3] = {n1[0], n1[1], 1.0}, x2[3] = {n2[0], n2[1], 1.0};
    double Ex1[3], Etx2[3];
    for (int r = 0; r < 3; ++r) {
        Ex1[r] = E[3 * r] * x1[0] + E[3 * r + 1] * x1[1] + E[3 * r + 2] * x1[2];
        Etx2[r] = E[r] * x2[0] + E[3 + r] * x2[1] + E[6 + r] * x2[2];
    }
    const double e = x2[0] * Ex1[0] + x2[1] * Ex1[1] + x2[2] * Ex1[2];
    const double den = Ex1[0] * Ex1[0] + Ex1[1] * Ex1[1] + Etx2[0] * Etx2[0] + Etx2[1] * Etx2[1];
    return den > 0 ? e * e / den : 0.0;
}

// Linear (DLT) triangulation of one correspondence from two 3x4 projections
// on normalised coordinates: the unit vector minimising |A x|, i.e. the
// eigenvector of the smallest eigenvalue of AᵀA (cyclic Jacobi).  Returns
// false when the homogeneous coordinate vanishes.
inline bool triangulate(const double P1[12], const double P2[12], const double n1[2], const double n2[2],
                        double X[3]) {
    double A[4][4];
    const double* Ps[2] = {P1, P2};
    const double* ns[2] = {n1, n2};
    for (int v = 0; v < 2; ++v)
        for (int c = 0; c < 4; ++c) {
            A[2 * v][c] = ns[v][0] * Ps[v][8 + c] - Ps[v][c];
            A[2 * v + 1][c] = ns[v][1] * Ps[v][8 + c] - Ps[v][4 + c];
        }
    double M[4][4], V[4][4];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
            double s = 0;
            for (int k = 0; k < 4; ++k) s += A[k][r] * A[k][c];
            M[r][c] = s;
            V[r][c] = r == c ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 30; ++sweep) {
        double off = 0, diag = 0;
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) (r == c ? diag : off) += M[r][c] * M[r][c];
        if (off <= 1e-30 * diag) break;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) {
                if (M[p][q] == 0.0) continue;
                const double th = (M[q][q] - M[p][p]) / (2.0 * M[p][q]);
                const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 4; ++k) {   // M <- Jᵀ M J
                    const double mkp = M[k][p], mkq = M[k][q];
                    M[k][p] = c * mkp - s * mkq;
                    M[k][q] = s * mkp + c * mkq;
                }
                for (int k = 0; k < 4; ++k) {
                    const double mpk = M[p][k], mqk = M[q][k];
                    M[p][k] = c * mpk - s * mqk;
                    M[q][k] = s * mpk + c * mqk;
                }
                for (int k = 0; k < 4; ++k) {
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
    }
    int m = 0;
    for (int k = 1; k < 4; ++k)
        if (M[k][k] < M[m][m]) m = k;
    const double w = V[3][m];
    if (!(std::fabs(w) > 1e-12)) return false;
    for (int a = 0; a < 3; ++a) X[a] = V[a][m] / w;
    return std::isfinite(X[0]) && std::isfinite(X[1]) && std::isfinite(X[2]);
}

// Pose of a camera from 2D-3D correspondences (stand-in for solvePnPRansac's
// refined pose): Gauss-Newton on the reprojection error from `pose`
// (the caller's prior), rotation updated on the left (R <- exp[d]x R), Huber
// weights at huber_px so stray matches do not pull; then the inliers within
// inlier_px are counted.  Returns the inlier count; pose is left unchanged
// when fewer than 4 correspondences lie in front of the camera.
inline int64_t refine_pose(const Camera& cam, std::array<double, 6>& pose, const std::vector<const double*>& X,
                           const std::vector<Point2d>& uv, double huber_px, double inlier_px) {
    double R[9], t[3] = {pose[3], pose[4], pose[5]};
    rot::aa_to_matrix(pose.data(), R);
    auto residual = [&](const double* Xw, const Point2d& o, double r[2], double P[3], double RX[3]) {
        for (int a = 0; a < 3; ++a) RX[a] = R[3 * a] * Xw[0] + R[3 * a + 1] * Xw[1] + R[3 * a + 2] * Xw[2];
        for (int a = 0; a < 3; ++a) P[a] = RX[a] + t[a];
        if (!(P[2] > 0)) return false;
        r[0] = cam.fx * P[0] / P[2] + cam.cx - o.x;
        r[1] = cam.fy * P[1] / P[2] + cam.cy - o.y;
        return true;
    };
    for (int it = 0; it < 10; ++it) {
        double H[6][7] = {};
        int64_t used = 0;
        for (std::size_t k = 0; k < X.size(); ++k) {
            double r[2], P[3], RX[3];
            if (!residual(X[k], uv[k], r, P, RX)) continue;
            ++used;
            const double iz = 1.0 / P[2];
            const double JP[2][3] = {{cam.fx * iz, 0, -cam.fx * P[0] * iz * iz},
                                     {0, cam.fy * iz, -cam.fy * P[1] * iz * iz}};
            // d(exp[d]x R X)/dd = -[RX]x
            const double S[3][3] = {{0, RX[2], -RX[1]}, {-RX[2], 0, RX[0]}, {RX[1], -RX[0], 0}};
            double J[2][6];
            for (int i = 0; i < 2; ++i)
                for (int c = 0; c < 3; ++c) {
                    J[i][c] = JP[i][0] * S[0][c] + JP[i][1] * S[1][c] + JP[i][2] * S[2][c];
                    J[i][3 + c] = JP[i][c];
                }
            const double e = std::sqrt(r[0] * r[0] + r[1] * r[1]);
            const double w = e <= huber_px ? 1.0 : huber_px / e;
            for (int a = 0; a < 6; ++a) {
                for (int b = 0; b < 6; ++b) H[a][b] += w * (J[0][a] * J[0][b] + J[1][a] * J[1][b]);
                H[a][6] -= w * (J[0][a] * r[0] + J[1][a] * r[1]);
            }
        }
        if (used < 4) return 0;
        // Gaussian elimination with partial pivoting on [H | -g]
        for (int c = 0; c < 6; ++c) {
            int piv = c;
            for (int r = c + 1; r < 6; ++r)
                if (std::fabs(H[r][c]) > std::fabs(H[piv][c])) piv = r;
            if (!(std::fabs(H[piv][c]) > 0)) return 0;
            if (piv != c)
                for (int k = 0; k < 7; ++k) std::swap(H[c][k], H[piv][k]);
            for (int r = c + 1; r < 6; ++r) {
                const double f = H[r][c] / H[c][c];
                for (int k = c; k < 7; ++k) H[r][k] -= f * H[c][k];
            }
        }
        double d[6];
        for (int c = 5; c >= 0; --c) {
            double s = H[c][6];
            for (int k = c + 1; k < 6; ++k) s -= H[c][k] * d[k];
            d[c] = s / H[c][c];
        }
        double dR[9], Rn[9];
        rot::aa_to_matrix(d, dR);
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c)
                Rn[3 * r + c] = dR[3 * r] * R[c] + dR[3 * r + 1] * R[3 + c] + dR[3 * r + 2] * R[6 + c];
        for (int a = 0; a < 9; ++a) R[a] = Rn[a];
        for (int a = 0; a < 3; ++a) t[a] += d[3 + a];
        double n2 = 0;
        for (double v : d) n2 += v * v;
        if (n2 < 1e-24) break;
    }
    double w[3];
    rot::matrix_to_aa(R, w);
    pose = {w[0], w[1], w[2], t[0], t[1], t[2]};
    int64_t inliers = 0;
    for (std::size_t k = 0; k < X.size(); ++k) {
        double r[2], P[3], RX[3];
        if (residual(X[k], uv[k], r, P, RX) && std::sqrt(r[0] * r[0] + r[1] * r[1]) <= inlier_px) ++inliers;
    }
    return inliers;
}

}  // namespace geom

// One image of the sequence as the loop receives it: what
// Image::detectAndCompute (Image.h:39-41) would leave behind, plus the pose
// the geometric solver would return for it (stand-in, see above).
struct SeqImage {
    std::vector<Point2d> keypoints;
    std::vector<uint8_t> descriptors;   // [n][128]
    std::array<double, 6> pose_prior{};
};

struct SeqOptions {
    double epipolar_px = 4.0;     // essential-matrix inlier threshold (stand-in)
    double pnp_reproj_px = 8.0;   // solvePnPRansac reprojectionError (:179)
    double max_depth = 100.0;     // recoverPose distanceThresh (:118)
    int64_t min_pnp_inliers = 30; // :191
    BundleAdjusterOptions ba;     // BundleAdjuster() (:167-174); verbose off by default
    SeqOptions() { ba.verbose = false; }
};

template <class Backend>
class BasicSequentialActuator {
   public:
    using Clock = std::chrono::steady_clock;
    BasicSequentialActuator(Backend be, Camera::Ptr camera, SeqOptions opt = SeqOptions())
        : be_(std::move(be)), camera_(std::move(camera)), opt_(opt), world_(std::make_shared<WorldStructure>()) {}

    WorldStructure::Ptr getWorld() const { return world_; }
    const sfm_seq_step& lastStep() const { return step_; }
    const std::vector<DMatch>& lastLocalMatches() const { return local_; }
    const std::vector<DMatch>& lastGlobalMatches() const { return global_; }
    const std::vector<Image::Ptr>& images() const { return images_; }
    Camera::Ptr camera() const { return camera_; }
    Backend& backend() { return be_; }

    // :85-136
    void init(const SeqImage& a, const SeqImage& b) {
        begin_step(1);
        auto im1 = make_image(a), im2 = make_image(b);
        world_->addImage(im1);
        world_->addImage(im2);
        cur_frame_ = std::make_shared<LocalFrame>(im1, im2);
        auto t0 = Clock::now();
        step_.local_kept = (int64_t)cur_frame_->matchFeatureAndFilter(be_.matcher());
        step_.local_raw = (int64_t)cur_frame_->rawMatchCount();
        local_ = cur_frame_->getMatches();
        auto t1 = Clock::now();
        im1->setPose({});            // image_ptr1->setTcw({})
        im2->setPose(b.pose_prior);  // recoverPose's (R, t) (stand-in)
        std::vector<uint8_t> inl;
        std::vector<std::array<double, 3>> pts;
        geometry(im1, im2, true, inl, pts);
        savePointCloudToWorld(inl, pts);
        cur_frame_.reset();
        step_.kept = 1;
        step_.seconds_local_match = secs(t0, t1);
        step_.seconds_geometry = secs(t1, Clock::now());
        end_step();
    }

    // :138-224; returns false when the image is dropped (< min PnP inliers)
    bool addSingleImage(const SeqImage& next) {
        begin_step((int32_t)images_.size());
        auto im1 = world_->getLocalFrames().back()->getImage2();
        auto im2 = make_image(next);
        world_->addImage(im2);
        cur_frame_ = std::make_shared<LocalFrame>(im1, im2);
        auto t0 = Clock::now();
        step_.local_kept = (int64_t)cur_frame_->matchFeatureAndFilter(be_.matcher());
        step_.local_raw = (int64_t)cur_frame_->rawMatchCount();
        local_ = cur_frame_->getMatches();
        auto t1 = Clock::now();
        GlobalFrame gf(world_, im2);
        step_.global_kept = (int64_t)gf.matchFeatureAndFilter(be_.matcher());
        step_.global_raw = (int64_t)gf.rawMatchCount();
        global_ = gf.getMatches();
        auto t2 = Clock::now();
        // solvePnPRansac (stand-in): the pose refined from the prior on the
        // 2D-3D matches, inliers by reprojection
        std::vector<const double*> X3;
        std::vector<Point2d> x2;
        for (const auto& m : global_) {
            X3.push_back(gf.get_world_points()[m.queryIdx]->world_pos_.data());
            x2.push_back(im2->keypoints[m.trainIdx]);
        }
        std::array<double, 6> pose = next.pose_prior;
        const int64_t inliers = geom::refine_pose(*camera_, pose, X3, x2, 0.5 * opt_.pnp_reproj_px, opt_.pnp_reproj_px);
        im2->setPose(pose);
        step_.pnp_inliers = inliers;
        if (inliers < opt_.min_pnp_inliers) {   // "current frame has bad matched points, dropping."
            step_.kept = 0;
            step_.seconds_local_match = secs(t0, t1);
            step_.seconds_global_match = secs(t1, t2);
            step_.seconds_geometry = secs(t2, Clock::now());
            end_step();
            return false;
        }
        std::vector<uint8_t> inl;
        std::vector<std::array<double, 3>> pts;
        geometry(im1, im2, false, inl, pts);
        savePointCloudToWorld(inl, pts);
        step_.kept = 1;
        step_.seconds_local_match = secs(t0, t1);
        step_.seconds_global_match = secs(t1, t2);
        step_.seconds_geometry = secs(t2, Clock::now());
        end_step();
        return true;
    }

    // :226-229 — a fresh BundleAdjuster per call
    void bundleAdjustment() {
        auto t0 = Clock::now();
        auto adjuster = be_.make_adjuster(opt_.ba);
        adjuster(world_);
        step_.ba = adjuster.summary();
        step_.ba_rc = adjuster.lastError();
        step_.ba_images = adjuster.lastImages();
        step_.ba_points = adjuster.lastPoints();
        step_.ba_observations = adjuster.lastObservations();
        step_.seconds_ba = secs(t0, Clock::now());
    }

   private:
    static double secs(Clock::time_point a, Clock::time_point b) {
        return std::chrono::duration<double>(b - a).count();
    }
    void begin_step(int32_t image) {
        step_ = sfm_seq_step{};
        step_.image = image;
        step_.ba_rc = 1;   // no bundle adjustment yet for this step
        local_.clear();
        global_.clear();
    }
    void end_step() {
        step_.world_points = (int64_t)world_->points().size();
        step_.world_observations = world_->observationCount();
    }
    Image::Ptr make_image(const SeqImage& s) {
        auto im = std::make_shared<Image>(camera_);
        im->keypoints = s.keypoints;
        im->descriptors = s.descriptors;
        images_.push_back(im);
        return im;
    }
    // stand-ins for the OpenCV geometry: inlier mask + triangulated points of
    // every local match (see the header comment)
    void geometry(const Image::Ptr& im1, const Image::Ptr& im2, bool cheirality, std::vector<uint8_t>& inl,
                  std::vector<std::array<double, 3>>& pts) {
        const double f = 0.5 * (camera_->fx + camera_->fy);
        const double thr2 = (opt_.epipolar_px / f) * (opt_.epipolar_px / f);
        double E[9], P1[12], P2[12];
        geom::essential(im1->pose(), im2->pose(), E);
        geom::pose_matrix(im1->pose(), P1);
        geom::pose_matrix(im2->pose(), P2);
        inl.assign(local_.size(), 0);
        pts.assign(local_.size(), {0, 0, 0});
        int64_t n_in = 0;
        for (std::size_t k = 0; k < local_.size(); ++k) {
            const auto& m = local_[k];
            double n1[2], n2[2], X[3];
            geom::normalise(*camera_, im1->keypoints[m.queryIdx], n1);
            geom::normalise(*camera_, im2->keypoints[m.trainIdx], n2);
            bool ok = geom::sampson2(E, n1, n2) <= thr2;
            const bool tri = geom::triangulate(P1, P2, n1, n2, X);
            if (ok && cheirality) {   // recoverPose: in front of both cameras, within distanceThresh
                double c1[3], c2[3];
                ok = tri;
                if (ok) {
                    geom::to_camera(im1->pose(), X, c1);
                    geom::to_camera(im2->pose(), X, c2);
                    ok = c1[2] > 0 && c2[2] > 0 && c1[2] < opt_.max_depth && c2[2] < opt_.max_depth;
                }
            }
            if (ok && !tri) ok = false;   // a point at infinity cannot enter the world
            inl[k] = ok;
            n_in += ok;
            if (tri) pts[k] = {X[0], X[1], X[2]};
        }
        step_.epipolar_inliers = n_in;
    }

    // :25-72
    void savePointCloudToWorld(const std::vector<uint8_t>& inl, const std::vector<std::array<double, 3>>& pts) {
        world_->addLocalFrame(cur_frame_);
        auto im1 = cur_frame_->getImage1(), im2 = cur_frame_->getImage2();
        for (std::size_t k = 0; k < local_.size(); ++k) {
            if (!inl[k]) continue;
            const auto& m = local_[k];
            std::vector<uint8_t> desc(im2->descriptors.begin() + 128 * (std::size_t)m.trainIdx,
                                      im2->descriptors.begin() + 128 * (std::size_t)m.trainIdx + 128);
            auto it = im1->kpt_wpt_idx_map_.find((std::size_t)m.queryIdx);
            if (it != im1->kpt_wpt_idx_map_.end()) {   // a point seen before: extend its track
                auto wp = world_->getPointFromIdx(it->second);
                world_->setLastDescriptor(it->second, std::move(desc));
                world_->addObservation(wp, im2, im2->keypoints[m.trainIdx]);
                im2->kpt_wpt_idx_map_[(std::size_t)m.trainIdx] = it->second;
                ++step_.extended_obs;
                continue;
            }
            const auto idx = world_->addPoint(pts[k], std::move(desc));
            auto wp = world_->getPointFromIdx(idx);
            world_->addObservation(wp, im1, im1->keypoints[m.queryIdx]);
            world_->addObservation(wp, im2, im2->keypoints[m.trainIdx]);
            im1->kpt_wpt_idx_map_[(std::size_t)m.queryIdx] = idx;
            im2->kpt_wpt_idx_map_[(std::size_t)m.trainIdx] = idx;
            ++step_.new_points;
        }
    }

    Backend be_;
    Camera::Ptr camera_;
    SeqOptions opt_;
    WorldStructure::Ptr world_;
    LocalFrame::Ptr cur_frame_;
    std::vector<Image::Ptr> images_;
    std::vector<DMatch> local_, global_;
    sfm_seq_step step_{};
};

// Every world point's observations in point-index order: the sequence index
// of the observing image and the observed pixel (sfm_seq_observations).
template <class Act>
int seq_observations(const Act& act, int32_t* img, double* uv, int64_t cap, int64_t* n) {
    auto w = act.getWorld();
    std::vector<std::pair<WorldPoint::Idx, WorldPoint::Ptr>> pts(w->points().begin(), w->points().end());
    std::sort(pts.begin(), pts.end(), [](auto& a, auto& b) { return a.first < b.first; });
    std::unordered_map<const Image*, int32_t> seq_idx;
    for (std::size_t k = 0; k < act.images().size(); ++k) seq_idx[act.images()[k].get()] = (int32_t)k;
    int64_t m = 0;
    for (auto& [i, p] : pts)
        for (auto& [im, o] : p->observed_frames_) {
            if (m < cap) {
                if (img) img[m] = seq_idx.at(im.get());
                if (uv) { uv[2 * m] = o.x; uv[2 * m + 1] = o.y; }
            }
            ++m;
        }
    *n = m;
    return SFM_OK;
}

}  // namespace sfm
