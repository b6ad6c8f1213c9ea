// BundleAdjuster (src/adjuster/BundleAdjuster.h:32-188) over a solver policy.
//
// BasicBundleAdjuster<Solver> does what the reference's class does around
// ceres::Solve: loadDataFromWorld (:82-98) + problem assembly (:100-123) into
// plain SoA arrays, the solve, updateWorld (:143-156) only when the solution
// is usable (:128-131, :179-184), clear (:158-164).  The solver policy is
//   int  solve(const sfm_ba_problem&, double* extr, double* intr, double* X,
//              const sfm_ba_options&, sfm_ba_summary&);   // SFM_OK / SFM_ERR_*
//   const char* last_error() const;
// sfm.hpp binds it to the GPU (sfm_ba_solve); the loop oracle binds it to the
// CPU restatement.  Header-only.
#pragma once
#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../../include/sfmcore.h"
#include "frames.hpp"
#include "pool.hpp"
#include "world.hpp"

namespace sfm {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& where, const char* msg = "")
        : std::runtime_error(where + ": " + std::to_string(c) + " " + msg), code(c) {}
};

struct BundleAdjusterOptions {
    bool fixed_writeback = false;  // false: reproduce Image::setIntrinsic's ZYX-Euler quirk
    bool verbose = true;           // print the reference's statistics block
    // A solve that could not run at all (bad input, device, RCCL, a shape the
    // build does not take) is not the reference's "solution not usable"
    // outcome: it is always reported on stderr with the solver's message, and
    // thrown as sfm::Error when set.
    bool throw_on_error = false;
    sfm_ba_options solver{};
    BundleAdjusterOptions() {
        solver.max_num_iterations = 50; solver.max_num_consecutive_invalid_steps = 5;
        solver.jacobi_scaling = 1; solver.reserved = 0;
        solver.function_tolerance = 1e-6; solver.gradient_tolerance = 1e-10;
        solver.parameter_tolerance = 1e-8; solver.initial_trust_region_radius = 1e4;
        solver.max_trust_region_radius = 1e16; solver.min_trust_region_radius = 1e-32;
        solver.min_relative_decrease = 1e-3; solver.min_lm_diagonal = 1e-6;
        solver.max_lm_diagonal = 1e32;
    }
};

template <class Solver>
class BasicBundleAdjuster {
   public:
    using Options = BundleAdjusterOptions;
    explicit BasicBundleAdjuster(Solver solver, Options opt = Options()) : solver_(std::move(solver)), opt_(opt) {}

    void operator()(WorldStructure::Ptr& world) {  // :176-186
        // SFM_TIMING=1 (diagnostic): the adjuster's own phases on stderr
        static const bool timing = std::getenv("SFM_TIMING") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        load(world);
        const auto t1 = std::chrono::steady_clock::now();
        const bool ok = solve();
        const auto t2 = std::chrono::steady_clock::now();
        if (ok) update();
        const auto t3 = std::chrono::steady_clock::now();
        clear();
        if (timing) {
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            std::fprintf(stderr, "[timing] adjuster: load %.2f ms, solve %.2f ms, update %.2f ms, clear %.2f ms\n",
                         ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, std::chrono::steady_clock::now()));
        }
    }
    const sfm_ba_summary& summary() const { return summary_; }
    int lastError() const { return last_rc_; }   // SFM_OK or the last solve code
    // size of the last problem (images with a pose block, points, observations)
    int64_t lastImages() const { return last_n_img_; }
    int64_t lastPoints() const { return last_n_pt_; }
    int64_t lastObservations() const { return last_n_obs_; }
    Options& options() { return opt_; }

   private:
    // loadDataFromWorld (:82-98) + problem assembly (:100-123)
    void load(const WorldStructure::Ptr& world) {
        for (const auto& im : images_) img_slot_[im->getIdx()] = -1;   // (normally cleared already)
        images_.clear(); cams_.clear(); extr_.clear(); intr_.clear();
        cam_index_.clear(); img_cam_.clear();
        auto add_cam = [&](const Camera::Ptr& c, bool zero) {
            auto it = cam_index_.find(c.get());
            if (it != cam_index_.end()) return it->second;
            const int k = (int)cams_.size();
            cam_index_[c.get()] = k;
            cams_.push_back(c);
            const auto v = zero ? std::array<double, 4>{0, 0, 0, 0} : c->getIntrinsic();
            intr_.insert(intr_.end(), v.begin(), v.end());
            return k;
        };
        // image -> problem index by the image's own index (a vector, not a hash
        // lookup per observation)
        auto add_img = [&](const Image::Ptr& im, bool zero_pose) {
            const std::size_t id = im->getIdx();
            if (id >= img_slot_.size()) img_slot_.resize(id + 1, -1);
            if (img_slot_[id] >= 0) return img_slot_[id];
            const int k = (int)images_.size();
            img_slot_[id] = k;
            images_.push_back(im);
            const auto p = zero_pose ? std::array<double, 6>{} : im->pose();
            extr_.insert(extr_.end(), p.begin(), p.end());
            img_cam_.push_back(-1);
            return k;
        };
        // Images are numbered in creation order (Image::getIdx(), the photo
        // order of the sequence), the poses of the local frames' second images
        // copied and every other observed image's pose block zero (:85-98,
        // :118-119).  Ceres orders parameter blocks itself, so the numbering
        // is free; creation order makes each call's problem an extension of
        // the previous call's (a new image, new points and new observations
        // appended, nothing renumbered), which the plan cache of sfm_ba_solve
        // reuses ("Grown problems"), and keeps the orbit's
        // cameras in band order.  (Until round 5 the local frames came first
        // and the sequence's first photo last.)
        std::vector<std::pair<Image::Ptr, bool>> imgs;   // (image, pose copied)
        // points in index order (the reference iterates its unordered_map).
        // The walk over the world is a pointer chase (every point and its
        // observation list are separate heap blocks), so it runs on host
        // threads over point ranges, each prefetching a few points ahead:
        //   pass 1: observations per point, and the images each range meets
        //           first, in order (merged in range order, that is the
        //           problem's image order of a serial walk: first appearance);
        //   pass 2: every range writes its points' X, image indices and uv.
        // The adjuster keeps plain pointers (the world owns the points for the
        // whole call), so no reference counts move.
        const std::vector<WorldPoint::Ptr>& pts = world->pointsByIdx();
        const std::size_t np = pts.size();
        const int nr = (int)std::max<std::size_t>(1, std::min<std::size_t>(PlanPool::width(), np / 4096));
        std::vector<std::vector<const Image::Ptr*>> first(nr);   // into the world's lists
        points_.resize(np);
        X_.resize(3 * np);
        off_.assign(np + 1, 0);
        auto ranges = [&](auto&& fn) {   // on the worker pool (pool.hpp)
            pool_ranges((int64_t)np, nr, [&](int64_t k0, int64_t k1, int r) { fn(r, (std::size_t)k0, (std::size_t)k1); });
        };
        constexpr std::size_t kAhead = 8;
        auto prefetch = [&](std::size_t k, std::size_t k1) {
            if (k + 2 * kAhead < k1) __builtin_prefetch(pts[k + 2 * kAhead].get());
            if (k + kAhead < k1) {
                const auto& of = pts[k + kAhead]->observed_frames_;
                __builtin_prefetch(of.data());
                __builtin_prefetch(reinterpret_cast<const char*>(of.data()) + 64);
                __builtin_prefetch(reinterpret_cast<const char*>(of.data()) + 128);
            }
        };
        ranges([&](int r, std::size_t k0, std::size_t k1) {
            std::vector<char> seen;
            for (std::size_t k = k0; k < k1; ++k) {
                prefetch(k, k1);
                WorldPoint* p = pts[k].get();
                points_[k] = p;
                off_[k + 1] = (int64_t)p->observed_frames_.size();
                for (auto& ob : p->observed_frames_) {
                    const std::size_t id = ob.first->getIdx();
                    if (id >= seen.size()) seen.resize(id + 1, 0);
                    if (!seen[id]) { seen[id] = 1; first[r].push_back(&ob.first); }
                }
            }
        });
        for (std::size_t k = 0; k < np; ++k) off_[k + 1] += off_[k];
        // image_extrinsic_[image] / camera_intrinsics_[camera] are operator[]:
        // unseen blocks are inserted as zeros (:118-119)
        for (auto& f : world->local_frames_) imgs.push_back({f->getImage2(), true});
        for (const auto& f : first)
            for (const Image::Ptr* im : f) imgs.push_back({*im, false});
        // a camera keeps its intrinsics when any local frame's image uses it
        // (loaded first, :85-98); only cameras of other images are zero blocks
        for (auto& f : world->local_frames_) add_cam(f->getImage2()->getCamera(), false);
        std::stable_sort(imgs.begin(), imgs.end(),
                         [](const auto& a, const auto& b) { return a.first->getIdx() < b.first->getIdx(); });
        for (const auto& e : imgs) {
            const Image::Ptr& im = e.first;
            const std::size_t id = im->getIdx();
            if (id < img_slot_.size() && img_slot_[id] >= 0) continue;   // (a local frame's image, also observed)
            const int k = add_img(im, !e.second);
            img_cam_[k] = add_cam(im->getCamera(), true);
        }
        const_img_ = world->local_frames_.empty() ? -1 : img_slot_[world->local_frames_.front()->getImage2()->getIdx()];
        const int64_t nobs = off_[np];
        obs_img_.resize(nobs);
        uv_.resize(2 * nobs);
        ranges([&](int, std::size_t k0, std::size_t k1) {
            for (std::size_t k = k0; k < k1; ++k) {
                prefetch(k, k1);
                const WorldPoint* p = points_[k];
                for (int a = 0; a < 3; ++a) X_[3 * k + a] = p->world_pos_[a];
                int64_t o = off_[k];
                for (auto& ob : p->observed_frames_) {
                    obs_img_[o] = img_slot_[ob.first->getIdx()];
                    uv_[2 * o] = ob.second.x;
                    uv_[2 * o + 1] = ob.second.y;
                    ++o;
                }
            }
        });
    }
    bool solve() {
        sfm_ba_problem pr{};
        pr.n_img = (int32_t)images_.size();
        pr.n_intr = (int32_t)cams_.size();
        pr.n_pt = (int64_t)points_.size();
        pr.n_obs = (int64_t)obs_img_.size();
        pr.pt_offsets = off_.data();
        pr.obs_img = obs_img_.data();
        pr.obs_uv = uv_.data();
        pr.img_intr = img_cam_.data();
        pr.const_img = const_img_;
        pr.huber_a = 4.0;
        last_n_img_ = pr.n_img; last_n_pt_ = pr.n_pt; last_n_obs_ = pr.n_obs;
        summary_ = sfm_ba_summary{};
        if (pr.n_img == 0 || pr.n_intr == 0) return false;
        const int rc = solver_.solve(pr, extr_.data(), intr_.data(), X_.data(), opt_.solver, summary_);
        last_rc_ = rc;
        if (rc != SFM_OK && rc != SFM_ERR_SOLVER && rc != SFM_ERR_NOT_FINITE) {
            std::fprintf(stderr, "Bundle Adjustment failed: %s (code %d)\n", solver_.last_error(), rc);
            if (opt_.throw_on_error) throw Error(rc, "bundle adjustment", solver_.last_error());
            return false;
        }
        if (rc != SFM_OK || !summary_.usable) {   // !IsSolutionUsable (:128-131)
            if (opt_.verbose) std::printf("Bundle Adjustment failed.\n");
            return false;
        }
        if (opt_.verbose)
            std::printf("Bundle Adjustment statistics (approximated RMSE):\n    #views: %zu\n    #residuals: %lld\n"
                        "    Initial RMSE: %g\n    Final RMSE: %g\n    Time (s): %g\n",
                        images_.size(), (long long)summary_.num_residuals, summary_.rmse_initial,
                        summary_.rmse_final, summary_.seconds);
        return true;
    }
    void update() {  // updateWorld (:143-156)
        const std::size_t np = points_.size();
        const int nr = (int)std::max<std::size_t>(1, std::min<std::size_t>(PlanPool::width(), np / 4096));
        pool_ranges((int64_t)np, nr, [&](int64_t k0, int64_t k1, int) {
            for (int64_t k = k0; k < k1; ++k) {
                if (k + 8 < k1) __builtin_prefetch(points_[k + 8], 1);
                points_[k]->setPos({X_[3 * k], X_[3 * k + 1], X_[3 * k + 2]});
            }
        });
        for (std::size_t k = 0; k < images_.size(); ++k) {
            std::array<double, 6> p;
            for (int a = 0; a < 6; ++a) p[a] = extr_[6 * k + a];
            images_[k]->setIntrinsic(p, opt_.fixed_writeback);
        }
        for (std::size_t k = 0; k < cams_.size(); ++k)
            cams_[k]->setIntrinsic({intr_[4 * k], intr_[4 * k + 1], intr_[4 * k + 2], intr_[4 * k + 3]});
    }
    void clear() {  // :158-164
        for (const auto& im : images_) img_slot_[im->getIdx()] = -1;
        images_.clear(); cams_.clear(); points_.clear();
    }

    Solver solver_;
    Options opt_;
    std::vector<Image::Ptr> images_;
    std::vector<Camera::Ptr> cams_;
    std::vector<WorldPoint*> points_;   // owned by the world during the call
    std::vector<int> img_slot_;   // Image::getIdx() -> problem image index or -1
    std::unordered_map<const Camera*, int> cam_index_;
    std::vector<int32_t> img_cam_, obs_img_;
    std::vector<double> extr_, intr_, X_, uv_;
    std::vector<int64_t> off_;
    int32_t const_img_ = -1;
    int last_rc_ = SFM_OK;
    int64_t last_n_img_ = 0, last_n_pt_ = 0, last_n_obs_ = 0;
    sfm_ba_summary summary_{};
};

}  // namespace sfm
