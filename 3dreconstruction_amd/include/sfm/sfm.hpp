// Reference-shaped C++ surface over libsfmcore.so (C-ABI include/sfmcore.h):
//
//   BundleAdjuster        src/adjuster/BundleAdjuster.h:32-188
//   Matcher               cv::BFMatcher(NORM_L2, crossCheck=true) as created by
//                         SequentialActuator.h:77 (exact mutual nearest neighbour)
//   LocalFrame/GlobalFrame src/frame/LocalFrame.h:19-83, GlobalFrame.h:15-160
//   sparse::sparseBuilder src/sparseBuilder/sparseBuilder.h:14-39 — matchPair()
//                         (exhaustive pairs, .cpp:758-807) and match()
//                         (Matcher_Regions(0.8, BRUTE_FORCE_L2), .cpp:809-1023)
//                         file-staged over <base>/output/matches in OpenMVG's
//                         formats (csrc/mvg_io.cpp), or on in-memory regions.
//
// Header-only; link with -lsfmcore.  Errors: the reference prints and leaves
// the world untouched on BA failure (BundleAdjuster.h:128-131); so does this
// façade.  Matching failures throw sfm::Error.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../../include/sfmcore.h"
#include "world.hpp"

namespace sfm {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& where)
        : std::runtime_error(where + ": " + std::to_string(c) + " " + sfm_last_error()), code(c) {}
};

inline void check(int rc, const char* where) {
    if (rc != SFM_OK) throw Error(rc, where);
}

// One HIP device (+ RCCL communicator for landmark-sharded BA).
class Context {
   public:
    explicit Context(int device = 0, int rank = 0, int world = 1, const uint8_t* comm_id = nullptr) {
        sfm_ctx_opts o{};
        o.device = device; o.rank = rank; o.world_size = world; o.comm_id = comm_id;
        check(sfm_ctx_create(&o, &ctx_), "sfm_ctx_create");
    }
    ~Context() { sfm_ctx_destroy(ctx_); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    sfm_ctx* get() const { return ctx_; }
    // the reference constructs a BundleAdjuster per call; share one context per thread
    static Context& thread_default() {
        thread_local Context c(0);
        return c;
    }

   private:
    sfm_ctx* ctx_ = nullptr;
};

class LocalFrame {
   public:
    using Ptr = std::shared_ptr<LocalFrame>;
    LocalFrame(Image::Ptr image1, Image::Ptr image2) : image1_(std::move(image1)), image2_(std::move(image2)) {}
    Image::Ptr getImage1() const { return image1_; }
    Image::Ptr getImage2() const { return image2_; }
    const std::vector<DMatch>& getMatches() const { return matches_; }
    template <class M> std::size_t matchFeature(M& matcher);
    std::vector<DMatch> filterMatches() const;
    template <class M> std::size_t matchFeatureAndFilter(M& matcher) {
        matchFeature(matcher);
        matches_ = filterMatches();
        return matches_.size();
    }

   private:
    Image::Ptr image1_, image2_;
    std::vector<DMatch> matches_;
};

// ---------------------------------------------------------------------------
// Exact descriptor matcher on the GPU (stands in for the cv::BFMatcher).
// ---------------------------------------------------------------------------
class Matcher {
   public:
    explicit Matcher(Context& ctx = Context::thread_default()) : ctx_(&ctx) {}
    // knnMatch(query, train, out, k=1) with crossCheck: rows without a mutual
    // partner are empty (LocalFrame.h:37-44 skips them).
    void knnMatch(const std::vector<uint8_t>& query, const std::vector<uint8_t>& train,
                  std::vector<std::vector<DMatch>>& out, int k = 1) const {
        if (k != 1) throw std::invalid_argument("crossCheck matcher supports k = 1 only");
        const int nq = (int)(query.size() / 128), nt = (int)(train.size() / 128);
        std::vector<int32_t> idx(std::max(nq, 1)), d2(std::max(nq, 1));
        sfm_match_options o{SFM_MATCH_MUTUAL, 0.8f};
        check(sfm_match_dense(ctx_->get(), query.data(), nq, train.data(), nt, &o, idx.data(), d2.data()),
              "sfm_match_dense");
        out.assign(nq, {});
        for (int q = 0; q < nq; ++q)
            if (idx[q] >= 0) out[q].push_back(DMatch{q, idx[q], 0, std::sqrt((float)d2[q])});
    }
    Context& context() const { return *ctx_; }

   private:
    Context* ctx_;
};

template <class M>
std::size_t LocalFrame::matchFeature(M& matcher) {
    if (!matches_.empty()) matches_.clear();  // "Rematch feature" warning in the reference
    std::vector<std::vector<DMatch>> v;
    matcher.knnMatch(image1_->descriptors, image2_->descriptors, v, 1);
    for (auto& row : v)
        if (!row.empty()) matches_.push_back(row[0]);
    return matches_.size();
}

// keep d <= 4 * min d (LocalFrame.h:49-64); empty input -> empty (the
// reference dereferences min_element of an empty vector)
inline std::vector<DMatch> LocalFrame::filterMatches() const {
    std::vector<DMatch> good;
    if (matches_.empty()) return good;
    const float mn = std::min_element(matches_.begin(), matches_.end(),
                                      [](const DMatch& a, const DMatch& b) { return a.distance < b.distance; })
                         ->distance;
    for (const auto& m : matches_)
        if (m.distance <= 4 * mn) good.push_back(m);
    return good;
}

class GlobalFrame {
   public:
    GlobalFrame(const WorldStructure::Ptr& world, Image::Ptr image) : image_(std::move(image)) {
        std::vector<std::pair<WorldPoint::Idx, WorldPoint::Ptr>> pts(world->world_points_.begin(),
                                                                     world->world_points_.end());
        std::sort(pts.begin(), pts.end(), [](auto& a, auto& b) { return a.first < b.first; });
        for (auto& p : pts) world_points_.push_back(p.second);
    }
    template <class M> std::size_t matchFeature(M& matcher) {
        matches_.clear();
        std::vector<uint8_t> q;
        for (auto& p : world_points_) q.insert(q.end(), p->last_descriptor_.begin(), p->last_descriptor_.end());
        std::vector<std::vector<DMatch>> v;
        matcher.knnMatch(q, image_->descriptors, v, 1);
        for (auto& row : v)
            if (!row.empty()) matches_.push_back(row[0]);
        return matches_.size();
    }
    // drop d > 3 * min d (GlobalFrame.h:45-60)
    std::vector<DMatch> filterMatches() const {
        std::vector<DMatch> good;
        if (matches_.empty()) return good;
        float mn = matches_[0].distance;
        for (auto& m : matches_) mn = std::min(mn, m.distance);
        for (auto& m : matches_)
            if (!(m.distance > 3 * mn)) good.push_back(m);
        return good;
    }
    template <class M> std::size_t matchFeatureAndFilter(M& matcher) {
        matchFeature(matcher);
        matches_ = filterMatches();
        return matches_.size();
    }
    const std::vector<WorldPoint::Ptr>& get_world_points() const { return world_points_; }
    const std::vector<DMatch>& getMatches() const { return matches_; }

   private:
    std::vector<DMatch> matches_;
    Image::Ptr image_;
    std::vector<WorldPoint::Ptr> world_points_;
};

// ---------------------------------------------------------------------------
// BundleAdjuster (BundleAdjuster.h:32-188)
// ---------------------------------------------------------------------------
class BundleAdjuster {
   public:
    struct Options {
        bool fixed_writeback = false;  // false: reproduce Image::setIntrinsic's ZYX-Euler quirk
        bool verbose = true;           // print the reference's statistics block
        // A solve that could not run at all (bad input, device, RCCL) is not
        // the reference's "solution not usable" outcome: it is always reported
        // on stderr with sfm_last_error(), and thrown as sfm::Error when set.
        bool throw_on_error = false;
        sfm_ba_options solver{};
        Options() { sfm_ba_default_options(&solver); }
    };
    explicit BundleAdjuster(Context& ctx = Context::thread_default(), Options opt = Options())
        : ctx_(&ctx), opt_(opt) {}

    void operator()(WorldStructure::Ptr& world) {  // :176-186
        load(world);
        if (solve()) update();
        clear();
    }
    const sfm_ba_summary& summary() const { return summary_; }
    int lastError() const { return last_rc_; }   // SFM_OK or the last sfm_ba_solve code

   private:
    // loadDataFromWorld (:82-98) + problem assembly (:100-123)
    void load(const WorldStructure::Ptr& world) {
        world_ = world;
        images_.clear(); cams_.clear(); extr_.clear(); intr_.clear();
        img_index_.clear(); cam_index_.clear();
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
        auto add_img = [&](const Image::Ptr& im, bool zero_pose) {
            auto it = img_index_.find(im.get());
            if (it != img_index_.end()) return it->second;
            const int k = (int)images_.size();
            img_index_[im.get()] = k;
            images_.push_back(im);
            const auto p = zero_pose ? std::array<double, 6>{} : im->pose();
            extr_.insert(extr_.end(), p.begin(), p.end());
            img_cam_.push_back(-1);
            return k;
        };
        img_cam_.clear();
        for (auto& f : world->local_frames_) {
            const int k = add_img(f->getImage2(), false);
            img_cam_[k] = add_cam(f->getImage2()->getCamera(), false);
        }
        const_img_ = world->local_frames_.empty() ? -1 : 0;
        std::vector<std::pair<WorldPoint::Idx, WorldPoint::Ptr>> pts(world->world_points_.begin(),
                                                                     world->world_points_.end());
        std::sort(pts.begin(), pts.end(), [](auto& a, auto& b) { return a.first < b.first; });
        points_.clear(); X_.clear(); off_.assign(1, 0); obs_img_.clear(); uv_.clear();
        for (auto& [idx, p] : pts) {
            points_.push_back(p);
            X_.insert(X_.end(), p->world_pos_.begin(), p->world_pos_.end());
            for (auto& [im, uv] : p->observed_frames_) {
                // image_extrinsic_[image] / camera_intrinsics_[camera] are
                // operator[]: unseen blocks are inserted as zeros (:118-119)
                const int k = add_img(im, true);
                if (img_cam_[k] < 0) img_cam_[k] = add_cam(im->getCamera(), true);
                obs_img_.push_back(k);
                uv_.push_back(uv.x);
                uv_.push_back(uv.y);
            }
            off_.push_back((int64_t)obs_img_.size());
        }
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
        if (pr.n_img == 0 || pr.n_intr == 0) return false;
        const int rc = sfm_ba_solve(ctx_->get(), &pr, extr_.data(), intr_.data(), X_.data(), &opt_.solver, &summary_);
        last_rc_ = rc;
        if (rc != SFM_OK && rc != SFM_ERR_SOLVER && rc != SFM_ERR_NOT_FINITE) {
            std::fprintf(stderr, "Bundle Adjustment failed: %s (code %d)\n", sfm_last_error(), rc);
            if (opt_.throw_on_error) throw Error(rc, "sfm_ba_solve");
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
        for (std::size_t k = 0; k < points_.size(); ++k) points_[k]->setPos({X_[3 * k], X_[3 * k + 1], X_[3 * k + 2]});
        for (std::size_t k = 0; k < images_.size(); ++k) {
            std::array<double, 6> p;
            for (int a = 0; a < 6; ++a) p[a] = extr_[6 * k + a];
            images_[k]->setIntrinsic(p, opt_.fixed_writeback);
        }
        for (std::size_t k = 0; k < cams_.size(); ++k)
            cams_[k]->setIntrinsic({intr_[4 * k], intr_[4 * k + 1], intr_[4 * k + 2], intr_[4 * k + 3]});
    }
    void clear() {
        world_ = nullptr;
        images_.clear(); cams_.clear(); points_.clear();
    }

    Context* ctx_;
    Options opt_;
    WorldStructure::Ptr world_;
    std::vector<Image::Ptr> images_;
    std::vector<Camera::Ptr> cams_;
    std::vector<WorldPoint::Ptr> points_;
    std::unordered_map<const Image*, int> img_index_;
    std::unordered_map<const Camera*, int> cam_index_;
    std::vector<int32_t> img_cam_, obs_img_;
    std::vector<double> extr_, intr_, X_, uv_;
    std::vector<int64_t> off_;
    int32_t const_img_ = -1;
    int last_rc_ = SFM_OK;
    sfm_ba_summary summary_{};
};

namespace sparse {

struct IndMatch {  // openMVG::matching::IndMatch
    uint32_t i_, j_;
};
using Pair = std::pair<uint32_t, uint32_t>;
using PairWiseMatches = std::map<Pair, std::vector<IndMatch>>;

// sparse::sparseBuilder (sparseBuilder.h:14-39).  Constructed on a base path
// like the reference's, matchPair() / match() are the file-staged stages of
// sparseBuilder.cpp:758-1023 over <base>/output/matches (sfm_data.json,
// image_describer.json, <stem>.desc/.feat, pairs.bin -> matches.putative.bin,
// preemptive_pairs.txt), with the GPU matcher in place of the OpenMVG
// collection matcher.  Errors print and return, as the reference's
// OPENMVG_LOG_ERROR + return does (:825-878); lastError() keeps the code.
// exhaustive() / matchRegions() are the same stages on in-memory regions.
class sparseBuilder {
   public:
    explicit sparseBuilder(Context& ctx = Context::thread_default()) : ctx_(&ctx) {}
    explicit sparseBuilder(const std::string& base_path, Context& ctx = Context::thread_default())
        : ctx_(&ctx), matches_dir_(base_path + "/output/matches") {}

    const std::string& matchesDir() const { return matches_dir_; }
    int lastError() const { return last_rc_; }

    // exhaustivePairs(#views) -> pairs.bin (:758-807)
    void matchPair() {
        last_rc_ = sfm_sparse_match_pair(matches_dir_.c_str());
        if (last_rc_ != SFM_OK) std::fprintf(stderr, "matchPair failed: %s\n", sfm_last_error());
    }
    // sNearestMatchingMethod (:814, :911-925) -> SFM_MATCH_*: "AUTO" on SIFT
    // regions is Cascade_Hashing_Matcher_Regions, "BRUTEFORCEL2" is
    // Matcher_Regions(BRUTE_FORCE_L2); others are not provided (-1).
    static int matchingMode(const std::string& method) {
        if (method == "AUTO" || method == "CASCADEHASHINGL2" || method == "FASTCASCADEHASHINGL2")
            return SFM_MATCH_CASCADE;
        if (method == "BRUTEFORCEL2") return SFM_MATCH_RATIO;
        return -1;
    }
    // match() over pairs.bin (:809-1023), fDistRatio = 0.8f, method "AUTO"
    void match(float dist_ratio = 0.8f, bool force = false, const std::string& method = "AUTO") {
        const int mode = matchingMode(method);
        if (mode < 0) {
            last_rc_ = SFM_ERR_UNSUPPORTED;
            std::fprintf(stderr, "match failed: unsupported nearest matching method %s\n", method.c_str());
            return;
        }
        sfm_sparse_match_opts o{mode, dist_ratio, force ? 1 : 0, 1, {0, 0}};
        last_rc_ = sfm_sparse_match(ctx_->get(), matches_dir_.c_str(), &o, &stats_);
        if (last_rc_ != SFM_OK) std::fprintf(stderr, "match failed: %s\n", sfm_last_error());
    }
    const sfm_sparse_match_stats& stats() const { return stats_; }

    // in-memory regions: per view, n x 128 uint8 descriptors
    void setRegions(std::vector<std::vector<uint8_t>> regions) { regions_ = std::move(regions); }
    // exhaustivePairs(N) (:786)
    std::vector<Pair> exhaustive() const {
        std::vector<Pair> p;
        const uint32_t n = (uint32_t)regions_.size();
        for (uint32_t i = 0; i < n; ++i)
            for (uint32_t j = i + 1; j < n; ++j) p.emplace_back(i, j);
        return p;
    }
    PairWiseMatches matchRegions(const std::vector<Pair>& pairs, float dist_ratio = 0.8f,
                                 const std::string& method = "AUTO") const {
        const int mode = matchingMode(method);
        if (mode < 0) throw Error(SFM_ERR_UNSUPPORTED, "unsupported nearest matching method " + method);
        std::vector<uint8_t> desc;
        std::vector<int64_t> off(1, 0);
        for (auto& r : regions_) {
            desc.insert(desc.end(), r.begin(), r.end());
            off.push_back(off.back() + (int64_t)(r.size() / 128));
        }
        sfm_match_plan* plan = nullptr;
        check(sfm_match_plan_create(ctx_->get(), desc.data(), off.data(), (int32_t)regions_.size(), &plan),
              "sfm_match_plan_create");
        std::vector<int32_t> pv;
        for (auto& p : pairs) { pv.push_back((int32_t)p.first); pv.push_back((int32_t)p.second); }
        sfm_match_options o{mode, dist_ratio};
        int64_t total = 0;
        int rc = sfm_match_plan_run(plan, pv.data(), (int64_t)pairs.size(), &o, &total);
        std::vector<int64_t> counts(pairs.size());
        std::vector<uint32_t> ii(std::max<int64_t>(total, 1)), jj(ii.size());
        std::vector<int32_t> dd(ii.size());
        if (rc == SFM_OK) rc = sfm_match_plan_fetch(plan, counts.data(), ii.data(), jj.data(), dd.data());
        sfm_match_plan_destroy(plan);
        check(rc, "sfm_match_plan");
        PairWiseMatches out;
        int64_t k = 0;
        for (std::size_t p = 0; p < pairs.size(); ++p) {
            auto& v = out[pairs[p]];
            for (int64_t c = 0; c < counts[p]; ++c, ++k) v.push_back(IndMatch{ii[k], jj[k]});
        }
        return out;
    }

   private:
    Context* ctx_;
    std::string matches_dir_;
    int last_rc_ = SFM_OK;
    sfm_sparse_match_stats stats_{};
    std::vector<std::vector<uint8_t>> regions_;
};

}  // namespace sparse
}  // namespace sfm
