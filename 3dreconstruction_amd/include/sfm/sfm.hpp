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
#include "actuator.hpp"
#include "adjuster.hpp"
#include "frames.hpp"
#include "world.hpp"

namespace sfm {

inline void check(int rc, const char* where) {
    if (rc != SFM_OK) throw Error(rc, where, sfm_last_error());
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
    // the same over float rows, the cv::Mat CV_32F cv::SIFT produces
    // (LocalFrame.h:38, Image.h:39-41): integer-valued rows take the exact u8
    // path, others the f32 one (sfm_match_dense_f32)
    void knnMatch(const std::vector<float>& query, const std::vector<float>& train,
                  std::vector<std::vector<DMatch>>& out, int k = 1) const {
        if (k != 1) throw std::invalid_argument("crossCheck matcher supports k = 1 only");
        const int nq = (int)(query.size() / 128), nt = (int)(train.size() / 128);
        std::vector<int32_t> idx(std::max(nq, 1));
        std::vector<float> d2(std::max(nq, 1));
        sfm_match_options o{SFM_MATCH_MUTUAL, 0.8f};
        check(sfm_match_dense_f32(ctx_->get(), query.data(), nq, train.data(), nt, &o, idx.data(), d2.data()),
              "sfm_match_dense_f32");
        out.assign(nq, {});
        for (int q = 0; q < nq; ++q)
            if (idx[q] >= 0) out[q].push_back(DMatch{q, idx[q], 0, std::sqrt(d2[q])});
    }
    Context& context() const { return *ctx_; }

   private:
    Context* ctx_;
};

// ---------------------------------------------------------------------------
// BundleAdjuster (BundleAdjuster.h:32-188) on the GPU solver
// ---------------------------------------------------------------------------
struct GpuSolver {
    Context* ctx;
    int solve(const sfm_ba_problem& pr, double* extr, double* intr, double* X, const sfm_ba_options& o,
              sfm_ba_summary& s) const {
        return sfm_ba_solve(ctx->get(), &pr, extr, intr, X, &o, &s);
    }
    const char* last_error() const { return sfm_last_error(); }
};

class BundleAdjuster : public BasicBundleAdjuster<GpuSolver> {
   public:
    explicit BundleAdjuster(Context& ctx = Context::thread_default(), Options opt = Options())
        : BasicBundleAdjuster<GpuSolver>(GpuSolver{&ctx}, opt) {}
};

// ---------------------------------------------------------------------------
// SequentialActuator (SequentialActuator.h:16-236) on the GPU matcher and
// adjuster (BASELINE.json config C5)
// ---------------------------------------------------------------------------
struct GpuSeqBackend {
    Matcher m;
    Context* ctx;
    Matcher& matcher() { return m; }
    BundleAdjuster make_adjuster(const BundleAdjusterOptions& o) const { return BundleAdjuster(*ctx, o); }
};

class SequentialActuator : public BasicSequentialActuator<GpuSeqBackend> {
   public:
    explicit SequentialActuator(Camera::Ptr camera, Context& ctx = Context::thread_default(),
                                SeqOptions opt = SeqOptions())
        : BasicSequentialActuator<GpuSeqBackend>(GpuSeqBackend{Matcher(ctx), &ctx}, std::move(camera), opt) {}
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

    // filter() (:1025-1280) with its settings: sGeometricModel "f" ->
    // GeometricFilter_FMatrix_AC(4.0, imax_iteration = 2048), no guided
    // matching: matches.putative.bin -> matches.f.bin
    void filter(double precision = 4.0, int max_iterations = 2048) {
        sfm_fmatrix_opts o{precision, max_iterations, 0};
        last_rc_ = sfm_sparse_filter(ctx_->get(), matches_dir_.c_str(), &o, &filter_stats_);
        if (last_rc_ != SFM_OK) std::fprintf(stderr, "filter failed: %s\n", sfm_last_error());
    }
    const sfm_sparse_filter_stats& filterStats() const { return filter_stats_; }

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
    sfm_sparse_filter_stats filter_stats_{};
    std::vector<std::vector<uint8_t>> regions_;
};

}  // namespace sparse
}  // namespace sfm
