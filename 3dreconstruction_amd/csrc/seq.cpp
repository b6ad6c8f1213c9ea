// C-ABI of the incremental loop (include/sfmcore.h sfm_seq_*): the
// SequentialActuator of include/sfm/actuator.hpp bound to this library's GPU
// matcher (sfm_match_dense, MUTUAL = BFMatcher crossCheck) and GPU solver
// (sfm_ba_solve), one fresh adjuster per bundleAdjustment() call as
// src/actuator/SequentialActuator.h:226-229 makes it.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "../include/sfm/actuator.hpp"
#include "common.h"

namespace {

struct CtxMatcher {
    sfm_ctx* ctx;
    // cv::BFMatcher(NORM_L2, crossCheck).knnMatch(query, train, out, 1)
    void knnMatch(const std::vector<uint8_t>& query, const std::vector<uint8_t>& train,
                  std::vector<std::vector<sfm::DMatch>>& out, int /*k*/) const {
        const int nq = (int)(query.size() / 128), nt = (int)(train.size() / 128);
        std::vector<int32_t> idx(std::max(nq, 1)), d2(std::max(nq, 1));
        sfm_match_options o{SFM_MATCH_MUTUAL, 0.8f};
        const int rc = sfm_match_dense(ctx, query.data(), nq, train.data(), nt, &o, idx.data(), d2.data());
        if (rc != SFM_OK) throw sfm::SfmError{rc};
        out.assign(nq, {});
        for (int q = 0; q < nq; ++q)
            if (idx[q] >= 0) out[q].push_back(sfm::DMatch{q, idx[q], 0, std::sqrt((float)d2[q])});
    }
};

// SFM_SEQ_DUMP=<dir> (diagnostic): every 100th solve's problem, and the one
// after it (a consecutive pair: the grown-structure relation), is written to
// <dir>/ba_<call>.bin (int64 n_img n_intr n_pt n_obs const_img, then
// pt_offsets, obs_img, obs_uv, img_intr) for replaying the planner offline
void dump_problem(const sfm_ba_problem& pr) {
    static const char* dir = std::getenv("SFM_SEQ_DUMP");
    static std::atomic<int> calls{0};   // sequences may solve on several threads
    if (!dir) return;
    const int call = calls.fetch_add(1);
    if (call % 100 != 99 && !(call >= 100 && call % 100 == 0)) return;
    char path[512];
    std::snprintf(path, sizeof path, "%s/ba_%03d.bin", dir, call);
    FILE* f = std::fopen(path, "wb");
    if (!f) return;
    const int64_t h[5] = {pr.n_img, pr.n_intr, pr.n_pt, pr.n_obs, pr.const_img};
    std::fwrite(h, sizeof h, 1, f);
    std::fwrite(pr.pt_offsets, sizeof(int64_t), (size_t)pr.n_pt + 1, f);
    std::fwrite(pr.obs_img, sizeof(int32_t), (size_t)pr.n_obs, f);
    std::fwrite(pr.obs_uv, sizeof(double), 2 * (size_t)pr.n_obs, f);
    std::fwrite(pr.img_intr, sizeof(int32_t), (size_t)pr.n_img, f);
    std::fclose(f);
}

struct CtxSolver {
    sfm_ctx* ctx;
    int solve(const sfm_ba_problem& pr, double* extr, double* intr, double* X, const sfm_ba_options& o,
              sfm_ba_summary& s) const {
        dump_problem(pr);
        return sfm_ba_solve(ctx, &pr, extr, intr, X, &o, &s);
    }
    const char* last_error() const { return sfm_last_error(); }
};

struct Backend {
    CtxMatcher m;
    CtxMatcher& matcher() { return m; }
    sfm::BasicBundleAdjuster<CtxSolver> make_adjuster(const sfm::BundleAdjusterOptions& o) const {
        return sfm::BasicBundleAdjuster<CtxSolver>(CtxSolver{m.ctx}, o);
    }
};

using Actuator = sfm::BasicSequentialActuator<Backend>;

sfm::SeqImage to_image(const sfm_seq_image* im) {
    SFM_REQUIRE(im && im->n_kp >= 0 && (im->n_kp == 0 || (im->kp_xy && im->desc)), SFM_ERR_INVALID_ARG,
                "sfm_seq: bad image");
    sfm::SeqImage s;
    s.keypoints.resize(im->n_kp);
    for (int32_t k = 0; k < im->n_kp; ++k) s.keypoints[k] = {im->kp_xy[2 * k], im->kp_xy[2 * k + 1]};
    s.descriptors.assign(im->desc, im->desc + (size_t)im->n_kp * 128);
    for (int a = 0; a < 6; ++a) s.pose_prior[a] = im->pose_prior[a];
    return s;
}

}  // namespace

struct sfm_seq {
    std::unique_ptr<Actuator> act;
    bool initialised = false;
};

extern "C" void sfm_seq_default_options(sfm_seq_options* o) {
    if (!o) return;
    std::memset(o, 0, sizeof *o);
    o->fx = o->fy = 2905.88;    // src/main.cpp:124
    o->cx = 1416.0;             // src/main.cpp:59
    o->cy = 1064.0;
    const sfm::SeqOptions d;
    o->epipolar_px = d.epipolar_px;
    o->pnp_reproj_px = d.pnp_reproj_px;
    o->max_depth = d.max_depth;
    o->min_pnp_inliers = d.min_pnp_inliers;
    o->fixed_writeback = 0;
    sfm_ba_default_options(&o->ba);
}

extern "C" int sfm_seq_create(sfm_ctx* ctx, const sfm_seq_options* opts, sfm_seq** out) {
    return sfm::guarded([&] {
        SFM_REQUIRE(ctx && out, SFM_ERR_INVALID_ARG, "sfm_seq_create: bad arguments");
        sfm_seq_options o;
        if (opts) o = *opts; else sfm_seq_default_options(&o);
        SFM_REQUIRE(o.fx > 0 && o.fy > 0 && o.epipolar_px > 0 && o.pnp_reproj_px > 0, SFM_ERR_INVALID_ARG,
                    "sfm_seq_create: bad options");
        sfm::SeqOptions so;
        so.epipolar_px = o.epipolar_px;
        so.pnp_reproj_px = o.pnp_reproj_px;
        so.max_depth = o.max_depth;
        so.min_pnp_inliers = o.min_pnp_inliers;
        so.ba.fixed_writeback = o.fixed_writeback != 0;
        so.ba.solver = o.ba;
        auto cam = std::make_shared<sfm::Camera>(o.fx, o.fy, o.cx, o.cy);
        auto s = std::make_unique<sfm_seq>();
        s->act = std::make_unique<Actuator>(Backend{CtxMatcher{ctx}}, cam, so);
        *out = s.release();
        return SFM_OK;
    });
}

extern "C" int sfm_seq_init(sfm_seq* s, const sfm_seq_image* a, const sfm_seq_image* b) {
    return sfm::guarded([&] {
        SFM_REQUIRE(s && !s->initialised, SFM_ERR_INVALID_ARG, "sfm_seq_init: bad handle or already initialised");
        s->act->init(to_image(a), to_image(b));
        s->initialised = true;
        return SFM_OK;
    });
}

extern "C" int sfm_seq_add_image(sfm_seq* s, const sfm_seq_image* im, int32_t* kept) {
    return sfm::guarded([&] {
        SFM_REQUIRE(s && s->initialised, SFM_ERR_INVALID_ARG, "sfm_seq_add_image: call sfm_seq_init first");
        const bool k = s->act->addSingleImage(to_image(im));
        if (kept) *kept = k ? 1 : 0;
        return SFM_OK;
    });
}

extern "C" int sfm_seq_bundle_adjust(sfm_seq* s, sfm_ba_summary* summary) {
    return sfm::guarded([&] {
        SFM_REQUIRE(s && s->initialised, SFM_ERR_INVALID_ARG, "sfm_seq_bundle_adjust: call sfm_seq_init first");
        sfm::PhaseTimer tm("sfm_seq_bundle_adjust");
        s->act->bundleAdjustment();
        tm.mark("total");
        const auto& st = s->act->lastStep();
        if (summary) *summary = st.ba;
        // "solution not usable" is the reference's printed-and-continue outcome
        // (BundleAdjuster.h:128-131); anything else is a hard failure
        if (st.ba_rc != SFM_OK && st.ba_rc != SFM_ERR_SOLVER && st.ba_rc != SFM_ERR_NOT_FINITE) return (int)st.ba_rc;
        return SFM_OK;
    });
}

extern "C" int sfm_seq_last_step(sfm_seq* s, sfm_seq_step* step) {
    return sfm::guarded([&] {
        SFM_REQUIRE(s && step, SFM_ERR_INVALID_ARG, "null argument");
        *step = s->act->lastStep();
        return SFM_OK;
    });
}

extern "C" int sfm_seq_matches(sfm_seq* s, int32_t which, int32_t* query, int32_t* train, float* dist,
                               int64_t cap, int64_t* n) {
  return sfm::guarded([&] {
    SFM_REQUIRE(s && n && (which == 0 || which == 1), SFM_ERR_INVALID_ARG, "bad argument");
    const auto& v = which == 0 ? s->act->lastLocalMatches() : s->act->lastGlobalMatches();
    *n = (int64_t)v.size();
    if (!query && !train && !dist) return SFM_OK;
    const int64_t m = std::min<int64_t>(cap, (int64_t)v.size());
    for (int64_t k = 0; k < m; ++k) {
        if (query) query[k] = v[k].queryIdx;
        if (train) train[k] = v[k].trainIdx;
        if (dist) dist[k] = v[k].distance;
    }
    return SFM_OK;
  });
}

extern "C" int sfm_seq_world(sfm_seq* s, double* X, int64_t* n_obs, int64_t cap_pts, int64_t* n_pts,
                             double* poses, int32_t cap_img, int32_t* n_img, double* intr4) {
  return sfm::guarded([&] {
    SFM_REQUIRE(s, SFM_ERR_INVALID_ARG, "null sequence");
    auto w = s->act->getWorld();
    std::vector<std::pair<sfm::WorldPoint::Idx, sfm::WorldPoint::Ptr>> pts(w->points().begin(), w->points().end());
    std::sort(pts.begin(), pts.end(), [](auto& a, auto& b) { return a.first < b.first; });
    if (n_pts) *n_pts = (int64_t)pts.size();
    const auto& ims = s->act->images();
    if (n_img) *n_img = (int32_t)ims.size();
    for (int64_t k = 0; k < std::min<int64_t>(cap_pts, (int64_t)pts.size()); ++k) {
        if (X) for (int a = 0; a < 3; ++a) X[3 * k + a] = pts[k].second->world_pos_[a];
        if (n_obs) n_obs[k] = (int64_t)pts[k].second->observed_frames_.size();
    }
    if (poses)
        for (int32_t k = 0; k < std::min<int32_t>(cap_img, (int32_t)ims.size()); ++k)
            for (int a = 0; a < 6; ++a) poses[6 * k + a] = ims[k]->pose()[a];
    if (intr4) {
        const auto v = s->act->camera()->getIntrinsic();
        for (int a = 0; a < 4; ++a) intr4[a] = v[a];
    }
    return SFM_OK;
  });
}

extern "C" int sfm_seq_observations(sfm_seq* s, int32_t* img, double* uv, int64_t cap, int64_t* n) {
    return sfm::guarded([&] {
        SFM_REQUIRE(s && n, SFM_ERR_INVALID_ARG, "null argument");
        return seq_observations(*s->act, img, uv, cap, n);
    });
}

extern "C" int sfm_seq_destroy(sfm_seq* s) {
    delete s;
    return SFM_OK;
}
