// Levenberg-Marquardt driver for the gfx950 BA kernels and the BA C-ABI.
//
// Mirrors BundleAdjuster::operator() (src/adjuster/BundleAdjuster.h:176-186):
// parameters are copied in, solved, and written back only if the solution is
// usable (:128-131, :143-156).  The trust-region control flow is the Ceres
// 2.2 TrustRegionMinimizer + LevenbergMarquardtStrategy restated in
// oracle/ba_oracle.cpp; every decision here is taken on the host from scalars
// the kernels reduce on the device (one device->host sync per iteration), so
// the accept/reject sequence follows the oracle's decision for decision.
//
// Multi-GPU (world_size > 1): each rank owns a landmark block (contiguous
// range of the camera-sorted point order); per iteration the reduced camera
// system and the E-part scalars are summed with RCCL all-reduce over xGMI and
// every rank solves the (identical) RCS redundantly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <limits>
#include <vector>
#include <unordered_map>
#include <thread>
#include <mutex>

#include "ba_bcr.h"
#include "ba_kernels.h"
#include "ba_order.h"
#include "ba_plan.h"
#include "common.h"
#include "../include/sfm/pool.hpp"

using namespace sfm;

struct sfm_ba_plan {
    sfm_ctx* ctx = nullptr;
    BAHostPlan hp;
    DevProblem P{};
    DBuf<int32_t> gram_img;
    DBuf<int32_t> pt_off, obs_img, obs_slot, img_obs_ptr, img_colc,
        img_coli, img_intr, intr_col, blk_img, blk_intr, free_img;
    DBuf<double> obs_uv;
    DBuf<ChunkDesc> chunks;
    DBuf<int32_t> group_off;   // tile groups of chunks
    DBuf<ReduceTarget> targets;
    DBuf<FlatTerm> terms;
    DBuf<double> X0, Xa, Xb, extr0, intr0, ea, eb, ia, ib;
    DBuf<CamPre> cpa, cpb;
    DBuf<double> scaleE, scaleF, gram, rcs, Lcol, Larrow, zF, yF, Wg, part_u, part_s,
        part_t, part_f, scal, bcr_buf, fin_part;
    DBuf<unsigned> fin_count;
    DBuf<int32_t> long_targets;
    DBuf<int32_t> gblk_off, gblk_col, gblk_z;   // general points
    DBuf<int64_t> gz_off;
    DBuf<int32_t> zbatch, zlong;
    DBuf<PTerm> pterms;
    DBuf<double> Zbuf, dense_buf;
    std::vector<int32_t> dense_meta;   // the dense dataflow solve's schedule (host copy, dense_flow_plan)
    DenseArgs dense;
    DBuf<double> lpart;           // long-target segment partials [n_lseg][36]
    DBuf<unsigned> lcount;        // per long target: segment tickets of the fused reduce
    DBuf<int32_t> plong_targets;  // long product-term targets, offsets, segments
    DBuf<double> plpart;          // their segment partials [n_plseg][36]
    DBuf<int32_t> img_pt;         // image-ordered observations (image Gram pass)
    DBuf<double> img_uv;
    DBuf<unsigned long long> stamps;   // SFM_SCHUR_STAMPS=1 diagnostic
    DBuf<unsigned long long> bcr_stamps;   // SFM_BCR_STAMPS=1 diagnostic
    DBuf<double> scal_g;                   // [world][kScMaxEnd] gathered partial scalars
    // plan-cache refresh (sfm_ba_solve): shard -> problem point / observation
    // maps (built on the first refresh) and staging for the new values
    DBuf<int32_t> pt_src, obs_src;
    DBuf<int64_t> src_off;
    DBuf<double> raw_uv, raw_X;
    BcrArgs bcr;
    unsigned bcr_epoch = 0;   // RCS solves so far (the back-substitution flags' epoch, BCR or dense)
    bool use_bcr = false;
    int64_t rcs_n = 0;
    double* scal_h = nullptr;  // pinned, host-mapped: [kScCount] + finalize sequence word
    double* scal_dev = nullptr;   // its device address
    unsigned long long fin_seq = 0;
    std::vector<sfm_ba_iter> trace;
    double last_ms[8] = {0};
    double schur_ms_total = 0;
    int64_t schur_launches = 0;
    bool cur_is_a = true;
    ~sfm_ba_plan() {
        if (scal_h) pinned_free(scal_h);
    }
};

namespace {

template <class T, class V>
void up(DBuf<T>& d, const V& h, hipStream_t s) {
    d.alloc(std::max<size_t>(h.size(), 1));
    d.upload(h.data(), h.size(), s);
}

// Page-locked staging for the plan's pageable host vectors: each is copied
// into it and uploaded from there, so every upload is an asynchronous DMA
// (a hipMemcpyAsync from pageable memory stages synchronously, per call).
// Blocks stay put until the staging is destroyed, after the stream's sync.
struct Staging {
    std::vector<HostVec<char>> blocks;
    size_t used = 0;
    template <class T>
    const T* put(const T* p, size_t n) {
        const size_t bytes = n * sizeof(T);
        if (blocks.empty() || used + bytes > blocks.back().size()) {
            blocks.emplace_back();
            blocks.back().resize(std::max<size_t>(bytes, (size_t)1 << 20));
            used = 0;
        }
        char* d = blocks.back().data() + used;
        std::memcpy(d, p, bytes);
        used += (bytes + 255) & ~(size_t)255;
        return reinterpret_cast<const T*>(d);
    }
};
template <class T, class A>
void up(Staging& st, DBuf<T>& d, const std::vector<T, A>& h, hipStream_t s) {
    d.alloc(std::max<size_t>(h.size(), 1));
    if (!h.empty()) d.upload(st.put(h.data(), h.size()), h.size(), s);
}

// the plan cache of sfm_ba_solve grows plans (SFM_BA_NO_PLAN_CACHE: no
// cache, nothing kept for it; SFM_BA_NO_GROWN_PLAN: exact reuse only)
bool cache_enabled_for_growth() {
    static const bool on = std::getenv("SFM_BA_NO_PLAN_CACHE") == nullptr && std::getenv("SFM_BA_NO_GROWN_PLAN") == nullptr;
    return on;
}

// The plan of a problem: from scratch, or -- seed set (sfm_ba_solve's plan
// cache, a problem grown from the previous call's, GrowPrev) -- grown from
// the seed plan (build_plan_grown: the same arrays; the measurements are
// gathered into shard order on the device).  Returns false, with nothing
// done and the seed intact, when the seed cannot seed this problem.
bool create_plan(sfm_ba_plan* pl, const sfm_ba_problem& prob, const double* extr, const double* intr,
                 const double* X, sfm_ba_plan* seed = nullptr, const GrowPrev* prev = nullptr) {
    sfm_ctx* ctx = pl->ctx;
    hipStream_t s = ctx->stream;
    BAHostPlan& h = pl->hp;
    PhaseTimer tm("create_plan");
    h.on_shard_ready = [&](BAHostPlan& hp) {
        up(pl->pt_off, hp.pt_off, s);
        up(pl->obs_img, hp.obs_img, s);
        up(pl->obs_slot, hp.obs_slot, s);
        if (!hp.uv_on_device) up(pl->obs_uv, hp.obs_uv, s);
    };
    PlanOpts po;
    po.force_dense = (ctx->flags & SFM_CTX_BA_DENSE_RCS) != 0;
    po.tile80 = (ctx->flags & SFM_CTX_BA_TILE80) != 0;
    if (seed) {
        if (!build_plan_grown(prob, *prev, seed->hp, h, po)) {
            h.on_shard_ready = nullptr;
            return false;
        }
    } else {
        build_plan(prob, ctx->rank, ctx->world, h, po);
    }
    h.on_shard_ready = nullptr;
    tm.mark(seed ? "build_plan_grown" : "build_plan");
    if (h.uv_on_device && h.n_sobs > 0) {
        // the measurements into shard order on the device, through the
        // shard -> problem maps the plan cache's refresh uses too
        std::vector<int32_t> ps(h.n_spt);
        for (int64_t k = 0; k < h.n_spt; ++k) ps[k] = (int32_t)h.spt_global[k];
        up(pl->pt_src, ps, s);
        pl->src_off.alloc(prob.n_pt + 1);
        pl->src_off.upload(prob.pt_offsets, prob.n_pt + 1, s);
        pl->obs_src.alloc(h.n_sobs);
        DBuf<int32_t> gperm;   // back to the context's cache, stream-ordered
        if (!h.gobs_perm.empty()) up(gperm, h.gobs_perm, s);
        ba_obs_source(pl->pt_src.p, pl->src_off.p, pl->pt_off.p, (int32_t)h.n_spt, (int32_t)h.n_cpt,
                      h.gobs_perm.empty() ? nullptr : gperm.p, pl->obs_src.p, s);
        pl->raw_uv.alloc(2 * (size_t)prob.n_obs);
        SFM_HIP(hipMemcpyAsync(pl->raw_uv.p, prob.obs_uv, 2 * (size_t)prob.n_obs * 8, hipMemcpyHostToDevice, s));
        pl->obs_uv.alloc(2 * (size_t)h.n_sobs);
        ba_gather_uv(pl->obs_src.p, pl->raw_uv.p, (int32_t)h.n_sobs, pl->obs_uv.p, s);
        tm.mark("gather_uv");
    }
    Staging st;
    up(st, pl->chunks, h.chunks, s);
    up(st, pl->group_off, h.group_off, s);
    up(st, pl->img_obs_ptr, h.img_obs_ptr, s);
    if (!h.gram_img.empty()) up(st, pl->gram_img, h.gram_img, s);
    pl->img_pt.alloc(std::max<int64_t>(h.n_sobs, 1));
    pl->img_uv.alloc(2 * std::max<int64_t>(h.n_sobs, 1));
    ba_image_order(pl->obs_img.p, pl->obs_uv.p, pl->pt_off.p, (int32_t)h.n_sobs, (int32_t)h.n_spt, prob.n_img,
                   pl->img_pt.p, pl->img_uv.p, s);
    up(st, pl->img_colc, h.img_colc, s);
    up(st, pl->img_coli, h.img_coli, s);
    {
        std::vector<int32_t> ic(std::max(prob.n_intr, 1), -1);
        for (int q = 0; q < prob.n_intr; ++q)
            if (h.intr_blk[q] >= 0) ic[q] = (int32_t)(h.nb + (int64_t)h.iw * h.intr_blk[q]);
        up(st, pl->intr_col, ic, s);
    }
    up(st, pl->img_intr, h.img_intr, s);
    up(st, pl->blk_img, h.blk_img, s);
    up(st, pl->blk_intr, h.blk_intr, s);
    {   // images without camera columns (the gauge image, unobserved images)
        std::vector<int32_t> fr;
        for (int t = 0; t < prob.n_img; ++t)
            if (h.img_colc[t] < 0) fr.push_back(t);
        pl->P.n_free = (int32_t)fr.size();
        up(st, pl->free_img, fr, s);
    }
    if (h.zero_targets.empty()) {
        up(st, pl->targets, h.targets, s);
    } else {   // the zero list after the real targets, one buffer
        std::vector<ReduceTarget> all(h.targets);
        all.insert(all.end(), h.zero_targets.begin(), h.zero_targets.end());
        up(st, pl->targets, all, s);
    }
    up(st, pl->gblk_off, h.gblk_off, s);
    up(st, pl->gblk_col, h.gblk_col, s);
    up(st, pl->gblk_z, h.gblk_z, s);
    up(st, pl->gz_off, h.gz_off, s);
    up(st, pl->zbatch, h.zbatch, s);
    up(st, pl->zlong, h.zlong, s);
    up(pl->pterms, h.pterms, s);
    pl->Zbuf.alloc(h.n_z + 2);   // (+2: preduce's 16-byte pieces read one double past an odd block)
    HostVec<double> xs(3 * std::max<int64_t>(h.n_spt, 1));
    for (int64_t k = 0; k < h.n_spt; ++k)
        for (int a = 0; a < 3; ++a) xs[3 * k + a] = X[3 * h.spt_global[k] + a];
    up(pl->X0, xs, s);
    pl->Xa.alloc(xs.size());
    pl->Xb.alloc(xs.size());
    std::vector<double> e(extr, extr + 6 * (size_t)prob.n_img), in(intr, intr + (size_t)h.iw * prob.n_intr);
    up(st, pl->extr0, e, s);
    up(st, pl->intr0, in, s);
    pl->ea.alloc(e.size()); pl->eb.alloc(e.size());
    pl->ia.alloc(in.size()); pl->ib.alloc(in.size());
    pl->cpa.alloc(prob.n_img); pl->cpb.alloc(prob.n_img);
    const int64_t nF = std::max<int64_t>(h.nF, 1);
    pl->scaleE.alloc(xs.size());
    pl->scaleF.alloc(nF);
    // per-chunk Schur tiles and per-image Gram slices share one buffer so the
    // reduction terms address every source with a single offset
    const size_t n_tiles = std::max<size_t>(h.n_group(), 1) * kTileR * kTileR;
    const size_t fw = 6 + (size_t)h.iw;   // F columns of an image block
    const size_t o_u = n_tiles, o_ub = o_u + fw * fw * (size_t)prob.n_img * kGramSeg,
                 o_ucn = o_ub + fw * (size_t)prob.n_img * kGramSeg,
                 n_gram = o_ucn + fw * (size_t)prob.n_img * kGramSeg;
    pl->gram.alloc(n_gram);
    // the image blocks of images without observations in this shard are never
    // written (the Gram pass runs over the others) but may be reduce sources
    // (one rank: every image's U terms): zero once, they stay zero
    SFM_HIP(hipMemsetAsync(pl->gram.p + o_u, 0, (n_gram - o_u) * sizeof(double), s));
    // the terms arrive resolved against this buffer (build_plan, same layout)
    up(pl->terms, h.terms, s);
    // RCS: band + arrow + corner, or dense; the parts of a dense S no target
    // writes stay zero from here on
    pl->rcs_n = h.n_sband + h.n_sarrow + h.n_scorner + h.n_sdense + 3 * h.nF + 1;
    pl->rcs.alloc(pl->rcs_n);
    pl->rcs.zero(s);
    const int Dp = h.D + 1;
    if (!h.dense) {
        pl->Lcol.alloc(std::max<size_t>((size_t)h.ncam * Dp * 36, 1));
        pl->Larrow.alloc(std::max<size_t>((size_t)h.ncam * h.nintr * 24, 1));
    }
    pl->zF.alloc(nF);
    pl->yF.alloc(nF);
    pl->part_u.alloc(2 * (size_t)prob.n_img * kGramSeg);
    pl->part_u.zero(s);   // the slots of images without observations stay zero (no Gram workgroup)
    pl->part_s.alloc(2 * std::max<size_t>(h.chunks.size() + h.n_gpt, 1));
    pl->scal.alloc(kScCount);
    pl->scal.zero(s);
    if (ctx->comm) {
        pl->scal_g.alloc((size_t)ctx->world * kScMaxEnd);
    }
    pl->scal_h = static_cast<double*>(pinned_alloc((kScCount + 1) * sizeof(double)));
    std::memset(pl->scal_h, 0, (kScCount + 1) * sizeof(double));
    SFM_HIP(hipHostGetDevicePointer((void**)&pl->scal_dev, pl->scal_h, 0));

    DevProblem& P = pl->P;
    P.n_img = prob.n_img; P.n_intr = prob.n_intr;
    P.n_spt = (int32_t)h.n_spt; P.n_sobs = (int32_t)h.n_sobs;
    P.n_chunk = (int32_t)h.chunks.size();
    P.gram_seg = h.gram_seg;
    P.chunk_pts_max = 0;
    for (const ChunkDesc& c : h.chunks) P.chunk_pts_max = std::max(P.chunk_pts_max, c.pt_end - c.pt_begin);
    {
        // step_kernel lanes per point: two (profiles/r04/l_split: C4 1062-1067
        // / 1076-1078 LM-iters/s with 1 / 2, rank 0 of N = 8 2145-2148 / 2191-
        // 2198 / 2175-2177 / 2128 with 1 / 2 / 4 / 8; adjacent lanes read
        // adjacent observations).  SFM_CTX_BA_STEP_LANES overrides (A/B,
        // tests); the longest chunk must fit the kernel's 256 threads
        int sp = ctx->step_lanes() ? ctx->step_lanes() : 2;
        while (sp > 1 && P.chunk_pts_max * sp > 256) sp /= 2;
        P.step_split = sp;
    }
    P.n_group = (int32_t)h.n_group();
    P.n_cpt = (int32_t)h.n_cpt; P.n_gpt = (int32_t)h.n_gpt;
    P.gz_max = (int32_t)h.gz_max;
    P.dense = h.dense ? 1 : 0;
    P.gblk_off = pl->gblk_off.p; P.gblk_col = pl->gblk_col.p; P.gblk_z = pl->gblk_z.p;
    P.gz_off = pl->gz_off.p; P.pterms = pl->pterms.p; P.Z = pl->Zbuf.p;
    P.zbatch = pl->zbatch.p; P.n_zbatch = (int32_t)(h.zbatch.size() / 2);
    P.zlong = pl->zlong.p; P.n_zlong = (int32_t)h.zlong.size();
    P.tile_nt = h.tile_nt;
    P.ncam = h.ncam; P.nintr = h.nintr; P.D = h.D;
    P.nb = h.nb; P.nF = h.nF;
    P.huber_a = prob.huber_a;
    P.cam_model = prob.camera_model;
    P.iw = h.iw;
    P.pt_off = pl->pt_off.p; P.obs_img = pl->obs_img.p;
    P.obs_slot = pl->obs_slot.p; P.obs_uv = pl->obs_uv.p; P.chunks = pl->chunks.p;
    P.group_off = pl->group_off.p;
    P.img_obs_ptr = pl->img_obs_ptr.p;
    P.gram_img = pl->gram_img.p; P.n_gram_img = (int32_t)h.gram_img.size();
    P.img_pt = pl->img_pt.p; P.img_uv = pl->img_uv.p;
    P.img_colc = pl->img_colc.p; P.img_coli = pl->img_coli.p; P.img_intr = pl->img_intr.p;
    P.intr_col = pl->intr_col.p;
    P.blk_img = pl->blk_img.p;
    P.free_img = pl->free_img.p;
    P.targets = pl->targets.p; P.terms = pl->terms.p; P.n_targets = (int32_t)h.targets.size();
    P.n_zero = (int32_t)h.zero_targets.size();
    {
        // reduce_kernel waves per target from the mean term count of the
        // targets it sums: C4 24 at N = 1, 50 at N = 4, 92 at N = 8
        // (profiles/r04/m_redw: N = 1 1072 / 1063 / 1046 LM-iters/s with 1 / 2
        // / 4 waves, rank 0 of N = 8 2123-2132 / 2215-2226 / 2244-2245;
        // SFM_CTX_BA_REDUCE_WAVES overrides: A/B, tests)
        int64_t nt = 0, nterm = 0;
        for (const ReduceTarget& T : h.targets) {
            const int32_t n = T.c_end - T.c_begin;
            if (n <= reduce_long_threshold()) { ++nt; nterm += n; }
        }
        const int64_t mean = nt > 0 ? nterm / nt : 0;
        P.red_waves = ctx->reduce_waves() ? ctx->reduce_waves() : mean >= 80 ? 4 : mean >= 40 ? 2 : 1;
        P.red_split = (ctx->flags & SFM_CTX_BA_SPLIT_REDUCE) ? 1 : 0;
    }
    {
        // long targets: [n_long targets | n_long+1 segment offsets | n_seg (long idx, term begin)]
        std::vector<int32_t> lt, off{0}, seg;
        for (size_t t = 0; t < h.targets.size(); ++t) {
            const int32_t b0 = h.targets[t].c_begin, n = h.targets[t].c_end - b0;
            if (n <= reduce_long_threshold()) continue;
            for (int32_t k = 0; k < n; k += kReduceSeg) {
                seg.push_back((int32_t)lt.size());
                seg.push_back(b0 + k);
            }
            lt.push_back((int32_t)t);
            off.push_back((int32_t)(seg.size() / 2));
        }
        P.n_long = (int32_t)lt.size();
        P.n_lseg = (int32_t)(seg.size() / 2);
        std::vector<int32_t> all(lt);
        all.insert(all.end(), off.begin(), off.end());
        all.insert(all.end(), seg.begin(), seg.end());
        up(st, pl->long_targets, all, s);
        P.long_targets = pl->long_targets.p;
        P.lseg_off = P.long_targets + P.n_long;
        P.lseg = P.lseg_off + P.n_long + 1;
        pl->lpart.alloc(36 * std::max<size_t>(P.n_lseg, 1));
        P.lpart = pl->lpart.p;
        pl->lcount.alloc(std::max<size_t>(P.n_long, 1));
        pl->lcount.zero(s);
        P.lcount = pl->lcount.p;
    }
    {
        // the same for long product-term lists (general points)
        std::vector<int32_t> lt, off{0}, seg;
        for (size_t t = 0; t < h.targets.size(); ++t) {
            const int32_t b0 = h.targets[t].p_begin, n = h.targets[t].p_end - b0;
            if (n <= preduce_long_threshold()) continue;
            for (int32_t k = 0; k < n; k += kReduceSeg) {
                seg.push_back((int32_t)lt.size());
                seg.push_back(b0 + k);
            }
            lt.push_back((int32_t)t);
            off.push_back((int32_t)(seg.size() / 2));
        }
        P.n_plong = (int32_t)lt.size();
        P.n_plseg = (int32_t)(seg.size() / 2);
        std::vector<int32_t> all(lt);
        all.insert(all.end(), off.begin(), off.end());
        all.insert(all.end(), seg.begin(), seg.end());
        up(st, pl->plong_targets, all, s);
        P.plong_targets = pl->plong_targets.p;
        P.plseg_off = P.plong_targets + P.n_plong;
        P.plseg = P.plseg_off + P.n_plong + 1;
        pl->plpart.alloc(36 * std::max<size_t>(P.n_plseg, 1));
        P.plpart = pl->plpart.p;
    }
    P.scaleE = pl->scaleE.p; P.scaleF = pl->scaleF.p; P.tiles = pl->gram.p;
    P.U = P.tiles + o_u; P.Ub = P.tiles + o_ub; P.Ucn = P.tiles + o_ucn;
    P.src = pl->gram.p;
    P.Sband = pl->rcs.p;
    P.Sarrow = P.Sband + h.n_sband;
    P.Scorner = P.Sarrow + h.n_sarrow;
    P.Sdense = P.Scorner + h.n_scorner;
    P.rhs = P.Sdense + h.n_sdense;
    P.bF = P.rhs + h.nF;
    P.cnF = P.bF + h.nF;
    P.Lcol = pl->Lcol.p; P.Larrow = pl->Larrow.p; P.zF = pl->zF.p; P.yF = pl->yF.p;
    if (!h.dense) {
        bool lds = true;
        solve_lds_bytes(P, &lds);
        if (!lds) pl->Wg.alloc(solve_window_doubles(P));
    }
    P.Wglobal = pl->Wg.p;
    P.part_u = pl->part_u.p; P.part_s = pl->part_s.p;
    pl->part_t.alloc((size_t)kPartT * std::max(ba_step_blocks(P), 1));
    P.part_t = pl->part_t.p;
    P.scal = pl->scal.p;
    pl->fin_part.alloc(16 * 12);
    pl->fin_count.alloc(1);
    pl->fin_count.zero(s);
    P.fin_part = pl->fin_part.p;
    P.fin_count = pl->fin_count.p;
    // (SFM_CTX_BA_SEQ_BAND: the sequential band solver, 4-wide intrinsics arrows only)
    pl->use_bcr = !h.dense && bcr_supported(P) && (!(ctx->flags & SFM_CTX_BA_SEQ_BAND) || P.iw != 4);
    SFM_REQUIRE(h.dense || pl->use_bcr || P.iw == 4, SFM_ERR_UNSUPPORTED, "band solver: 4-wide intrinsics only");
    if (h.dense) {
        dense_setup(pl->dense, P);
        pl->dense.chain = (ctx->flags & SFM_CTX_BA_DENSE_CHAIN) != 0;
        // (the exact tile pattern needs every block's target: one rank lists
        // only the blocks its shard touches, so a multi-rank plan keeps the
        // structural pattern -- every rank then plans the same schedule)
        const std::vector<char> exact =
            ctx->world == 1 ? dense_tile_pattern(h.targets, P.nF, pl->dense.nt) : std::vector<char>();
        pl->dense_meta = dense_flow_plan(pl->dense, P, exact.empty() ? nullptr : &exact);   // the dataflow solve's schedule (host)
        pl->dense_buf.alloc(dense_doubles(pl->dense));
        dense_bind(pl->dense, pl->dense_buf.p);
        // failure words, tickets, flags and granules: zeroed once (the dataflow
        // solve clears its failure words itself after each verdict)
        SFM_HIP(hipMemsetAsync(pl->dense.fail, 0, 8 * sizeof(double) + sizeof(unsigned) * dense_flag_words(pl->dense), s));
        if (!pl->dense_meta.empty())
            SFM_HIP(hipMemcpyAsync(const_cast<int32_t*>(pl->dense.meta), pl->dense_meta.data(),
                                   pl->dense_meta.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
        if (std::getenv("SFM_DENSE_STAMPS")) {
            pl->bcr_stamps.alloc(32);   // chain phases [0, 8), chol_inv64's [8, 24), real time [24, 28)
            pl->bcr_stamps.zero(s);
            pl->dense.stamps = pl->bcr_stamps.p;
        }
    }
    // candidate partials: the BCR back substitution forms them per super-block
    // (+ one slot for the intrinsics), the other solvers through cand_kernel
    if (pl->use_bcr) {
        BcrArgs tmp;
        bcr_setup(tmp, P);
        P.n_fblk = tmp.N + 1;
    } else {
        P.n_fblk = ba_cand_blocks(P);
    }
    pl->part_f.alloc(3 * (size_t)P.n_fblk);
    P.part_f = pl->part_f.p;
    if (pl->use_bcr) {
        bcr_setup(pl->bcr, P);
        pl->bcr.split = (ctx->flags & SFM_CTX_BA_SPLIT_BCR) != 0;
        pl->bcr_buf.alloc(bcr_doubles(pl->bcr));
        bcr_bind(pl->bcr, pl->bcr_buf.p);
        // failure words, counters and y flags: zeroed once (each solve's last
        // kernels reset what they used)
        SFM_HIP(hipMemsetAsync(pl->bcr.fail, 0, 8 * sizeof(double) + sizeof(unsigned) * (size_t)pl->bcr.N, s));
        // the back substitution's tagged y granules (tags = solve epochs from 1)
        SFM_HIP(hipMemsetAsync(pl->bcr.Y, 0, sizeof(double) * bcr_y_granules(pl->bcr), s));
        // the fused top's tagged corner sums (slot N of the partials; tags = solve epochs from 1)
        SFM_HIP(hipMemsetAsync(pl->bcr.part + (size_t)pl->bcr.N * 512, 0, 512 * sizeof(double), s));
        if (std::getenv("SFM_BCR_STAMPS")) {
            pl->bcr_stamps.alloc(16);
            pl->bcr_stamps.zero(s);
            pl->bcr.stamps = pl->bcr_stamps.p;
        }
    }
    if (std::getenv("SFM_SCHUR_STAMPS")) pl->stamps.alloc(6 * std::max<size_t>(h.chunks.size(), 1));
    tm.mark("alloc+upload");
    SFM_HIP(hipStreamSynchronize(s));
    // the observation staging goes back to the cache (the uploads are done);
    // a plan that can seed a grown one keeps its shard arrays (obs_img,
    // obs_slot and the reduce plan's terms: build_plan_grown takes their
    // unchanged prefix)
    if (!(h.grow.ok && cache_enabled_for_growth())) {
        h.obs_img = HostVec<int32_t>();
        h.obs_slot = HostVec<int32_t>();
        h.pterms = HostVec<PTerm>();
        h.terms = HostVec<FlatTerm>();
        h.grow = PlanGrowState();
    }
    h.obs_uv = HostVec<double>();
    tm.mark("sync");
    return true;
}

// New values for a plan whose problem structure is unchanged (the plan
// cache of sfm_ba_solve): measurements, points, poses and intrinsics are
// uploaded as the caller holds them and gathered into the plan's shard order
// on the device; the image-ordered copy is rebuilt.  Everything structural
// (order, chunks, reduce plan, RCS layout) is kept.
void refresh_values(sfm_ba_plan* pl, const sfm_ba_problem& prob, const double* extr, const double* intr,
                    const double* X) {
    sfm_ctx* ctx = pl->ctx;
    hipStream_t s = ctx->stream;
    BAHostPlan& h = pl->hp;
    PhaseTimer tm("refresh_values");
    if (!pl->obs_src.p && h.n_sobs > 0) {
        std::vector<int32_t> ps(h.n_spt);
        for (int64_t k = 0; k < h.n_spt; ++k) ps[k] = (int32_t)h.spt_global[k];
        up(pl->pt_src, ps, s);
        pl->src_off.alloc(prob.n_pt + 1);
        pl->src_off.upload(prob.pt_offsets, prob.n_pt + 1, s);
        pl->obs_src.alloc(h.n_sobs);
        DBuf<int32_t> gperm;   // back to the context's cache, stream-ordered
        if (!h.gobs_perm.empty()) up(gperm, h.gobs_perm, s);
        ba_obs_source(pl->pt_src.p, pl->src_off.p, pl->pt_off.p, (int32_t)h.n_spt, (int32_t)h.n_cpt,
                      h.gobs_perm.empty() ? nullptr : gperm.p, pl->obs_src.p, s);
        tm.mark("maps");
    }
    if (h.n_sobs > 0) {
        if (pl->raw_uv.n < 2 * (size_t)prob.n_obs) pl->raw_uv.alloc(2 * (size_t)prob.n_obs);
        SFM_HIP(hipMemcpyAsync(pl->raw_uv.p, prob.obs_uv, 2 * (size_t)prob.n_obs * 8, hipMemcpyHostToDevice, s));
        ba_gather_uv(pl->obs_src.p, pl->raw_uv.p, (int32_t)h.n_sobs, pl->obs_uv.p, s);
        ba_image_order(pl->obs_img.p, pl->obs_uv.p, pl->pt_off.p, (int32_t)h.n_sobs, (int32_t)h.n_spt, prob.n_img,
                       pl->img_pt.p, pl->img_uv.p, s);
    }
    if (h.n_spt > 0) {
        if (pl->raw_X.n < 3 * (size_t)prob.n_pt) pl->raw_X.alloc(3 * (size_t)prob.n_pt);
        SFM_HIP(hipMemcpyAsync(pl->raw_X.p, X, 3 * (size_t)prob.n_pt * 8, hipMemcpyHostToDevice, s));
        ba_gather_points(pl->pt_src.p, pl->raw_X.p, (int32_t)h.n_spt, pl->X0.p, s);
    }
    SFM_HIP(hipMemcpyAsync(pl->extr0.p, extr, 6 * (size_t)prob.n_img * 8, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(pl->intr0.p, intr, (size_t)h.iw * prob.n_intr * 8, hipMemcpyHostToDevice, s));
    pl->P.huber_a = prob.huber_a;
    tm.mark("upload+gather");
}

// Wait for finalize_kernel's publish of the iteration scalars (sequence word
// after the values, system-scope release): a host spin on pinned memory
// instead of a blit + stream synchronisation per LM iteration.  A long wait
// falls back to the stream synchronisation, which also reports a failed launch.
void wait_scalars(const double* host, unsigned long long seq, hipStream_t s) {
    const auto* word = reinterpret_cast<const unsigned long long*>(host + kScCount);
    auto published = [&] { return __atomic_load_n(word, __ATOMIC_ACQUIRE) == seq; };
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spins = 0; !published(); ++spins) {
        __builtin_ia32_pause();
        if ((spins & 1023) == 1023 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) {
            SFM_HIP(hipStreamSynchronize(s));
            SFM_REQUIRE(published(), SFM_ERR_DEVICE, "iteration scalars were not published");
            break;
        }
    }
}

struct IterState {
    double* X; double* Xc; double* e; double* ec; double* in; double* inc; CamPre* cp; CamPre* cpc;
};

int run_plan(sfm_ba_plan* pl, const sfm_ba_options& O, sfm_ba_summary* sum) {
    sfm_ctx* ctx = pl->ctx;
    hipStream_t s = ctx->stream;
    BAHostPlan& h = pl->hp;
    DevProblem& P = pl->P;
    P.min_diag = O.min_lm_diagonal;
    P.max_diag = O.max_lm_diagonal;
    P.lm_min_rel = O.min_relative_decrease;
    P.lm_ftol = O.function_tolerance;
    P.lm_ptol = O.parameter_tolerance;
    const auto t0 = std::chrono::steady_clock::now();
    std::memset(sum, 0, sizeof *sum);
    sum->num_residuals = 2 * h.n_obs;
    pl->trace.clear();
    pl->schur_ms_total = 0;
    pl->schur_launches = 0;

    // working buffers: a = current point, b = candidate
    IterState S{pl->Xa.p, pl->Xb.p, pl->ea.p, pl->eb.p, pl->ia.p, pl->ib.p, pl->cpa.p, pl->cpb.p};
    const size_t ne = 6 * (size_t)h.n_img, ni = (size_t)h.iw * h.n_intr, nx = 3 * (size_t)h.n_spt;
    // the working point from the plan's initial values, and the unit column
    // scales of the unscaled iteration-0 pass, in one launch (three blits and
    // two fills were five launches and, at a shard's size, host-bound gaps
    // between them)
    {
        SegList L;
        L.add(S.X, pl->X0.p, (int64_t)nx);
        L.add(S.e, pl->extr0.p, (int64_t)ne);
        L.add(S.in, pl->intr0.p, (int64_t)ni);
        L.add(pl->scaleF.p, nullptr, std::max<int64_t>(h.nF, 1), 1.0);
        L.add(pl->scaleE.p, nullptr, (int64_t)nx, 1.0);
        ba_segs(L, s);
    }

    auto allreduce_rcs = [&] {
        ctx_allreduce(ctx, pl->rcs.p, pl->rcs_n, 0, s);
    };
    auto relinearize = [&] {
        ba_image_gram(P, S.cp, S.in, S.X, s);
    };
    // ---- iteration zero: Jacobi scaling from the corrected Jacobian at x0 ----
    ba_campre(S.e, h.n_img, S.cp, s);
    if (O.jacobi_scaling) {
        relinearize();                 // unscaled column norms of the F blocks
        if (ctx->world > 1 && h.dense)
            ba_fill(pl->rcs.p, (int64_t)pl->rcs_n, 0.0, s);   // dense: its targets are this shard's blocks only
        ba_reduce(P, true, s);
        allreduce_rcs();
        ba_fscale(P, s);
        ba_gram_rescale(P, s);         // = relinearize() at the new scales
        // the point scales come from the first Schur pass (schur_kernel<SE>)
    } else {
        relinearize();
    }

    // one rank: the scalars come back through host-mapped memory (wait_scalars);
    // several: the device all-gather / host all-reduce below
    // (with an RCCL communicator, even a 1-rank one, the scalars go through
    // the all-gather and publish_gathered_kernel instead)
    P.scal_host = (!ctx->comm && (ctx->world == 1 || ctx->no_exchange)) ? pl->scal_dev : nullptr;
    // Speculative Gram pass (round 5): where the device combines the scalars
    // (finalize_kernel at one rank, publish_gathered_kernel over RCCL) it
    // also takes the host's accept decision (lm_spec_accept), and the Gram
    // pass at the candidate is launched right behind it, gated on that flag --
    // so after an accepted step the pass runs while the host polls and
    // decides, instead of after (the host-to-launch gap was 8 us at rank 0 of
    // N = 8 and 16 us at C4 per accepted step, profiles/r05/*/iter_gaps_*).
    // The host compares the flag with its own decision: it runs the pass if
    // the device skipped it, and redoes it at the current point if the device
    // ran it for a step the host rejects, so no result depends on the flag.
    const bool spec_gram = !(ctx->flags & SFM_CTX_BA_NO_SPEC_GRAM) &&
                           (P.scal_host != nullptr || (ctx->comm && !ctx->host_allreduce));
    P.spec_force = (ctx->flags & SFM_CTX_DIAG_SPEC_ALWAYS) ? 1 : 0;
    double radius = O.initial_trust_region_radius, decrease_factor = 2.0;
    int consecutive_invalid = 0;
    double x_cost = 0.0, x_norm = 0.0;
    bool relin_pending = true;   // Finalize of iteration 0 / of an accepted step pending
    sfm_ba_iter pending{};
    pending.iteration = 0; pending.step_is_valid = 1; pending.step_is_successful = 1;
    int term = -1;
    hipEvent_t* ev = ctx_events(ctx);   // the Schur launch timing of steps 1 and 2
    int last_iter = 0;

    auto finalize = [&](const sfm_ba_iter& cur, double gmax) -> int {
        pl->trace.push_back(cur);
        last_iter = cur.iteration;
        if (cur.step_is_successful) sum->successful_steps++; else sum->unsuccessful_steps++;
        if (cur.iteration >= O.max_num_iterations) return SFM_TERM_NO_CONVERGENCE;
        if (gmax <= O.gradient_tolerance) return SFM_TERM_CONVERGENCE;
        if (radius < O.min_trust_region_radius) return SFM_TERM_CONVERGENCE;
        return -1;
    };

    double prev_gmax = 0.0;
    int step_no = 0;
    // SFM_SCHUR_TIME_ALL (measurement): time every Schur launch after the first
    const bool time_all = std::getenv("SFM_SCHUR_TIME_ALL") != nullptr;
    while (term < 0) {
        // ---- one step on the device ------------------------------------------
        // the Schur launch is timed with events only on request
        // (SFM_SCHUR_TIME_ALL, measurement: every launch but the first, which
        // also forms the point scales): an event pair costs ~12 us of stream
        // serialisation, which an untimed solve should not pay
        const bool first = step_no == 0;
        const bool timed = time_all && step_no >= 1;
        ++step_no;
        if (timed) SFM_HIP(hipEventRecord(ev[0], s));
        ba_schur(P, S.cp, S.in, S.X, radius, s, pl->stamps.p, O.jacobi_scaling && first);
        if (timed) SFM_HIP(hipEventRecord(ev[1], s));
        // across ranks each shard writes only the blocks its own points touch,
        // so the summed system of the last iteration is cleared first
        if (ctx->world > 1 && h.dense)
            ba_fill(pl->rcs.p, (int64_t)pl->rcs_n, 0.0, s);   // dense: its targets are this shard's blocks only
        ba_reduce(P, false, s);
        allreduce_rcs();
        if (P.dense) dense_solve(pl->dense, P, radius, s, ++pl->bcr_epoch);
        else if (pl->use_bcr)   // (the candidates: formed by its back substitution)
            bcr_solve(pl->bcr, P, radius, s, ++pl->bcr_epoch, BcrCand{S.e, S.in, S.ec, S.inc, S.cpc});
        else ba_solve(P, radius, s);
        if (ctx->fail_solve_wait) ba_fill(P.scal + kScSolveFail, 1, kSolveWaitTimeout, s);   // diagnostic
        if (!pl->use_bcr) ba_cand(P, S.e, S.in, S.ec, S.inc, S.cpc, s);
        ba_step(P, S.cp, S.in, S.cpc, S.inc, S.X, S.Xc, radius, s);
        const unsigned long long seq = ++pl->fin_seq;
        ba_finalize(P, s, seq);
        if (P.scal_host) {
            if (spec_gram) ba_image_gram(P, S.cpc, S.inc, S.Xc, s, P.scal + kScAccept);
            wait_scalars(pl->scal_h, seq, s);
        } else if (ctx->comm && !ctx->host_allreduce) {
            // one RCCL collective: gather every rank's partial scalars; a
            // one-wave kernel sums (rank order) / maxes them and publishes to
            // host-mapped memory, polled as at one rank (no copy, no sync)
            SFM_REQUIRE(rccl_allgather_f64(ctx->comm, P.scal, pl->scal_g.p, kScMaxEnd, s) == 0, SFM_ERR_COMM,
                        "RCCL all-gather failed");
            ba_publish_gathered(P, pl->scal_g.p, ctx->world, P.scal, pl->scal_dev, s, seq);
            if (spec_gram) ba_image_gram(P, S.cpc, S.inc, S.Xc, s, P.scal + kScAccept);
            wait_scalars(pl->scal_h, seq, s);
        } else {
            if (ctx->world > 1) {
                ctx_allreduce(ctx, P.scal + kScSumBegin, kScSumEnd - kScSumBegin, 0, s);
                ctx_allreduce(ctx, P.scal + kScMaxBegin, kScMaxEnd - kScMaxBegin, 1, s);
            }
            SFM_HIP(hipMemcpyAsync(pl->scal_h, P.scal, kScCount * 8, hipMemcpyDeviceToHost, s));
            SFM_HIP(hipStreamSynchronize(s));
        }
        if (timed) {
            SFM_HIP(hipEventSynchronize(ev[1]));
            float ms = 0.f;
            SFM_HIP(hipEventElapsedTime(&ms, ev[0], ev[1]));
            pl->schur_ms_total += ms;
            pl->schur_launches++;
            pl->last_ms[0] = ms;
        }
        const double* sc = pl->scal_h;
        // the speculative pass at the candidate ran (spec_gram and the device accepted)
        const bool spec_ran = spec_gram && sc[kScAccept] != 0.0;

        // ---- Finalize of the previous accepted iteration (needs g, x at x) ----
        if (relin_pending) {
            relin_pending = false;
            x_cost = sc[kScCost];
            if (pending.iteration == 0) {
                sum->initial_cost = x_cost;
                if (sc[kScBadX] != 0.0 || !std::isfinite(x_cost)) {
                    term = SFM_TERM_FAILURE;
                    sum->termination = term;
                    set_error("residual evaluation at the initial point is not finite");
                    sum->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                    return SFM_ERR_NOT_FINITE;
                }
            }
            x_norm = std::sqrt(sc[kScXnorm2E] + sc[kScXnorm2F]);
            pending.cost = x_cost;
            pending.gradient_max_norm = std::max(sc[kScGmaxE], sc[kScGmaxF]);
            pending.trust_region_radius = radius;
            prev_gmax = pending.gradient_max_norm;
            term = finalize(pending, pending.gradient_max_norm);
            if (term >= 0) break;
        }

        // ---- this iteration -----------------------------------------------------
        sfm_ba_iter cur{};
        cur.iteration = last_iter + 1;
        const double model_change = -sc[kScModelAcc];
        cur.model_cost_change = model_change;
        SFM_REQUIRE(sc[kScSolveFail] != kSolveWaitTimeout, SFM_ERR_DEVICE,
                    "RCS solve: a dataflow wait timed out (workgroups not co-resident; another context holding the CUs?)");
        const bool finite = sc[kScSolveFail] == 0.0 && sc[kScStepBad] == 0.0 && std::isfinite(model_change);
        cur.step_is_valid = finite && model_change > 0.0;
        if (!cur.step_is_valid) {
            if (++consecutive_invalid >= O.max_num_consecutive_invalid_steps) { term = SFM_TERM_FAILURE; break; }
            if (spec_ran) relinearize();   // (the device's copy of the decision differed: U back at x)
            radius = radius / decrease_factor;
            decrease_factor *= 2.0;
            cur.cost = x_cost;
            cur.gradient_max_norm = prev_gmax;
            cur.trust_region_radius = radius;
            term = finalize(cur, prev_gmax);
            continue;
        }
        consecutive_invalid = 0;
        const double cand_cost = sc[kScCandBad] != 0.0 ? std::numeric_limits<double>::max() : sc[kScCandCost];
        cur.step_norm = std::sqrt(sc[kScStepnorm2E] + sc[kScStepnorm2F]);
        if (cur.step_norm <= O.parameter_tolerance * (x_norm + O.parameter_tolerance)) { term = SFM_TERM_CONVERGENCE; break; }
        cur.cost_change = x_cost - cand_cost;
        if (std::fabs(cur.cost_change) <= O.function_tolerance * x_cost) { term = SFM_TERM_CONVERGENCE; break; }
        cur.relative_decrease = cand_cost >= std::numeric_limits<double>::max()
                                    ? std::numeric_limits<double>::lowest()
                                    : (x_cost - cand_cost) / model_change;
        if (cur.relative_decrease > O.min_relative_decrease) {
            std::swap(S.X, S.Xc); std::swap(S.e, S.ec); std::swap(S.in, S.inc); std::swap(S.cp, S.cpc);
            cur.step_is_successful = 1;
            const double q = cur.relative_decrease;
            radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * q - 1.0, 3));
            radius = std::min(O.max_trust_region_radius, radius);
            decrease_factor = 2.0;
            if (!spec_ran) relinearize();   // (else already run at the candidate, now the current point)
            relin_pending = true;
            pending = cur;
            continue;   // Finalize after the gradient at the new x is known
        }
        cur.step_is_successful = 0;
        if (spec_ran) relinearize();   // (the device's copy of the decision differed: U back at x)
        cur.cost = cand_cost;
        cur.gradient_max_norm = prev_gmax;
        radius = radius / decrease_factor;
        decrease_factor *= 2.0;
        cur.trust_region_radius = radius;
        term = finalize(cur, prev_gmax);
    }
    if (pl->bcr.stamps) {  // diagnostic: average cycles per odd block, all levels
        unsigned long long st[16];
        SFM_HIP(hipMemcpy(st, pl->bcr.stamps, sizeof st, hipMemcpyDeviceToHost));
        const double n = st[4] ? (double)st[4] : 1.0;
        std::fprintf(stderr, "[bcr stamps] cycles/odd block: loads %.0f load+update %.0f chol %.0f (diag16 %.0f, "
                     "pivots alone %.0f) to X copy %.0f total %.0f over %llu; windows 0..3 pivot wave %.0f %.0f %.0f "
                     "%.0f, slowest helper %.0f %.0f %.0f %.0f\n",
                     st[5] / n, st[2] / n, st[1] / n, st[0] / n, st[7] / n, st[6] / n, st[3] / n, st[4],
                     st[12] / n, st[13] / n, st[14] / n, st[15] / n, st[8] / n, st[9] / n, st[10] / n, st[11] / n);
    }
    if (pl->dense.stamps) {  // diagnostic: dataflow chain, average cycles per block column
        unsigned long long st[32];
        SFM_HIP(hipMemcpy(st, pl->dense.stamps, sizeof st, hipMemcpyDeviceToHost));
        const double n = st[6] ? (double)st[6] : 1.0, ns = st[27] ? (double)st[27] : 1.0;
        std::fprintf(stderr, "[dense stamps] cycles/column: wait S+D %.0f  L + X out %.0f  update %.0f  sync %.0f  "
                     "factor %.0f (diag16 %.0f, pivots %.0f)  last X %.0f  over %llu columns; per solve: chain "
                     "%.2f us, chain end to x_0 %.2f us over %llu solves\n",
                     st[0] / n, st[1] / n, st[2] / n, st[3] / n, st[4] / n, st[8] / n, st[15] / n, st[5] / n, st[6],
                     st[24] / ns / 100.0, st[25] / ns / 100.0, st[27]);
    }
    if (pl->stamps.p) {  // diagnostic: average phase cycles per chunk (last Schur launch)
        std::vector<unsigned long long> st(pl->stamps.n);
        SFM_HIP(hipMemcpy(st.data(), pl->stamps.p, st.size() * 8, hipMemcpyDeviceToHost));
        double avg[6] = {0};
        for (size_t c = 0; c < h.chunks.size(); ++c)
            for (int k = 0; k < 6; ++k) avg[k] += (double)st[6 * c + k] / h.chunks.size();
        std::fprintf(stderr, "[schur stamps] cycles/chunk zero %.0f A %.0f B %.0f C %.0f D %.0f tail %.0f\n",
                     avg[0], avg[1], avg[2], avg[3], avg[4], avg[5]);
    }
    pl->cur_is_a = S.X == pl->Xa.p;   // download() reads whichever set is current
    sum->termination = term;
    sum->usable = term != SFM_TERM_FAILURE;
    sum->iterations = pl->trace.empty() ? 0 : pl->trace.back().iteration;
    sum->final_cost = sum->initial_cost;
    for (const auto& it : pl->trace)
        if (it.step_is_successful) sum->final_cost = std::min(sum->final_cost, it.cost);
    sum->rmse_initial = sum->num_residuals ? std::sqrt(sum->initial_cost / sum->num_residuals) : 0.0;
    sum->rmse_final = sum->num_residuals ? std::sqrt(sum->final_cost / sum->num_residuals) : 0.0;
    sum->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (term == SFM_TERM_FAILURE) set_error("bundle adjustment failed (solution not usable)");
    return term == SFM_TERM_FAILURE ? SFM_ERR_SOLVER : SFM_OK;
}

void download(sfm_ba_plan* pl, double* extr, double* intr, double* X) {
    hipStream_t s = pl->ctx->stream;
    const BAHostPlan& h = pl->hp;
    const double* e = pl->cur_is_a ? pl->ea.p : pl->eb.p;
    const double* in = pl->cur_is_a ? pl->ia.p : pl->ib.p;
    const double* x = pl->cur_is_a ? pl->Xa.p : pl->Xb.p;
    if (extr) SFM_HIP(hipMemcpyAsync(extr, e, 6 * (size_t)h.n_img * 8, hipMemcpyDeviceToHost, s));
    if (intr) SFM_HIP(hipMemcpyAsync(intr, in, (size_t)h.iw * h.n_intr * 8, hipMemcpyDeviceToHost, s));
    // (page-locked, cached staging: a DMA, and no page faults on a fresh
    // vector per call -- the incremental loop downloads after every solve)
    HostVec<double> xs(3 * (size_t)h.n_spt);
    if (X && h.n_spt) SFM_HIP(hipMemcpyAsync(xs.data(), x, xs.size() * 8, hipMemcpyDeviceToHost, s));
    SFM_HIP(hipStreamSynchronize(s));
    if (X) {
        const int64_t n = h.n_spt;
        const int nt = n < 16384 ? 1 : std::min<int>(8, (int)(n / 8192));
        auto part = [&](int t) {
            for (int64_t k = n * t / nt; k < n * (t + 1) / nt; ++k)
                for (int a = 0; a < 3; ++a) X[3 * h.spt_global[k] + a] = xs[3 * k + a];
        };
        if (nt == 1) part(0);
        else PlanPool::get().run(nt, part);
    }
}

}  // namespace

extern "C" void sfm_ba_default_options(sfm_ba_options* o) {
    if (!o) return;
    std::memset(o, 0, sizeof *o);
    o->max_num_iterations = 50;
    o->max_num_consecutive_invalid_steps = 5;
    o->jacobi_scaling = 1;
    o->function_tolerance = 1e-6;
    o->gradient_tolerance = 1e-10;
    o->parameter_tolerance = 1e-8;
    o->initial_trust_region_radius = 1e4;
    o->max_trust_region_radius = 1e16;
    o->min_trust_region_radius = 1e-32;
    o->min_relative_decrease = 1e-3;
    o->min_lm_diagonal = 1e-6;
    o->max_lm_diagonal = 1e32;
}

extern "C" int sfm_ba_plan_create(sfm_ctx* ctx, const sfm_ba_problem* prob, const double* extr,
                                  const double* intr, const double* X, sfm_ba_plan** out) {
    return guarded([&] {
        SFM_REQUIRE(ctx && prob && extr && intr && (X || prob->n_pt == 0) && out, SFM_ERR_INVALID_ARG,
                    "null argument");
        CtxScope scope_(ctx);
        auto* pl = new sfm_ba_plan;
        pl->ctx = ctx;
        try {
            create_plan(pl, *prob, extr, intr, X);
        } catch (...) {
            delete pl;
            throw;
        }
        *out = pl;
        return SFM_OK;
    });
}

extern "C" int sfm_ba_plan_run(sfm_ba_plan* pl, const sfm_ba_options* opts, sfm_ba_summary* sum) {
    return guarded([&] {
        SFM_REQUIRE(pl && sum, SFM_ERR_INVALID_ARG, "null argument");
        CtxScope scope_(pl->ctx);
        sfm_ba_options O;
        if (opts) O = *opts; else sfm_ba_default_options(&O);
        return run_plan(pl, O, sum);
    });
}

extern "C" int sfm_ba_plan_download(sfm_ba_plan* pl, double* extr, double* intr, double* X) {
    return guarded([&] {
        SFM_REQUIRE(pl, SFM_ERR_INVALID_ARG, "null plan");
        CtxScope scope_(pl->ctx);
        download(pl, extr, intr, X);
        return SFM_OK;
    });
}

extern "C" int sfm_ba_plan_destroy(sfm_ba_plan* pl) {
    return guarded([&] {
        if (!pl) return SFM_OK;
        CtxScope scope_(pl->ctx);
        PhaseTimer tm("sfm_ba_plan_destroy");
        (void)hipStreamSynchronize(pl->ctx->stream);
        tm.mark("sync");
        delete pl;
        tm.mark("delete");
        return SFM_OK;
    });
}

extern "C" int sfm_ba_plan_get_info(sfm_ba_plan* pl, sfm_ba_plan_info* info) {
    return guarded([&] {
        SFM_REQUIRE(pl && info, SFM_ERR_INVALID_ARG, "null argument");
        const BAHostPlan& h = pl->hp;
        std::memset(info, 0, sizeof *info);
        info->shard_pt_begin = h.bounds[h.rank];
        info->shard_pt_end = h.bounds[h.rank + 1];
        info->shard_obs = h.n_sobs;
        info->n_chunks = (int32_t)h.chunks.size();
        info->band_blocks = h.D;
        info->n_cam_active = h.ncam;
        info->n_intr_active = h.nintr;
        info->rcs_dim = h.nF;
        for (int k = 0; k < 8; ++k) info->last_kernel_ms[k] = pl->last_ms[k];
        info->schur_flops_per_iter = h.schur_flops;
        info->schur_launches = pl->schur_launches;
        info->schur_ms_total = pl->schur_ms_total;
        info->rcs_solver = h.dense ? SFM_RCS_DENSE : pl->use_bcr ? SFM_RCS_BCR : SFM_RCS_SEQ_BAND;
        info->tile_rows = 16 * h.tile_nt;
        return SFM_OK;
    });
}

extern "C" int sfm_ba_plan_get_trace(sfm_ba_plan* pl, sfm_ba_iter* out, int32_t cap, int32_t* n) {
    return guarded([&] {
        SFM_REQUIRE(pl && n, SFM_ERR_INVALID_ARG, "null argument");
        const int32_t m = (int32_t)std::min<size_t>(pl->trace.size(), cap > 0 ? cap : 0);
        for (int32_t k = 0; k < m; ++k) out[k] = pl->trace[k];
        *n = m;
        return SFM_OK;
    });
}

namespace {

// ---- plan cache of sfm_ba_solve -------------------------------------------
// The reference builds a fresh problem per BundleAdjuster call
// (SequentialActuator.h:226-229); when the problem's structure (points,
// observation images, intrinsics assignment, gauge, model) equals the last
// one solved on this context -- a world that did not grow since the last
// call, or a caller re-solving the same problem -- the plan is reused and
// only the values are refreshed.  Keyed by an exact comparison, never a hash.
// SFM_BA_NO_PLAN_CACHE=1 disables it; sfm_ba_cache_clear releases it.
struct PlanKey {
    int32_t n_img = -1, n_intr = 0, const_img = 0, model = 0;
    int64_t n_pt = 0, n_obs = 0;
    std::vector<int64_t> pt_offsets;
    std::vector<int32_t> obs_img, img_intr;

    template <class T>
    static bool same(const T* a, const T* b, int64_t n) {
        if (n <= 0) return true;
        const int64_t kPar = 1 << 20;
        if (n < kPar) return std::memcmp(a, b, (size_t)n * sizeof(T)) == 0;
        const int nt = 8;
        std::atomic<bool> ok{true};
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
                if (std::memcmp(a + lo, b + lo, (size_t)(hi - lo) * sizeof(T)) != 0) ok = false;
            });
        for (auto& x : th) x.join();
        return ok;
    }
    bool matches(const sfm_ba_problem& P) const {
        return n_img == P.n_img && n_intr == P.n_intr && const_img == P.const_img && model == P.camera_model &&
               n_pt == P.n_pt && n_obs == P.n_obs && same(pt_offsets.data(), P.pt_offsets, P.n_pt + 1) &&
               same(img_intr.data(), P.img_intr, P.n_img) && same(obs_img.data(), P.obs_img, P.n_obs);
    }
    void assign(const sfm_ba_problem& P) {
        n_img = P.n_img; n_intr = P.n_intr; const_img = P.const_img; model = P.camera_model;
        n_pt = P.n_pt; n_obs = P.n_obs;
        pt_offsets.assign(P.pt_offsets, P.pt_offsets + P.n_pt + 1);
        obs_img.assign(P.obs_img, P.obs_img + P.n_obs);
        img_intr.assign(P.img_intr, P.img_intr + P.n_img);
    }
};

struct CacheEntry {
    sfm_ba_plan* plan = nullptr;
    PlanKey key;
};

std::mutex g_cache_mu;
std::unordered_map<const sfm_ctx*, CacheEntry>& plan_cache() {
    static auto* m = new std::unordered_map<const sfm_ctx*, CacheEntry>;
    return *m;
}

bool cache_enabled() {
    static const bool on = std::getenv("SFM_BA_NO_PLAN_CACHE") == nullptr;
    return on;
}

// take the context's cached plan out of the cache (nullptr if none)
sfm_ba_plan* cache_take(const sfm_ctx* ctx, PlanKey* key) {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    auto it = plan_cache().find(ctx);
    if (it == plan_cache().end()) return nullptr;
    sfm_ba_plan* pl = it->second.plan;
    *key = std::move(it->second.key);
    plan_cache().erase(it);
    return pl;
}

void cache_put(const sfm_ctx* ctx, sfm_ba_plan* pl, PlanKey&& key) {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    CacheEntry& e = plan_cache()[ctx];
    e.plan = pl;
    e.key = std::move(key);
}

}  // namespace

void sfm::ba_cache_release(sfm_ctx* ctx) {
    PlanKey k;
    if (sfm_ba_plan* pl = cache_take(ctx, &k)) sfm_ba_plan_destroy(pl);
}

extern "C" int sfm_ba_cache_stats(sfm_ctx* ctx, int64_t* reused, int64_t* grown, int64_t* fresh) {
    return guarded([&] {
        SFM_REQUIRE(ctx, SFM_ERR_INVALID_ARG, "null ctx");
        if (reused) *reused = ctx->plans_reused;
        if (grown) *grown = ctx->plans_grown;
        if (fresh) *fresh = ctx->plans_fresh;
        return SFM_OK;
    });
}

extern "C" int sfm_ba_cache_clear(sfm_ctx* ctx) {
    return guarded([&] {
        SFM_REQUIRE(ctx, SFM_ERR_INVALID_ARG, "null ctx");
        ba_cache_release(ctx);
        return SFM_OK;
    });
}

extern "C" int sfm_ba_solve(sfm_ctx* ctx, const sfm_ba_problem* prob, double* extr, double* intr,
                            double* X, const sfm_ba_options* opts, sfm_ba_summary* sum) {
    if (!ctx || !prob || !extr || !intr || (!X && prob->n_pt > 0)) {
        set_error("null argument");
        return SFM_ERR_INVALID_ARG;
    }
    sfm::PhaseTimer tm("sfm_ba_solve");
    sfm_ba_plan* pl = nullptr;
    PlanKey key;
    bool hit = false;
    sfm_ba_plan* seed_pl = nullptr;   // a cached plan of another structure (a grown problem's seed?)
    if (cache_enabled()) {
        pl = cache_take(ctx, &key);
        if (pl) {
            hit = key.matches(*prob);
            if (!hit) {
                seed_pl = pl;
                pl = nullptr;
            }
        }
        tm.mark("cache_lookup");
    }
    int rc = SFM_OK;
    if (hit) {
        rc = guarded([&] {
            CtxScope scope_(ctx);
            refresh_values(pl, *prob, extr, intr, X);
            return SFM_OK;
        });
        tm.mark("refresh");
        ++ctx->plans_reused;
        if (rc != SFM_OK) {
            sfm_ba_plan_destroy(pl);
            return rc;
        }
    } else {
        // a problem grown from the cached plan's (the next BundleAdjuster call
        // of SequentialActuator, SequentialActuator.h:226-229): the cached
        // plan seeds the new one (build_plan_grown), else a fresh plan
        sfm_ba_plan* grown = nullptr;
        if (seed_pl && cache_enabled_for_growth()) {
            GrowPrev gp;
            gp.n_img = key.n_img; gp.n_intr = key.n_intr; gp.const_img = key.const_img; gp.model = key.model;
            gp.n_pt = key.n_pt; gp.n_obs = key.n_obs;
            gp.pt_offsets = key.pt_offsets.data(); gp.obs_img = key.obs_img.data(); gp.img_intr = key.img_intr.data();
            rc = guarded([&] {
                CtxScope scope_(ctx);
                (void)hipStreamSynchronize(ctx->stream);   // the seed's last solve has finished with its buffers
                auto* np = new sfm_ba_plan;
                np->ctx = ctx;
                try {
                    if (create_plan(np, *prob, extr, intr, X, seed_pl, &gp)) grown = np;
                    else delete np;
                } catch (...) {
                    delete np;
                    throw;
                }
                return SFM_OK;
            });
            tm.mark(grown ? "grown" : "not_grown");
        }
        if (seed_pl) sfm_ba_plan_destroy(seed_pl);
        if (rc != SFM_OK) return rc;
        if (grown) {
            pl = grown;
            ++ctx->plans_grown;
        } else {
            rc = sfm_ba_plan_create(ctx, prob, extr, intr, X, &pl);
            tm.mark("create");
            if (rc != SFM_OK) return rc;
            ++ctx->plans_fresh;
        }
        if (cache_enabled()) key.assign(*prob);
    }
    rc = sfm_ba_plan_run(pl, opts, sum);
    tm.mark("run");
    if (sum && sum->usable) {  // BundleAdjuster::updateWorld only on success (:179-184)
        const int rc2 = sfm_ba_plan_download(pl, extr, intr, X);
        if (rc == SFM_OK) rc = rc2;
    }
    tm.mark("download");
    // a device or communication error leaves the plan suspect: not kept
    const bool keep = cache_enabled() && rc != SFM_ERR_DEVICE && rc != SFM_ERR_COMM;
    if (keep) cache_put(ctx, pl, std::move(key));
    else sfm_ba_plan_destroy(pl);
    tm.mark(keep ? "cached" : "destroy");
    return rc;
}

extern "C" int sfm_ba_dense_schedule(const sfm_ba_problem* prob, int32_t* out, int64_t cap, int64_t* n_words,
                                     int32_t* shape) {
    using namespace sfm;
    return guarded([&] {
        SFM_REQUIRE(prob && n_words && shape && cap >= 0 && (out || cap == 0), SFM_ERR_INVALID_ARG, "bad arguments");
        BAHostPlan h;
        build_plan(*prob, 0, 1, h);
        DevProblem P{};
        P.ncam = h.ncam; P.nintr = h.nintr; P.D = h.D; P.nb = h.nb; P.nF = h.nF; P.iw = h.iw;
        DenseArgs d;
        dense_setup(d, P);
        const std::vector<char> exact = h.dense ? dense_tile_pattern(h.targets, P.nF, d.nt) : std::vector<char>();
        const std::vector<int32_t> meta = h.dense ? dense_flow_plan(d, P, &exact) : std::vector<int32_t>();
        shape[0] = d.nt; shape[1] = d.nch; shape[2] = d.ntask; shape[3] = (h.dense && d.flow) ? 1 : 0;
        shape[4] = (int32_t)h.nF; shape[5] = (int32_t)h.nb; shape[6] = h.D;
        *n_words = (int64_t)meta.size();
        if ((int64_t)meta.size() <= cap && !meta.empty()) std::memcpy(out, meta.data(), meta.size() * sizeof(int32_t));
        return SFM_OK;
    });
}
