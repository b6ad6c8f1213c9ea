// Host-side planning of a BA problem for the gfx950 kernels.
#pragma once
#include <cstdint>
#include <functional>
#include <vector>

#include "../../include/sfmcore.h"
#include "ba_types.h"
#include "common.h"

namespace sfm {

// What a plan keeps so that the next call's plan, on a problem grown from this
// one (sfm_ba_solve's plan cache: SequentialActuator's next BA call, one image
// and its points added), can take its unchanged prefix instead of planning it
// again (build_plan_grown).  World 1 only.
struct PlanGrowState {
    bool ok = false;                         // this plan can seed a grown one
    std::vector<int32_t> span_lo, span_hi;   // every problem point's active camera span
    std::vector<char> used;                  // observed images
    int32_t lb = 0;                          // longest track, in distinct active cameras, minus one
    std::vector<char> ck;                    // chunkable flag per sorted position
    int64_t n_ck = 0;                        // classified chunkable points (n_cpt unless the chunking was dropped)
    int64_t rlen = 0;                        // chunking range length (points)
    int chunk_pts = 0;
    int cap = 0;                             // tile rows of the kept one-height chunking (0: none)
    std::vector<int32_t> seg_nch;            // its chunks per range
    std::vector<int64_t> seg_flops;          // its algorithmic flops per range
    std::vector<int32_t> seg_own, seg_obs;   // per range: largest tile rows / observations of a point
    std::vector<int64_t> gflops;             // algorithmic flops per general point
};

struct BAHostPlan {
    // ---- global (identical on every rank) ---------------------------------
    int32_t n_img = 0, n_intr = 0;
    int64_t n_pt = 0, n_obs = 0;
    std::vector<int32_t> cam_blk;    // image -> active camera block or -1
    std::vector<int32_t> intr_blk;   // intrinsic -> active block or -1
    std::vector<int32_t> blk_img;    // camera block -> image
    std::vector<int32_t> blk_intr;   // intr block -> intrinsic
    std::vector<int32_t> img_colc;   // image -> global F column of its pose or -1
    std::vector<int32_t> img_coli;   // image -> global F column of its intrinsics
    std::vector<int32_t> img_intr;
    int32_t ncam = 0, nintr = 0, D = 0;
    int64_t nb = 0, na = 0, nF = 0;
    int32_t iw = 4;                  // doubles per intrinsics block (RADIAL3: 6)
    std::vector<int64_t> order, bounds;  // sorted points / rank ranges
    int32_t rank = 0, world = 1;

    int32_t nFB = 0;                 // F blocks: cameras 0..ncam-1, intrinsics ncam..
    bool dense = false;              // RCS storage + solver: dense (true) or band + arrow (BCR)
    int64_t n_sdense = 0;            // nF * nF when dense

    // ---- shard ------------------------------------------------------------
    // Shard points [0, n_cpt) are handled by Schur chunks (tile rows, LDS
    // staging); [n_cpt, n_spt) are general points (any track length,
    // duplicate views, many intrinsics), one wavefront each, whose
    // eliminated rows Z go to a buffer and reach the RCS as product terms.
    int64_t n_spt = 0, n_sobs = 0;
    int64_t n_cpt = 0, n_gpt = 0;
    int32_t gram_seg = kGramSeg < 3 ? kGramSeg : 3;   // image Gram workgroups per image (1..kGramSeg)
    std::vector<int32_t> gram_img;   // images with observations in this shard (the Gram pass's images)
    std::vector<int32_t> gblk_off;   // [n_gpt+1] block range of a general point
    std::vector<int32_t> gblk_col;   // F column of each of its blocks (6 rows: camera, 4: intrinsics)
    std::vector<int32_t> gblk_z;     // element offset of the block's Z rows within the point's Z
    std::vector<int64_t> gz_off;     // [n_gpt+1] Z buffer range of a point: blocks, then w (3)
    int64_t n_z = 0, gz_max = 0;     // Z doubles in all / of the largest point
    // Z kernels: batches of consecutive general points of <= kZShortObs
    // observations each, <= 64 observations and <= kZBatchPts points per batch
    // (one wave, one lane per observation), and the longer points (one wave
    // per point, rounds of 64)
    std::vector<int32_t> zbatch;     // [n][2] general point range [g0, g1)
    std::vector<int32_t> zlong;      // general point ids
    std::vector<int64_t> spt_global;  // shard point -> global point id
    // a general point's observations are re-sorted by image (chunk points keep
    // the problem's order): gobs_perm[s - pt_off[n_cpt]] = the problem-local
    // index (within its point) of shard observation s; empty when every
    // general point was already in image order.  The plan cache's value
    // refresh maps new measurements through it (ba_obs_source).
    std::vector<int32_t> gobs_perm;
    // observation-sized arrays live in page-locked staging memory while a
    // context is bound (HostVec, common.h): uploaded, then released
    HostVec<int32_t> pt_off;          // [n_spt+1]
    HostVec<int32_t> obs_img, obs_slot;
    HostVec<double> obs_uv;
    std::vector<ChunkDesc> chunks;
    // tile groups: chunks [group_off[g], group_off[g+1]) share one slot
    // layout and one tile (index g); <= kGroupChunks chunks each
    std::vector<int32_t> group_off;
    int64_t n_group() const { return group_off.empty() ? 0 : (int64_t)group_off.size() - 1; }
    int32_t tile_nt = 5;              // 16-row MFMA tiles per chunk side (4 or 5)
    std::vector<int32_t> img_obs_ptr;  // [n_img+1] shard observations per image (prefix)

    // ---- reduce plan ------------------------------------------------------
    std::vector<ReduceTarget> targets;
    std::vector<ReduceTarget> zero_targets;   // world > 1: blocks other shards write (zeroed by the reduce)
    std::vector<int32_t> row_tgt;    // [nFB + 1] first matrix target of every F-block row (grown plans)
    HostVec<FlatTerm> terms;         // resolved against the solver's source buffer (default-initialised)
    HostVec<PTerm> pterms;           // uploaded as it is: page-locked staging
    int64_t n_sband = 0, n_sarrow = 0, n_scorner = 0;
    int64_t schur_flops = 0;    // algorithmic flops of one Schur pass
    // called by build_plan once pt_off / obs_img / obs_slot / obs_uv are final
    // (their upload then overlaps the rest of the planning)
    std::function<void(BAHostPlan&)> on_shard_ready;
    int64_t schur_bytes = 0;    // algorithmic HBM bytes of one Schur pass
    // obs_uv is left empty (grown plans): the caller gathers the measurements
    // into shard order on the device (ba_obs_source, ba_gather_uv)
    bool uv_on_device = false;
    // grown plans: the sorted positions taken over from the seed plan unchanged
    // (diagnostics, tests)
    int64_t reused_pts = 0;
    int64_t reused_chunks = 0, reused_gpts = 0;   // chunks / general points taken from the seed
    PlanGrowState grow;
};

// The previous problem's structure (the plan cache's key of sfm_ba_solve).
struct GrowPrev {
    int32_t n_img = 0, n_intr = 0, const_img = 0, model = 0;
    int64_t n_pt = 0, n_obs = 0;
    const int64_t* pt_offsets = nullptr;
    const int32_t* obs_img = nullptr;
    const int32_t* img_intr = nullptr;
};

// Engine choices the planner takes from the context (SFM_CTX_BA_*): the
// dense RCS for a narrow band, 80-row Schur tiles for every chunk.
struct PlanOpts {
    bool force_dense = false;
    bool tile80 = false;
};

// Validates the problem and fills every field.  Throws SfmError.
void build_plan(const sfm_ba_problem& prob, int rank, int world, BAHostPlan& plan, const PlanOpts& opts = {});

// The plan of `prob` when it grows `prev` (the problem `seed` was built for):
// the same images, intrinsics map and gauge with images, points and
// observations appended only (every point keeps its observations, in order,
// and may gain new ones at the end).  The sorted points before the first one
// the growth moves keep their classification, shard arrays, chunks (whole
// chunking ranges) and general-point blocks, taken from `seed`; the rest and
// the reduce plan are planned as build_plan plans them, so the result equals
// build_plan(prob, 0, 1, ...) array for array (tests: sfm_ba_grown_digest).
// World 1.  The measurements are not gathered on the host (uv_on_device).
// Returns false, with `seed` untouched, when prob does not grow prev or seed
// cannot seed it (then build_plan).  `seed` is consumed otherwise.  Throws
// SfmError.
bool build_plan_grown(const sfm_ba_problem& prob, const GrowPrev& prev, BAHostPlan& seed, BAHostPlan& plan,
                      const PlanOpts& opts = {});

// FNV-1a digest of every plan array the device uses (diagnostics, tests)
uint64_t plan_digest(const BAHostPlan& h, bool with_uv);

// Every point's active camera span [lo, hi) under a camera order ((ncam, 0):
// no active camera): the partition's sort keys.
struct PointSpans {
    std::vector<int32_t> lo, hi;
};

// Landmark-block partition (sfm_ba_partition); spans: precomputed keys (optional).
void partition_points(const sfm_ba_problem& prob, const std::vector<int32_t>& cam_blk, int world,
                      std::vector<int64_t>& order, std::vector<int64_t>& bounds, const PointSpans* spans = nullptr);

// Image -> active camera block (-1: constant or unobserved) in the RCS order:
// image order, or reverse Cuthill-McKee over the camera co-visibility graph
// when that gives a narrower band.  *D_out = the block half-bandwidth.
// spans / used_out (optional): every point's span under the returned order,
// and the observed-image flags, from the same passes.
std::vector<int32_t> camera_blocks(const sfm_ba_problem& prob, int32_t* ncam_out, int32_t* D_out,
                                   PointSpans* spans = nullptr, std::vector<char>* used_out = nullptr,
                                   int32_t* lb_out = nullptr, bool* rcm_out = nullptr);

// Largest camera half-bandwidth the block-cyclic-reduction solver takes.
constexpr int kBandMaxD = 10;

}  // namespace sfm
