// Host-side planning of a BA problem for the gfx950 kernels.
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/sfmcore.h"
#include "ba_types.h"

namespace sfm {

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
    std::vector<int64_t> order, bounds;  // sorted points / rank ranges
    int32_t rank = 0, world = 1;

    // ---- shard ------------------------------------------------------------
    int64_t n_spt = 0, n_sobs = 0;
    std::vector<int64_t> spt_global;  // shard point -> global point id
    std::vector<int32_t> pt_off;      // [n_spt+1]
    std::vector<int32_t> obs_img, obs_pt, obs_slot;
    std::vector<double> obs_uv;
    std::vector<ChunkDesc> chunks;
    int32_t tile_nt = 5;              // 16-row MFMA tiles per chunk side (4 or 5)
    std::vector<int32_t> img_obs_ptr, img_obs;
    std::vector<int32_t> img_pt;      // image order: point of each observation
    std::vector<double> img_uv;       // image order: its measurement

    // ---- reduce plan ------------------------------------------------------
    std::vector<ReduceTarget> targets;
    std::vector<ReduceTerm> terms;
    int64_t n_sband = 0, n_sarrow = 0, n_scorner = 0;
    int64_t schur_flops = 0;    // algorithmic flops of one Schur pass
    int64_t schur_bytes = 0;    // algorithmic HBM bytes of one Schur pass
};

// Validates the problem and fills every field.  Throws SfmError.
void build_plan(const sfm_ba_problem& prob, int rank, int world, BAHostPlan& plan);

// Landmark-block partition (sfm_ba_partition).
void partition_points(const sfm_ba_problem& prob, const std::vector<int32_t>& cam_blk, int world,
                      std::vector<int64_t>& order, std::vector<int64_t>& bounds);

}  // namespace sfm
