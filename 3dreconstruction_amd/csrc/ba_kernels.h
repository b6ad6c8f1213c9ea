// Launch wrappers for the BA kernels (ba_kernels.hip), called by the LM
// driver (ba_solver.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ba_types.h"

namespace sfm {

// Scalar slots produced by ba_finalize (one double each).
enum : int {
    kScCost = 0, kScXnorm2E, kScModelAcc, kScCandCost, kScStepnorm2E,  // summed over ranks
    kScBadX, kScGmaxE, kScCandBad, kScStepBad, kScSolveFail,             // max over ranks
    kScXnorm2F, kScStepnorm2F, kScGmaxF,                                 // replicated
    kScAccept,   // the device's copy of the host's accept decision (lm_spec_accept), 1 / 0
    kScCount
};
// kScSolveFail: 0 solved, 1 numerical failure (an invalid LM step),
// kSolveWaitTimeout a dataflow solve's wait timed out (a device error).  Max
// over ranks although every rank solves the same system: a numerical failure
// is replicated, but a wait timeout depends on which workgroups were resident
// on that rank's GPU, and every rank has to see it to leave the LM loop
// together (a rank that stopped alone would leave the others waiting in the
// next iteration's collective).
constexpr double kSolveWaitTimeout = 2.0;
constexpr int kScSumBegin = 0, kScSumEnd = 5, kScMaxBegin = 5, kScMaxEnd = 10;
constexpr int kPartT = 5;  // per step block: model acc, cand cost, step norm^2, step bad, cand bad

struct DevProblem {
    int32_t n_img, n_intr, n_spt, n_sobs, n_chunk, ncam, nintr, D;
    int32_t n_group;                // tile groups (one Schur workgroup and one tile each)
    int32_t n_cpt, n_gpt;           // chunk points [0, n_cpt), general points [n_cpt, n_spt)
    int32_t gz_max;                 // Z doubles of the largest general point
    int32_t dense;                  // RCS stored dense (Sdense) rather than band + arrow
    int32_t tile_nt;    // 16-row MFMA tiles per chunk side: 4 (64 F rows) or 5 (76 + w row)
    int32_t cam_model;  // SFM_CAM_* residual model
    int32_t iw;         // doubles per intrinsics block (4; RADIAL3 6)
    int32_t chunk_pts_max;   // longest Schur chunk (points)
    int32_t step_split;  // lanes per point in step_kernel (1, 2, 4, 8)
    int32_t n_zero;     // world > 1: targets[n_targets, n_targets + n_zero) are cleared, not summed
    int32_t red_waves;  // waves per target in reduce_kernel (1, 2, 4)
    int32_t red_split;  // SFM_CTX_BA_SPLIT_REDUCE: long targets in their own two launches
    int32_t gram_seg;   // image Gram workgroups per image (1..kGramSeg; U / Ub / Ucn / part_u stride)
    int32_t n_gram_img;          // images with observations in this shard
    const int32_t* gram_img;     // [n_gram_img] their indices (the Gram pass's workgroups)
    int64_t nb, nF;
    double huber_a, min_diag, max_diag;
    // LM options the device's accept decision needs (lm_spec_accept)
    double lm_min_rel, lm_ftol, lm_ptol;
    int32_t spec_force;   // SFM_CTX_DIAG_SPEC_ALWAYS (tests): the device's decision forced to accept
    // shard data
    const int32_t* pt_off;
    const int32_t* obs_img;
    const int32_t* obs_slot;
    const double* obs_uv;
    const ChunkDesc* chunks;
    const int32_t* group_off;       // [n_group + 1] chunk range of a tile group
    const int32_t* img_obs_ptr;
    const int32_t* img_pt;          // image order (img_obs_ptr): point, measurement
    const double* img_uv;
    const int32_t* img_colc;
    const int32_t* img_coli;
    const int32_t* img_intr;
    const int32_t* intr_col;        // [n_intr] first F column of the intrinsic block or -1
    const int32_t* blk_img;         // [ncam] image of each camera block (BCR back substitution's candidates)
    const int32_t* free_img;        // [n_free] images without camera columns (their candidate is a copy)
    int32_t n_free;
    const ReduceTarget* targets;
    const FlatTerm* terms;
    const double* src;              // contiguous [tiles | U | Ub | Ucn] the terms index
    int32_t n_targets;
    int32_t n_long;                 // targets with > reduce_long_threshold() terms
    const int32_t* long_targets;    // [n_long] target ids
    int32_t n_lseg;                 // kReduceSeg-term segments of the long targets
    const int32_t* lseg_off;        // [n_long+1] segment ranges per long target
    const int32_t* lseg;            // [n_lseg][2] (long index, first term)
    double* lpart;                  // [n_lseg][36] segment partial sums
    unsigned* lcount;               // [n_long] segments done this launch (the last one combines; reset by it)
    // general points (ba_plan.h): blocks, Z layout, product terms
    const int32_t* gblk_off;        // [n_gpt+1]
    const int32_t* gblk_col;        // F column of each block
    const int32_t* gblk_z;          // block's offset within the point's Z
    const int64_t* gz_off;          // [n_gpt+1]
    // general points split for the Z kernels: batches of consecutive short
    // points (zbatch_kernel, one wave each) and the rest (zpoint_kernel)
    int32_t n_zbatch, n_zlong;
    const int32_t* zbatch;          // [n_zbatch][2] general point range [g0, g1)
    const int32_t* zlong;           // [n_zlong] general point
    const PTerm* pterms;
    double* Z;                      // general points' eliminated rows, w after each point's blocks
    int32_t n_plong;                // targets with > preduce_long_threshold() product terms
    const int32_t* plong_targets;   // [n_plong] target ids
    int32_t n_plseg;                // kReduceSeg-term segments of their product-term lists
    const int32_t* plseg_off;       // [n_plong+1]
    const int32_t* plseg;           // [n_plseg][2] (long index, first product term)
    double* plpart;                 // [n_plseg][36]
    // state
    double* scaleE;     // [3*n_spt]
    double* scaleF;     // [nF]
    double* tiles;      // [n_group][80][80]
    double* U;          // [n_img * kGramSeg][FW * FW], FW = 6 + iw
    double* Ub;         // [n_img * kGramSeg][FW]
    double* Ucn;        // [n_img * kGramSeg][FW]
    double* Sband;      // [ncam][D+1][36]
    double* Sarrow;     // [nintr][ncam][24]
    double* Scorner;    // [nintr][nintr][16]
    double* Sdense;     // [nF][nF], lower triangle (dense mode)
    double* rhs;        // [nF]
    double* bF;         // [nF]
    double* cnF;        // [nF]
    double* Lcol;       // [ncam][D+1][36]
    double* Larrow;     // [ncam][nintr][24]
    double* zF;         // [nF]
    double* yF;         // [nF]
    double* Wglobal;    // solve window when it does not fit LDS
    double* part_u;     // [n_img][2]
    double* part_s;     // [n_chunk + n_gpt][2]
    double* part_t;     // [n_step_blocks][kPartT]
    double* part_f;     // [n_fblk][3] candidate partials (cand_kernel's workgroups, or BCR: block i, then
                        // [N] for the intrinsics)
    int32_t n_fblk;
    double* scal;       // [kScCount]
    double* fin_part;   // [16][12] finalize_kernel's workgroup partials
    unsigned* fin_count;   // its ticket (zeroed once; the last workgroup resets it)
    double* scal_host;  // device view of host-mapped [kScCount + 1] (+ sequence word), or null
};

void ba_campre(const double* extr, int n_img, CamPre* out, hipStream_t s);
// U blocks, cost and non-finite flag at (cp, intr, X); scaled with scaleF.
// gate (device, optional): the pass runs only if *gate != 0 (the speculative
// pass at the candidate, gated by finalize's kScAccept)
void ba_image_gram(const DevProblem& P, const CamPre* cp, const double* intr, const double* X,
                   hipStream_t s, const double* gate = nullptr);
// Jacobi scaling at iteration 0: scaleF from the reduced cnF (after ba_reduce
// of an unscaled pass); scaleE comes from ba_schur(..., scale_e = true).
void ba_fscale(const DevProblem& P, hipStream_t s);
// U / Ub / Ucn of a unit-scale ba_image_gram pass -> the same pass at scaleF
void ba_gram_rescale(const DevProblem& P, hipStream_t s);
void ba_fill(double* p, int64_t n, double v, hipStream_t s);
// several copies / fills in one launch (a solve's start: the working point
// from the plan's initial values, unit scales)
struct Seg {
    double* dst;
    const double* src;   // null: fill with v
    int64_t n;
    double v;
};
struct SegList {
    static constexpr int kSegs = 6;
    Seg seg[kSegs];
    int n = 0;
    void add(double* d, const double* src, int64_t cnt, double v = 0.0) {
        if (cnt > 0) seg[n++] = Seg{d, src, cnt, v};
    }
};
void ba_segs(const SegList& L, hipStream_t s);
// stamps (diagnostic builds only, else nullptr): per chunk 6 phase cycle sums
// scale_e: also form the Jacobi point scales (scaleE) in this pass (the
// solve's first pass, replacing ba_point_scale)
void ba_schur(const DevProblem& P, const CamPre* cp, const double* intr, const double* X,
              double radius, hipStream_t s, unsigned long long* stamps = nullptr, bool scale_e = false);
void ba_reduce(const DevProblem& P, bool vectors_only, hipStream_t s);
void ba_solve(const DevProblem& P, double radius, hipStream_t s);
// candidate cameras/intrinsics and their CamPre; F-part norm/gradient partials
// into part_f (summed by ba_finalize)
constexpr int kCandThreads = 256;
int ba_cand_blocks(const DevProblem& P);
void ba_cand(const DevProblem& P, const double* extr, const double* intr, double* cand_extr,
             double* cand_intr, CamPre* cand_cp, hipStream_t s);
void ba_step(const DevProblem& P, const CamPre* cp, const double* intr, const CamPre* cp_cand,
             const double* intr_cand, const double* X, double* X_cand, double radius,
             hipStream_t s);
// seq: written to scal_host[kScCount] after the scalars when scal_host is set
void ba_finalize(const DevProblem& P, hipStream_t s, unsigned long long seq = 0);
// world > 1 (RCCL): combine the all-gathered scalars in rank order and publish them
void ba_publish_gathered(const DevProblem& P, const double* gathered, int world, double* scal, double* scal_host,
                         hipStream_t s, unsigned long long seq);
size_t solve_lds_bytes(const DevProblem& P, bool* use_lds);
size_t solve_window_doubles(const DevProblem& P);
int ba_step_blocks(const DevProblem& P);
constexpr int kGStepThreads = 128;   // general points per step workgroup
int reduce_long_threshold();
int preduce_long_threshold();
constexpr int kReduceSeg = 256;   // terms per long-target segment (one workgroup)

}  // namespace sfm
