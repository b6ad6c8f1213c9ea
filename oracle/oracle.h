/*
 * oracle.h — CPU restatement of the reference semantics.  TEST
 * INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
 * bench.py cpu_baseline leg as the checker / CPU baseline.  The product
 * (libsfmcore.so) never links, loads or calls anything here.
 *
 * PARITY STATUS: parity unpinned.  The reference's BA arithmetic lives in
 * Ceres 2.2 (CMakeLists.txt:32) and its matchers in OpenMVG (unpinned,
 * un-vendored) and OpenCV 4 — none is present in /root/reference or in this
 * image, and the reference ships no tests or golden outputs for either path
 * (SURVEY.md §4, §8c).  This file restates:
 *   - src/adjuster/BundleAdjuster.h:33-69 (ReprojectCost), :109 (Huber 4),
 *     :105 (gauge), :125-139 (Solve + RMSE definition) with the published
 *     Ceres 2.2 TrustRegionMinimizer / LevenbergMarquardtStrategy /
 *     SchurEliminator control flow (documented in oracle/ba_oracle.cpp),
 *     and src/adjuster/SnavelyReprojectionError.h:16-54 (BAL residual model,
 *     SURVEY.md §8(f) row 4) and OpenMVG's PINHOLE_CAMERA_RADIAL3 residual
 *     (sparseBuilder.cpp:1292-1299) as alternative residuals;
 *   - OpenMVG Matcher_Regions(BRUTE_FORCE_L2) ratio matching as selected by
 *     src/sparseBuilder/sparseBuilder.cpp:919-921 with fDistRatio 0.8 (:812);
 *   - OpenMVG Cascade_Hashing_Matcher_Regions(0.8), the "AUTO" default of
 *     src/sparseBuilder/sparseBuilder.cpp:811-814,911-914 (cascade_oracle.cpp);
 *   - OpenCV BFMatcher(NORM_L2, crossCheck) knnMatch(k=1) as used by
 *     src/frame/LocalFrame.h:31-47 and src/frame/GlobalFrame.h:22-43.
 * The only reference-produced artefacts available are VLFeat descriptors
 * compiled from src/nonFree/sift/vl (oracle/build_ref.sh), used as golden
 * matcher inputs.
 */
#ifndef SFM_ORACLE_H
#define SFM_ORACLE_H
#include <stdint.h>
#include "../include/sfmcore.h"

#ifdef __cplusplus
extern "C" {
#endif
/* the C-ABI is the only exported surface (libraries build with hidden default visibility) */
#pragma GCC visibility push(default)

/* op: 0 = sum, 1 = max.  In-place over buf[n]. */
typedef void (*orc_allreduce_fn)(void* user, double* buf, int64_t n, int32_t op);

/* Full LM solve.  shard_pts (optional) = the global point ids this rank owns
 * (in processing order); NULL = all points.  allreduce may be NULL for a
 * single rank.  n_threads: OpenMP threads for the per-point work. */
int orc_ba_solve(const sfm_ba_problem* prob, double* extr, double* intr, double* X,
                 const sfm_ba_options* opts, sfm_ba_summary* summary,
                 sfm_ba_iter* trace, int32_t trace_cap, int32_t* trace_n,
                 const int64_t* shard_pts, int64_t n_shard_pts,
                 orc_allreduce_fn allreduce, void* user, int32_t n_threads);

/* Cost 1/2 sum rho(|r|^2) and raw residuals r (2*n_obs, may be NULL). */
int orc_ba_cost(const sfm_ba_problem* prob, const double* extr, const double* intr,
                const double* X, double* cost, double* residuals);

/* Residual and Jacobian of one observation, J row-major 2x13 over
 * (fx,fy,cx,cy | w0,w1,w2,t0,t1,t2 | X0,X1,X2).  mode 0: analytic (the
 * formulas the oracle and the GPU use), mode 1: forward-mode dual numbers
 * through a restatement of BundleAdjuster.h:40-65 and
 * ceres::AngleAxisRotatePoint (the Ceres AutoDiff path). */
int orc_ba_jacobian(int32_t mode, const double* intr, const double* extr, const double* X,
                    const double* uv, double* r, double* J);

/* Same for a residual model SFM_CAM_* (SNAVELY: SnavelyReprojectionError.h,
 * intrinsics {f, l1, l2, -}, J column 3 is zero; RADIAL3: OpenMVG
 * Pinhole_Intrinsic_Radial_K3, {f, ppx, ppy, k1, k2, k3}, J row-major 2x15). */
int orc_ba_jacobian_model(int32_t model, int32_t mode, const double* intr, const double* extr,
                          const double* X, const double* uv, double* r, double* J);

/* Dense single-pair matching: same contract as sfm_match_dense. */
int orc_match_dense(const uint8_t* a, int32_t n_a, const uint8_t* b, int32_t n_b,
                    int32_t mode, float ratio, int32_t* match_idx, int32_t* match_d2);

/* The same on n_threads OpenMP threads. */
int orc_match_dense_mt(const uint8_t* a, int32_t n_a, const uint8_t* b, int32_t n_b,
                       int32_t mode, float ratio, int32_t n_threads, int32_t* match_idx,
                       int32_t* match_d2);

/* Incremental loop oracle (seq_oracle.cpp): sfm_seq_* semantics with the CPU
 * matcher and solver. */
typedef struct orc_seq orc_seq;
int orc_seq_create(const sfm_seq_options* opts, int32_t n_threads, orc_seq** out);
int orc_seq_init(orc_seq* s, const sfm_seq_image* a, const sfm_seq_image* b);
int orc_seq_add_image(orc_seq* s, const sfm_seq_image* im, int32_t* kept);
int orc_seq_bundle_adjust(orc_seq* s, sfm_ba_summary* summary);
int orc_seq_last_step(orc_seq* s, sfm_seq_step* step);
int orc_seq_matches(orc_seq* s, int32_t which, int32_t* query, int32_t* train, float* dist,
                    int64_t cap, int64_t* n);
int orc_seq_world(orc_seq* s, double* X, int64_t* n_obs, int64_t cap_pts, int64_t* n_pts,
                  double* poses, int32_t cap_img, int32_t* n_img, double* intr4);
int orc_seq_observations(orc_seq* s, int32_t* img, double* uv, int64_t cap, int64_t* n);
int orc_seq_destroy(orc_seq* s);
/* Overwrite the numeric state (X[3*n_pts] in point-index order, poses[6*n_img]
 * in sequence order, the camera's intr4) of a loop with identical topology. */
int orc_seq_set_state(orc_seq* s, const double* X, int64_t n_pts, const double* poses, int32_t n_img,
                      const double* intr4);

/* Float descriptors (sfm_match_dense_f32's restatement): RATIO / MUTUAL. */
int orc_match_dense_f32(const float* a, int32_t n_a, const float* b, int32_t n_b, int32_t mode,
                        float ratio, int32_t n_threads, int32_t* match_idx, float* match_d2);
/* All-pairs, compacted (counts per pair; matches sorted by (i,j)).
 * Two calls: counts only when i/j/d2 are NULL. */
int orc_match_pairs(const uint8_t* desc, const int64_t* offsets, int32_t n_img,
                    const int32_t* pairs, int64_t n_pairs, int32_t mode, float ratio,
                    int32_t n_threads, int64_t* counts, uint32_t* i, uint32_t* j, int32_t* d2);

/* Cascade hashing (SFM_MATCH_CASCADE, cascade_oracle.cpp): per query of J,
 * idx/dist[p * stride + q] = matched row of I or -1 / its L2^2 or -1. */
int orc_cascade_pairs(const uint8_t* desc, const int64_t* offsets, int32_t n_img,
                      const int32_t* pairs, int64_t n_pairs, float ratio, int32_t n_threads,
                      int64_t stride, int32_t* idx, int32_t* dist);
/* IndMatchDecorator<float>::getDeduplicated: (i, j)-sorted matches and
 * [n][4] keypoints (x, y, scale, orientation) of both images -> survivors in
 * the decorator's std::set order. */
int orc_dedup_decorator(const uint32_t* i, const uint32_t* j, int64_t n, const float* feat_i,
                        const float* feat_j, uint32_t* out_i, uint32_t* out_j, int64_t* n_out);
/* CascadeHasher::Init projections, float [188][128]. */
int orc_cascade_projections(float* out);

/* sfm_fmatrix_ac semantics (fmat_oracle.cpp: OpenMVG GeometricFilter_FMatrix_AC
 * + ACRANSAC restated), OpenMP over pairs. */
int orc_fmatrix_ac(int64_t n_pairs, const int64_t* off, const double* xy, const int32_t* wh,
                   const sfm_fmatrix_opts* opts, sfm_fmatrix_result* results, int32_t* inliers,
                   int32_t n_threads);
/* std::mt19937(default_seed) + std::uniform_int_distribution<uint32_t>(lo[k], hi[k]) */
int orc_uniform_draws(const uint32_t* lo, const uint32_t* hi, int64_t n, uint32_t* out);
/* fn 0: the filter's log10, 1: its cube root */
int orc_det_math(int32_t fn, const double* x, int64_t n, double* out);
/* seven-point solver on 7 normalised correspondences: F[9 * n_models] */
int orc_seven_point(const double* x1, const double* x2, double* F, int32_t* n_models);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif
