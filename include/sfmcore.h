/*
 * sfmcore.h — C-ABI of the MI355X-native bundle-adjustment and descriptor
 * matching core (libsfmcore.so).
 *
 * This is the drop-in boundary for the two hot paths of
 * RainbowXXX/3DReconstruction (reference tree, read-only):
 *
 *   BA   : src/adjuster/BundleAdjuster.h:100-141  (ceres::Solve over the
 *          whole WorldStructure; ReprojectCost :33-69, HuberLoss(4) :109,
 *          gauge :105, options :167-174, write-back :143-156)
 *   Match: src/sparseBuilder/sparseBuilder.cpp:758-807 (matchPair,
 *          exhaustive pairs) and :809-1023 (match, Matcher_Regions(0.8,
 *          BRUTE_FORCE_L2) :919-921), plus the legacy exact matcher
 *          src/frame/LocalFrame.h:31-47 / GlobalFrame.h:22-43
 *          (cv::BFMatcher(NORM_L2, crossCheck) knnMatch k=1).
 *
 * Conventions
 *   - Plain pointers and sizes only; every buffer is caller owned.  No
 *     allocation crosses the ABI.  Nothing here throws.
 *   - Every function returns 0 (SFM_OK) on success or a negative SFM_ERR_*
 *     code; sfm_last_error() returns a thread-local message for the last
 *     failure on the calling thread.
 *   - One sfm_ctx per thread (contexts are independent; a context is not
 *     re-entrant).  A context owns its HIP device, stream(s) and, when
 *     world_size > 1, an RCCL communicator over xGMI.
 *   - Functions marked [cpu] never touch the GPU and work without one.
 */
#ifndef SFMCORE_H
#define SFMCORE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
/* the C-ABI is the only exported surface (libraries build with hidden default visibility) */
#pragma GCC visibility push(default)

#define SFM_OK                 0
#define SFM_ERR_INVALID_ARG   -1
#define SFM_ERR_DEVICE        -2   /* HIP runtime error / no gfx950 device      */
#define SFM_ERR_NOT_FINITE    -3   /* non-finite residual at the initial point   */
#define SFM_ERR_UNSUPPORTED   -4   /* problem shape outside this build's kernels */
#define SFM_ERR_COMM          -5   /* RCCL failure                               */
#define SFM_ERR_OOM           -6
#define SFM_ERR_SOLVER        -7   /* LM terminated with FAILURE (not usable)    */

/* [cpu] library identification and last error message (thread local). */
const char* sfm_version(void);
const char* sfm_last_error(void);

/* ------------------------------------------------------------------------ */
/* Context                                                                   */
/* ------------------------------------------------------------------------ */
typedef struct sfm_ctx sfm_ctx;

/* Host-side all-reduce hook: reduce buf[n] across all ranks in place,
 * op 0 = sum, 1 = max; return 0 on success. */
typedef int32_t (*sfm_allreduce_fn)(void* user, double* buf, int64_t n, int32_t op);

typedef struct sfm_ctx_opts {
    int32_t device;          /* HIP device ordinal (local to the process)      */
    int32_t rank;            /* 0 .. world_size-1                              */
    int32_t world_size;      /* 1 = single GPU; >1 = landmark-sharded BA       */
    int32_t flags;           /* SFM_CTX_* bits (0 = defaults)                  */
    const uint8_t* comm_id;  /* 128-byte RCCL unique id from rank 0's
                                sfm_comm_unique_id(); NULL when world_size==1
                                or when `allreduce` is given (at world_size 1
                                it builds a 1-rank communicator: the RCCL
                                exchanges run and are identities)             */
    sfm_allreduce_fn allreduce; /* optional (world_size > 1, comm_id NULL):
                                the per-iteration exchanges are staged through
                                pinned host memory and handed to this hook
                                (MPI, gloo, ...) instead of RCCL over xGMI   */
    void* allreduce_user;
} sfm_ctx_opts;

/* sfm_ctx_opts.flags.  SFM_CTX_TUNE_HOST_MALLOC (opt-in): keep freed host memory in
 * the process heap (glibc M_MMAP_THRESHOLD at its 32 MiB maximum, and
 * M_TRIM_THRESHOLD).  Unmapping a large host buffer stalls the process's next
 * GPU operation for 10-30 ms while the driver invalidates its mappings, which
 * an incremental loop (BA, then matching, per image) pays every step; the
 * price is that the heap does not shrink, so a long-running host application
 * leaves it off (the default: its malloc settings are not touched). */
#define SFM_CTX_TUNE_HOST_MALLOC 1
/* Diagnostic only: world_size > 1 with every exchange a no-op (no RCCL, no
 * hook).  The context plans and runs rank `rank`'s landmark shard alone, so
 * its kernels and wall time are what that rank spends in an N-GPU run minus
 * the collectives; the solve is not the global one (bench.py --fake-world). */
#define SFM_CTX_DIAG_NO_EXCHANGE 2
/* Diagnostic only (error-path tests): every reduced-camera-system solve of
 * this context reports that one of its dataflow waits timed out, as when
 * another context holds the CUs a persistent solve kernel needs.  The solve
 * verdict is max-reduced over ranks with the other per-iteration maxima, so
 * every rank of a sharded solve then returns SFM_ERR_DEVICE together instead
 * of the others waiting in the next collective. */
#define SFM_CTX_DIAG_FAIL_SOLVE_WAIT 4
/* Measurement: sfm_fmatrix_ac brackets its kernel with HIP events (after
 * draining its uploads) so that sfm_ctx_last_kernel_ms can report the kernel
 * alone.  Off by default: the extra stream synchronisation and event pair are
 * not part of the filter's production path. */
#define SFM_CTX_TIME_KERNELS 8
/* Diagnostic only (tests): the device's copy of the LM accept decision is
 * forced to "accept", so the speculative Gram pass at the candidate runs after
 * every step and the host has to redo it at the current point for each step
 * it rejects (the path a device / host disagreement would take). */
#define SFM_CTX_DIAG_SPEC_ALWAYS (1 << 11)
/* BA engine shape (A/B measurement and tests; 0 = the measured defaults).
 * Every alternative is exact: the launch-shape bits and the per-point /
 * per-target lane counts change only how the same sums are launched
 * (bit-identical results, or sums in another fixed order), the solver bits
 * pick the other direct solver of the same reduced camera system.  They are
 * read when a plan is created (sfm_ba_plan_create, sfm_ba_solve); there are
 * no environment switches for any of them.
 *   SFM_CTX_BA_DENSE_RCS     blocked dense Cholesky even for a narrow band
 *   SFM_CTX_BA_SEQ_BAND      the sequential block-band solver instead of
 *                            cyclic reduction (4-wide intrinsics arrows)
 *   SFM_CTX_BA_TILE80        80-row Schur tiles for every chunk
 *   SFM_CTX_BA_SPLIT_REDUCE  the RCS reduction in three launches (short
 *                            targets, long-target segments, their combine)
 *   SFM_CTX_BA_SPLIT_BCR     cyclic reduction's top, corner and every
 *                            back-substitution level as separate launches
 *   SFM_CTX_BA_DENSE_CHAIN   the dense factorisation and back substitution
 *                            as launch chains instead of dataflow kernels
 *   SFM_CTX_BA_NO_SPEC_GRAM  the Gram pass after an accepted step launched by
 *                            the host after its decision, not speculatively
 *   SFM_CTX_BA_STEP_LANES(n) n = 1, 2, 4, 8 lanes per point in the step pass
 *   SFM_CTX_BA_REDUCE_WAVES(n) n = 1, 2, 4 waves per reduce target
 * (a field of 0 means the planner's default; any other n gives the field
 * value 7, which sfm_ctx_create rejects with SFM_ERR_INVALID_ARG) */
#define SFM_CTX_BA_DENSE_RCS      (1 << 4)
#define SFM_CTX_BA_SEQ_BAND       (1 << 5)
#define SFM_CTX_BA_TILE80         (1 << 6)
#define SFM_CTX_BA_SPLIT_REDUCE   (1 << 7)
#define SFM_CTX_BA_SPLIT_BCR      (1 << 8)
#define SFM_CTX_BA_DENSE_CHAIN    (1 << 9)
#define SFM_CTX_BA_NO_SPEC_GRAM   (1 << 10)
#define SFM_CTX_BA_STEP_LANES(n)  (((n) == 8 ? 4 : (n) == 4 ? 3 : (n) == 2 ? 2 : (n) == 1 ? 1 : 7) << 12)
#define SFM_CTX_BA_REDUCE_WAVES(n) (((n) == 4 ? 3 : (n) == 2 ? 2 : (n) == 1 ? 1 : 7) << 15)

/* [cpu] fill out[128] with a fresh RCCL unique id (rank 0 only). */
int sfm_comm_unique_id(uint8_t* out128);
int sfm_ctx_create(const sfm_ctx_opts* opts, sfm_ctx** out);
int sfm_ctx_destroy(sfm_ctx* ctx);
int sfm_ctx_synchronize(sfm_ctx* ctx);

/* ------------------------------------------------------------------------ */
/* Bundle adjustment                                                         */
/*                                                                          */
/* Residual (BundleAdjuster.h:40-65): P = R(w) X + t (ceres::AngleAxisRotate- */
/* Point), u = fx P0/P2 + cx, v = fy P1/P2 + cy, r = (u - obs.x, v - obs.y).   */
/* Parameter blocks: extr[6*n_img] = {w0,w1,w2,t0,t1,t2} per image,          */
/* intr[4*n_intr] = {fx,fy,cx,cy} (camera_model selects others), X[3*n_pt].   */
/* Loss HuberLoss(huber_a).                                                  */
/* ------------------------------------------------------------------------ */
typedef struct sfm_ba_problem {
    int32_t n_img;           /* posed images (extrinsic blocks)                */
    int32_t n_intr;          /* intrinsic blocks (Camera objects)              */
    int64_t n_pt;            /* world points                                   */
    int64_t n_obs;           /* observations = residual blocks                 */
    const int64_t* pt_offsets;/* [n_pt+1] landmark-major: obs of point p are
                                 pt_offsets[p] .. pt_offsets[p+1]-1          */
    const int32_t* obs_img;  /* [n_obs] image of each observation              */
    const double*  obs_uv;   /* [2*n_obs] observed pixel (x, y)                */
    const int32_t* img_intr; /* [n_img] intrinsic block of each image          */
    int32_t const_img;       /* gauge: image whose pose is held constant
                                (BundleAdjuster.h:105); -1 for none          */
    int32_t camera_model;    /* SFM_CAM_* residual model (0 = the reference's
                                ReprojectCost)                               */
    double huber_a;          /* HuberLoss scale a (reference: 4.0); <=0: none  */
} sfm_ba_problem;

/* Residual models (sfm_ba_problem.camera_model).  The intrinsics blocks of
 * intr[] are 4 doubles wide, except RADIAL3's 6 (sfm_ba_intr_width()):
 *   SFM_CAM_PINHOLE  BundleAdjuster.h:33-69 ReprojectCost, {fx, fy, cx, cy}:
 *                    r = (fx P0/P2 + cx - u, fy P1/P2 + cy - v)
 *   SFM_CAM_SNAVELY  src/adjuster/SnavelyReprojectionError.h:16-54 (BAL /
 *                    Bundler), {f, l1, l2, -}: p = (-P0/P2, -P1/P2),
 *                    r = f (1 + |p|^2 (l1 + l2 |p|^2)) p - (u, v); the 4th
 *                    double is not a parameter (never read, never moved).
 *   SFM_CAM_RADIAL3  OpenMVG Pinhole_Intrinsic_Radial_K3 with ADJUST_ALL, as
 *                    reconstruction() selects it (sparseBuilder.cpp:1292-1299;
 *                    ResidualErrorFunctor_Pinhole_Intrinsic_Radial_K3),
 *                    {f, ppx, ppy, k1, k2, k3}: x = P0/P2, y = P1/P2,
 *                    c = 1 + k1 r2 + k2 r2^2 + k3 r2^3 (r2 = x^2 + y^2),
 *                    r = (ppx + f x c - u, ppy + f y c - v).  Solved through
 *                    the general-point path and the dense reduced camera
 *                    system. */
#define SFM_CAM_PINHOLE 0
#define SFM_CAM_SNAVELY 1
#define SFM_CAM_RADIAL3 2
/* [cpu] doubles per intrinsics block of a model (4, or 6 for RADIAL3);
 * 0 for an unknown model. */
int sfm_ba_intr_width(int32_t camera_model);

typedef struct sfm_ba_options {  /* ceres::Solver::Options semantics      */
    int32_t max_num_iterations;            /* 50   */
    int32_t max_num_consecutive_invalid_steps; /* 5 */
    int32_t jacobi_scaling;                /* 1    */
    int32_t reserved;
    double function_tolerance;             /* 1e-6 */
    double gradient_tolerance;             /* 1e-10 */
    double parameter_tolerance;            /* 1e-8 */
    double initial_trust_region_radius;    /* 1e4  */
    double max_trust_region_radius;        /* 1e16 */
    double min_trust_region_radius;        /* 1e-32 */
    double min_relative_decrease;          /* 1e-3 */
    double min_lm_diagonal;                /* 1e-6 */
    double max_lm_diagonal;                /* 1e32 */
} sfm_ba_options;

/* ceres::TerminationType subset */
#define SFM_TERM_CONVERGENCE     0
#define SFM_TERM_NO_CONVERGENCE  1
#define SFM_TERM_FAILURE         2

typedef struct sfm_ba_summary {
    double initial_cost;     /* 1/2 sum rho(|r|^2) at the input parameters     */
    double final_cost;
    int64_t num_residuals;   /* 2 * n_obs                                      */
    int32_t iterations;      /* ceres summary.iterations.size()-1 (iteration 0
                                is the initial evaluation)                    */
    int32_t successful_steps;/* counts iteration 0, as Ceres does             */
    int32_t unsuccessful_steps;
    int32_t termination;     /* SFM_TERM_*                                     */
    int32_t usable;          /* summary.IsSolutionUsable()                     */
    int32_t reserved;
    double rmse_initial;     /* sqrt(initial_cost/num_residuals), the metric
                                BundleAdjuster.h:137 prints                  */
    double rmse_final;       /* sqrt(final_cost/num_residuals)  (:138)         */
    double seconds;          /* wall time of the LM loop                        */
} sfm_ba_summary;

/* One entry per minimizer iteration (ceres::IterationSummary subset); used to
 * compare accept/reject sequences between implementations. */
typedef struct sfm_ba_iter {
    int32_t iteration;
    int32_t step_is_valid;
    int32_t step_is_successful;
    int32_t reserved;
    double cost;
    double cost_change;
    double model_cost_change;
    double relative_decrease;
    double trust_region_radius;  /* radius after the iteration's update */
    double step_norm;
    double gradient_max_norm;
} sfm_ba_iter;

/* [cpu] Ceres defaults as used by BundleAdjuster() (BundleAdjuster.h:167-174). */
void sfm_ba_default_options(sfm_ba_options* opts);

/* One-shot: upload, solve, and (only if usable) write extr/intr/X back —
 * mirrors BundleAdjuster::operator() (BundleAdjuster.h:176-186).  With
 * world_size>1 every rank passes the full problem; each rank solves the
 * landmark shard sfm_ba_partition assigns it and writes back the cameras and
 * its own points only. */
int sfm_ba_solve(sfm_ctx* ctx, const sfm_ba_problem* prob,
                 double* extr, double* intr, double* X,
                 const sfm_ba_options* opts, sfm_ba_summary* summary);
/* sfm_ba_solve keeps its last plan in the context: a later call whose problem
 * has the same structure (n_*, pt_offsets, obs_img, img_intr, const_img,
 * camera_model -- compared exactly) reuses it and only uploads the new values
 * (a world that did not grow since the previous BundleAdjuster call,
 * SequentialActuator.h:226-229).  A call whose problem grows the cached one
 * (the same images, intrinsics map, gauge and model, with images, points and
 * observations only appended: every point keeps its observations in order
 * and may gain new ones at the end -- the next call of the incremental loop,
 * SequentialActuator.h:226-229 after addSingleImage, main.cpp:99-108) plans
 * only what the growth moved and takes the rest from the cached plan, with
 * the same result as a fresh plan bit for bit (world 1).  This releases that
 * plan (its device memory); sfm_ctx_destroy does too.  SFM_BA_NO_PLAN_CACHE=1
 * turns the cache off, SFM_BA_NO_GROWN_PLAN=1 the growth only. */
int sfm_ba_cache_clear(sfm_ctx* ctx);
/* [diagnostic] sfm_ba_solve calls on this context that reused the cached plan
 * as it was, grew it, or planned from scratch. */
int sfm_ba_cache_stats(sfm_ctx* ctx, int64_t* reused, int64_t* grown, int64_t* fresh);

/* Resident variant (used by the benchmark): the plan uploads the problem and
 * the initial parameters once; every sfm_ba_plan_run restarts from those
 * initial parameters with all data already in HBM. */
typedef struct sfm_ba_plan sfm_ba_plan;
int sfm_ba_plan_create(sfm_ctx* ctx, const sfm_ba_problem* prob,
                       const double* extr, const double* intr, const double* X,
                       sfm_ba_plan** out);
int sfm_ba_plan_run(sfm_ba_plan* plan, const sfm_ba_options* opts,
                    sfm_ba_summary* summary);
int sfm_ba_plan_download(sfm_ba_plan* plan, double* extr, double* intr, double* X);
int sfm_ba_plan_destroy(sfm_ba_plan* plan);

typedef struct sfm_ba_plan_info {
    int64_t shard_pt_begin, shard_pt_end;   /* rank's range in sorted order   */
    int64_t shard_obs;                      /* observations on this rank      */
    int32_t n_chunks;                       /* Schur work chunks              */
    int32_t band_blocks;                    /* block half-bandwidth D of S    */
    int32_t n_cam_active, n_intr_active;    /* RCS blocks                     */
    int64_t rcs_dim;                        /* 6*n_cam_active+w*n_intr_active */
    double  last_kernel_ms[8];              /* per-phase device time of the
                                               last iteration (HIP events)   */
    int64_t schur_flops_per_iter;           /* algorithmic flops, Schur kernel*/
    int64_t schur_launches;                 /* timed Schur launches, last run  */
    double  schur_ms_total;                 /* their summed kernel time (HIP
                                               events; only with the
                                               SFM_SCHUR_TIME_ALL diagnostic:
                                               an event pair serialises the
                                               stream, 0 launches otherwise) */
    int32_t rcs_solver;                     /* SFM_RCS_* the plan solves with  */
    int32_t tile_rows;                      /* Schur chunk tile height (64/80) */
} sfm_ba_plan_info;
/* sfm_ba_plan_info.rcs_solver */
#define SFM_RCS_BCR       0   /* block cyclic reduction of the band + arrow   */
#define SFM_RCS_DENSE     1   /* blocked dense Cholesky                      */
#define SFM_RCS_SEQ_BAND  2   /* sequential block-band Cholesky              */
int sfm_ba_plan_get_info(sfm_ba_plan* plan, sfm_ba_plan_info* info);
/* Iteration log of the last sfm_ba_plan_run (n <= cap entries written). */
int sfm_ba_plan_get_trace(sfm_ba_plan* plan, sfm_ba_iter* out, int32_t cap, int32_t* n);

/* [cpu] Structure the planner chooses for a problem (no device needed):
 * Schur chunks vs general points (any track length, repeated views, many
 * intrinsics blocks), camera half-bandwidth after ordering, and the reduced
 * camera system's form (dense = 1: blocked dense Cholesky; 0: block-banded
 * cyclic reduction). */
typedef struct sfm_ba_plan_shape {
    int32_t n_chunks, band_blocks, dense, n_cam_active, n_intr_active, tile_rows;
    int64_t n_chunk_pts, n_general_pts, rcs_dim, n_targets, n_terms, n_pterms;
} sfm_ba_plan_shape;
int sfm_ba_describe(const sfm_ba_problem* prob, int32_t rank, int32_t world_size, sfm_ba_plan_shape* out);

/* [cpu] Diagnostic (tests): plans `prob` twice -- from scratch, and grown
 * from the plan of `prev` (sfm_ba_solve's path when a problem extends the
 * previous call's: SequentialActuator::bundleAdjustment after
 * addSingleImage, src/actuator/SequentialActuator.h:226-229) -- and returns
 * the FNV-1a digest of every plan array the device reads in each (the
 * measurements excluded: a grown plan gathers them on the device).
 * *reused = the sorted points the grown plan took over from prev's plan, -1
 * when prob does not grow prev or prev's plan cannot seed it (digest_grown
 * then 0). */
int sfm_ba_grown_digest(const sfm_ba_problem* prev, const sfm_ba_problem* prob, uint64_t* digest_fresh,
                        uint64_t* digest_grown, int64_t* reused);

/* [cpu] Diagnostic (tests): the schedule of the dense RCS dataflow solve
 * (dense_flow_kernel) for `prob`'s plan, as the device reads it: permuted
 * tile order | previous column per chain | link / D / S bits | lookahead row
 * | chain 0 list | chain 1 list | the two lengths | tasks (kind << 24 | i << 12
 * | j, in execution order) | the tile pattern of L (nt * nt bytes).  Copies it
 * to out when *n_words <= cap (cap 0: size query).  shape[7] = {nt, chains,
 * tasks, 1 if the dataflow solve runs, nF, nb, camera half-bandwidth}; no schedule (n_words 0) for a
 * band problem or a system over the dataflow solve's size. */
int sfm_ba_dense_schedule(const sfm_ba_problem* prob, int32_t* out, int64_t cap, int64_t* n_words, int32_t* shape);

/* [cpu] Landmark-block partition: contiguous point ranges of the
 * (min-camera)-sorted point order with ~equal observation counts.
 * order[n_pt] receives the sorted point order, bounds[world_size+1] the
 * ranges into it. */
int sfm_ba_partition(const sfm_ba_problem* prob, int32_t world_size,
                     int64_t* order, int64_t* bounds);

/* [cpu] Deterministic synthetic scenes.  Two calls: first with
 * NULL arrays to get sizes, then with caller-allocated arrays.  vis_mode 0 =
 * banded orbit visibility (k consecutive cameras), 1 = random k cameras,
 * 2 = closed orbit (k consecutive cameras modulo n_cam).
 * gt_* receive ground truth, extr/intr/X the perturbed initial point. */
typedef struct sfm_synth_ba_config {
    int32_t n_cam, k, vis_mode, n_intr;   /* n_intr 1 = shared intrinsics      */
    int64_t n_pt;
    uint64_t seed;
    double noise_px, outlier_frac;        /* 0.5, 0.01                         */
    double perturb_rot, perturb_t, perturb_X, perturb_f; /* .01,.05,.05,5      */
    int32_t const_img;                    /* gauge (1)                          */
    int32_t camera_model;                 /* SFM_CAM_*; SNAVELY: f 1000,
                                             l1 -0.08, l2 0.02 (+ perturbation);
                                             RADIAL3: pinhole f / principal point,
                                             k1 -0.05, k2 0.01, k3 -0.002
                                             (intr / gt_intr 6 doubles a block) */
} sfm_synth_ba_config;
int sfm_synth_ba(const sfm_synth_ba_config* cfg,
                 int64_t* pt_offsets, int32_t* obs_img, double* obs_uv,
                 int32_t* img_intr, double* extr, double* intr, double* X,
                 double* gt_extr, double* gt_intr, double* gt_X,
                 int64_t* n_obs_out);

/* ------------------------------------------------------------------------ */
/* Descriptor matching (128-D uint8 SIFT/RootSIFT, exact integer L2^2)       */
/* ------------------------------------------------------------------------ */
#define SFM_MATCH_RATIO   0   /* Matcher_Regions(0.8, BRUTE_FORCE_L2): for each
                                 query j of image J, top-2 over image I; keep
                                 if d1 < fl32(ratio*ratio)*d2; emit (i, j)   */
#define SFM_MATCH_MUTUAL  1   /* BFMatcher(NORM_L2, crossCheck) knnMatch k=1:
                                 keep (i, j) iff j = NN_J(i) and i = NN_I(j) */
#define SFM_MATCH_CASCADE 2   /* Cascade_Hashing_Matcher_Regions(0.8), the
                                 "AUTO" default (sparseBuilder.cpp:811-814,
                                 911-914): per query j of J, candidates of I
                                 sharing one of 6 hash buckets, top-10 by
                                 Hamming distance re-ranked by exact L2^2,
                                 ratio test as RATIO; emit (i, j).  The
                                 zero-mean descriptor is taken over the
                                 images of the run's pair list.             */

typedef struct sfm_match_options {
    int32_t mode;            /* SFM_MATCH_*                                    */
    float ratio;             /* fDistRatio (sparseBuilder.cpp:812): 0.8f       */
} sfm_match_options;

/* Single image pair, dense output (behind LocalFrame/GlobalFrame::matchFeature).
 * Descriptors are row-major [n][128] uint8.  For RATIO the database is `a`
 * and the queries are `b` (OpenMVG: regions I vs queries J); for MUTUAL `a`
 * is the OpenCV query set and `b` the train set.  Outputs, per row of `b`
 * (RATIO) or per row of `a` (MUTUAL): the matched index in the other set or
 * -1, and the exact squared L2 distance of that match. */
int sfm_match_dense(sfm_ctx* ctx, const uint8_t* a, int32_t n_a,
                    const uint8_t* b, int32_t n_b,
                    const sfm_match_options* opts,
                    int32_t* match_idx, int32_t* match_d2);

/* The same with float descriptors: the cv::Mat CV_32F rows cv::SIFT gives
 * LocalFrame/GlobalFrame::matchFeature (src/frame/LocalFrame.h:38,
 * GlobalFrame.h:28-34, src/component/Image.h:39-41).  OpenCV's SIFT stores
 * saturate_cast<uchar> values in them, so rows whose every value is an
 * integer in [0, 255] are converted exactly and matched on the u8 path
 * (distances exact integers, < 2^24, hence exact floats).  Any other input is
 * matched in f32: d = sum_k (a_k - b_k)^2 accumulated as an fmaf chain in k
 * order (first minimum wins), bit for bit the oracle's restatement; OpenCV's
 * own SIMD summation order is not pinned for such input.  match_d2 is the
 * squared distance (DMatch.distance = sqrtf of it), -1 where unmatched. */
int sfm_match_dense_f32(sfm_ctx* ctx, const float* a, int32_t n_a,
                        const float* b, int32_t n_b,
                        const sfm_match_options* opts,
                        int32_t* match_idx, float* match_d2);

/* All-pairs matching over a resident descriptor collection. */
typedef struct sfm_match_plan sfm_match_plan;
/* desc: concatenated [sum n_img][128] uint8; desc_offsets[n_img+1]. */
int sfm_match_plan_create(sfm_ctx* ctx, const uint8_t* desc,
                          const int64_t* desc_offsets, int32_t n_img,
                          sfm_match_plan** out);
/* Float collection (the rules of sfm_match_dense_f32; SFM_MATCH_CASCADE
 * needs integer-valued descriptors and returns SFM_ERR_UNSUPPORTED
 * otherwise). */
int sfm_match_plan_create_f32(sfm_ctx* ctx, const float* desc,
                              const int64_t* desc_offsets, int32_t n_img,
                              sfm_match_plan** out);
/* pairs[2*n_pairs] = (I, J).  Results stay on the device. */
int sfm_match_plan_run(sfm_match_plan* plan, const int32_t* pairs,
                       int64_t n_pairs, const sfm_match_options* opts,
                       int64_t* total_matches);
/* SFM_MATCH_CASCADE tables (codes, buckets, zero-mean descriptor) for the
 * images of this pair list, as Cascade_Hashing_Matcher_Regions::Match builds
 * them for its whole pair list.  Later CASCADE runs whose images are a subset
 * reuse them, so a list split over ranks or batches matches exactly as the
 * whole list does; a run touching other images re-hashes for its own list. */
int sfm_match_plan_cascade_index(sfm_match_plan* plan, const int32_t* pairs,
                                 int64_t n_pairs);
/* Fetch: counts[n_pairs]; i/j/d2[total] pair-ordered, each pair's matches
 * sorted by (i, j) as openMVG IndMatch::getDeduplicated leaves them (the
 * keypoint-coordinate decorator is applied by sfm_sparse_match only). */
int sfm_match_plan_fetch(sfm_match_plan* plan, int64_t* counts,
                         uint32_t* i, uint32_t* j, int32_t* d2);
/* The same with float squared distances (any collection; a non-integer f32
 * collection has only this one). */
int sfm_match_plan_fetch_f32(sfm_match_plan* plan, int64_t* counts,
                             uint32_t* i, uint32_t* j, float* d2);
/* Order-independent digest of the last run's results (checksum of per-pair
 * checksums) computed on the device. */
int sfm_match_plan_digest(sfm_match_plan* plan, uint64_t* digest);
int sfm_match_plan_get_last_ms(sfm_match_plan* plan, double* kernel_ms,
                               int64_t* launches);
int sfm_match_plan_destroy(sfm_match_plan* plan);

/* [cpu] exhaustive pair list of openMVG exhaustivePairs(N)
 * (sparseBuilder.cpp:786): all (i, j), 0 <= i < j < N, in i-major order.
 * pairs[2 * N*(N-1)/2]. */
int sfm_exhaustive_pairs(int32_t n_img, int32_t* pairs);

/* [cpu] Deterministic synthetic RootSIFT-like descriptors for config C3:
 * n_img frames x n_kp descriptors; frames share landmark descriptors with
 * their neighbours (true correspondences) plus integer noise. */
int sfm_synth_descriptors(int32_t n_img, int32_t n_kp, uint64_t seed,
                          uint8_t* desc /* [n_img*n_kp*128] */);

/* ------------------------------------------------------------------------ */
/* Incremental loop: SequentialActuator (src/actuator/SequentialActuator.h)  */
/* as src/main.cpp:99-108 drives it (BASELINE.json config C5):               */
/*   init(img0, img1); bundleAdjustment();                                  */
/*   for i >= 2 { addSingleImage(img_i); bundleAdjustment(); }               */
/* LocalFrame mutual matching + 4*min filter and GlobalFrame world-point     */
/* matching + 3*min filter run on the GPU matcher (sfm_match_dense MUTUAL);  */
/* bundleAdjustment is a fresh BundleAdjuster over the whole world per call  */
/* (:226-229) on the GPU solver (sfm_ba_solve).  The OpenCV geometry          */
/* (findEssentialMat / recoverPose / solvePnPRansac) is out of scope: each   */
/* image carries the pose that solver would return (pose_prior) and the      */
/* inlier masks are geometric checks against the current poses (the C++      */
/* header include/sfm/actuator.hpp documents each stand-in).                 */
/* ------------------------------------------------------------------------ */
typedef struct sfm_seq_image {
    int32_t n_kp;
    int32_t reserved;
    const double* kp_xy;     /* [2*n_kp] keypoint pixel coordinates           */
    const uint8_t* desc;     /* [n_kp*128] descriptors (RootSIFT uchar)       */
    double pose_prior[6];    /* Tcw as angle-axis + t (the geometric solver's
                                output; image 0's is ignored: Tcw = I)       */
} sfm_seq_image;

typedef struct sfm_seq_options {
    double fx, fy, cx, cy;   /* the one shared Camera (main.cpp:91,124)       */
    double epipolar_px;      /* essential-matrix inlier threshold, px (4.0)   */
    double pnp_reproj_px;    /* solvePnPRansac reprojectionError (8.0, :179)  */
    double max_depth;        /* recoverPose distanceThresh (100)              */
    int64_t min_pnp_inliers; /* drop the image below this (30, :191)          */
    int32_t fixed_writeback; /* 0: Image::setIntrinsic ZYX-Euler quirk (the
                                reference); 1: store the angle-axis          */
    int32_t reserved;
    sfm_ba_options ba;       /* BundleAdjuster() solver options               */
} sfm_seq_options;

/* What one init / addSingleImage (+ the following bundleAdjustment) did. */
typedef struct sfm_seq_step {
    int32_t image;              /* sequence index of the new image           */
    int32_t kept;               /* 0: dropped (< min_pnp_inliers)            */
    int64_t local_raw, local_kept;     /* LocalFrame matches before / after
                                          the 4*min filter                  */
    int64_t global_raw, global_kept;   /* GlobalFrame, 3*min filter          */
    int64_t pnp_inliers, epipolar_inliers;
    int64_t new_points, extended_obs;  /* savePointCloudToWorld             */
    int64_t world_points, world_observations;
    sfm_ba_summary ba;          /* last bundleAdjustment of this step        */
    int32_t ba_rc;              /* its return code (1: not run yet)          */
    int32_t reserved;
    int64_t ba_images, ba_points, ba_observations;   /* its problem size    */
    double seconds_local_match, seconds_global_match, seconds_geometry, seconds_ba;
} sfm_seq_step;

typedef struct sfm_seq sfm_seq;
/* [cpu] SequentialActuator defaults + BundleAdjuster() options. */
void sfm_seq_default_options(sfm_seq_options* opts);
int sfm_seq_create(sfm_ctx* ctx, const sfm_seq_options* opts, sfm_seq** out);
int sfm_seq_init(sfm_seq* seq, const sfm_seq_image* img0, const sfm_seq_image* img1);
/* *kept = 0 when the image was dropped (fewer than min_pnp_inliers). */
int sfm_seq_add_image(sfm_seq* seq, const sfm_seq_image* img, int32_t* kept);
int sfm_seq_bundle_adjust(sfm_seq* seq, sfm_ba_summary* summary);
int sfm_seq_last_step(sfm_seq* seq, sfm_seq_step* step);
/* The last step's filtered matches: which 0 = LocalFrame (query = image1
 * keypoint, train = image2 keypoint), 1 = GlobalFrame (query = world point in
 * index order, train = image keypoint).  dist = sqrt of the exact L2^2. */
int sfm_seq_matches(sfm_seq* seq, int32_t which, int32_t* query, int32_t* train,
                    float* dist, int64_t cap, int64_t* n);
/* World state: points in index order (X[3*n]), the observation count of
 * each (n_obs[n]), every image's pose in sequence order (poses[6*n_img]) and
 * the shared camera's {fx, fy, cx, cy}.  NULL arrays: sizes only. */
int sfm_seq_world(sfm_seq* seq, double* X, int64_t* n_obs, int64_t cap_pts, int64_t* n_pts,
                  double* poses, int32_t cap_img, int32_t* n_img, double* intr4);
/* Every world point's observations, points in index order (counts from
 * sfm_seq_world's n_obs): the observing image's sequence index and the pixel. */
int sfm_seq_observations(sfm_seq* seq, int32_t* img, double* uv, int64_t cap, int64_t* n);
int sfm_seq_destroy(sfm_seq* seq);

/* [cpu] Synthetic closed-orbit image sequence for C5: cameras on a circle of
 * radius 10 around a cube of landmarks (side 4), looking at its centre, all
 * with the reference intrinsics (fx = fy = 2905.88, cx 1416, cy 1064).  Each
 * landmark faces a direction and is seen from an arc of consecutive images
 * (tracks of ~track_mean images), detected with detect_prob; its observed
 * descriptor is a RootSIFT-like base with desc_noise_dims entries moved by up
 * to +-desc_noise_amp.  n_clutter unmatched keypoints per image.  Keypoint
 * order is shuffled per image.  pose_prior = ground-truth Tcw relative to
 * image 0 (the reconstruction's world frame) + N(0, prior_rot^2) rad /
 * N(0, prior_t^2) noise; image 0's is exactly zero. */
typedef struct sfm_synth_orbit_config {
    int32_t n_img, n_clutter;
    int64_t n_landmarks;
    double track_mean, detect_prob, noise_px;
    int32_t desc_noise_dims, desc_noise_amp;
    double prior_rot, prior_t;
    uint64_t seed;
} sfm_synth_orbit_config;
/* Two calls: NULL arrays return *n_kp only.  landmark[n_kp] (optional):
 * ground-truth landmark of each keypoint or -1 for clutter; gt_X (optional,
 * [3*n_landmarks]) landmark positions in the image-0 frame. */
int sfm_synth_orbit_image(const sfm_synth_orbit_config* cfg, int32_t img, int32_t* n_kp,
                          double* kp_xy, uint8_t* desc, double* pose_prior,
                          int64_t* landmark, double* gt_X);

/* ------------------------------------------------------------------------ */
/* File-staged sparseBuilder flow.                   */
/* The reference's matchPair()/match() (sparseBuilder.cpp:758-1023) talk to  */
/* each other through files in <base>/output/matches written by OpenMVG's    */
/* Load/Save (cereal).  These functions read and write the same layouts      */
/* natively (restated from OpenMVG's published code; OpenMVG is un-vendored, */
/* so byte parity is unpinned — DESIGN.md §3).  Pass NULL output arrays to   */
/* query sizes first.                                                        */
/* ------------------------------------------------------------------------ */
typedef struct sfm_mvg_view {  /* openMVG::sfm::View                         */
    uint32_t id_view, id_intrinsic, id_pose, width, height;
    char img_path[500];        /* View::s_Img_path = local_path/filename      */
} sfm_mvg_view;

/* [cpu] VIEWS of an sfm_data.json (Load(sfm_data, ..., VIEWS), :773, :835),
 * sorted by id_view. */
int sfm_mvg_load_views(const char* sfm_data_json, sfm_mvg_view* views,
                       int32_t cap, int32_t* n_views);
/* [cpu] image_describer.json names 128-D uint8 SIFT_Regions (:851-856);
 * other region types return SFM_ERR_UNSUPPORTED. */
int sfm_mvg_check_describer(const char* image_describer_json);
/* [cpu] <stem>.desc: uint64 count, count x 128 uint8 (saveDescsToBinFile). */
int sfm_mvg_read_desc(const char* path, uint8_t* desc, int64_t cap_rows, int64_t* n_rows);
int sfm_mvg_write_desc(const char* path, const uint8_t* desc, int64_t n_rows);
/* [cpu] <stem>.feat: text "x y scale orientation" per keypoint (SIOPointFeature). */
int sfm_mvg_read_feat(const char* path, float* xyso /* [4*n] */, int64_t cap_rows, int64_t* n_rows);
/* [cpu] pairs.bin (text despite its name): loadPairs(N, ...) / savePairs
 * (:801, :948): lines "I J1 J2 ...", stored as sorted unique (min, max). */
int sfm_mvg_load_pairs(const char* path, int32_t n_views, int32_t* pairs, int64_t cap,
                       int64_t* n_pairs);
int sfm_mvg_save_pairs(const char* path, const int32_t* pairs, int64_t n_pairs);
/* [cpu] PairWiseMatches Save/Load (:986, :896): ".bin" = cereal
 * PortableBinary (uint8 1; uint64 #pairs; per pair uint32 I, J, uint64 n,
 * n x (uint32 i, j)), ".txt" = "I J\nn\ni j\n...".  pairs strictly increasing. */
int sfm_mvg_save_matches(const char* path, const int32_t* pairs, int64_t n_pairs,
                         const int64_t* counts, const uint32_t* i, const uint32_t* j);
int sfm_mvg_load_matches(const char* path, int32_t* pairs, int64_t* counts,
                         uint32_t* i, uint32_t* j, int64_t cap_pairs, int64_t cap_matches,
                         int64_t* n_pairs, int64_t* n_matches);

/* [cpu] sparseBuilder::matchPair(): <matches_dir>/pairs.bin =
 * exhaustivePairs(#views of sfm_data.json). */
int sfm_sparse_match_pair(const char* matches_dir);

typedef struct sfm_sparse_match_opts {
    int32_t mode;      /* SFM_MATCH_CASCADE = "AUTO", the reference's default
                          (:814, :911-914); SFM_MATCH_RATIO = "BRUTEFORCEL2"
                          (:919-921); NULL opts select CASCADE             */
    float ratio;       /* fDistRatio 0.8f (:812)                              */
    int32_t force;     /* 0: reload an existing matches.putative.bin (:890)   */
    int32_t dedup_xy;  /* 1: drop matches whose keypoint coordinates repeat
                          (IndMatchDecorator, needs <stem>.feat)             */
    int32_t reserved[2];
} sfm_sparse_match_opts;
typedef struct sfm_sparse_match_stats {
    int64_t n_views, n_pairs_in, n_pairs_out, n_matches;
    int32_t reloaded, reserved;
} sfm_sparse_match_stats;
/* sparseBuilder::match(), file-staged: sfm_data.json + image_describer.json
 * + <stem>.desc/.feat + pairs.bin -> GPU matcher ->
 * matches.putative.bin (non-empty pairs) + preemptive_pairs.txt.
 * pairs.bin must exist (the reference's loadPairs fails without it, :957-960:
 * SFM_ERR_INVALID_ARG).  opts NULL = {CASCADE ("AUTO"), 0.8f, 0, 1}.
 * dedup_xy keeps the survivors in the order OpenMVG's
 * IndMatchDecorator::getDeduplicated leaves them (std::set over its
 * coordinate comparator, inserted in (i, j) order). */
int sfm_sparse_match(sfm_ctx* ctx, const char* matches_dir, const sfm_sparse_match_opts* opts,
                     sfm_sparse_match_stats* stats);

/* ------------------------------------------------------------------------ */
/* Geometric filter                                  */
/* sparseBuilder::filter() (sparseBuilder.cpp:1025-1280) runs                */
/* GeometricFilter_FMatrix_AC(4.0, 2048) (:1179-1186) over every putative    */
/* pair: OpenMVG's a-contrario RANSAC (ACRANSAC) with the 7-point            */
/* fundamental-matrix solver, keeping a pair iff it has > 2.5 * 7 inliers.   */
/* Restated from OpenMVG's published code (un-vendored: parity unpinned,     */
/* DESIGN.md §3); the GPU runs one workgroup per pair.                       */
/* ------------------------------------------------------------------------ */
typedef struct sfm_fmatrix_opts {
    double precision;         /* 4.0 px: upper bound of the a-contrario threshold */
    int32_t max_iterations;   /* 2048 (imax_iteration, :1040)                     */
    int32_t reserved;
} sfm_fmatrix_opts;
typedef struct sfm_fmatrix_result {
    double F[9];          /* row-major, pixels: x_J' F x_I = 0 (when n_inliers > 0)  */
    double error_max;     /* a-contrario threshold in px (ACRANSAC .first)          */
    double min_nfa;       /* log10 NFA of the best model (ACRANSAC .second)         */
    int32_t n_inliers;    /* > 17 when the pair is kept, else 0                     */
    int32_t iterations;   /* RANSAC iterations run                                  */
} sfm_fmatrix_result;
/* n_pairs independent pairs.  Pair q's putative correspondences are
 * k = off[q] .. off[q+1]-1 with xy[4k..4k+3] = (x_I, y_I, x_J, y_J) in pixels
 * (MatchesPairToMat order = the putative IndMatch order); wh[4q..4q+3] =
 * (width_I, height_I, width_J, height_J).  inliers[off[q] + t],
 * t < results[q].n_inliers: the kept correspondences (indices into the pair's
 * list) in OpenMVG's vec_inliers order (ascending residual).  opts NULL =
 * {4.0, 2048}.  Pairs of any size (sort buffers move from LDS to global
 * memory above 8192 correspondences); a pair whose RANSAC would draw more than
 * 2^18 random numbers (2048 iterations draw about 15,000) returns
 * SFM_ERR_UNSUPPORTED. */
int sfm_fmatrix_ac(sfm_ctx* ctx, int64_t n_pairs, const int64_t* off, const double* xy,
                   const int32_t* wh, const sfm_fmatrix_opts* opts,
                   sfm_fmatrix_result* results, int32_t* inliers);

/* Device time (HIP events on the context's stream) of the kernel of the
 * context's last sfm_fmatrix_ac call, without its host normalisation,
 * uploads and downloads (measurement; no reference counterpart).  Only a
 * context created with SFM_CTX_TIME_KERNELS times it; -1 otherwise. */
int sfm_ctx_last_kernel_ms(sfm_ctx* ctx, double* ms);

/* sparseBuilder::filter(), file-staged: sfm_data.json (view sizes) +
 * <stem>.feat + matches.putative.bin -> sfm_fmatrix_ac ->
 * matches.f.bin (kept pairs, each pair's IndMatches in vec_inliers order).
 * opts NULL = {4.0, 2048}. */
typedef struct sfm_sparse_filter_stats {
    int64_t n_pairs_in, n_pairs_out, n_matches_in, n_matches_out;
} sfm_sparse_filter_stats;
int sfm_sparse_filter(sfm_ctx* ctx, const char* matches_dir, const sfm_fmatrix_opts* opts,
                      sfm_sparse_filter_stats* stats);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif /* SFMCORE_H */
