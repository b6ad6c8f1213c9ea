"""ctypes mirror of include/sfmcore.h (plumbing for tests and bench.py).

The product is libsfmcore.so (HIP kernels + C-ABI); this module only
describes its structs and loads it.  Loading order matters on ROCm: torch
ships its own libamdhip64.so.7 / librccl.so.1 and both libraries must share
one HIP runtime, so torch is imported (if available) before the library.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libsfmcore.so")

SFM_OK = 0
SFM_ERR_INVALID_ARG = -1
SFM_ERR_DEVICE = -2
SFM_ERR_NOT_FINITE = -3
SFM_ERR_UNSUPPORTED = -4
SFM_ERR_COMM = -5
SFM_ERR_OOM = -6
SFM_ERR_SOLVER = -7

SFM_TERM_CONVERGENCE = 0
SFM_TERM_NO_CONVERGENCE = 1
SFM_TERM_FAILURE = 2

SFM_CAM_PINHOLE = 0
SFM_CAM_SNAVELY = 1
SFM_CAM_RADIAL3 = 2

SFM_CTX_TUNE_HOST_MALLOC = 1
SFM_CTX_DIAG_NO_EXCHANGE = 2
SFM_CTX_DIAG_FAIL_SOLVE_WAIT = 4
SFM_CTX_TIME_KERNELS = 8
SFM_CTX_BA_DENSE_RCS = 1 << 4
SFM_CTX_BA_SEQ_BAND = 1 << 5
SFM_CTX_BA_TILE80 = 1 << 6
SFM_CTX_BA_SPLIT_REDUCE = 1 << 7
SFM_CTX_BA_SPLIT_BCR = 1 << 8
SFM_CTX_BA_NO_SPEC_GRAM = 1 << 10
SFM_CTX_DIAG_SPEC_ALWAYS = 1 << 11
SFM_CTX_BA_DENSE_CHAIN = 1 << 9


def SFM_CTX_BA_STEP_LANES(n):
    return {1: 1, 2: 2, 4: 3, 8: 4}[n] << 12


def SFM_CTX_BA_REDUCE_WAVES(n):
    return {1: 1, 2: 2, 4: 3}[n] << 15


SFM_RCS_BCR, SFM_RCS_DENSE, SFM_RCS_SEQ_BAND = 0, 1, 2

SFM_MATCH_RATIO = 0
SFM_MATCH_MUTUAL = 1
SFM_MATCH_CASCADE = 2

i32p = C.POINTER(C.c_int32)
i64p = C.POINTER(C.c_int64)
u32p = C.POINTER(C.c_uint32)
f32p = C.POINTER(C.c_float)
u64p = C.POINTER(C.c_uint64)
u8p = C.POINTER(C.c_uint8)
f64p = C.POINTER(C.c_double)


class CtxOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("rank", C.c_int32), ("world_size", C.c_int32),
                ("flags", C.c_int32), ("comm_id", u8p),
                ("allreduce", C.c_void_p), ("allreduce_user", C.c_void_p)]


# int32_t (*)(void* user, double* buf, int64_t n, int32_t op)
ALLREDUCE_HOOK = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.POINTER(C.c_double), C.c_int64, C.c_int32)


class BAProblem(C.Structure):
    _fields_ = [("n_img", C.c_int32), ("n_intr", C.c_int32), ("n_pt", C.c_int64),
                ("n_obs", C.c_int64), ("pt_offsets", i64p), ("obs_img", i32p),
                ("obs_uv", f64p), ("img_intr", i32p), ("const_img", C.c_int32),
                ("camera_model", C.c_int32), ("huber_a", C.c_double)]


class BAOptions(C.Structure):
    _fields_ = [("max_num_iterations", C.c_int32),
                ("max_num_consecutive_invalid_steps", C.c_int32),
                ("jacobi_scaling", C.c_int32), ("reserved", C.c_int32),
                ("function_tolerance", C.c_double), ("gradient_tolerance", C.c_double),
                ("parameter_tolerance", C.c_double),
                ("initial_trust_region_radius", C.c_double),
                ("max_trust_region_radius", C.c_double),
                ("min_trust_region_radius", C.c_double),
                ("min_relative_decrease", C.c_double), ("min_lm_diagonal", C.c_double),
                ("max_lm_diagonal", C.c_double)]


class BASummary(C.Structure):
    _fields_ = [("initial_cost", C.c_double), ("final_cost", C.c_double),
                ("num_residuals", C.c_int64), ("iterations", C.c_int32),
                ("successful_steps", C.c_int32), ("unsuccessful_steps", C.c_int32),
                ("termination", C.c_int32), ("usable", C.c_int32), ("reserved", C.c_int32),
                ("rmse_initial", C.c_double), ("rmse_final", C.c_double),
                ("seconds", C.c_double)]


class BAIter(C.Structure):
    _fields_ = [("iteration", C.c_int32), ("step_is_valid", C.c_int32),
                ("step_is_successful", C.c_int32), ("reserved", C.c_int32),
                ("cost", C.c_double), ("cost_change", C.c_double),
                ("model_cost_change", C.c_double), ("relative_decrease", C.c_double),
                ("trust_region_radius", C.c_double), ("step_norm", C.c_double),
                ("gradient_max_norm", C.c_double)]


class BAPlanInfo(C.Structure):
    _fields_ = [("shard_pt_begin", C.c_int64), ("shard_pt_end", C.c_int64),
                ("shard_obs", C.c_int64), ("n_chunks", C.c_int32),
                ("band_blocks", C.c_int32), ("n_cam_active", C.c_int32),
                ("n_intr_active", C.c_int32), ("rcs_dim", C.c_int64),
                ("last_kernel_ms", C.c_double * 8), ("schur_flops_per_iter", C.c_int64),
                ("schur_launches", C.c_int64), ("schur_ms_total", C.c_double),
                ("rcs_solver", C.c_int32), ("tile_rows", C.c_int32)]


class BAPlanShape(C.Structure):
    _fields_ = [("n_chunks", C.c_int32), ("band_blocks", C.c_int32), ("dense", C.c_int32),
                ("n_cam_active", C.c_int32), ("n_intr_active", C.c_int32), ("tile_rows", C.c_int32),
                ("n_chunk_pts", C.c_int64), ("n_general_pts", C.c_int64), ("rcs_dim", C.c_int64),
                ("n_targets", C.c_int64), ("n_terms", C.c_int64), ("n_pterms", C.c_int64)]


class SynthBAConfig(C.Structure):
    _fields_ = [("n_cam", C.c_int32), ("k", C.c_int32), ("vis_mode", C.c_int32),
                ("n_intr", C.c_int32), ("n_pt", C.c_int64), ("seed", C.c_uint64),
                ("noise_px", C.c_double), ("outlier_frac", C.c_double),
                ("perturb_rot", C.c_double), ("perturb_t", C.c_double),
                ("perturb_X", C.c_double), ("perturb_f", C.c_double),
                ("const_img", C.c_int32), ("camera_model", C.c_int32)]


class MatchOptions(C.Structure):
    _fields_ = [("mode", C.c_int32), ("ratio", C.c_float)]


class MvgView(C.Structure):
    _fields_ = [("id_view", C.c_uint32), ("id_intrinsic", C.c_uint32), ("id_pose", C.c_uint32),
                ("width", C.c_uint32), ("height", C.c_uint32), ("img_path", C.c_char * 500)]


class SparseMatchOpts(C.Structure):
    _fields_ = [("mode", C.c_int32), ("ratio", C.c_float), ("force", C.c_int32),
                ("dedup_xy", C.c_int32), ("reserved", C.c_int32 * 2)]


class SparseMatchStats(C.Structure):
    _fields_ = [("n_views", C.c_int64), ("n_pairs_in", C.c_int64), ("n_pairs_out", C.c_int64),
                ("n_matches", C.c_int64), ("reloaded", C.c_int32), ("reserved", C.c_int32)]


class SeqImage(C.Structure):
    _fields_ = [("n_kp", C.c_int32), ("reserved", C.c_int32), ("kp_xy", f64p), ("desc", u8p),
                ("pose_prior", C.c_double * 6)]


class SeqOptions(C.Structure):
    _fields_ = [("fx", C.c_double), ("fy", C.c_double), ("cx", C.c_double), ("cy", C.c_double),
                ("epipolar_px", C.c_double), ("pnp_reproj_px", C.c_double),
                ("max_depth", C.c_double), ("min_pnp_inliers", C.c_int64),
                ("fixed_writeback", C.c_int32), ("reserved", C.c_int32), ("ba", BAOptions)]


class SeqStep(C.Structure):
    _fields_ = [("image", C.c_int32), ("kept", C.c_int32),
                ("local_raw", C.c_int64), ("local_kept", C.c_int64),
                ("global_raw", C.c_int64), ("global_kept", C.c_int64),
                ("pnp_inliers", C.c_int64), ("epipolar_inliers", C.c_int64),
                ("new_points", C.c_int64), ("extended_obs", C.c_int64),
                ("world_points", C.c_int64), ("world_observations", C.c_int64),
                ("ba", BASummary), ("ba_rc", C.c_int32), ("reserved", C.c_int32),
                ("ba_images", C.c_int64), ("ba_points", C.c_int64), ("ba_observations", C.c_int64),
                ("seconds_local_match", C.c_double), ("seconds_global_match", C.c_double),
                ("seconds_geometry", C.c_double), ("seconds_ba", C.c_double)]


class SynthOrbitConfig(C.Structure):
    _fields_ = [("n_img", C.c_int32), ("n_clutter", C.c_int32), ("n_landmarks", C.c_int64),
                ("track_mean", C.c_double), ("detect_prob", C.c_double), ("noise_px", C.c_double),
                ("desc_noise_dims", C.c_int32), ("desc_noise_amp", C.c_int32),
                ("prior_rot", C.c_double), ("prior_t", C.c_double), ("seed", C.c_uint64)]


class FMatrixOpts(C.Structure):
    _fields_ = [("precision", C.c_double), ("max_iterations", C.c_int32), ("reserved", C.c_int32)]


class FMatrixResult(C.Structure):
    _fields_ = [("F", C.c_double * 9), ("error_max", C.c_double), ("min_nfa", C.c_double),
                ("n_inliers", C.c_int32), ("iterations", C.c_int32)]


class SparseFilterStats(C.Structure):
    _fields_ = [("n_pairs_in", C.c_int64), ("n_pairs_out", C.c_int64), ("n_matches_in", C.c_int64),
                ("n_matches_out", C.c_int64)]


def default_options():
    o = BAOptions()
    o.max_num_iterations = 50
    o.max_num_consecutive_invalid_steps = 5
    o.jacobi_scaling = 1
    o.function_tolerance = 1e-6
    o.gradient_tolerance = 1e-10
    o.parameter_tolerance = 1e-8
    o.initial_trust_region_radius = 1e4
    o.max_trust_region_radius = 1e16
    o.min_trust_region_radius = 1e-32
    o.min_relative_decrease = 1e-3
    o.min_lm_diagonal = 1e-6
    o.max_lm_diagonal = 1e32
    return o


# (name, restype, argtypes) for every symbol declared in include/sfmcore.h
SIGNATURES = [
    ("sfm_version", C.c_char_p, []),
    ("sfm_last_error", C.c_char_p, []),
    ("sfm_comm_unique_id", C.c_int, [u8p]),
    ("sfm_ctx_create", C.c_int, [C.POINTER(CtxOpts), C.POINTER(C.c_void_p)]),
    ("sfm_ctx_destroy", C.c_int, [C.c_void_p]),
    ("sfm_ctx_last_kernel_ms", C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    ("sfm_ctx_synchronize", C.c_int, [C.c_void_p]),
    ("sfm_ba_default_options", None, [C.POINTER(BAOptions)]),
    ("sfm_ba_solve", C.c_int, [C.c_void_p, C.POINTER(BAProblem), f64p, f64p, f64p,
                               C.POINTER(BAOptions), C.POINTER(BASummary)]),
    ("sfm_ba_cache_clear", C.c_int, [C.c_void_p]),
    ("sfm_ba_cache_stats", C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    ("sfm_ba_plan_create", C.c_int, [C.c_void_p, C.POINTER(BAProblem), f64p, f64p, f64p,
                                     C.POINTER(C.c_void_p)]),
    ("sfm_ba_plan_run", C.c_int, [C.c_void_p, C.POINTER(BAOptions), C.POINTER(BASummary)]),
    ("sfm_ba_plan_download", C.c_int, [C.c_void_p, f64p, f64p, f64p]),
    ("sfm_ba_plan_destroy", C.c_int, [C.c_void_p]),
    ("sfm_ba_plan_get_info", C.c_int, [C.c_void_p, C.POINTER(BAPlanInfo)]),
    ("sfm_ba_plan_get_trace", C.c_int, [C.c_void_p, C.POINTER(BAIter), C.c_int32, i32p]),
    ("sfm_ba_intr_width", C.c_int, [C.c_int32]),
    ("sfm_ba_partition", C.c_int, [C.POINTER(BAProblem), C.c_int32, i64p, i64p]),
    ("sfm_ba_describe", C.c_int, [C.POINTER(BAProblem), C.c_int32, C.c_int32, C.POINTER(BAPlanShape)]),
    ("sfm_ba_grown_digest", C.c_int, [C.POINTER(BAProblem), C.POINTER(BAProblem), C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64), C.POINTER(C.c_int64)]),
    ("sfm_ba_dense_schedule", C.c_int, [C.POINTER(BAProblem), i32p, C.c_int64, i64p, i32p]),
    ("sfm_synth_ba", C.c_int, [C.POINTER(SynthBAConfig), i64p, i32p, f64p, i32p, f64p,
                               f64p, f64p, f64p, f64p, f64p, i64p]),
    ("sfm_match_dense", C.c_int, [C.c_void_p, u8p, C.c_int32, u8p, C.c_int32,
                                  C.POINTER(MatchOptions), i32p, i32p]),
    ("sfm_match_dense_f32", C.c_int, [C.c_void_p, f32p, C.c_int32, f32p, C.c_int32,
                                      C.POINTER(MatchOptions), i32p, f32p]),
    ("sfm_match_plan_create", C.c_int, [C.c_void_p, u8p, i64p, C.c_int32,
                                        C.POINTER(C.c_void_p)]),
    ("sfm_match_plan_create_f32", C.c_int, [C.c_void_p, f32p, i64p, C.c_int32,
                                            C.POINTER(C.c_void_p)]),
    ("sfm_match_plan_fetch_f32", C.c_int, [C.c_void_p, i64p, u32p, u32p, f32p]),
    ("sfm_match_plan_run", C.c_int, [C.c_void_p, i32p, C.c_int64, C.POINTER(MatchOptions),
                                     i64p]),
    ("sfm_match_plan_fetch", C.c_int, [C.c_void_p, i64p, u32p, u32p, i32p]),
    ("sfm_match_plan_cascade_index", C.c_int, [C.c_void_p, i32p, C.c_int64]),
    ("sfm_match_plan_digest", C.c_int, [C.c_void_p, u64p]),
    ("sfm_match_plan_get_last_ms", C.c_int, [C.c_void_p, f64p, i64p]),
    ("sfm_match_plan_destroy", C.c_int, [C.c_void_p]),
    ("sfm_exhaustive_pairs", C.c_int, [C.c_int32, i32p]),
    ("sfm_synth_descriptors", C.c_int, [C.c_int32, C.c_int32, C.c_uint64, u8p]),
    ("sfm_mvg_load_views", C.c_int, [C.c_char_p, C.POINTER(MvgView), C.c_int32, i32p]),
    ("sfm_mvg_check_describer", C.c_int, [C.c_char_p]),
    ("sfm_mvg_read_desc", C.c_int, [C.c_char_p, u8p, C.c_int64, i64p]),
    ("sfm_mvg_write_desc", C.c_int, [C.c_char_p, u8p, C.c_int64]),
    ("sfm_mvg_read_feat", C.c_int, [C.c_char_p, C.POINTER(C.c_float), C.c_int64, i64p]),
    ("sfm_mvg_load_pairs", C.c_int, [C.c_char_p, C.c_int32, i32p, C.c_int64, i64p]),
    ("sfm_mvg_save_pairs", C.c_int, [C.c_char_p, i32p, C.c_int64]),
    ("sfm_mvg_save_matches", C.c_int, [C.c_char_p, i32p, C.c_int64, i64p, u32p, u32p]),
    ("sfm_mvg_load_matches", C.c_int, [C.c_char_p, i32p, i64p, u32p, u32p, C.c_int64, C.c_int64,
                                       i64p, i64p]),
    ("sfm_seq_default_options", None, [C.POINTER(SeqOptions)]),
    ("sfm_seq_create", C.c_int, [C.c_void_p, C.POINTER(SeqOptions), C.POINTER(C.c_void_p)]),
    ("sfm_seq_init", C.c_int, [C.c_void_p, C.POINTER(SeqImage), C.POINTER(SeqImage)]),
    ("sfm_seq_add_image", C.c_int, [C.c_void_p, C.POINTER(SeqImage), i32p]),
    ("sfm_seq_bundle_adjust", C.c_int, [C.c_void_p, C.POINTER(BASummary)]),
    ("sfm_seq_last_step", C.c_int, [C.c_void_p, C.POINTER(SeqStep)]),
    ("sfm_seq_matches", C.c_int, [C.c_void_p, C.c_int32, i32p, i32p, f32p, C.c_int64, i64p]),
    ("sfm_seq_world", C.c_int, [C.c_void_p, f64p, i64p, C.c_int64, i64p, f64p, C.c_int32, i32p,
                                f64p]),
    ("sfm_seq_observations", C.c_int, [C.c_void_p, i32p, f64p, C.c_int64, i64p]),
    ("sfm_seq_destroy", C.c_int, [C.c_void_p]),
    ("sfm_synth_orbit_image", C.c_int, [C.POINTER(SynthOrbitConfig), C.c_int32, i32p, f64p, u8p,
                                        f64p, i64p, f64p]),
    ("sfm_sparse_match_pair", C.c_int, [C.c_char_p]),
    ("sfm_sparse_match", C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(SparseMatchOpts),
                                   C.POINTER(SparseMatchStats)]),
    ("sfm_fmatrix_ac", C.c_int, [C.c_void_p, C.c_int64, i64p, f64p, i32p, C.POINTER(FMatrixOpts),
                                 C.POINTER(FMatrixResult), i32p]),
    ("sfm_sparse_filter", C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(FMatrixOpts),
                                    C.POINTER(SparseFilterStats)]),
]

_lib = None


def load(path=None):
    """Load libsfmcore.so (after torch, so both share one HIP runtime)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    try:
        import torch  # noqa: F401  (shares libamdhip64.so.7 / librccl.so.1)
    except Exception:
        pass
    p = path or os.environ.get("SFMCORE_LIB") or LIB_PATH   # override: A/B of library builds
    if not os.path.exists(p):
        raise RuntimeError(f"libsfmcore.so not built: {p} (run __graft_entry__.build())")
    lib = C.CDLL(p, mode=C.RTLD_GLOBAL)
    missing = []
    for name, res, args in SIGNATURES:
        try:
            fn = getattr(lib, name)
        except AttributeError:
            missing.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    lib.missing_symbols = missing
    if path is None:
        _lib = lib
    return lib


def ptr(a, t):
    """numpy array -> ctypes pointer (None for None)."""
    if a is None:
        return None
    return a.ctypes.data_as(t)
