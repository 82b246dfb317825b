"""ctypes mirror of include/imls_gpu.h (the C ABI) — structures, enums and library loading.

The product library is ``csrc/libimls_gpu.so`` (hand-written HIP for gfx950).  There is no CPU
fallback: `load_library()` raises if the library is missing, and every compute entry point of
the library returns IMLS_ERR_DEVICE when no MI355X is visible.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

PKG_DIR = pathlib.Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "csrc" / "libimls_gpu.so"

IMLS_OK, IMLS_ERR_ARG, IMLS_ERR_DEVICE, IMLS_ERR_STATE, IMLS_ERR_UNSUPPORTED, IMLS_ERR_CAPACITY = 0, -1, -2, -3, -4, -5
IMLS_MATCH_IMLS, IMLS_MATCH_PLANE_ICP = 0, 1
IMLS_SOLVE_LS, IMLS_SOLVE_RANSAC, IMLS_SOLVE_WEIGHTED_LS, IMLS_SOLVE_DRPM = 0, 1, 2, 3
IMLS_FINAL_LS, IMLS_FINAL_WEIGHTED_LS, IMLS_FINAL_DRPM = 0, 1, 2
IMLS_FRAME_MAX_ITERS, IMLS_FRAME_CONVERGED, IMLS_FRAME_TOO_FEW, IMLS_FRAME_SOLVE_FAILED = 0, 1, 2, 3
REJECT_NAMES = ("no_normal", "too_far", "invalid_normal", "normal_constraint", "mls_fail", "nan_inf_height")
IMLS_NUM_REJ = 6
# imls_set_option (include/imls_gpu.h "runtime options"): option ids and the traversal values
(IMLS_OPT_TRAVERSAL, IMLS_OPT_LIST_REUSE, IMLS_OPT_TEMPORAL_SEED, IMLS_OPT_LEAF_SIZE, IMLS_OPT_FIRST_PACKET,
 IMLS_OPT_FIRST_PACKET_ITERS, IMLS_OPT_FIRST_PACKET_BATCHED, IMLS_OPT_TV_SKIN, IMLS_OPT_FORCE_FALLBACK) = range(9)
IMLS_TRAVERSAL_AUTO, IMLS_TRAVERSAL_PACKETS, IMLS_TRAVERSAL_WAVE_PER_QUERY, IMLS_TRAVERSAL_LANE = 0, 1, 2, 3
OPTION_IDS = {"traversal": IMLS_OPT_TRAVERSAL, "list_reuse": IMLS_OPT_LIST_REUSE,
              "temporal_seed": IMLS_OPT_TEMPORAL_SEED, "leaf_size": IMLS_OPT_LEAF_SIZE,
              "first_packet": IMLS_OPT_FIRST_PACKET, "first_packet_iters": IMLS_OPT_FIRST_PACKET_ITERS,
              "first_packet_batched": IMLS_OPT_FIRST_PACKET_BATCHED, "tv_skin": IMLS_OPT_TV_SKIN,
              "force_fallback": IMLS_OPT_FORCE_FALLBACK}

STATUS_NAMES = {0: "IMLS_OK", -1: "IMLS_ERR_ARG", -2: "IMLS_ERR_DEVICE", -3: "IMLS_ERR_STATE",
                -4: "IMLS_ERR_UNSUPPORTED", -5: "IMLS_ERR_CAPACITY"}

_i32, _u32, _f64, _f32 = C.c_int32, C.c_uint32, C.c_double, C.c_float


class ImlsParams(C.Structure):
    """Field-for-field mirror of `imls_params` (include/imls_gpu.h)."""
    _fields_ = [
        ("matching_method", _i32), ("correspond_number", _i32),
        ("h", _f64), ("r", _f64),
        ("get_normals", _i32), ("search_number_normal", _i32),
        ("r_normal", _f64),
        ("use_projected_distance", _i32), ("normal_angle_constraint", _i32),
        ("r_proj", _f64), ("angle_diff_threshold", _f64),
        ("search_number", _i32), ("use_tensor_voting", _i32), ("tensor_k", _i32),
        ("recompute_normal_count_mode", _i32),
        ("tensor_sigma", _f64), ("tensor_distance_threshold", _f64),
        ("picp_r", _f64), ("picp_r_proj", _f64), ("picp_angle_diff_threshold", _f64),
        ("picp_use_projected_distance", _i32), ("picp_normal_angle_constraint", _i32),
        ("solve_method", _i32), ("iterations", _i32),
        ("delta_dist_threshold", _f64), ("delta_angle_threshold", _f64), ("ls_threshold", _f64),
        ("ransac_max_iterations", _i32), ("ransac_final_method", _i32),
        ("ransac_distance_threshold", _f64), ("ransac_min_inliers_percentage", _f64),
        ("ransac_huber_threshold", _f64), ("ransac_ls_threshold", _f64),
        ("drpm_threshold", _f64), ("drpm_stdev_points", _f64), ("drpm_stdev_normals", _f64),
        ("ransac_seed", _u32),
        ("transform_normal", _i32), ("max_queue_size", _i32),
        ("_reserved", _i32 * 4),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if not k.startswith("_")}


class ImlsIterTrace(C.Structure):
    _fields_ = [("delta", _f64 * 16), ("pose", _f64 * 16), ("reject", C.c_uint64 * IMLS_NUM_REJ),
                ("n_valid", C.c_uint64), ("n_kept", C.c_uint64)]


def default_params() -> ImlsParams:
    """The reference's shipped config.json values (laser_odometry section), matching
    imls_default_params() in the library; computed here too so CPU-only code needs no GPU."""
    p = ImlsParams()
    p.matching_method = IMLS_MATCH_IMLS
    p.correspond_number = 6
    p.h, p.r = 1.0, 3.0
    p.get_normals, p.search_number_normal, p.r_normal = 1, 10, 1.0
    p.use_projected_distance, p.r_proj = 0, 0.8
    p.normal_angle_constraint, p.angle_diff_threshold = 1, 30.0
    p.search_number = 20
    p.use_tensor_voting, p.tensor_k, p.tensor_sigma, p.tensor_distance_threshold = 0, 50, 0.2, 0.6
    p.recompute_normal_count_mode = 0
    p.picp_r, p.picp_r_proj, p.picp_angle_diff_threshold = 1.5, 0.8, 30.0
    p.picp_use_projected_distance, p.picp_normal_angle_constraint = 0, 1
    p.solve_method = IMLS_SOLVE_RANSAC
    p.iterations = 30
    p.delta_dist_threshold, p.delta_angle_threshold = 0.001, 0.0001745353
    p.ls_threshold = 0.02
    p.ransac_max_iterations, p.ransac_final_method = 5000, IMLS_FINAL_DRPM
    p.ransac_distance_threshold, p.ransac_min_inliers_percentage = 0.8, 0.95
    p.ransac_huber_threshold, p.ransac_ls_threshold = 0.648, 0.02
    p.drpm_threshold, p.drpm_stdev_points, p.drpm_stdev_normals = 0.05, 0.02, 0.05
    p.ransac_seed = 1
    p.transform_normal, p.max_queue_size = 0, 1
    return p


class ImlsFrontParams(C.Structure):
    _fields_ = [("n_scans", _i32), ("minimum_range", _f32), ("maximum_range", _f32), ("scan_period", _f32),
                ("is_dense", _i32)]


def default_front_params(n_scans: int | None = None) -> "ImlsFrontParams":
    p = ImlsFrontParams()
    load_library().imls_default_front_params(C.byref(p))
    if n_scans is not None:
        p.n_scans = n_scans
    return p


class ImlsPcaParams(C.Structure):
    """imls_pca_params (include/imls_gpu.h): scan_registration.compute_normal_method.pca +
    presample_method.geometric_features (config.json, read at scan_registration.cpp:1140-1145, 1451)."""
    _fields_ = [("window_size", C.c_int32), ("iter_step", C.c_int32), ("knn_distance_threshold", C.c_float),
                ("neighbor_scan", C.c_int32), ("distance_threshold", C.c_float),
                ("valid_points_threshold", C.c_float), ("use_all_points", C.c_int32),
                ("planarity_threshold", C.c_float)]


IMLS_PCA_PLANE_INVALID, IMLS_PCA_CANDIDATE = 1, 2


def default_pca_params() -> ImlsPcaParams:
    """The shipped config.json values (imls_default_pca_params() in the library)."""
    p = ImlsPcaParams()
    p.window_size, p.iter_step, p.knn_distance_threshold, p.neighbor_scan = 3, 1, 10.0, 0
    p.distance_threshold, p.valid_points_threshold = 0.02, 0.8
    p.use_all_points, p.planarity_threshold = 1, 0.05
    return p


class ImlsSampleParams(C.Structure):
    """imls_sample_params (include/imls_gpu.h): scan_registration.sample_method (config.json,
    read at scan_registration.cpp:784-799)."""
    _fields_ = [("method", C.c_int32), ("r", C.c_float), ("r_proj", C.c_float), ("max_total_points", C.c_int32),
                ("azimuth_bins", C.c_int32), ("elevation_bins", C.c_int32), ("min_points_per_bin", C.c_int32),
                ("max_points_per_bin", C.c_int32), ("sampling_strategy", C.c_int32), ("shuffle_seed", C.c_uint32),
                ("rand_seed", C.c_uint32)]


IMLS_SAMPLE_NORMAL, IMLS_SAMPLE_MAJOR_AXIS = 0, 1
SAMPLE_FPS, SAMPLE_RANDOM = 0, 1


def default_sample_params(method: int = IMLS_SAMPLE_MAJOR_AXIS) -> ImlsSampleParams:
    """The shipped config.json values (imls_default_sample_params() in the library)."""
    p = ImlsSampleParams()
    p.method = method
    p.r, p.r_proj, p.max_total_points = 0.5, 1.5, 2000
    p.azimuth_bins = p.elevation_bins = 8
    p.min_points_per_bin = 20
    if method == IMLS_SAMPLE_NORMAL:
        p.max_points_per_bin, p.sampling_strategy = 100, SAMPLE_RANDOM
    else:
        p.max_points_per_bin, p.sampling_strategy = 200, SAMPLE_FPS
    p.shuffle_seed, p.rand_seed = 0, 1
    return p


class ImlsPairInput(C.Structure):
    """imls_pair_input (include/imls_gpu.h)."""
    _fields_ = [("src_xyz", C.c_void_p), ("src_nrm", C.c_void_p), ("n_src", C.c_size_t),
                ("tgt_xyz", C.c_void_p), ("tgt_nrm", C.c_void_p), ("n_tgt", C.c_size_t),
                ("stride_floats", C.c_size_t)]


def _bind(lib: C.CDLL) -> C.CDLL:
    P, VP, SZ = C.POINTER, C.c_void_p, C.c_size_t
    sig = {
        "imls_abi_version": (C.c_int, []),
        "imls_default_params": (None, [P(ImlsParams)]),
        "imls_create": (VP, [C.c_int, P(ImlsParams)]),
        "imls_destroy": (None, [VP]),
        "imls_set_params": (C.c_int, [VP, P(ImlsParams)]),
        "imls_last_error": (C.c_char_p, [VP]),
        "imls_set_stream": (C.c_int, [VP, VP]),
        "imls_synchronize": (C.c_int, [VP]),
        "imls_set_target": (C.c_int, [VP, VP, VP, SZ, SZ, P(SZ)]),
        "imls_set_source": (C.c_int, [VP, VP, VP, SZ, SZ, P(SZ), VP]),
        "imls_set_target_device": (C.c_int, [VP, VP, SZ, P(SZ)]),
        "imls_set_source_device": (C.c_int, [VP, VP, SZ, P(SZ)]),
        "imls_set_target_tensors": (C.c_int, [VP, VP, SZ, SZ]),
        "imls_set_target_tensors_device": (C.c_int, [VP, VP, SZ]),
        "imls_tv_encode_pca": (None, [VP, VP, SZ, C.c_int32, VP]),
        "imls_project": (C.c_int, [VP, VP, VP, VP, VP, VP, P(SZ), VP]),
        "imls_solve": (C.c_int, [VP, VP, P(C.c_int)]),
        "imls_solve_correspondences": (C.c_int, [VP, C.c_int32, VP, VP, VP, VP, SZ, VP, P(C.c_int)]),
        "imls_register_frame": (C.c_int, [VP, VP, P(C.c_int), P(C.c_int), VP]),
        "imls_register_frame_async": (C.c_int, [VP]),
        "imls_register_frame_result": (C.c_int, [VP, VP, P(C.c_int), P(C.c_int), VP]),
        "imls_enable_timing": (C.c_int, [VP, C.c_int]),
        "imls_enable_stats": (C.c_int, [VP, C.c_int]),
        "imls_kernel_timing": (C.c_int, [VP, C.c_int, P(C.c_double), P(C.c_uint64)]),
        "imls_reset_timing": (C.c_int, [VP]),
        "imls_index_stats": (C.c_int, [VP, VP]),
        "imls_traversal_stats": (C.c_int, [VP, VP]),
        "imls_default_pca_params": (None, [P(ImlsPcaParams)]),
        "imls_default_front_params": (None, [P(ImlsFrontParams)]),
        "imls_scan_front_end": (C.c_int, [VP, P(ImlsFrontParams), VP, SZ, SZ, VP, VP, VP, P(SZ)]),
        "imls_ring_normals_pca": (C.c_int, [VP, P(ImlsPcaParams), VP, SZ, VP, C.c_int32, VP, VP, VP, VP, VP, VP,
                                            P(SZ), VP]),
        "imls_default_sample_params": (None, [P(ImlsSampleParams), C.c_int32]),
        "imls_batch_create": (VP, [C.c_int, P(ImlsParams), C.c_int32]),
        "imls_batch_destroy": (None, [VP]),
        "imls_batch_last_error": (C.c_char_p, [VP]),
        "imls_register_batch": (C.c_int, [VP, SZ, VP, VP, VP, VP]),
        "imls_register_frames": (C.c_int, [VP, SZ, VP, VP, VP, VP]),
        "imls_register_frames_async": (C.c_int, [VP, SZ]),
        "imls_register_frames_result": (C.c_int, [VP, VP, VP, VP, VP]),
        "imls_sample_point_cloud": (C.c_int, [VP, P(ImlsSampleParams), VP, VP, SZ, SZ, VP, SZ, VP, SZ, SZ, VP, P(SZ),
                                              VP]),
        "imls_seed_rng": (C.c_int, [VP, C.c_uint32]),
        "imls_get_rng_state": (C.c_int, [VP, VP]),
        "imls_set_rng_state": (C.c_int, [VP, VP]),
        "imls_map_push": (C.c_int, [VP, VP, VP, SZ, SZ, P(SZ)]),
        "imls_map_push_device": (C.c_int, [VP, VP, SZ, P(SZ)]),
        "imls_map_clear": (C.c_int, [VP]),
        "imls_map_size": (C.c_int, [VP, P(SZ), P(SZ)]),
        "imls_set_defer": (C.c_int, [VP, C.c_int]),
        "imls_set_option": (C.c_int, [VP, C.c_int32, C.c_double]),
        "imls_get_option": (C.c_int, [VP, C.c_int32, P(C.c_double)]),
        "imls_capture_correspondences": (C.c_int, [VP, C.c_int]),
        "imls_captured_correspondences": (C.c_int, [VP, C.c_int, SZ, VP, VP, VP, VP, P(SZ)]),
        "imls_timing_origin": (C.c_int, [VP]),
        "imls_timing_intervals": (C.c_int, [VP, C.c_int, VP, SZ, P(SZ)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


ABI_SYMBOLS = (
    "imls_abi_version", "imls_default_params", "imls_create", "imls_destroy", "imls_set_params",
    "imls_last_error", "imls_set_stream", "imls_synchronize", "imls_set_target", "imls_set_source",
    "imls_set_target_device", "imls_set_source_device", "imls_set_target_tensors",
    "imls_set_target_tensors_device", "imls_tv_encode_pca", "imls_project", "imls_solve",
    "imls_solve_correspondences", "imls_register_frame", "imls_register_frame_async",
    "imls_register_frame_result", "imls_enable_timing", "imls_kernel_timing", "imls_reset_timing",
    "imls_index_stats", "imls_traversal_stats", "imls_default_pca_params", "imls_ring_normals_pca",
    "imls_default_sample_params", "imls_sample_point_cloud", "imls_batch_create", "imls_batch_destroy",
    "imls_batch_last_error", "imls_register_batch", "imls_seed_rng", "imls_get_rng_state",
    "imls_set_rng_state", "imls_map_push", "imls_map_push_device", "imls_map_clear", "imls_map_size",
    "imls_register_frames", "imls_register_frames_async", "imls_register_frames_result",
    "imls_default_front_params", "imls_scan_front_end", "imls_enable_stats", "imls_set_defer",
    "imls_timing_origin", "imls_timing_intervals", "imls_capture_correspondences",
    "imls_captured_correspondences", "imls_set_option", "imls_get_option",
)

_LIB = None


def load_library(path: os.PathLike | None = None) -> C.CDLL:
    """Load libimls_gpu.so.  Raises (never falls back) when it is missing."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    # IMLS_LIB_PATH: a diagnostic build of the same library (e.g. make debug → csrc/debug/)
    p = pathlib.Path(path) if path else pathlib.Path(os.environ.get("IMLS_LIB_PATH", LIB_PATH))
    if not p.exists():
        raise RuntimeError(f"HIP extension missing: {p} (run __graft_entry__.build())")
    lib = _bind(C.CDLL(str(p)))
    if path is None:
        _LIB = lib
    return lib


class ImlsError(RuntimeError):
    def __init__(self, status: int, msg: str = ""):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status
