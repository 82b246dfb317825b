"""config.json ↔ imls_params.

Accepts the reference's config.json layout unchanged (the ``laser_odometry`` section that
laser_odometry.cpp reads at 487-518, 570, 606, 640-641 and the dispatcher 183-243) plus one new
key, ``laser_odometry.backend`` ("hip" — the only backend this package ships).  Method names are
the reference's strings: matching "IMLS" / "plane_ICP"; solving "LS" / "RANSAC" / "Ceres" / "ICP" /
"Teaser"; RANSAC final "LS" / "Weighted LS" / "DRPM".
"""
from __future__ import annotations

import json
import pathlib

from . import _abi

DEFAULT_CONFIG = pathlib.Path(__file__).resolve().parent / "config" / "config.json"

MATCHING = {"IMLS": _abi.IMLS_MATCH_IMLS, "plane_ICP": _abi.IMLS_MATCH_PLANE_ICP}
# The top-level solve_method names the reference's dispatcher accepts (laser_odometry.cpp:183-272).
# "Weighted LS" is only a RANSAC final method there: as a top-level name it hits "Invalid
# SOLVE_METHOD!", so it is rejected here too (the C ABI's IMLS_SOLVE_WEIGHTED_LS is an extension
# for callers that want a unit-weight WLS loop, never produced from a config file).
SOLVING = {"LS": _abi.IMLS_SOLVE_LS, "RANSAC": _abi.IMLS_SOLVE_RANSAC}
FINAL = {"LS": _abi.IMLS_FINAL_LS, "Weighted LS": _abi.IMLS_FINAL_WEIGHTED_LS, "DRPM": _abi.IMLS_FINAL_DRPM}
# Third-party solver engines (solver.cpp:25-72, 387-483): outside the GPU path.
UNSUPPORTED_SOLVERS = ("Ceres", "ICP", "Teaser")


class ConfigError(ValueError):
    pass


def load(path: str | pathlib.Path | None = None) -> dict:
    """Parse a config file.  Like common.cpp:8-17 a missing file raises (runtime_error there)."""
    p = pathlib.Path(path) if path else DEFAULT_CONFIG
    if not p.exists():
        raise FileNotFoundError(f"cannot open config file: {p}")
    with open(p) as f:
        return json.load(f)


def params_from_config(cfg: dict) -> _abi.ImlsParams:
    """Build imls_params from the reference key paths.  Unknown method names raise ConfigError.
    Deliberate change, documented in INTEGRATION.md: the reference prints "Invalid
    MATCHING_METHOD!" / "Invalid SOLVE_METHOD!" and keeps running with every frame's solve failing
    (rPose = I for every frame); this fails once, at configuration time."""
    lo = cfg["laser_odometry"]
    mm = lo["matching_method"]
    sm = lo["solve_method"]
    p = _abi.default_params()
    if mm["method"] not in MATCHING:
        raise ConfigError(f"Invalid MATCHING_METHOD! {mm['method']!r}")
    p.matching_method = MATCHING[mm["method"]]
    p.correspond_number = int(mm["correspond_number"])
    im = mm["IMLS"]
    p.h, p.r = float(im["h"]), float(im["r"])
    tv = im["use_tensor_voting"]
    p.use_tensor_voting, p.tensor_k = int(bool(tv["enabled"])), int(tv["k"])
    p.tensor_sigma, p.tensor_distance_threshold = float(tv["sigma"]), float(tv["distance_threshold"])
    gn = im["get_normals"]
    p.get_normals, p.r_normal, p.search_number_normal = int(bool(gn["enabled"])), float(gn["r_normal"]), int(gn["search_number_normal"])
    pd = im["use_projected_distance"]
    p.use_projected_distance, p.r_proj = int(bool(pd["enabled"])), float(pd["r_proj"])
    nac = im["normal_angle_constraint"]
    p.normal_angle_constraint, p.angle_diff_threshold = int(bool(nac["enabled"])), float(nac["angle_diff_threshold"])
    p.search_number = int(im["IMLS function"]["search_number"])
    pi = mm.get("plane_ICP")
    if pi:
        p.picp_r = float(pi["r"])
        p.picp_use_projected_distance = int(bool(pi["use_projected_distance"]["enabled"]))
        p.picp_r_proj = float(pi["use_projected_distance"]["r_proj"])
        p.picp_normal_angle_constraint = int(bool(pi["normal_angle_constraint"]["enabled"]))
        p.picp_angle_diff_threshold = float(pi["normal_angle_constraint"]["angle_diff_threshold"])
    method = sm["method"]
    if method in UNSUPPORTED_SOLVERS:
        raise ConfigError(f"solve_method {method!r} is a third-party solver engine outside the GPU path")
    if method not in SOLVING:
        raise ConfigError(f"Invalid SOLVE_METHOD! {method!r}")
    p.solve_method = SOLVING[method]
    p.iterations = int(sm["iterations"])
    p.delta_dist_threshold = float(sm["delta_dist_threshold"])
    p.delta_angle_threshold = float(sm["delta_angle_threshold"])
    p.ls_threshold = float(sm["LS"]["threshold"])
    rs = sm["RANSAC"]
    p.ransac_max_iterations = int(rs["max_iterations"])
    p.ransac_distance_threshold = float(rs["distance_threshold"])
    p.ransac_min_inliers_percentage = float(rs["min_inliers_percentage"])
    p.ransac_huber_threshold = float(rs["huber_threshold"])
    if rs["final_solve_method"] not in FINAL:
        raise ConfigError(f"Invalid FINAL_SOLVE_METHOD in RANSAC! {rs['final_solve_method']!r}")
    p.ransac_final_method = FINAL[rs["final_solve_method"]]
    p.ransac_ls_threshold = float(rs["LS_threshold"])
    p.drpm_threshold = float(rs["DRPM_threshold"])
    p.drpm_stdev_points = float(rs["DRPM_stdev_points"])
    p.drpm_stdev_normals = float(rs["DRPM_stdev_normals"])
    p.transform_normal = int(bool(lo.get("transform_normal", False)))
    p.max_queue_size = int(lo.get("max_queue_size", 1))
    backend = lo.get("backend", "hip")
    if backend != "hip":
        raise ConfigError(f"laser_odometry.backend {backend!r}: only 'hip' is shipped")
    return p


def bench_params(iterations: int = 20) -> _abi.ImlsParams:
    """shipped IMLS parameters, LS (t = 0.02), fixed iteration count
    (delta thresholds −1 so the convergence test never fires)."""
    p = params_from_config(load())
    p.solve_method = _abi.IMLS_SOLVE_LS
    p.iterations = iterations
    p.delta_dist_threshold = -1.0
    p.delta_angle_threshold = -1.0
    return p
