"""Host-side mirror of the reference operator interface, over the HIP C ABI (libimls_gpu.so).

Same names, argument meaning and error behaviour as the reference's C++ API so code (and
tests) read like the reference:

  IMLSICPMatcher              imls_icp.h:45-147  (setSourcePointCloud, setTargetPointCloud,
                                                   setParameters, ProjSourcePtToSurface)
  SolveMotionEstimationProblemLS / WeightedLS    solver.h:84-98
  solveMotionEstimationProblem(method, ...)      laser_odometry.cpp:173-275 (string dispatch)
  LaserOdometry                                  laser_odometry.cpp:416-683 minus ROS: map FIFO
                                                 (accumulateTargetCloud 116-136), per-frame
                                                 registration, global pose chaining (649-658)
  savePoseToFile / saveMatchedPointsToFile       saver.cpp:46-54, 113-133 (text formats)

Clouds are numpy structured arrays of synth.POINT_DTYPE (the 48-byte pcl::PointXYZINormal
record) or float arrays shaped (N, 6) = x y z nx ny nz.  Every compute call runs on the GPU;
there is no CPU fallback — without an MI355X the context cannot be created and this raises.
"""
from __future__ import annotations

import ctypes as C
import math
from collections import deque
from typing import Optional

import numpy as np

from . import _abi
from . import config as _config
from .synth import POINT_DTYPE


def _as_xyzn(cloud) -> np.ndarray:
    """(N, 6) float32 contiguous x y z nx ny nz from a PointXYZINormal array or an (N, 6) array."""
    if isinstance(cloud, np.ndarray) and cloud.dtype == POINT_DTYPE:
        out = np.empty((cloud.size, 6), np.float32)
        for k, f in enumerate(("x", "y", "z", "normal_x", "normal_y", "normal_z")):
            out[:, k] = cloud[f]
        return out
    a = np.ascontiguousarray(cloud, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] != 6:
        raise ValueError("cloud must be a PointXYZINormal array or shaped (N, 6)")
    return a


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class ImlsContext:
    """RAII wrapper of one `imls_ctx` (one per host thread; not thread-safe, like the reference)."""

    def __init__(self, params: Optional[_abi.ImlsParams] = None, device: int = 0):
        self.lib = _abi.load_library()
        self.params = params if params is not None else _config.params_from_config(_config.load())
        if self.params.solve_method == _abi.IMLS_SOLVE_RANSAC:
            # the shipped config's solver; the fused GPU loop needs an LS-family method here
            p = _abi.ImlsParams.from_buffer_copy(self.params)
            p.solve_method = _abi.IMLS_SOLVE_LS
            self.params = p
        self.ctx = self.lib.imls_create(device, C.byref(self.params))
        if not self.ctx:
            raise _abi.ImlsError(_abi.IMLS_ERR_DEVICE, f"imls_create(device={device}) failed: no MI355X visible "
                                                       "(the GPU path has no CPU fallback)")
        self.n_target = 0
        self.n_source = 0

    # -- plumbing -------------------------------------------------------------------------------
    def _check(self, rc: int):
        if rc != _abi.IMLS_OK:
            msg = self.lib.imls_last_error(self.ctx)
            raise _abi.ImlsError(rc, msg.decode() if msg else "")

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.imls_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_params(self, p: _abi.ImlsParams):
        self._check(self.lib.imls_set_params(self.ctx, C.byref(p)))
        self.params = p

    def set_stream(self, hip_stream: int | None):
        self._check(self.lib.imls_set_stream(self.ctx, C.c_void_p(hip_stream or 0)))

    def synchronize(self):
        self._check(self.lib.imls_synchronize(self.ctx))

    # -- clouds ---------------------------------------------------------------------------------
    def set_target(self, cloud) -> int:
        a = _as_xyzn(cloud)
        n = C.c_size_t()
        self._check(self.lib.imls_set_target(self.ctx, _ptr(a), C.c_void_p(a.ctypes.data + 12), a.shape[0], 6, C.byref(n)))
        self.n_target = n.value
        return n.value

    def set_target_tensors(self, tensors):
        """Tensor-voting input tensors of the last set_target's points: (n, 6) float32
        (xx, xy, xz, yy, yz, zz) — VoteForAny's encode(AWARE_TENSOR) input (imls_icp.cpp:179)."""
        t = np.ascontiguousarray(tensors, dtype=np.float32)
        if t.ndim != 2 or t.shape[1] != 6:
            raise ValueError("tensors must be (n, 6)")
        self._check(self.lib.imls_set_target_tensors(self.ctx, _ptr(t), t.shape[0], 6))

    def set_target_tensors_device(self, ten6_ptr: int, n: int):
        self._check(self.lib.imls_set_target_tensors_device(self.ctx, C.c_void_p(ten6_ptr), n))

    def set_source(self, cloud):
        a = _as_xyzn(cloud)
        n = C.c_size_t()
        kept = np.zeros(a.shape[0], np.uint32)
        self._check(self.lib.imls_set_source(self.ctx, _ptr(a), C.c_void_p(a.ctypes.data + 12), a.shape[0], 6,
                                             C.byref(n), _ptr(kept)))
        self.n_source = n.value
        return kept[: n.value]

    def set_target_device(self, soa6_ptr: int, n: int) -> int:
        k = C.c_size_t()
        self._check(self.lib.imls_set_target_device(self.ctx, C.c_void_p(soa6_ptr), n, C.byref(k)))
        self.n_target = k.value
        return k.value

    def set_source_device(self, soa6_ptr: int, n: int) -> int:
        k = C.c_size_t()
        self._check(self.lib.imls_set_source_device(self.ctx, C.c_void_p(soa6_ptr), n, C.byref(k)))
        self.n_source = k.value
        return k.value

    # -- matching / solving -------------------------------------------------------------------
    def project(self, pose=None):
        N = max(self.n_source, 1)
        pose = np.ascontiguousarray(np.eye(4) if pose is None else pose, dtype=np.float64).reshape(16)
        x = np.zeros((N, 3), np.float32); y = np.zeros((N, 3), np.float32); n = np.zeros((N, 3), np.float32)
        idx = np.zeros(N, np.uint32); rej = np.zeros(6, np.uint64); nv = C.c_size_t()
        self._check(self.lib.imls_project(self.ctx, _ptr(pose), _ptr(x), _ptr(y), _ptr(n), _ptr(idx), C.byref(nv), _ptr(rej)))
        k = nv.value
        return x[:k], y[:k], n[:k], idx[:k], rej

    def solve(self):
        D = np.zeros(16); ok = C.c_int()
        self._check(self.lib.imls_solve(self.ctx, _ptr(D), C.byref(ok)))
        return bool(ok.value), D.reshape(4, 4)

    def solve_correspondences(self, method: int, s, d, n, weights=None):
        s, d, n = (np.ascontiguousarray(a, dtype=np.float64).reshape(-1, 3) for a in (s, d, n))
        w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
        D = np.zeros(16); ok = C.c_int()
        self._check(self.lib.imls_solve_correspondences(self.ctx, method, _ptr(s), _ptr(d), _ptr(n),
                                                        None if w is None else _ptr(w), len(s), _ptr(D), C.byref(ok)))
        return bool(ok.value), D.reshape(4, 4)

    def register_frame(self):
        it = max(self.params.iterations, 1)
        trace = (_abi.ImlsIterTrace * it)()
        pose = np.zeros(16); iters = C.c_int(); status = C.c_int()
        self._check(self.lib.imls_register_frame(self.ctx, _ptr(pose), C.byref(iters), C.byref(status), trace))
        return dict(pose=pose.reshape(4, 4), iters=iters.value, status=status.value,
                    trace=[trace[k] for k in range(iters.value)])

    def register_frame_async(self):
        self._check(self.lib.imls_register_frame_async(self.ctx))

    def register_frame_result(self):
        it = max(self.params.iterations, 1)
        trace = (_abi.ImlsIterTrace * it)()
        pose = np.zeros(16); iters = C.c_int(); status = C.c_int()
        self._check(self.lib.imls_register_frame_result(self.ctx, _ptr(pose), C.byref(iters), C.byref(status), trace))
        self.last_trace = [trace[k] for k in range(iters.value)]
        return pose.reshape(4, 4), iters.value, status.value

    # -- instrumentation ------------------------------------------------------------------------
    def ring_normals_pca(self, xyz, ring_sizes, pca_params: Optional[_abi.ImlsPcaParams] = None) -> dict:
        """scan_registration.cpp's "pca" normal estimation + geometric-features presample (1136-1229,
        279-327, 1481-1489) on the ring-concatenated cloud `laserCloud` (1064-1069).
        xyz: (n, 3+) float32 (stride = its row length); ring_sizes: points per scan line.
        Returns the filteredLaserCloud rows: index (into xyz; = PCA centre + 5, the reference's own
        offset), normal, evals, evecs (3x3 column-major), features (8), flags (IMLS_PCA_*), plus
        the pca_failure / plane-check counters."""
        a = np.ascontiguousarray(xyz, dtype=np.float32)
        if a.ndim != 2 or a.shape[1] < 3:
            raise ValueError("xyz must be (n, >=3)")
        rs = np.ascontiguousarray(ring_sizes, dtype=np.int32)
        if int(rs.sum()) != a.shape[0]:
            raise ValueError("ring sizes must sum to the number of points")
        p = pca_params if pca_params is not None else _abi.default_pca_params()
        n = max(a.shape[0], 1)
        idx = np.zeros(n, np.uint32); nrm = np.zeros((n, 3), np.float32); ev = np.zeros((n, 3), np.float32)
        evec = np.zeros((n, 9), np.float32); feat = np.zeros((n, 8), np.float32); fl = np.zeros(n, np.uint8)
        cnt = np.zeros(2, np.uint64); nout = C.c_size_t()
        self._check(self.lib.imls_ring_normals_pca(self.ctx, C.byref(p), _ptr(a), a.shape[1], _ptr(rs), len(rs),
                                                   _ptr(idx), _ptr(nrm), _ptr(ev), _ptr(evec), _ptr(feat), _ptr(fl),
                                                   C.byref(nout), _ptr(cnt)))
        k = nout.value
        return dict(index=idx[:k], normal=nrm[:k], evals=ev[:k], evecs=evec[:k], features=feat[:k], flags=fl[:k],
                    pca_failure=int(cnt[0]), plane_invalid=int(cnt[1]))

    def sample_point_cloud(self, xyz, nrm, candidates, last_xyz=None,
                           sample_params: Optional[_abi.ImlsSampleParams] = None):
        """samplePointCloud "normal" / "major_axis" (scan_registration.cpp:761-806) of the filtered
        cloud (xyz, nrm: (n, 3) float32) restricted to `candidates`, against the previous frame's
        cloud last_xyz (major_axis).  Returns (sampled indices in the reference's order, bin weights)."""
        a = np.ascontiguousarray(np.asarray(xyz, np.float32)[:, :3])
        nn = np.ascontiguousarray(np.asarray(nrm, np.float32)[:, :3])
        if a.shape != nn.shape:
            raise ValueError("xyz and nrm must have the same shape")
        cand = np.ascontiguousarray(candidates, dtype=np.int32)
        last = np.ascontiguousarray(np.zeros((0, 3)) if last_xyz is None else np.asarray(last_xyz)[:, :3],
                                    dtype=np.float32)
        p = sample_params if sample_params is not None else _abi.default_sample_params()
        nb = p.azimuth_bins * p.elevation_bins
        out = np.zeros(len(cand) + nb + 1, np.int32); w = np.zeros(nb, np.float32); k = C.c_size_t()
        self._check(self.lib.imls_sample_point_cloud(self.ctx, C.byref(p), _ptr(a), _ptr(nn), 3, a.shape[0],
                                                     _ptr(cand), len(cand), _ptr(last), 3, last.shape[0],
                                                     _ptr(out), C.byref(k), _ptr(w)))
        return out[:k.value], w

    def enable_timing(self, on=True):
        self._check(self.lib.imls_enable_timing(self.ctx, int(on)))

    def reset_timing(self):
        self._check(self.lib.imls_reset_timing(self.ctx))

    def kernel_timing(self, kernel: int):
        ms = C.c_double(); n = C.c_uint64()
        self._check(self.lib.imls_kernel_timing(self.ctx, kernel, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def index_stats(self) -> dict:
        out = np.zeros(8, np.uint64)
        self._check(self.lib.imls_index_stats(self.ctx, _ptr(out)))
        keys = ("points", "leaves", "leaf_slots", "levels", "sum_kq", "nn_found", "queries", "bucket")
        return {k: int(v) for k, v in zip(keys, out)}

    def traversal_stats(self) -> dict:
        out = np.zeros(8, np.uint64)
        self._check(self.lib.imls_traversal_stats(self.ctx, _ptr(out)))
        keys = ("sum_kq", "nn_found", "leaves_visited", "inner_visited", "waves", "uncertified", "verlet_reused")
        return {k: int(v) for k, v in zip(keys, out)}


# ================================================================================================
# Reference-shaped API
# ================================================================================================
class ImlsBatch:
    """Many independent scan pairs kept in flight over `streams` contexts (imls_register_batch):
    each pair is registered exactly as set_target + set_source + register_frame."""

    def __init__(self, params: Optional[_abi.ImlsParams] = None, device: int = 0, streams: int = 4):
        self.lib = _abi.load_library()
        p = params if params is not None else _abi.default_params()
        self._params = p
        self.b = self.lib.imls_batch_create(device, C.byref(p), streams)
        if not self.b:
            raise _abi.ImlsError(_abi.IMLS_ERR_DEVICE, "imls_batch_create failed (no MI355X?)")

    def close(self):
        if getattr(self, "b", None):
            self.lib.imls_batch_destroy(self.b)
            self.b = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def register(self, pairs):
        """pairs: list of (source_cloud, target_cloud) in any layout set_source/set_target accept.
        Returns (poses (n,4,4), iterations (n,), statuses (n,))."""
        keep, arr = [], (_abi.ImlsPairInput * max(len(pairs), 1))()
        for k, (src, tgt) in enumerate(pairs):
            s, t = _as_xyzn(src), _as_xyzn(tgt)
            keep += [s, t]
            arr[k] = _abi.ImlsPairInput(s.ctypes.data, s.ctypes.data + 12, s.shape[0],
                                        t.ctypes.data, t.ctypes.data + 12, t.shape[0], 6)
        n = len(pairs)
        poses = np.zeros((max(n, 1), 16)); iters = np.zeros(max(n, 1), np.int32); st = np.zeros(max(n, 1), np.int32)
        rc = self.lib.imls_register_batch(self.b, n, arr, _ptr(poses), _ptr(iters), _ptr(st))
        if rc != 0:
            raise _abi.ImlsError(rc, (self.lib.imls_batch_last_error(self.b) or b"").decode())
        return poses[:n].reshape(n, 4, 4), iters[:n], st[:n]


class IMLSICPMatcher:
    """Drop-in mirror of IMLSICPMatcher (imls_icp.h:45-147) backed by the HIP path.

    The reference mutates its boost::shared_ptr clouds in place (NaN erase; erase of unmatched
    points); numpy arrays cannot shrink in place, so the mutating calls RETURN the new clouds."""

    def __init__(self, params: Optional[_abi.ImlsParams] = None, device: int = 0):
        p = params if params is not None else _config.params_from_config(_config.load())
        self._ctx = ImlsContext(p, device)
        self._source = None
        self._target = None

    @property
    def context(self) -> ImlsContext:
        return self._ctx

    def setParameters(self, _iter, _h, _r, _r_normal, _r_proj, _useTensorVoting, _isGetNormals, _useProjectedDistance,
                      _tensor_k, _tensor_sigma, _tensor_distance_threshold, _search_number_normal, _search_number,
                      _normal_angle_constraint, _angle_diff_threshold, _output_dir=""):
        """imls_icp.cpp:146-168 (16 parameters, same order)."""
        p = _abi.ImlsParams.from_buffer_copy(self._ctx.params)
        p.iterations, p.h, p.r, p.r_normal, p.r_proj = int(_iter), float(_h), float(_r), float(_r_normal), float(_r_proj)
        p.use_tensor_voting, p.get_normals = int(bool(_useTensorVoting)), int(bool(_isGetNormals))
        p.use_projected_distance, p.tensor_k = int(bool(_useProjectedDistance)), int(_tensor_k)
        p.tensor_sigma, p.tensor_distance_threshold = float(_tensor_sigma), float(_tensor_distance_threshold)
        p.search_number_normal, p.search_number = int(_search_number_normal), int(_search_number)
        p.normal_angle_constraint, p.angle_diff_threshold = int(bool(_normal_angle_constraint)), float(_angle_diff_threshold)
        self._ctx.set_params(p)

    @staticmethod
    def _finite(cloud):
        if isinstance(cloud, np.ndarray) and cloud.dtype == POINT_DTYPE:
            return cloud[np.isfinite(cloud["x"]) & np.isfinite(cloud["y"]) & np.isfinite(cloud["z"])]
        a = _as_xyzn(cloud)
        return a[np.isfinite(a[:, :3]).all(axis=1)]

    def setSourcePointCloud(self, cloud):
        """imls_icp.cpp:74-78; returns the NaN-filtered cloud (the reference filters in place)."""
        self._source = self._finite(cloud)
        self._ctx.set_source(self._source)
        return self._source

    def setTargetPointCloud(self, cloud):
        """imls_icp.cpp:80-103: NaN filter + index build."""
        self._target = self._finite(cloud)
        self._ctx.set_target(self._target)
        return self._target

    def ProjSourcePtToSurface(self, in_cloud, timestamp: str = "", i: int = 0, pose=None):
        """imls_icp.cpp:496-745.  `in_cloud` is the source as set by setSourcePointCloud; the GPU
        applies `pose` itself (laser_odometry.cpp:527-549 transforms before the call).  Returns
        (in_cloud_kept, out_cloud, reject_counters): in_cloud_kept holds the transformed source
        points that found a match, out_cloud their projections y with the NN-1 normals."""
        x, y, n, idx, rej = self._ctx.project(pose)
        src = in_cloud if in_cloud is not None else self._source
        keep = src[idx].copy() if isinstance(src, np.ndarray) and src.dtype == POINT_DTYPE else np.zeros(len(idx), POINT_DTYPE)
        keep["x"], keep["y"], keep["z"] = x[:, 0], x[:, 1], x[:, 2]
        out = np.zeros(len(idx), POINT_DTYPE)
        out["x"], out["y"], out["z"] = y[:, 0], y[:, 1], y[:, 2]
        out["normal_x"], out["normal_y"], out["normal_z"] = n[:, 0], n[:, 1], n[:, 2]
        return keep, out, dict(zip(_abi.REJECT_NAMES, map(int, rej)))


def tv_encode_pca(evals, evecs, k: int = 50) -> np.ndarray:
    """The reference's tensor encoding of PCA features (scan_registration.cpp:358-381) via the
    library's host helper: evals (n, 3), evecs (n, 9) column-major 3×3 → tensors (n, 6)."""
    ev = np.ascontiguousarray(evals, dtype=np.float32)
    ec = np.ascontiguousarray(evecs, dtype=np.float32)
    out = np.zeros((ev.shape[0], 6), np.float32)
    _abi.load_library().imls_tv_encode_pca(_ptr(ev), _ptr(ec), ev.shape[0], int(k), _ptr(out))
    return out


def _triples(v) -> np.ndarray:
    return np.ascontiguousarray(v, dtype=np.float64).reshape(-1, 3)


_SOLVER_CTX: Optional[ImlsContext] = None


def _solver_ctx() -> ImlsContext:
    global _SOLVER_CTX
    if _SOLVER_CTX is None:
        p = _config.params_from_config(_config.load())
        p.solve_method = _abi.IMLS_SOLVE_LS
        _SOLVER_CTX = ImlsContext(p)
    return _SOLVER_CTX


def SolveMotionEstimationProblemLS(source_cloud, ref_cloud, ref_normals, timestamp: str = "", threshold: float = 0.02):
    """solver.cpp:74-166 → (flag, deltaTrans 4×4)."""
    ctx = _solver_ctx()
    p = _abi.ImlsParams.from_buffer_copy(ctx.params)
    p.ls_threshold = float(threshold)
    p.solve_method = _abi.IMLS_SOLVE_LS
    ctx.set_params(p)
    return ctx.solve_correspondences(_abi.IMLS_SOLVE_LS, _triples(source_cloud), _triples(ref_cloud), _triples(ref_normals))


def SolveMotionEstimationProblemWeightedLS(source_cloud, ref_cloud, ref_normals, weights, timestamp: str = ""):
    """solver.cpp:168-220 → (flag, deltaTrans 4×4)."""
    return _solver_ctx().solve_correspondences(_abi.IMLS_SOLVE_WEIGHTED_LS, _triples(source_cloud), _triples(ref_cloud),
                                               _triples(ref_normals), np.asarray(weights, dtype=np.float64))


def solveMotionEstimationProblem(solve_method: str, in_cloud_vec, ref_cloud_vec, ref_normal, timestamp: str = "",
                                 cfg: Optional[dict] = None):
    """laser_odometry.cpp:173-275: string dispatch with parameters read from the config."""
    cfg = cfg if cfg is not None else _config.load()
    sm = cfg["laser_odometry"]["solve_method"]
    if solve_method == "LS":
        return SolveMotionEstimationProblemLS(in_cloud_vec, ref_cloud_vec, ref_normal, timestamp, float(sm["LS"]["threshold"]))
    if solve_method in _config.UNSUPPORTED_SOLVERS or solve_method == "RANSAC":
        raise _abi.ImlsError(_abi.IMLS_ERR_UNSUPPORTED, f"solve_method {solve_method!r} is not on the GPU path")
    # the reference prints "Invalid SOLVE_METHOD!" and returns false
    return False, np.eye(4)


# ================================================================================================
# Per-frame driver (laser_odometry.cpp:416-683 without ROS / file I/O)
# ================================================================================================
class LaserOdometry:
    """Streams (filtered cloud, flat cloud) frames like processData: the first frame only seeds
    the map (Q13); every later frame registers its flat cloud against the FIFO map of the last
    `max_queue_size` filtered clouds (untransformed, oldest first — accumulateTargetCloud), and
    chains nowPose = prevLaserPose · rPose."""

    def __init__(self, params: Optional[_abi.ImlsParams] = None, device: int = 0):
        self.ctx = ImlsContext(params, device)
        self.queue: deque = deque()
        self.prev_pose = np.eye(4)
        self.frame_count = 0
        self.poses: list = []           # (timestamp, 4×4) per registered frame

    def process(self, filtered_cloud, flat_cloud, timestamp: str = ""):
        result = None
        if self.frame_count != 0:
            target = np.concatenate(list(self.queue)) if len(self.queue) > 1 else self.queue[0]
            self.ctx.set_target(target)
            self.ctx.set_source(flat_cloud)
            result = self.ctx.register_frame()
            now = self.prev_pose @ result["pose"]
            self.prev_pose = now
            self.poses.append((timestamp, now))
        self.queue.append(filtered_cloud)
        while len(self.queue) > max(1, self.ctx.params.max_queue_size):
            self.queue.popleft()
        self.frame_count += 1
        return result


def _quat_xyzw(R: np.ndarray):
    """Rotation matrix → (x, y, z, w) as Eigen::Quaterniond(Matrix3d) (Shepperd's method)."""
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        w, x, y, z = 0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = math.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0) * 2
        q = [0.0, 0.0, 0.0]
        q[i] = 0.25 * s
        q[j] = (R[j, i] + R[i, j]) / s
        q[k] = (R[k, i] + R[i, k]) / s
        w = (R[k, j] - R[j, k]) / s
        x, y, z = q
    return x, y, z, w


def savePoseToFile(pose, filename: str, timestamp: str):
    """saver.cpp:46-54: append `ts tx ty tz qx qy qz qw`, fixed, 6 decimals."""
    P = np.asarray(pose, dtype=np.float64)
    x, y, z, w = _quat_xyzw(P[:3, :3])
    with open(filename, "a") as f:
        f.write(f"{timestamp} {P[0, 3]:.6f} {P[1, 3]:.6f} {P[2, 3]:.6f} {x:.6f} {y:.6f} {z:.6f} {w:.6f}\n")


def saveMatchedPointsToFile(source_cloud, matched_cloud, filename: str):
    """saver.cpp:113-133: append `sx sy sz yx yy yz` per pair (default 6-significant-digit stream)."""
    s, d = _triples(source_cloud), _triples(matched_cloud)
    with open(filename, "a") as f:
        for a, b in zip(s, d):
            f.write(" ".join(f"{v:.6g}" for v in (*a, *b)) + "\n")
