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
from . import wire as _wire
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


_XYZ_OFF = POINT_DTYPE.fields["x"][1]
_NRM_OFF = POINT_DTYPE.fields["normal_x"][1]


def _cloud_args(cloud):
    """(keep-alive array, xyz pointer, normal pointer, n, stride in floats) for the C ABI's strided
    clouds: a contiguous PointXYZINormal array — or a PointCloud2 message of one (wire.py: the
    /laser_cloud_filtered, /laser_cloud_flat wire format) — is passed in place (the reference's
    48-byte PCL record, stride 12: no host copy); anything else as a packed (N, 6) float32 array."""
    if isinstance(cloud, _wire.PointCloud2):
        sv = _wire.strided_view(cloud)
        if sv is None:
            cloud = _wire.xyzinormal_from_msg(cloud)
        else:
            buf, xo, no, n, stride = sv
            return buf, C.c_void_p(buf.ctypes.data + xo), C.c_void_p(buf.ctypes.data + no), n, stride
    if isinstance(cloud, np.ndarray) and cloud.dtype == POINT_DTYPE and cloud.flags.c_contiguous and cloud.ndim == 1:
        base = cloud.ctypes.data
        return cloud, C.c_void_p(base + _XYZ_OFF), C.c_void_p(base + _NRM_OFF), cloud.size, POINT_DTYPE.itemsize // 4
    a = _as_xyzn(cloud)
    return a, C.c_void_p(a.ctypes.data), C.c_void_p(a.ctypes.data + 12), a.shape[0], 6


class ImlsContext:
    """RAII wrapper of one `imls_ctx` (one per host thread; not thread-safe, like the reference)."""

    def __init__(self, params: Optional[_abi.ImlsParams] = None, device: int = 0):
        self.lib = _abi.load_library()
        self.params = params if params is not None else _config.params_from_config(_config.load())
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
    # count=False: the C call returns without waiting for the NaN-filtered count (the rest of the
    # index build is deferred to the first use), so many contexts' uploads overlap; returns None.
    def set_target(self, cloud, count: bool = True):
        _keep, px, pn, m, stride = _cloud_args(cloud)
        n = C.c_size_t()
        self._check(self.lib.imls_set_target(self.ctx, px, pn, m, stride, C.byref(n) if count else None))
        self.n_target = n.value if count else None
        return self.n_target

    def set_target_tensors(self, tensors):
        """Tensor-voting input tensors of the last set_target's points: (n, 6) float32
        (xx, xy, xz, yy, yz, zz) — VoteForAny's encode(AWARE_TENSOR) input (imls_icp.cpp:179)."""
        t = np.ascontiguousarray(tensors, dtype=np.float32)
        if t.ndim != 2 or t.shape[1] != 6:
            raise ValueError("tensors must be (n, 6)")
        self._check(self.lib.imls_set_target_tensors(self.ctx, _ptr(t), t.shape[0], 6))

    def set_target_tensors_device(self, ten6_ptr: int, n: int):
        self._check(self.lib.imls_set_target_tensors_device(self.ctx, C.c_void_p(ten6_ptr), n))

    def set_source(self, cloud, count: bool = True):
        """Returns the input index of every kept point (count=True) or None (deferred, see set_target)."""
        _keep, px, pn, m, stride = _cloud_args(cloud)
        if not count:
            self._check(self.lib.imls_set_source(self.ctx, px, pn, m, stride, None, None))
            self.n_source = None
            return None
        n = C.c_size_t()
        kept = np.zeros(m, np.uint32)
        self._check(self.lib.imls_set_source(self.ctx, px, pn, m, stride, C.byref(n), _ptr(kept)))
        self.n_source = n.value
        return kept[: n.value]

    def set_target_device(self, soa6_ptr: int, n: int, count: bool = True):
        k = C.c_size_t()
        self._check(self.lib.imls_set_target_device(self.ctx, C.c_void_p(soa6_ptr), n, C.byref(k) if count else None))
        self.n_target = k.value if count else None
        return self.n_target

    def set_source_device(self, soa6_ptr: int, n: int, count: bool = True):
        k = C.c_size_t()
        self._check(self.lib.imls_set_source_device(self.ctx, C.c_void_p(soa6_ptr), n, C.byref(k) if count else None))
        self.n_source = k.value if count else None
        return self.n_source

    # -- map FIFO (accumulateTargetCloud, laser_odometry.cpp:116-136) ---------------------------
    def map_push(self, cloud, count: bool = True):
        """accumulateTargetCloud(cloud, max_queue_size) + setTargetPointCloud(accumulatedTargetCloud):
        the scan joins the device-resident FIFO (only it crosses PCIe) and the index is rebuilt over
        the FIFO's scans, oldest first.  Returns the map size after the NaN filter (count=True)."""
        _keep, px, pn, m, stride = _cloud_args(cloud)
        n = C.c_size_t()
        np_ = C.byref(n) if count else None
        if m == 0:
            self._check(self.lib.imls_map_push(self.ctx, None, None, 0, 6, np_))
        else:
            self._check(self.lib.imls_map_push(self.ctx, px, pn, m, stride, np_))
        self.n_target = n.value if count else None
        return self.n_target

    def map_push_device(self, soa6_ptr: int, n: int, count: bool = True):
        k = C.c_size_t()
        self._check(self.lib.imls_map_push_device(self.ctx, C.c_void_p(soa6_ptr), n, C.byref(k) if count else None))
        self.n_target = k.value if count else None
        return self.n_target

    def map_clear(self):
        self._check(self.lib.imls_map_clear(self.ctx))

    def map_size(self):
        e, p = C.c_size_t(), C.c_size_t()
        self._check(self.lib.imls_map_size(self.ctx, C.byref(e), C.byref(p)))
        return e.value, p.value

    # -- RANSAC rand() stream ---------------------------------------------------------------------
    def seed_rng(self, seed: int):
        self._check(self.lib.imls_seed_rng(self.ctx, int(seed)))

    def rng_state(self) -> np.ndarray:
        st = np.zeros(34, np.int32)
        self._check(self.lib.imls_get_rng_state(self.ctx, _ptr(st)))
        return st

    def set_rng_state(self, state):
        st = np.ascontiguousarray(state, dtype=np.int32)
        if st.shape != (34,):
            raise ValueError("rand() state is int32[34]")
        self._check(self.lib.imls_set_rng_state(self.ctx, _ptr(st)))

    # -- matching / solving -------------------------------------------------------------------
    def project(self, pose=None):
        N = max(self.n_source if self.n_source is not None else self.index_stats()["queries"], 1)
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
    def scan_front_end(self, xyz, front_params: Optional[_abi.ImlsFrontParams] = None):
        """laserCloudHandler's front end (scan_registration.cpp:862-1069) on a raw sweep (n, 3+)
        float32 in the driver's order: NaN + range filter, ring assignment, relative time.  Returns
        (xyz (m, 3), intensity (m,), input index (m,), ring sizes) — laserCloud, ring-concatenated."""
        a = np.ascontiguousarray(xyz, dtype=np.float32)
        if a.ndim != 2 or a.shape[1] < 3:
            raise ValueError("xyz must be (n, >=3)")
        p = front_params if front_params is not None else _abi.default_front_params()
        n = a.shape[0]
        out = np.zeros((max(n, 1), 4), np.float32); idx = np.zeros(max(n, 1), np.uint32)
        rs = np.zeros(max(p.n_scans, 1), np.int32); m = C.c_size_t()
        self._check(self.lib.imls_scan_front_end(self.ctx, C.byref(p), _ptr(a), a.shape[1], n, _ptr(out), _ptr(idx),
                                                 _ptr(rs), C.byref(m)))
        k = m.value
        return out[:k, :3], out[:k, 3], idx[:k], rs[:p.n_scans]

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

    def enable_stats(self, on=True):
        """Collect the traversal / neighbour counters (traversal_stats, index_stats' sum_kq / nn_found)."""
        self._check(self.lib.imls_enable_stats(self.ctx, int(on)))

    def enable_timing(self, on=True):
        """on: False/0 off, True/1 every launch kind, 2 light (projection + solve events only)."""
        self._check(self.lib.imls_enable_timing(self.ctx, int(on)))

    def set_defer(self, on=True):
        """Count-less device loads read their buffer at first use (imls_set_defer)."""
        self._check(self.lib.imls_set_defer(self.ctx, int(bool(on))))

    def set_option(self, name, value):
        """A runtime option (imls_set_option): name from _abi.OPTION_IDS or an IMLS_OPT_* id."""
        opt = _abi.OPTION_IDS[name] if isinstance(name, str) else int(name)
        self._check(self.lib.imls_set_option(self.ctx, opt, float(value)))

    def get_option(self, name) -> float:
        opt = _abi.OPTION_IDS[name] if isinstance(name, str) else int(name)
        v = C.c_double()
        self._check(self.lib.imls_get_option(self.ctx, opt, C.byref(v)))
        return v.value

    def set_options(self, **opts):
        for k, v in opts.items():
            self.set_option(k, v)

    def capture_correspondences(self, on=True):
        """Keep every iteration's correspondences of register_frame (imls_capture_correspondences)."""
        self._check(self.lib.imls_capture_correspondences(self.ctx, int(bool(on))))

    def captured(self, it: int):
        """Iteration `it` of the last register_frame: (x, y, n, source index), source order."""
        nv = C.c_size_t()
        # size query first (all outputs NULL), then arrays of exactly that many rows
        self._check(self.lib.imls_captured_correspondences(self.ctx, int(it), 0, None, None, None, None, C.byref(nv)))
        N = nv.value
        x = np.zeros((N, 3), np.float32); y = np.zeros((N, 3), np.float32); n = np.zeros((N, 3), np.float32)
        idx = np.zeros(N, np.uint32)
        self._check(self.lib.imls_captured_correspondences(self.ctx, int(it), N, _ptr(x), _ptr(y), _ptr(n), _ptr(idx),
                                                           C.byref(nv)))
        return x, y, n, idx

    def timing_origin(self):
        """Process-wide origin of the timing intervals (imls_timing_origin)."""
        self._check(self.lib.imls_timing_origin(self.ctx))

    def timing_intervals(self, kernel: int) -> np.ndarray:
        """(n, 2) ms since the origin of every harvested launch of `kernel` (imls_timing_intervals)."""
        n = C.c_size_t()
        self._check(self.lib.imls_timing_intervals(self.ctx, kernel, None, 0, C.byref(n)))
        out = np.zeros((max(n.value, 1), 2))
        self._check(self.lib.imls_timing_intervals(self.ctx, kernel, _ptr(out), n.value, C.byref(n)))
        return out[: n.value]

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


def _ctx_array(contexts):
    arr = (C.c_void_p * max(len(contexts), 1))()
    for k, c in enumerate(contexts):
        arr[k] = c.ctx
    return arr


def register_frames_async(contexts):
    """Enqueue the frames loaded into `contexts` (set_target / map_push + set_source on each) as ONE
    launch sequence (imls_register_frames_async): every per-iteration kernel runs once for all
    frames.  Collect with register_frames_result(contexts)."""
    if not contexts:
        raise ValueError("no contexts")
    lead = contexts[0]
    lead._check(lead.lib.imls_register_frames_async(_ctx_array(contexts), len(contexts)))


class TraceView:
    """One frame's iteration records inside a batch's result array, read on access: a batch of
    1024 frames × 20 iterations would otherwise build 20k ctypes records in Python before the
    caller can enqueue its next batch (measured: ~16 ms of GPU idle per stream step)."""

    __slots__ = ("_arr", "_off", "_n")

    def __init__(self, arr, off: int, n: int):
        self._arr, self._off, self._n = arr, off, n

    def __len__(self):
        return self._n

    def __getitem__(self, j):
        if isinstance(j, slice):
            return [self[k] for k in range(*j.indices(self._n))]
        if j < 0:
            j += self._n
        if not 0 <= j < self._n:
            raise IndexError(j)
        return self._arr[self._off + j]

    def __iter__(self):
        return (self._arr[self._off + j] for j in range(self._n))


def register_frames_result(contexts):
    """(poses (n,4,4), iterations (n,), statuses (n,), traces [n sequences of ImlsIterTrace]).  The
    per-frame trace sequences are views into the batch's result array (records built on access)."""
    lead, n = contexts[0], len(contexts)
    it = max(lead.params.iterations, 1)
    poses = np.zeros((n, 16)); iters = np.zeros(n, np.int32); st = np.zeros(n, np.int32)
    tr = (_abi.ImlsIterTrace * (it * n))()
    lead._check(lead.lib.imls_register_frames_result(lead.ctx, _ptr(poses), _ptr(iters), _ptr(st), tr))
    traces = [TraceView(tr, k * it, int(iters[k])) for k in range(n)]
    for c, t in zip(contexts, traces):
        c.last_trace = t
    return poses.reshape(n, 4, 4), iters, st, traces


def register_frames(contexts):
    """imls_register_frames: register_frames_async + register_frames_result."""
    register_frames_async(contexts)
    return register_frames_result(contexts)


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
    """The free-function solvers' context (one per process, like the reference's free functions).
    Its RANSAC rand() stream runs on across every call, as the reference's process-wide rand()."""
    global _SOLVER_CTX
    if _SOLVER_CTX is None:
        _SOLVER_CTX = ImlsContext(_config.params_from_config(_config.load()))
    return _SOLVER_CTX


def SolveMotionEstimationProblemLS(source_cloud, ref_cloud, ref_normals, timestamp: str = "", threshold: float = 0.02):
    """solver.cpp:74-166 → (flag, deltaTrans 4×4)."""
    ctx = _solver_ctx()
    p = _abi.ImlsParams.from_buffer_copy(ctx.params)
    p.ls_threshold = float(threshold)
    ctx.set_params(p)
    return ctx.solve_correspondences(_abi.IMLS_SOLVE_LS, _triples(source_cloud), _triples(ref_cloud), _triples(ref_normals))


def SolveMotionEstimationProblemWeightedLS(source_cloud, ref_cloud, ref_normals, weights, timestamp: str = ""):
    """solver.cpp:168-220 → (flag, deltaTrans 4×4)."""
    return _solver_ctx().solve_correspondences(_abi.IMLS_SOLVE_WEIGHTED_LS, _triples(source_cloud), _triples(ref_cloud),
                                               _triples(ref_normals), np.asarray(weights, dtype=np.float64))


def SolveMotionEstimationProblemRANSAC(source_cloud, ref_cloud, ref_normals, timestamp: str = "",
                                       max_iterations: int = 5000, distance_threshold: float = 0.8,
                                       min_inliers_percentage: float = 0.95, huber_threshold: float = 0.648,
                                       final_solve_method: str = "DRPM", ls_threshold: float = 0.02,
                                       drpm_threshold: float = 0.05, drpm_stdev_points: float = 0.02,
                                       drpm_stdev_normals: float = 0.05):
    """solver.cpp:222-385 (+ the LS / Weighted LS / DRPM finals, 368-384, 486-603) → (flag, deltaTrans).
    An unknown final_solve_method returns False like solver.cpp:380-384."""
    if final_solve_method not in _config.FINAL:
        return False, np.eye(4)
    ctx = _solver_ctx()
    p = _abi.ImlsParams.from_buffer_copy(ctx.params)
    p.ransac_max_iterations = int(max_iterations)
    p.ransac_distance_threshold = float(distance_threshold)
    p.ransac_min_inliers_percentage = float(min_inliers_percentage)
    p.ransac_huber_threshold = float(huber_threshold)
    p.ransac_final_method = _config.FINAL[final_solve_method]
    p.ransac_ls_threshold = float(ls_threshold)
    p.drpm_threshold = float(drpm_threshold)
    p.drpm_stdev_points = float(drpm_stdev_points)
    p.drpm_stdev_normals = float(drpm_stdev_normals)
    ctx.set_params(p)
    return ctx.solve_correspondences(_abi.IMLS_SOLVE_RANSAC, _triples(source_cloud), _triples(ref_cloud),
                                     _triples(ref_normals))


def SolveMotionEstimationProblemDRPM(source_cloud, ref_cloud, ref_normals, weights, timestamp: str = "",
                                     threshold: float = 0.05, stdev_points: float = 0.02, stdev_normals: float = 0.05):
    """solver.cpp:499-603 (degeneracy-aware solve with DRPM probabilities) → (flag, deltaTrans)."""
    ctx = _solver_ctx()
    p = _abi.ImlsParams.from_buffer_copy(ctx.params)
    p.drpm_threshold, p.drpm_stdev_points, p.drpm_stdev_normals = float(threshold), float(stdev_points), float(stdev_normals)
    ctx.set_params(p)
    return ctx.solve_correspondences(_abi.IMLS_SOLVE_DRPM, _triples(source_cloud), _triples(ref_cloud),
                                     _triples(ref_normals), np.asarray(weights, dtype=np.float64))


def solveMotionEstimationProblem(solve_method: str, in_cloud_vec, ref_cloud_vec, ref_normal, timestamp: str = "",
                                 cfg: Optional[dict] = None):
    """laser_odometry.cpp:173-275: string dispatch with parameters read from the config each call."""
    cfg = cfg if cfg is not None else _config.load()
    sm = cfg["laser_odometry"]["solve_method"]
    if solve_method == "LS":
        return SolveMotionEstimationProblemLS(in_cloud_vec, ref_cloud_vec, ref_normal, timestamp, float(sm["LS"]["threshold"]))
    if solve_method == "RANSAC":
        rs = sm["RANSAC"]
        return SolveMotionEstimationProblemRANSAC(
            in_cloud_vec, ref_cloud_vec, ref_normal, timestamp, int(rs["max_iterations"]),
            float(rs["distance_threshold"]), float(rs["min_inliers_percentage"]), float(rs["huber_threshold"]),
            str(rs["final_solve_method"]), float(rs["LS_threshold"]), float(rs["DRPM_threshold"]),
            float(rs["DRPM_stdev_points"]), float(rs["DRPM_stdev_normals"]))
    if solve_method in _config.UNSUPPORTED_SOLVERS:
        raise _abi.ImlsError(_abi.IMLS_ERR_UNSUPPORTED, f"solve_method {solve_method!r} is not on the GPU path")
    # the reference prints "Invalid SOLVE_METHOD!" and returns false (laser_odometry.cpp:269-272)
    return False, np.eye(4)


# ================================================================================================
# Per-frame driver (laser_odometry.cpp:416-683 without ROS)
# ================================================================================================
def chain_pose(prev, rel) -> np.ndarray:
    """nowPose = prevLaserPose * rPose (laser_odometry.cpp:652) in Eigen's 4×4 product order
    (res(i,j) = ((a(i,0)b(0,j) + a(i,1)b(1,j)) + a(i,2)b(2,j)) + a(i,3)b(3,j)): identical doubles
    on every host, unlike a BLAS matmul."""
    a = np.asarray(prev, dtype=np.float64).reshape(4, 4).tolist()
    b = np.asarray(rel, dtype=np.float64).reshape(4, 4).tolist()
    return np.array([[((a[i][0] * b[0][j] + a[i][1] * b[1][j]) + a[i][2] * b[2][j]) + a[i][3] * b[3][j]
                      for j in range(4)] for i in range(4)])


class LaserOdometry:
    """processData (laser_odometry.cpp:416-683) minus ROS: per (filteredLaserCloud, flatCloud)
    frame, the first frame only seeds the map (Q13); every later frame registers its flat cloud
    against the map FIFO (rPose = I, the fused device loop), chains nowPose = prevLaserPose·rPose
    and appends it to `pose_file` (savePoseToFile, 659); then the filtered cloud joins the FIFO
    (accumulateTargetCloud, 663-664).  The FIFO lives in HBM (ImlsContext.map_push): only the new
    scan crosses PCIe each frame.  The context (and its RANSAC rand() stream) persists across frames."""

    def __init__(self, params: Optional[_abi.ImlsParams] = None, device: int = 0, pose_file: Optional[str] = None,
                 output_dir: Optional[str] = None, pipelined: Optional[bool] = None):
        self.ctx = ImlsContext(params, device)
        # pipelined (default for max_queue_size 1, the shipped config): two contexts alternate.  Frame
        # k registers on the one holding scan k−1's index while its own filtered scan goes to the
        # other — that push's pack, upload, NaN filter and index build run beside the registration.
        # The reference's work per frame is unchanged (accumulateTargetCloud after matching,
        # laser_odometry.cpp:663-664: only its start moves earlier, and the map the next frame sees is
        # the same scan); the RANSAC rand() stream is handed from one context to the other, so the
        # draws continue as in one context (tests/test_gpu_stream.py: poses bit-equal to one context)
        self._ctxs = [self.ctx]
        if pipelined is None:
            pipelined = self.ctx.params.max_queue_size == 1
        if pipelined and self.ctx.params.max_queue_size == 1:
            self._ctxs.append(ImlsContext(params, device))
        self._cur = 0                   # the context holding the map the next frame registers against
        # output_dir (opt-in): the reference's per-iteration outputs (laser_odometry.cpp:621-625) —
        # matched_points/<ts>_<i>.txt and imls_iter_results.txt under it, from the device trace and
        # the captured correspondences (the subdirectory is created here; the reference needs it
        # pre-created, config.json:173-176)
        self.output_dir = output_dir
        if output_dir:
            import os
            os.makedirs(os.path.join(output_dir, "matched_points"), exist_ok=True)
            for c in self._ctxs:
                c.capture_correspondences(True)
        self.prev_pose = np.eye(4)
        self.frame_count = 0
        self.pose_file = pose_file
        self.poses: list = []           # (timestamp, nowPose 4×4) per registered frame
        self.results: list = []         # (timestamp, rPose, iterations, status) per registered frame

    def close(self):
        for c in self._ctxs:
            c.close()

    @property
    def pipelined(self) -> bool:
        return len(self._ctxs) == 2

    @property
    def contexts(self) -> tuple:
        """Every context this driver registers on (two in pipelined mode, which alternate frame by
        frame).  `.ctx` is only the context of the current / last frame: a setting made through it
        reaches every other frame only, so apply settings to all of them (`apply`)."""
        return tuple(self._ctxs)

    def apply(self, fn):
        """fn(ctx) for every context (set_option, enable_stats, set_defer, kernel timing …)."""
        return [fn(c) for c in self._ctxs]

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def process(self, filtered_cloud, flat_cloud, timestamp: str = ""):
        # the reference's step timers (laser_odometry.cpp:418-420, 461-475, 660, 677): with output_dir,
        # "Frame time", "1. Preprocessing", "2. Matching and solving in flat points" (registered
        # frames only) and "Total time" are appended to laser_odometry_times.txt
        times = TimesLog(self.output_dir) if self.output_dir else None
        result = None
        n_flat = len(flat_cloud)
        ctx = self.ctx = self._ctxs[self._cur]
        nxt = self._ctxs[1 - self._cur] if self.pipelined else ctx   # where this frame's scan goes
        pushed = False
        registers = self.frame_count != 0 and n_flat != 0 and ctx.n_target != 0
        if registers:
            # the flat cloud's upload: this path's preprocessing.  Count-less: the registration waits
            # for the filter's count itself, so the host does not also wait here for the count and the
            # kept-index download (one stream synchronisation fewer before the first launch)
            ctx.set_source(flat_cloud, count=False)
        if times:
            times.frame(timestamp)
            times.step("1. Preprocessing")
        if self.frame_count != 0:
            if times:
                times.tic()                            # laser_odometry.cpp:482: step 2 starts here
            if not registers:
                # in_cloud / the map is empty: the first iteration's gate breaks with rPose = I (570-576)
                result = dict(pose=np.eye(4), iters=0, status=_abi.IMLS_FRAME_TOO_FEW, trace=[])
            elif nxt is not ctx:
                ctx.register_frame_async()
                nxt.map_push(filtered_cloud)           # this frame's accumulateTargetCloud, overlapped
                pushed = True
                pose, iters, status = ctx.register_frame_result()
                result = dict(pose=pose, iters=iters, status=status, trace=ctx.last_trace)
            else:
                result = ctx.register_frame()
            if registers and self.output_dir:
                self._save_iterations(result, timestamp)
            now = chain_pose(self.prev_pose, result["pose"])
            self.prev_pose = now
            self.poses.append((timestamp, now))
            self.results.append((timestamp, result["pose"], result["iters"], result["status"]))
            if self.pose_file:
                savePoseToFile(now, self.pose_file, timestamp)
            if times:
                times.step("2. Matching and solving in flat points")
        if not pushed:
            nxt.map_push(filtered_cloud)
        if nxt is not ctx:
            if ctx.params.solve_method == _abi.IMLS_SOLVE_RANSAC:
                nxt.set_rng_state(ctx.rng_state())      # one rand() stream across the frames
            self._cur = 1 - self._cur
        self.frame_count += 1
        if times:
            times.total("Total time")
        return result

    def _save_iterations(self, result, timestamp: str):
        """laser_odometry.cpp:621-625, for every iteration whose solve succeeded (the reference writes
        after the solver's flag check, before the convergence test): the correspondences the solver
        got (in_cloud_vec, ref_cloud_vec) and rPose after `rPose = Δ·rPose`."""
        import os
        for i in range(result["iters"]):
            x, y, _, _ = self.ctx.captured(i)
            saveMatchedPointsToFile(x, y, os.path.join(self.output_dir, "matched_points", f"{timestamp}_{i}.txt"))
            savePoseToFile(np.array(result["trace"][i].pose).reshape(4, 4),
                           os.path.join(self.output_dir, "imls_iter_results.txt"), timestamp)


class TimesLog:
    """TicToc::tocAndLog (tic_toc.h:28-38) as processData uses it (laser_odometry.cpp:418-420, 430,
    461-475, 482, 660, 677): two clocks started together (t_whole, t_step); t_step restarts (tic) at
    the start of step 1 and again at the start of step 2 (482), so "2." excludes "1."; a step line
    is the time since t_step's last tic, `<step>: <ms> ms` with std::fixed and 3 decimals, appended
    to <dir>/laser_odometry_times.txt.  One difference in what is inside step 2: in LaserOdometry's
    pipelined mode the next map's push (accumulateTargetCloud, 663-664) runs beside the registration,
    so its host work falls inside the step-2 interval (the reference times it after step 2)."""

    FILE = "laser_odometry_times.txt"

    def __init__(self, directory: str):
        import os
        import time
        self.path = os.path.join(directory, self.FILE)
        self._now = time.perf_counter
        self.t_whole = self.t_step = self._now()

    def _append(self, line: str):
        with open(self.path, "a") as f:
            f.write(line + "\n")

    def tic(self):
        self.t_step = self._now()

    def frame(self, timestamp: str):
        self._append(f"Frame time: {timestamp}")

    def step(self, name: str) -> float:
        ms = (self._now() - self.t_step) * 1000.0
        self._append(format_time_line(name, ms))
        return ms

    def total(self, name: str) -> float:
        ms = (self._now() - self.t_whole) * 1000.0
        self._append(format_time_line(name, ms))
        return ms


def format_time_line(step: str, ms: float) -> str:
    """tic_toc.h:34: `file << std::fixed << std::setprecision(3) << stepName << ": " << time << " ms"`."""
    return f"{step}: {ms:.3f} ms"


def _quat_xyzw(R) -> tuple:
    """Eigen::Quaterniond(Matrix3d) (Eigen's quaternionbase_assign_impl for a 3×3): the trace branch,
    else the largest-diagonal branch chosen with strict '>'."""
    m = np.asarray(R, dtype=np.float64).tolist()
    t = (m[0][0] + m[1][1]) + m[2][2]
    q = [0.0, 0.0, 0.0]
    if t > 0.0:
        t = math.sqrt(t + 1.0)
        w = 0.5 * t
        t = 0.5 / t
        q = [(m[2][1] - m[1][2]) * t, (m[0][2] - m[2][0]) * t, (m[1][0] - m[0][1]) * t]
    else:
        i = 0
        if m[1][1] > m[0][0]:
            i = 1
        if m[2][2] > m[i][i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = math.sqrt(((m[i][i] - m[j][j]) - m[k][k]) + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        w = (m[k][j] - m[j][k]) * t
        q[j] = (m[j][i] + m[i][j]) * t
        q[k] = (m[k][i] + m[i][k]) * t
    return q[0], q[1], q[2], w


def format_pose_line(pose, timestamp: str) -> str:
    """One savePoseToFile line: `ts tx ty tz qx qy qz qw`, std::fixed, 6 decimals."""
    P = np.asarray(pose, dtype=np.float64)
    x, y, z, w = _quat_xyzw(P[:3, :3])
    return f"{timestamp} {P[0, 3]:.6f} {P[1, 3]:.6f} {P[2, 3]:.6f} {x:.6f} {y:.6f} {z:.6f} {w:.6f}\n"


def savePoseToFile(pose, filename: str, timestamp: str):
    """saver.cpp:46-54: append `ts tx ty tz qx qy qz qw`, fixed, 6 decimals."""
    with open(filename, "a") as f:
        f.write(format_pose_line(pose, timestamp))


def saveMatchedPointsToFile(source_cloud, matched_cloud, filename: str):
    """saver.cpp:113-133: append `sx sy sz yx yy yz` per pair (default 6-significant-digit stream)."""
    s, d = _triples(source_cloud), _triples(matched_cloud)
    with open(filename, "a") as f:
        for a, b in zip(s, d):
            f.write(" ".join(_g6(v) for v in (*a, *b)) + "\n")


def _g6(v: float) -> str:
    """std::ostream's default float format (%g with precision 6; 'inf'/'nan' as glibc prints them)."""
    return "%g" % v
