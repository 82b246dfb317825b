"""Upstream producer, sampling: samplePointCloud "normal" / "major_axis"
(scan_registration.cpp:536-806) with farthestPointSampling (common.cpp:19-82) — CPU side: the C++
oracle on analytic cases.  Parity unpinned: randomSampling seeds std::mt19937 from
std::random_device in the reference (restated with a seed), FPS's first index comes from the
process's glibc rand() stream (restated from srand(rand_seed) per call)."""
import numpy as np

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi


def two_planes(n_each=300, seed=0):
    """A floor (normal +z) and a wall (normal +x): two histogram bins."""
    rng = np.random.default_rng(seed)
    floor = np.c_[rng.uniform(0, 10, n_each), rng.uniform(0, 10, n_each), np.zeros(n_each)]
    wall = np.c_[np.full(n_each, 5.0), rng.uniform(0, 10, n_each), rng.uniform(0, 3, n_each)]
    xyz = np.concatenate([floor, wall]).astype(np.float32)
    nrm = np.concatenate([np.tile([0, 0, 1.0], (n_each, 1)), np.tile([1.0, 0, 0], (n_each, 1))]).astype(np.float32)
    return xyz, nrm


def bin_of(nrm, az_bins=8, el_bins=8):
    az = np.arctan2(nrm[:, 1], nrm[:, 0]).astype(np.float32)
    az = np.where(az < 0, az + 2 * np.pi, az)
    el = np.arcsin(nrm[:, 2].astype(np.float64)) + np.pi / 2
    return (np.minimum((az / (2 * np.pi / az_bins)).astype(int), az_bins - 1) * el_bins
            + np.minimum((el / (np.pi / el_bins)).astype(int), el_bins - 1))


def test_normal_sampling_bins_and_fps():
    xyz, nrm = two_planes()
    cand = np.arange(len(xyz))
    p = _abi.default_sample_params(_abi.IMLS_SAMPLE_NORMAL)
    s, _ = oc.sample_point_cloud(xyz, nrm, cand, None, p)
    assert len(s) == 200 and len(set(s.tolist())) == 200          # two bins × max_points_per_bin 100
    b = bin_of(nrm[s])
    assert np.all(np.diff(b) >= 0)                                 # bin order (az-major, el-minor)
    p.sampling_strategy = _abi.SAMPLE_FPS
    f, _ = oc.sample_point_cloud(xyz, nrm, cand, None, p)
    assert len(f) == 200
    # FPS: every next sample is the farthest from the ones before (within its bin)
    for lo in (0, 100):
        pts = xyz[f[lo:lo + 100]].astype(np.float64)
        binpts = xyz[np.nonzero(bin_of(nrm) == bin_of(nrm[f[lo:lo + 1]])[0])[0]].astype(np.float64)
        for k in (1, 10, 50):
            dmin = np.min(np.linalg.norm(binpts[:, None] - pts[None, :k], axis=2), axis=1)
            assert np.isclose(np.linalg.norm(pts[k][None] - pts[:k], axis=1).min(), dmin.max())


def test_small_bins_kept_whole_and_dropped():
    xyz, nrm = two_planes(n_each=50)
    cand = np.r_[np.arange(10), np.arange(50, 100)]                # floor bin 10 < 20 → dropped; wall 50 ≤ 100 → whole
    p = _abi.default_sample_params(_abi.IMLS_SAMPLE_NORMAL)
    s, _ = oc.sample_point_cloud(xyz, nrm, cand, None, p)
    assert np.array_equal(s, np.arange(50, 100))


def test_major_axis_weights():
    xyz, nrm = two_planes(n_each=400)
    # the previous frame: the floor seen 0.2 m higher, the wall 0.6 m further → bin weights ∝ the offsets
    last = np.concatenate([xyz[:400] + [0, 0, 0.2], xyz[400:] + [0.6, 0, 0]]).astype(np.float32)
    p = _abi.default_sample_params(_abi.IMLS_SAMPLE_MAJOR_AXIS)
    s, w = oc.sample_point_cloud(xyz, nrm, np.arange(800), last, p)
    nz = np.sort(w[w > 0])
    assert len(nz) == 2 and np.isclose(w.sum(), 1.0, atol=1e-6)
    assert nz[1] > nz[0]                                             # the wall bin (larger offset) weighs more
    assert len(s) == sum(min(int(x * 2000), 400) for x in w if x > 0)
