"""The producer's front end (scan_registration.cpp:laserCloudHandler 862-1069) — CPU oracle
(oracle/scanreg_oracle.cpp oracle_scan_front_end), pinned against the synthetic sensor's own ground
truth: for a VLP-16 sweep (rings at −15° … +15° step 2°, the reference's 16-line formula recovers
them exactly) the ring of every point, the ring sizes and the in-ring order are known; relTime
spans [0, 1] over a clockwise revolution started anywhere (the halfPassed unwrap); the filters'
edge cases follow PCL / the reference (a dense cloud keeps its NaN points; NaN passes the range
test and is then dropped by the ring formula for 16 / 64 lines, but lands in ring 0 with 32).  The
GPU kernels are checked against this oracle in tests/test_gpu_front_end.py."""
import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi, synth


@pytest.fixture(scope="module")
def scene():
    return synth.make_scene(2), synth.trajectory(3, 2002)


def _fp(ns, lo=0.5, hi=100.0, dense=0):
    p = _abi.default_front_params(ns)
    p.minimum_range, p.maximum_range, p.is_dense = lo, hi, dense
    return p


def test_vlp16_rings_match_ground_truth(scene):
    sc, poses = scene
    cloud, flat = synth.scan(sc, synth.vlp16(), poses[1], 7, return_index=True)
    for start in (0.0, 123.4, 359.6):
        raw = synth.raw_sweep(sc, synth.vlp16(), poses[1], 7, start_deg=start)
        xyzi, idx, rs = oc.scan_front_end(raw, _fp(16))
        assert np.array_equal(rs, np.bincount(np.floor(cloud["intensity"]).astype(int), minlength=16))
        ring = np.repeat(np.arange(16), rs)
        assert np.array_equal(np.floor(xyzi[:, 3] + 1e-6).astype(int), ring)          # intensity = ring + 0.1·rel
        assert np.all(np.diff(idx.astype(np.int64)[ring == 3]) > 0)                     # input order within a ring
        assert np.array_equal(xyzi[:, :3], raw[idx])
        rel = (xyzi[:, 3] - ring) / 0.1
        assert rel.min() > -1e-3 and rel.max() < 1 + 1e-3                               # one revolution, unwrapped


def test_filters_and_nan_edge_cases(scene):
    sc, poses = scene
    raw = synth.raw_sweep(sc, synth.vlp16(), poses[1], 7, n_nan=6, n_close=4)
    n_nan = int(np.isnan(raw).any(axis=1).sum())
    xyzi, idx, rs = oc.scan_front_end(raw, _fp(16))
    assert not np.isin(idx, np.nonzero(np.isnan(raw).any(axis=1))[0]).any()
    assert np.all(np.linalg.norm(raw[idx], axis=1) >= 0.5)
    assert len(idx) == len(raw) - n_nan - 4
    # dense message: NaN points skip the NaN filter and pass the range test; 16 lines: int(NaN) = INT_MIN → dropped
    assert np.array_equal(oc.scan_front_end(raw, _fp(16, dense=1))[1], idx)
    # 32 lines: the nearest-angle search never updates on NaN → ring 0 (scanID's initial 0)
    xyzi32, idx32, rs32 = oc.scan_front_end(raw, _fp(32, dense=1))
    nan_rows = np.isnan(xyzi32[:, 0])
    assert nan_rows.sum() == n_nan and np.all(nan_rows[rs32[0]:] == False)  # noqa: E712
    # range thresholds: r² < min² and r² > max² drop, equality keeps (float arithmetic)
    pts = np.array([[0.5, 0, 0], [0.4999999, 0, 0], [100.0, 0, 0], [100.00001, 0, 0], [3, 0, 0.05]], np.float32)
    _, keep, _ = oc.scan_front_end(pts, _fp(16))
    assert list(keep) == [0, 2, 4]
    assert len(oc.scan_front_end(np.zeros((0, 3), np.float32), _fp(16))[0]) == 0
    assert len(oc.scan_front_end(np.full((5, 3), 0.01, np.float32), _fp(16))[0]) == 0    # nothing survives


def test_64_line_mapping(scene):
    """64 lines (the shipped launch file): 1/3° rings above −8.83°, 1/2° below, rings > 50 and
    angles outside [−24.33°, 2°] dropped (992-1003)."""
    sc, poses = scene
    raw = synth.raw_sweep(sc, synth.hdl64(), poses[1], 7, start_deg=250.0)
    xyzi, idx, rs = oc.scan_front_end(raw, _abi.default_front_params(64))
    ring = np.repeat(np.arange(64), rs)
    p = raw[idx].astype(np.float64)
    ang = np.degrees(np.arctan(p[:, 2] / np.hypot(p[:, 0], p[:, 1])))
    expect = np.where(ang >= -8.83, np.floor((2 - ang) * 3 + 0.5), 32 + np.floor((-8.83 - ang) * 2 + 0.5))
    assert np.mean(expect == ring) > 0.999 and ring.max() <= 50
