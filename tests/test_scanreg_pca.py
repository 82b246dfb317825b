"""Upstream producer: ring-neighbourhood PCA normals + geometric-features
presample (scan_registration.cpp:1136-1229, computeNormalPCA 158-229, findNearestPoint 117-136,
checkPlaneValidity 138-156, computeGeometricFeatures 279-327, erase 1481-1489) — CPU side: the C++
oracle against the committed golden fixture and the independent numpy restatement, and
analytic known-answer cases (parity unpinned: PCL/FLANN and Eigen are not in the container)."""
import pathlib

import numpy as np
import pytest

import imls_np
import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"


def plane_rings(n_rings=3, per_ring=30, dx=0.05, dy=0.1, z_of_ring=None, jitter=0.0, seed=0):
    """Scan lines along x on the plane z = 0, one line per y = i·dy (z_of_ring overrides a line's z)."""
    rng = np.random.default_rng(seed)
    pts = []
    for i in range(n_rings):
        x = np.arange(per_ring) * dx
        z = np.full(per_ring, 0.0 if z_of_ring is None else z_of_ring(i))
        p = np.stack([x, np.full(per_ring, i * dy), z], 1) + rng.normal(0, jitter, (per_ring, 3)) * (jitter > 0)
        pts.append(p)
    return np.concatenate(pts).astype(np.float32), np.full(n_rings, per_ring, np.int32)


def test_oracle_reproduces_golden():
    g = np.load(GOLDEN / "pca_vlp16.npz")
    o = oc.ring_pca(g["xyz"], g["sizes"], _abi.default_pca_params())
    for k in ("index", "normal", "evals", "flags", "margin"):
        assert np.array_equal(o[k], g[k]), k
    assert np.array_equal(o["features"][:, 5], g["planarity"])
    assert [o["pca_failure"], o["plane_invalid"]] == list(g["counters"])


def test_oracle_matches_numpy_restatement():
    g = np.load(GOLDEN / "pca_vlp16.npz")
    idx, nrm, lam, fl, fail, inv = imls_np.ring_pca_np(g["xyz"], g["sizes"])
    assert np.array_equal(idx, g["index"].astype(np.int64))
    assert fail == g["counters"][0]
    flip = fl != g["flags"]
    assert np.all(g["margin"][flip] < 1e-6)
    same = ~flip
    assert np.abs(np.sum(nrm[same] * g["normal"][same], 1)).min() > 1 - 1e-6
    ok = same & ((g["flags"] & _abi.IMLS_PCA_PLANE_INVALID) == 0)
    assert np.allclose(lam[ok], g["evals"][ok], rtol=1e-4, atol=1e-7)


def test_plane_known_answer():
    xyz, sizes = plane_rings()
    o = oc.ring_pca(xyz, sizes, _abi.default_pca_params())
    # only line 1 is processed (lines 1 … N−2), centres j = 5 … 24; rows carry index start + 5 + j (Q-SR1)
    assert np.array_equal(o["index"], 30 + 5 + np.arange(5, 25))
    assert o["pca_failure"] == 0 and o["plane_invalid"] == 0
    assert np.allclose(o["normal"], [0, 0, 1], atol=1e-6)
    assert np.all(o["evals"][:, 2] < 1e-9) and np.all(o["evals"][:, 0] >= o["evals"][:, 1])
    assert np.all(o["flags"] == _abi.IMLS_PCA_CANDIDATE)   # planarity = λ2/λ1 ≫ 0.05


def test_knn_threshold_failure_and_index_mode():
    # line 2 lifted 10 m: its NN squared distance 100 > knn_distance_threshold 10 → 14 < 21 window points
    xyz, sizes = plane_rings(z_of_ring=lambda i: 10.0 if i == 2 else 0.0)
    p = _abi.default_pca_params()
    o = oc.ring_pca(xyz, sizes, p)
    assert len(o["index"]) == 0 and o["pca_failure"] == 20
    p.neighbor_scan = 1    # "index": the neighbour is the same index, no distance test
    o = oc.ring_pca(xyz, sizes, p)
    assert len(o["index"]) == 20 and o["pca_failure"] == 0
    assert np.all(o["flags"] & _abi.IMLS_PCA_PLANE_INVALID)   # the lifted line breaks the plane


def test_use_all_points_and_size_gates():
    xyz, sizes = plane_rings(n_rings=4, jitter=0.05, seed=3)   # rough: most windows fail the plane check
    p = _abi.default_pca_params()
    a = oc.ring_pca(xyz, sizes, p)
    assert a["plane_invalid"] > 0
    inv = (a["flags"] & _abi.IMLS_PCA_PLANE_INVALID) != 0
    assert np.all(a["evals"][inv] == -1) and not np.any(a["flags"][inv] & _abi.IMLS_PCA_CANDIDATE)
    p.use_all_points = 0
    b = oc.ring_pca(xyz, sizes, p)
    assert np.array_equal(b["index"], a["index"][~inv])
    # a line shorter than 17 points disables itself and both neighbours (scanEnd − scanStart < 6)
    sizes2 = sizes.copy()
    xyz2 = np.concatenate([xyz[:30], xyz[30:46], xyz[60:]])
    sizes2[1] = 16
    c = oc.ring_pca(xyz2, sizes2, _abi.default_pca_params())
    assert len(c["index"]) == 0 and c["pca_failure"] == 0
