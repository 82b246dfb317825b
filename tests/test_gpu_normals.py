"""GPU parity of the recompute-normal path: get_normals=false.
  * count mode (the documented intent of Q1): every candidate's normal = ComputeNormal
    (imls_icp.cpp:753-794) of its kNN-search_number_normal within r_normal (self match excluded),
    computed on the device once per map and read like stored normals;
  * the reference's own (dead) mode: knn() returns 0, every candidate normal is ∞ → all rejected
    as invalid normals (imls_icp.cpp:418-421, 654-657, 672-679).
Normals are the same fp64 Jacobi arithmetic on both sides, so n is compared bit-exactly."""
import pathlib

import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import config, imls_icp

pytestmark = pytest.mark.gpu
GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"
Y_TOL = 1e-5
POSE_TOL = 1e-6


def golden(name):
    return dict(np.load(GOLDEN / f"{name}.npz"))


def soa_to_rows(soa6):
    return np.ascontiguousarray(np.asarray(soa6, np.float32).T)


def params(count_mode, iters=6, k_normal=10, r_normal=1.0):
    p = config.bench_params(iters)
    p.delta_dist_threshold = 0.001
    p.delta_angle_threshold = 0.0001745353
    p.get_normals = 0
    p.recompute_normal_count_mode = count_mode
    p.search_number_normal = k_normal
    p.r_normal = r_normal
    return p


@pytest.fixture(scope="module")
def ctx():
    c = imls_icp.ImlsContext(params(1))
    yield c
    c.close()


@pytest.mark.parametrize("name", ["vlp16_pair", "planetary_pair"])
@pytest.mark.parametrize("k_normal,r_normal", [(10, 1.0), (5, 0.5), (20, 2.0)])
def test_count_mode_projection(ctx, name, k_normal, r_normal):
    g = golden(name)
    p = params(1, k_normal=k_normal, r_normal=r_normal)
    ctx.set_params(p)
    ctx.set_target(soa_to_rows(g["tgt"]))
    ctx.set_source(soa_to_rows(g["src"]))
    for k in (0, 1):
        x, y, n, idx, rej = ctx.project(g[f"pose{k}"])
        wx, wy, wn, widx, wrej = oc.project(g["src"], g["tgt"], g[f"pose{k}"], p)
        assert np.array_equal(rej, wrej) and np.array_equal(idx, widx)
        assert np.array_equal(x, wx) and np.array_equal(n, wn)
        if len(idx):
            assert np.abs(y.astype(np.float64) - wy).max() <= Y_TOL
            assert np.allclose(np.linalg.norm(n, axis=1), 1.0, atol=1e-6) and (n[:, 2] >= 0).all()


def test_count_mode_frame(ctx):
    g = golden("vlp16_pair")
    p = params(1, iters=5)
    ctx.set_params(p)
    ctx.set_target(soa_to_rows(g["tgt"]))
    ctx.set_source(soa_to_rows(g["src"]))
    r = ctx.register_frame()
    want = oc.register_frame(g["src"], g["tgt"], p)
    assert r["iters"] == want["iters"] and r["status"] == want["status"]
    assert np.abs(r["pose"] - want["pose"]).max() < POSE_TOL


def test_dead_mode_rejects_everything(ctx):
    g = golden("vlp16_pair")
    p = params(0)
    ctx.set_params(p)
    ctx.set_target(soa_to_rows(g["tgt"]))
    ctx.set_source(soa_to_rows(g["src"]))
    x, y, n, idx, rej = ctx.project(g["pose1"])
    wx, wy, wn, widx, wrej = oc.project(g["src"], g["tgt"], g["pose1"], p)
    assert len(idx) == 0 and np.array_equal(rej, wrej) and rej[2] > 0
    r = ctx.register_frame()
    assert r["status"] == 2 and r["iters"] == 0   # too few correspondences at iteration 0
