"""GPU parity of the plane_ICP matcher (laser_odometry.cpp:277-413): NN-1
within its own radius, tangent-plane projection y = x − ((x−p)·n)·n, its own angle gate and reject
semantics (unfound → "no normal", no h gate), against the oracle on the golden pairs.
No exp/acos-dependent arithmetic feeds y here, so y is compared bit-exactly."""
import pathlib

import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi, config, imls_icp

pytestmark = pytest.mark.gpu
GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"
POSE_TOL = 1e-6


def golden(name):
    return dict(np.load(GOLDEN / f"{name}.npz"))


def soa_to_rows(soa6):
    return np.ascontiguousarray(np.asarray(soa6, np.float32).T)


def picp_params(iters=10, angle=1, solver=_abi.IMLS_SOLVE_LS):
    p = config.bench_params(iters)
    p.delta_dist_threshold = 0.001
    p.delta_angle_threshold = 0.0001745353
    p.matching_method = _abi.IMLS_MATCH_PLANE_ICP
    p.picp_normal_angle_constraint = angle
    p.solve_method = solver
    return p


@pytest.fixture(scope="module")
def ctx():
    c = imls_icp.ImlsContext(picp_params())
    yield c
    c.close()


@pytest.mark.parametrize("name", ["vlp16_pair", "planetary_pair"])
@pytest.mark.parametrize("angle", [0, 1])
def test_plane_icp_projection(ctx, name, angle):
    g = golden(name)
    p = picp_params(angle=angle)
    ctx.set_params(p)
    ctx.set_target(soa_to_rows(g["tgt"]))
    ctx.set_source(soa_to_rows(g["src"]))
    for k in (0, 1):
        x, y, n, idx, rej = ctx.project(g[f"pose{k}"])
        wx, wy, wn, widx, wrej = oc.project(g["src"], g["tgt"], g[f"pose{k}"], p)
        assert np.array_equal(rej, wrej) and np.array_equal(idx, widx)
        assert np.array_equal(x, wx) and np.array_equal(n, wn) and np.array_equal(y, wy)


@pytest.mark.parametrize("name", ["vlp16_pair", "planetary_pair"])
@pytest.mark.parametrize("solver", [_abi.IMLS_SOLVE_LS, _abi.IMLS_SOLVE_RANSAC])
def test_plane_icp_register_frame(ctx, name, solver):
    g = golden(name)
    p = picp_params(iters=8, solver=solver)
    ctx.set_params(p)
    ctx.seed_rng(p.ransac_seed)        # a fresh rand() stream, as the oracle frame starts one
    ctx.set_target(soa_to_rows(g["tgt"]))
    ctx.set_source(soa_to_rows(g["src"]))
    r = ctx.register_frame()
    want = oc.register_frame(g["src"], g["tgt"], p)
    assert r["iters"] == want["iters"] and r["status"] == want["status"]
    assert np.abs(r["pose"] - want["pose"]).max() < POSE_TOL
    for t, u in zip(r["trace"], want["trace"]):
        assert t.n_valid == u.n_valid and list(t.reject) == list(u.reject)
