"""GPU parity of the upstream producer's sampling (imls_sample_point_cloud; samplePointCloud
"normal" / "major_axis", scan_registration.cpp:536-806, farthestPointSampling common.cpp:19-82)
against the C++ oracle.  EXACT: sampled indices (order included) and the major_axis bin weights
bit-for-bit — the device evaluates the neighbour gates and the in-order float sums with the
oracle's operations and FPS's fp64 distances likewise; the host side (histogram, shuffles, glibc
rand() replay) follows the same seeds.  Parity unpinned vs the reference itself (random_device
seeding, process-wide rand() stream; see imls_gpu.h)."""
import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi, imls_icp, synth
from test_sample_point_cloud import two_planes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    with imls_icp.ImlsContext(device=0) as c:
        yield c


def producer_frames(model, k0=0, seed=0):
    """Two consecutive sweeps → (filtered xyz, normals, candidates) per frame, from the PCA oracle."""
    m = synth.vlp16() if model == "vlp16" else synth.hdl64()
    sc = synth.make_scene(seed)
    out = []
    for k in (k0, k0 + 1):
        cl = synth.scan(sc, m, synth.pose_xyyaw(k * 1.0, 0, np.radians(0.5 * k)), seed=100 + k)
        sizes = np.bincount(np.floor(cl["intensity"]).astype(np.int64), minlength=len(m.rings))
        xyz = np.stack([cl["x"], cl["y"], cl["z"]], 1).astype(np.float32)
        o = oc.ring_pca(xyz, sizes, _abi.default_pca_params())
        out.append((xyz[o["index"]], o["normal"], np.nonzero(o["flags"] & _abi.IMLS_PCA_CANDIDATE)[0]))
    return out


def check(ctx, xyz, nrm, cand, last, p):
    so, wo = oc.sample_point_cloud(xyz, nrm, cand, last, p)
    sg, wg = ctx.sample_point_cloud(xyz, nrm, cand, last, p)
    assert np.array_equal(so, sg), (len(so), len(sg))
    assert np.array_equal(wo.view(np.uint32), wg.view(np.uint32))
    return so


@pytest.mark.parametrize("method,strategy", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_two_planes(ctx, method, strategy):
    xyz, nrm = two_planes(n_each=400)
    last = np.concatenate([xyz[:400] + [0, 0, 0.2], xyz[400:] + [0.6, 0, 0]]).astype(np.float32)
    p = _abi.default_sample_params(method)
    p.sampling_strategy = strategy
    s = check(ctx, xyz, nrm, np.arange(800), last, p)
    assert len(s) > 0


@pytest.mark.parametrize("model", ["vlp16", "hdl64"])
@pytest.mark.parametrize("method,strategy", [(1, 0), (1, 1), (0, 0), (0, 1)])
def test_producer_frames(ctx, model, method, strategy):
    (x0, n0, c0), (x1, n1, c1) = producer_frames(model)
    p = _abi.default_sample_params(method)
    p.sampling_strategy = strategy
    p.shuffle_seed, p.rand_seed = 11, 7
    s = check(ctx, x1, n1, c1, x0, p)
    assert len(s) > 0 and len(set(s.tolist())) == len(s)


def test_edge_cases(ctx):
    xyz, nrm = two_planes(n_each=50)
    p = _abi.default_sample_params(1)
    check(ctx, xyz, nrm, np.arange(0), xyz, p)                   # no candidates
    check(ctx, xyz, nrm, np.arange(100), np.zeros((0, 3), np.float32), p)   # empty previous cloud: weights NaN
    check(ctx, xyz, nrm, np.arange(100), xyz + 5.0, p)           # nothing nearby: zero weights
    p.min_points_per_bin = 1
    p.max_total_points = 7                                        # k = 0 in some bins: FPS keeps its first index
    check(ctx, xyz, nrm, np.arange(100), xyz + [0, 0, 0.1], p)
