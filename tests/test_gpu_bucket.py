"""Leaves smaller than one wave (option leaf_size = 16 / 32 points per leaf) through the packet traversal.

The lockstep leaf scan counts a lane's already-listed points of the leaf before it builds the
listed-point mask.  That count must cover the leaf's own `cnt = min(B, M − base)`
points only: with B < 64 a 64-slot window also counts listed points of the FOLLOWING leaves, a lane
with one new candidate then looks like it has none, the candidate is dropped and the list's bound W
claims a point was searched when it was not.  The correspondences of every iteration
are compared with the CPU oracle (oracle/imls_oracle.cpp restates imls_icp.cpp:496-745, which has no
notion of leaves): validity masks and reject counters exact, x / n bit-exact, y within 1e-5 m; and a
whole registration's iterations, valid counts and reject counters exact, pose within 1e-6.
"""
import pathlib

import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi, config, imls_icp, synth

pytestmark = pytest.mark.gpu
GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"


@pytest.mark.parametrize("qwave", ["0", "1"], ids=["packets", "wave_per_query"])
@pytest.mark.parametrize("bucket", ["16", "32"])
@pytest.mark.parametrize("name", ["vlp16_pair", "planetary_pair"])
def test_small_leaves_match_oracle(name, bucket, qwave):
    """packets: the lockstep leaf scan; wave per query: the frontier traversal, whose leaf groups
    measure B / 8 points per lane (2 at B = 16)."""
    g = dict(np.load(GOLDEN / f"{name}.npz"))
    src, tgt = np.ascontiguousarray(g["src"]), np.ascontiguousarray(g["tgt"])
    p = config.bench_params(8)
    with imls_icp.ImlsContext(p) as ctx:
        ctx.set_options(leaf_size=int(bucket), traversal=_abi.IMLS_TRAVERSAL_PACKETS if qwave == "0"
                        else _abi.IMLS_TRAVERSAL_WAVE_PER_QUERY)
        ctx.set_target(np.ascontiguousarray(tgt.T))
        ctx.set_source(np.ascontiguousarray(src.T))
        assert ctx.index_stats()["bucket"] == int(bucket)
        for pose_t in [(0.0, 0.0, 0.0), (0.35, -0.2, 0.05)]:
            pose = np.eye(4)
            pose[:3, 3] = pose_t
            x, y, n, idx, rej = ctx.project(pose)
            ox, oy, on, oidx, orej = oc.project(src, tgt, pose, p)
            assert np.array_equal(idx, oidx)
            assert np.array_equal(rej, orej), (rej, orej)
            assert np.array_equal(x, ox) and np.array_equal(n, on)
            assert np.abs(y.astype(np.float64) - oy).max() <= 1e-5
        got = ctx.register_frame()
    want = oc.register_frame(src, tgt, p)
    assert got["iters"] == want["iters"] and got["status"] == want["status"]
    for tg, tw in zip(got["trace"], want["trace"]):
        assert tg.n_valid == tw.n_valid
        assert list(tg.reject) == list(tw.reject)
    assert np.abs(got["pose"] - want["pose"]).max() < 1e-6


def test_captured_correspondences_capacity_and_lifetime():
    """imls_captured_correspondences: sized from the captured frame (size query), refuses a capacity
    below its row count, refuses iterations past the frame's iters_run, and a later set_source drops
    the capture (no stale rows of an older, larger frame)."""
    g = dict(np.load(GOLDEN / "vlp16_pair.npz"))
    src, tgt = np.ascontiguousarray(g["src"]), np.ascontiguousarray(g["tgt"])
    p = config.bench_params(4)
    with imls_icp.ImlsContext(p) as ctx:
        ctx.set_target(np.ascontiguousarray(tgt.T))
        ctx.set_source(np.ascontiguousarray(src.T))
        ctx.capture_correspondences(True)
        r = ctx.register_frame()
        x, y, n, idx = ctx.captured(0)
        assert len(idx) == r["trace"][0].n_valid
        lib, c = ctx.lib, ctx.ctx
        import ctypes as C
        nv = C.c_size_t()
        small = np.zeros((max(len(idx) - 1, 1), 3), np.float32)
        rc = lib.imls_captured_correspondences(c, 0, len(idx) - 1, small.ctypes.data, None, None, None, C.byref(nv))
        assert rc != 0 and nv.value == len(idx)
        rc = lib.imls_captured_correspondences(c, r["iters"], 0, None, None, None, None, C.byref(nv))
        assert rc != 0
        # a smaller source: the capture of the larger frame must not be readable any more
        ctx.set_source(np.ascontiguousarray(src[:, : src.shape[1] // 2].T))
        rc = lib.imls_captured_correspondences(c, 0, 0, None, None, None, None, C.byref(nv))
        assert rc != 0
        r2 = ctx.register_frame()
        x2, _, _, idx2 = ctx.captured(0)
        assert len(idx2) == r2["trace"][0].n_valid and (idx2 < src.shape[1] // 2).all()
