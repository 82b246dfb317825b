"""GPU: many independent pairs through imls_register_batch (configs C/D: every frame restarts from
rPose = I against the raw previous scan, laser_odometry.cpp:484-485, 116-136).  Each pair's result
must equal — bit for bit — the single-context set_target + set_source + register_frame result
(every reduction walks rows in a fixed order, so the path is deterministic run to run), and the
error path must name the failing pair and drain the pairs in flight."""
import numpy as np
import pytest

from planetary_lidar_odometry_amd import _abi, config, imls_icp, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def stream_pairs():
    pairs = synth.make_pairs(5, "vlp16", map_scans=1, scene_seed=3, traj_seed=2003, noise_seed=1003)
    return [(synth.fps_subsample(q.source, 1500, seed=k), q.target) for k, q in enumerate(pairs)]


def test_batch_matches_single_context(stream_pairs):
    p = config.bench_params(8)
    p.delta_dist_threshold, p.delta_angle_threshold = 0.001, 0.0001745353   # shipped convergence test
    with imls_icp.ImlsBatch(p, streams=3) as b:
        poses, iters, status = b.register(stream_pairs)
        poses2, _, _ = b.register(stream_pairs[::-1])     # contexts reused in another order
    with imls_icp.ImlsContext(p) as c:
        for k, (src, tgt) in enumerate(stream_pairs):
            c.set_target(tgt)
            c.set_source(src)
            r = c.register_frame()
            assert np.array_equal(r["pose"], poses[k]), k
            assert r["iters"] == iters[k] and r["status"] == status[k]
            assert np.array_equal(r["pose"], poses2[len(stream_pairs) - 1 - k]), k


def test_batch_error_names_the_pair(stream_pairs):
    bad = list(stream_pairs)
    bad[3] = (np.zeros((0, 6), np.float32), bad[3][1])     # empty source
    with imls_icp.ImlsBatch(config.bench_params(3), streams=2) as b:
        with pytest.raises(_abi.ImlsError, match="pair 3"):
            b.register(bad)
        poses, _, _ = b.register(stream_pairs[:2])          # the batch is usable afterwards
        assert np.all(np.isfinite(poses))


def test_batch_ransac_independent_of_streams(stream_pairs):
    """The shipped RANSAC → DRPM solver draws from each context's rand() stream; imls_register_batch
    restarts it from params.ransac_seed before every pair, so a pair's result is the same whatever
    `streams` is and whatever its context registered before — equal to a fresh context's
    register_frame (laser_odometry.cpp:489: a fresh matcher per frame)."""
    p = config.params_from_config(config.load())          # RANSAC → DRPM
    p.iterations = 6
    res = []
    for streams in (1, 2, 4):
        with imls_icp.ImlsBatch(p, streams=streams) as b:
            res.append(b.register(stream_pairs))
    for k, (src, tgt) in enumerate(stream_pairs):
        with imls_icp.ImlsContext(p) as c:
            c.set_target(tgt)
            c.set_source(src)
            r = c.register_frame()
        for poses, iters, status in res:
            assert np.array_equal(r["pose"], poses[k]), k
            assert (r["iters"], r["status"]) == (iters[k], status[k]), k
