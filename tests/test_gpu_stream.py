"""Config C on a seeded synthetic stream: the per-frame driver (laser_odometry.cpp:
478-660 with nowPose = prevLaserPose·rPose, 649-658, and savePoseToFile, saver.cpp:46-54) and the
device-resident map FIFO (a18: accumulateTargetCloud, laser_odometry.cpp:116-136), end to end on
the GPU — producer (ring PCA + geometric-features presample + major_axis sampling, ≤ 2000 flat
points per frame) → LaserOdometry — against the CPU oracle run on the same frames.

Tolerances (stated per check): rPose per frame and the chained trajectory within 1e-6 (LS; the
device solves the normal equations by pivoted Cholesky where the oracle restates Eigen's
column-pivoted QR), 1e-5 through RANSAC→DRPM (device erfc); iteration counts and statuses equal;
the pose-file lines byte-identical to the oracle's formatting of the same poses.  Parity vs the
reference itself is unpinned (see oracle/imls_oracle.h)."""
import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi, config, imls_icp, producer, synth

pytestmark = pytest.mark.gpu


def stream_frames(model: str, n: int, scene_seed: int = 0, traj_seed: int = 2000):
    """n consecutive sweeps of one seeded trajectory, each in its own sensor frame."""
    sm = synth.hdl64() if model == "hdl64" else synth.vlp16()
    scene = synth.make_scene(scene_seed)
    poses = synth.trajectory(n + 5, traj_seed)
    return [synth.scan(scene, sm, poses[5 + k], seed=3000 + k) for k in range(n)], len(sm.rings)


def produce(sweeps, n_rings):
    """GPU producer → [(pcl_cloud, pcl_surface_cloud)] per frame."""
    out = []
    with imls_icp.ImlsContext(device=0) as pctx:
        sr = producer.ScanRegistration(ctx=pctx, shuffle_seed=5, rand_seed=3)
        for sw in sweeps:
            xyz, sizes, inten = producer.sweep_inputs(sw, n_rings)
            out.append(sr.process(xyz, sizes, inten))
    return out


def oracle_stream(frames, p, rand_state=None):
    """The oracle's processData over the same frames: host FIFO (deque of the last max_queue_size
    filtered clouds, oldest first; the reference's `if` pop), oracle register_frame per frame."""
    queue, prev, out = [], np.eye(4), []
    for k, (filtered, flat) in enumerate(frames):
        if k != 0:
            tgt = synth.soa(np.concatenate(queue))
            r = oc.register_frame(synth.soa(flat), tgt, p, rand_state=rand_state)
            prev = oc.chain_pose(prev, r["pose"])
            out.append((r["pose"], r["iters"], r["status"], prev))
        queue.append(filtered)
        if len(queue) > p.max_queue_size:
            queue.pop(0)
    return out


def run_gpu(frames, p, tmp_path, name):
    pose_file = tmp_path / f"{name}.txt"
    with imls_icp.LaserOdometry(p, device=0, pose_file=str(pose_file)) as lo:
        for k, (filtered, flat) in enumerate(frames):
            lo.process(filtered, flat, timestamp=f"{1317384506.0 + 0.1 * k:f}")
        return list(lo.results), list(lo.poses), pose_file.read_text().splitlines(keepends=True)


@pytest.fixture(scope="module")
def vlp_frames():
    sweeps, nr = stream_frames("vlp16", 12)
    return produce(sweeps, nr)


@pytest.fixture(scope="module")
def hdl_frames():
    sweeps, nr = stream_frames("hdl64", 10, scene_seed=1, traj_seed=2001)
    return produce(sweeps, nr)


def test_producer_stream_matches_oracle(vlp_frames):
    """The GPU producer's flat clouds are ≤ 2000 points (major_axis max_total_points) and equal the
    oracle producer's on the same sweeps, frame by frame (indices bit-exact)."""
    sweeps, nr = stream_frames("vlp16", 12)
    last = None
    for k, (sw, (filtered, flat)) in enumerate(zip(sweeps, vlp_frames)):
        xyz, sizes, _ = producer.sweep_inputs(sw, nr)
        o = oc.ring_pca(xyz, sizes, _abi.default_pca_params())
        fxyz = xyz[o["index"]]
        assert np.array_equal(fxyz[:, 0], filtered["x"]) and np.array_equal(o["normal"][:, 2], filtered["normal_z"])
        sp = _abi.default_sample_params(_abi.IMLS_SAMPLE_NORMAL if k == 0 else _abi.IMLS_SAMPLE_MAJOR_AXIS)
        sp.shuffle_seed, sp.rand_seed = (5 + 7919 * (k + 1)) & 0xFFFFFFFF, 3 + k
        cand = np.nonzero(o["flags"] & _abi.IMLS_PCA_CANDIDATE)[0]
        s, _ = oc.sample_point_cloud(fxyz, o["normal"], cand, last, sp)
        assert np.array_equal(fxyz[s][:, 1], flat["y"])
        assert 0 < len(flat) <= (6400 if k == 0 else 2000 + 64)
        last = fxyz


def _check_stream(gpu, ora, tol):
    results, poses, lines = gpu
    assert len(results) == len(ora) == len(poses) == len(lines)
    traj_err, prev = [], np.eye(4)
    for (ts, rp, it, st), (ts2, now), (orp, oit, ost, onow), line in zip(results, poses, ora, lines):
        assert (it, st) == (oit, ost), (ts, it, st, oit, ost)
        assert np.abs(rp - orp).max() < tol, (ts, np.abs(rp - orp).max())
        assert np.array_equal(now, oc.chain_pose(prev, rp))     # nowPose = prevLaserPose·rPose, Eigen order
        prev = now
        traj_err.append(np.linalg.norm(now[:3, 3] - onow[:3, 3]))
        # the pose file: byte-identical to the oracle's savePoseToFile formatting of the same pose,
        # and numerically the oracle trajectory's line within the tolerance
        assert line == oc.format_pose(now, ts2)
        assert np.abs(np.array(line.split()[1:], float) - np.array(oc.format_pose(onow, ts2).split()[1:], float)).max() \
            <= tol + 1.01e-6
    rmse = float(np.sqrt(np.mean(np.square(traj_err))))
    assert rmse <= tol, rmse
    return rmse


@pytest.mark.parametrize("queue", [1, 3])
def test_vlp16_stream_ls(vlp_frames, tmp_path, queue):
    p = config.params_from_config(config.load())
    p.solve_method = _abi.IMLS_SOLVE_LS
    p.max_queue_size = queue
    _check_stream(run_gpu(vlp_frames, p, tmp_path, f"ls{queue}"), oracle_stream(vlp_frames, p), 1e-6)


@pytest.mark.parametrize("queue", [1, 3])
def test_hdl64_stream_ls(hdl_frames, tmp_path, queue):
    """≥ 10 HDL-64 frames, ≤ 2000 producer-sampled queries per frame against the FIFO map."""
    p = config.params_from_config(config.load())
    p.solve_method = _abi.IMLS_SOLVE_LS
    p.max_queue_size = queue
    _check_stream(run_gpu(hdl_frames, p, tmp_path, f"hdl{queue}"), oracle_stream(hdl_frames, p), 1e-6)


def test_vlp16_stream_shipped_ransac_drpm(vlp_frames, tmp_path):
    """The shipped config (RANSAC → DRPM) over 5 frames: the device rand() stream runs on across
    ICP iterations and frames exactly as the oracle's carried glibc stream (one stream for the
    whole sequence, the reference's process-wide rand())."""
    p = config.params_from_config(config.load())
    assert p.solve_method == _abi.IMLS_SOLVE_RANSAC and p.ransac_final_method == _abi.IMLS_FINAL_DRPM
    frames = vlp_frames[:5]
    st = oc.rand_state(p.ransac_seed)
    _check_stream(run_gpu(frames, p, tmp_path, "ransac"), oracle_stream(frames, p, rand_state=st), 1e-5)


@pytest.mark.parametrize("solver", ["LS", "RANSAC"])
def test_pipelined_equals_one_context(vlp_frames, solver):
    """LaserOdometry's pipelined mode (max_queue_size 1: two contexts alternate, each frame's scan
    pushed to the other while it registers) gives the one-context loop's results bit for bit — the
    same maps, the same kernels, and for RANSAC the rand() stream handed over between the contexts."""
    p = config.params_from_config(config.load())
    if solver == "LS":
        p.solve_method = _abi.IMLS_SOLVE_LS
    p.max_queue_size = 1
    frames = vlp_frames[:6]
    out = {}
    for pipelined in (False, True):
        with imls_icp.LaserOdometry(p, device=0, pipelined=pipelined) as lo:
            assert lo.pipelined == pipelined
            for filtered, flat in frames:
                lo.process(filtered, flat)
            out[pipelined] = list(lo.results)
    assert len(out[False]) == len(out[True]) == len(frames) - 1
    for (t0, p0, i0, s0), (t1, p1, i1, s1) in zip(out[False], out[True]):
        assert (i0, s0) == (i1, s1) and np.array_equal(p0, p1)


def test_device_fifo_equals_host_concatenation(hdl_frames):
    """a18: the map assembled in HBM by map_push (only the new scan uploaded) gives bit-identical
    registrations to set_target on the host-concatenated map, as the FIFO rolls over."""
    p = config.bench_params(8)
    p.max_queue_size = 3
    with imls_icp.ImlsContext(p, device=0) as a, imls_icp.ImlsContext(p, device=0) as b:
        queue = []
        for k, (filtered, flat) in enumerate(hdl_frames[:6]):
            if k:
                b.set_target(np.concatenate(queue))
                a.set_source(flat)
                b.set_source(flat)
                ra, rb = a.register_frame(), b.register_frame()
                assert np.array_equal(ra["pose"], rb["pose"]) and ra["iters"] == rb["iters"]
            n_map = a.map_push(filtered)
            queue.append(filtered)
            if len(queue) > 3:
                queue.pop(0)
            assert a.map_size() == (len(queue), sum(len(q) for q in queue))
            assert n_map == sum(len(q) for q in queue)


def test_fifo_edge_cases(vlp_frames):
    """max_queue_size 0 empties the map (the reference's push-then-pop); map_clear; an empty scan."""
    filtered, flat = vlp_frames[1]
    p = config.bench_params(3)
    p.max_queue_size = 0
    with imls_icp.ImlsContext(p, device=0) as c:
        assert c.map_push(filtered) == 0 and c.map_size() == (0, 0)
        p.max_queue_size = 2
        c.set_params(p)
        assert c.map_push(filtered) == len(filtered)
        assert c.map_push(flat[:0]) == len(filtered)          # an empty scan is an entry of 0 points
        assert c.map_size() == (2, len(filtered))
        c.map_clear()
        assert c.map_size() == (0, 0)
    with imls_icp.LaserOdometry(p, device=0) as lo:            # empty flat cloud: rPose = I, TOO_FEW
        lo.process(filtered, flat)
        r = lo.process(filtered, flat[:0])
        assert r["status"] == _abi.IMLS_FRAME_TOO_FEW and np.array_equal(r["pose"], np.eye(4))


def test_per_iteration_outputs(vlp_frames, tmp_path):
    """LaserOdometry(output_dir=…): the reference's per-iteration files (laser_odometry.cpp:621-625)
    — matched_points/<ts>_<i>.txt (saveMatchedPointsToFile, saver.cpp:113-133) and
    imls_iter_results.txt (savePoseToFile of rPose after each successful solve) — one per
    iteration that solved.  Bytes: identical to the oracle's C++ formatting of the same values;
    values: the oracle's own correspondences of that iteration (count and x exact, y within 1e-5)
    and its per-iteration rPose (within 1e-6)."""
    p = config.params_from_config(config.load())
    p.solve_method = _abi.IMLS_SOLVE_LS
    frames = vlp_frames[:4]
    out = tmp_path / "out"
    n_lines = 0
    with imls_icp.LaserOdometry(p, device=0, output_dir=str(out)) as lo:
        for k, (filtered, flat) in enumerate(frames):
            ts = f"{1317384506.0 + 0.1 * k:f}"
            r = lo.process(filtered, flat, timestamp=ts)
            if k == 0:
                continue
            tgt, src = synth.soa(frames[k - 1][0]), synth.soa(flat)   # max_queue_size 1: previous scan
            iter_lines = (out / "imls_iter_results.txt").read_text().splitlines(keepends=True)
            assert len(iter_lines) == n_lines + r["iters"]
            for i in range(r["iters"]):
                x, y, _, _ = lo.ctx.captured(i)
                text = (out / "matched_points" / f"{ts}_{i}.txt").read_text()
                assert text == oc.format_matched(x, y)             # the reference's formatting, bytes
                corr = oc.register_frame(src, tgt, p, corr_iter=i)["corr"]
                assert len(x) == len(corr) and np.array_equal(x, corr[:, :3]), (ts, i)
                assert np.abs(y.astype(np.float64) - corr[:, 3:6]).max() <= 1e-5, (ts, i)
                pose_i = np.array(r["trace"][i].pose).reshape(4, 4)
                assert iter_lines[n_lines + i] == oc.format_pose(pose_i, ts)
            want = oc.register_frame(src, tgt, p)
            assert want["iters"] == r["iters"]
            for i in range(r["iters"]):
                assert np.abs(np.array(r["trace"][i].pose) - np.array(want["trace"][i].pose)).max() < 1e-6
            assert not (out / "matched_points" / f"{ts}_{r['iters']}.txt").exists()
            n_lines += r["iters"]
    # the reference's step timer log (laser_odometry.cpp:461-475, 660, 677; tic_toc.h:28-38)
    from test_times_log import check_times_log
    check_times_log((out / "laser_odometry_times.txt").read_text(),
                    [f"{1317384506.0 + 0.1 * k:f}" for k in range(len(frames))], first_registers=False)
