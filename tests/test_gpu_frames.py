"""GPU: imls_register_frames — the frames loaded into n contexts registered as ONE launch sequence
(every per-iteration kernel once for all frames, grid y = frame; SURVEY §8(b) "many independent
pairs per launch").  Frames are independent in the reference (rPose = I per frame against the raw
previous scan(s), laser_odometry.cpp:484-485, 116-136), so the contract is strict: every frame's
pose, iteration count, status and per-iteration trace must equal — bit for bit — what
imls_register_frame gives on that frame alone, whatever else shares the launch (other sizes, other
traversal / solver paths, frames that stop early)."""
import ctypes as C

import numpy as np
import pytest

from planetary_lidar_odometry_amd import _abi, config, imls_icp, synth

pytestmark = pytest.mark.gpu


def _params(iters=8, shipped_convergence=True):
    p = config.bench_params(iters)
    if shipped_convergence:
        p.delta_dist_threshold, p.delta_angle_threshold = 0.001, 0.0001745353
    return p


@pytest.fixture(scope="module")
def vlp_pairs():
    pairs = synth.make_pairs(4, "vlp16", map_scans=1, scene_seed=5, traj_seed=2005, noise_seed=1005)
    return pairs


@pytest.fixture(scope="module")
def hdl_pair():
    return synth.make_pairs(1, "hdl64", map_scans=1, scene_seed=6, traj_seed=2006, noise_seed=1006)[0]


def _single(p, frames):
    out = []
    with imls_icp.ImlsContext(p) as c:
        for src, tgt in frames:
            c.set_target(tgt)
            c.set_source(src)
            out.append(c.register_frame())
    return out


def _batched(p, frames, repeat=1, opts=None):
    ctxs = [imls_icp.ImlsContext(p) for _ in frames]
    for c in ctxs:
        c.set_options(**(opts or {}))
    try:
        res = None
        for _ in range(repeat):
            for c, (src, tgt) in zip(ctxs, frames):
                c.set_target(tgt)
                c.set_source(src)
            res = imls_icp.register_frames(ctxs)
        return res
    finally:
        for c in ctxs:
            c.close()


def _trace_equal(a, b):
    return (list(a.delta) == list(b.delta) and list(a.pose) == list(b.pose) and list(a.reject) == list(b.reject)
            and a.n_valid == b.n_valid and a.n_kept == b.n_kept)


def _check(p, frames, repeat=1):
    ref = _single(p, frames)
    poses, iters, status, traces = _batched(p, frames, repeat)
    for k, r in enumerate(ref):
        assert np.array_equal(r["pose"], poses[k]), (k, np.abs(r["pose"] - poses[k]).max())
        assert (r["iters"], r["status"]) == (iters[k], status[k]), k
        assert len(r["trace"]) == len(traces[k])
        assert all(_trace_equal(a, b) for a, b in zip(r["trace"], traces[k])), k
    return ref


def test_small_frames_one_launch(vlp_pairs):
    """≤ 2000-query frames (the config-C shape): wave-per-query traversal + one-block LS solve."""
    frames = [(synth.fps_subsample(q.source, 1500 + 100 * k, seed=k), q.target) for k, q in enumerate(vlp_pairs)]
    ref = _check(_params(), frames, repeat=2)
    assert any(r["status"] == _abi.IMLS_FRAME_CONVERGED for r in ref)     # frames stop at their own iteration


def test_mixed_paths_in_one_batch(vlp_pairs, hdl_pair):
    """Every per-frame path shares the launch: packets (> 16384 queries) and wave-per-query
    traversal, the grid LS chain (> 4096 rows) and the one-block solve."""
    frames = [
        (hdl_pair.source, hdl_pair.target),                                        # packets + chain
        (synth.fps_subsample(vlp_pairs[0].source, 1200, seed=1), vlp_pairs[0].target),   # qwave + small
        (vlp_pairs[1].source, vlp_pairs[1].target),                                # qwave + chain
        (synth.fps_subsample(hdl_pair.source, 30000, seed=2), hdl_pair.target),    # packets + chain
    ]
    _check(_params(6), frames)


def test_too_few_and_weighted_ls(vlp_pairs):
    """A frame that stops at the correspondence gate (TOO_FEW) next to running frames; weighted LS."""
    p = _params(5)
    frames = [(synth.fps_subsample(vlp_pairs[2].source, 1500, seed=3), vlp_pairs[2].target),
              (vlp_pairs[3].source[:12], vlp_pairs[3].target),
              (synth.fps_subsample(vlp_pairs[3].source, 1800, seed=4), vlp_pairs[3].target)]
    ref = _check(p, frames)
    assert ref[1]["status"] == _abi.IMLS_FRAME_TOO_FEW
    p.solve_method = _abi.IMLS_SOLVE_WEIGHTED_LS
    _check(p, frames)


def _check_fresh(p, frames):
    """Batched vs each frame alone in a FRESH context (a fresh seeded rand() stream per frame, as the
    batch's fresh contexts have): pose, iterations, status and trace bit for bit."""
    ref = []
    for src, tgt in frames:
        ref += _single(p, [(src, tgt)])
    poses, iters, status, traces = _batched(p, frames)
    for k, r in enumerate(ref):
        assert np.array_equal(r["pose"], poses[k]), (k, np.abs(r["pose"] - poses[k]).max())
        assert (r["iters"], r["status"]) == (iters[k], status[k]), k
        assert all(_trace_equal(a, b) for a, b in zip(r["trace"], traces[k])), k
    return ref


@pytest.mark.parametrize("final", [_abi.IMLS_FINAL_DRPM, _abi.IMLS_FINAL_LS, _abi.IMLS_FINAL_WEIGHTED_LS])
def test_ransac_frames_one_launch(vlp_pairs, final):
    """The shipped RANSAC → DRPM solver (and RANSAC's LS / weighted-LS finals) through the batched
    launch: every RANSAC step is one launch for all frames, each frame on its own context's rand()
    stream; a TOO_FEW frame shares the launch."""
    p = config.params_from_config(config.load())
    p.iterations = 4
    p.ransac_final_method = final
    frames = [(synth.fps_subsample(q.source, 1300 + 150 * k, seed=k), q.target) for k, q in enumerate(vlp_pairs[:3])]
    frames.append((vlp_pairs[3].source[:4], vlp_pairs[3].target))
    ref = _check_fresh(p, frames)
    assert ref[3]["status"] == _abi.IMLS_FRAME_TOO_FEW


def test_ransac_frames_all_chunks(vlp_pairs, hdl_pair):
    """No early exit (min inliers 100 %): every hypothesis chunk runs (16, 64, 256, …), strided over
    the batch's blocks; a large frame (grid inlier chain) next to small ones."""
    p = config.params_from_config(config.load())
    p.iterations = 2
    p.ransac_min_inliers_percentage = 1.0
    p.ransac_max_iterations = 700
    frames = [(synth.fps_subsample(hdl_pair.source, 6000, seed=7), hdl_pair.target),
              (synth.fps_subsample(vlp_pairs[0].source, 1500, seed=8), vlp_pairs[0].target)]
    _check_fresh(p, frames)
    # a frame above the one-block compaction size (three-kernel compaction for the whole batch)
    frames.append((synth.fps_subsample(hdl_pair.source, 20000, seed=9), hdl_pair.target))
    _check_fresh(p, frames)


def test_errors(vlp_pairs):
    src, tgt = vlp_pairs[0].source, vlp_pairs[0].target
    p, q = _params(3), _params(4)
    with imls_icp.ImlsContext(p) as a, imls_icp.ImlsContext(q) as b, imls_icp.ImlsContext(p) as c:
        for x in (a, b):
            x.set_target(tgt)
            x.set_source(src)
        with pytest.raises(_abi.ImlsError, match="params"):
            imls_icp.register_frames([a, b])
        c.set_target(tgt)
        with pytest.raises(_abi.ImlsError, match="set_source"):
            imls_icp.register_frames([a, c])
        with pytest.raises(_abi.ImlsError, match="twice"):
            imls_icp.register_frames([a, a])
        imls_icp.register_frames_async([a])
        with pytest.raises(_abi.ImlsError, match="pending"):
            a.register_frame_async()
        poses, _, _, _ = imls_icp.register_frames_result([a])
        assert np.all(np.isfinite(poses))
        assert np.array_equal(poses[0], a.register_frame()["pose"])     # usable afterwards, same answer


def test_plane_icp_frames(vlp_pairs):
    """The plane_ICP matcher (NN-1 tangent plane, angle gate on) through the batched launch."""
    p = _params(5)
    p.matching_method = _abi.IMLS_MATCH_PLANE_ICP
    p.picp_normal_angle_constraint = 1
    frames = [(synth.fps_subsample(q.source, 1500, seed=k), q.target) for k, q in enumerate(vlp_pairs[:3])]
    _check(p, frames)


def test_deferred_builds_match_counted(vlp_pairs):
    """set_target / set_source / map_push without a requested count return before the NaN filter's
    count is known (the rest of the build runs at first use): same registration as the counted calls;
    an all-NaN deferred target surfaces as the missing-target state error at first use."""
    p = _params(6)
    q = vlp_pairs[1]
    src = synth.fps_subsample(q.source, 1600, seed=9)
    with imls_icp.ImlsContext(p) as a, imls_icp.ImlsContext(p) as b:
        a.set_target(q.target)
        a.set_source(src)
        ra = a.register_frame()
        assert b.set_target(q.target, count=False) is None and b.set_source(src, count=False) is None
        rb = b.register_frame()
        assert np.array_equal(ra["pose"], rb["pose"]) and ra["iters"] == rb["iters"]
        b.map_push(q.target, count=False)
        b.set_source(src, count=False)
        assert np.array_equal(b.register_frame()["pose"], ra["pose"])
        x, y, n, idx, rej = b.project(np.eye(4))      # query count found without a counted set_source
        assert len(idx) > 0
        bad = np.array(q.target, copy=True)
        bad["x"] = np.nan
        b.set_target(bad, count=False)
        with pytest.raises(_abi.ImlsError, match="set_target"):
            b.register_frame()


def test_two_batches_in_flight(vlp_pairs):
    """Two disjoint batches in flight at once (the bench's double buffering): each equals its frames
    registered alone."""
    p = _params(6)
    frames = [(synth.fps_subsample(q.source, 1400, seed=20 + k), q.target) for k, q in enumerate(vlp_pairs)]
    ref = _single(p, frames)
    ctxs = [imls_icp.ImlsContext(p) for _ in frames]
    try:
        for c, (src, tgt) in zip(ctxs[:2], frames[:2]):
            c.set_target(tgt, count=False)
            c.set_source(src, count=False)
        imls_icp.register_frames_async(ctxs[:2])
        for c, (src, tgt) in zip(ctxs[2:], frames[2:]):
            c.set_target(tgt, count=False)
            c.set_source(src, count=False)
        imls_icp.register_frames_async(ctxs[2:])
        p1 = imls_icp.register_frames_result(ctxs[:2])[0]
        p2 = imls_icp.register_frames_result(ctxs[2:])[0]
        for k, pose in enumerate(list(p1) + list(p2)):
            assert np.array_equal(pose, ref[k]["pose"]), k
    finally:
        for c in ctxs:
            c.close()


def test_deferred_filters_in_large_batches(vlp_pairs):
    """With imls_set_defer on, a context defers its NaN filter to the first use: a batch filters and
    builds all its members in one launch sequence (device inputs, a queue-1 map pushed in place, NaN
    points in the maps); a member registered alone afterwards filters on its own.  Round 0 runs with
    the default (filters at once).  Every result equals a fresh single context fed the same clouds
    from the host."""
    p = _params(5)
    p.max_queue_size = 1
    frames = []
    for k in range(10):
        q = vlp_pairs[k % len(vlp_pairs)]
        tgt = np.array(q.target, copy=True)
        tgt["x"][k::17] = np.nan                      # the filter must drop these
        frames.append((synth.fps_subsample(q.source, 1200 + 37 * k, seed=30 + k), tgt))
    hip = _hip()
    dev = [(_DevSoa(hip, synth.soa(s)), _DevSoa(hip, synth.soa(t))) for s, t in frames]
    ref = _single(p, frames)
    ctxs = [imls_icp.ImlsContext(p) for _ in frames]
    try:
        for rnd in range(2):                          # round 0: filters at once; round 1: deferred
            for c, (sd, td) in zip(ctxs, dev):
                c.set_defer(rnd == 1)
                c.map_push_device(td.ptr, td.n, count=False)
                c.set_source_device(sd.ptr, sd.n, count=False)
            poses, iters, status, _ = imls_icp.register_frames(ctxs)
            for k, r in enumerate(ref):
                assert np.array_equal(r["pose"], poses[k]), (rnd, k)
                assert (r["iters"], r["status"]) == (iters[k], status[k]), (rnd, k)
        c = ctxs[3]                                   # alone, deferred filters on its own stream
        sd, td = dev[3]
        c.map_push_device(td.ptr, td.n, count=False)
        c.set_source_device(sd.ptr, sd.n, count=False)
        assert np.array_equal(c.register_frame()["pose"], ref[3]["pose"])
    finally:
        for c in ctxs:
            c.close()
        for a, b in dev:
            a.free()
            b.free()


def test_count_less_buffer_lifetime(vlp_pairs):
    """The lifetime of a count-less device load's buffer depends on imls_set_defer alone (never on
    what the context did before): defer off — once the context's stream has passed the call the
    caller may overwrite the buffer; defer on — after the first use has run (the registration's
    result) the context works on its own filtered copy.  Both with and without an earlier large
    batch on the context."""
    p = _params(5)
    p.max_queue_size = 1
    q = vlp_pairs[2]
    src = synth.fps_subsample(q.source, 1300, seed=41)
    ref = _single(p, [(src, q.target)])[0]
    hip = _hip()
    junk = np.full((6, max(src.size, q.target.size)), np.nan, np.float32)
    ctxs = [imls_icp.ImlsContext(p) for _ in range(9)]
    bufs = []
    try:
        for history in (False, True):
            if history:                               # a batch of 9 frames on these contexts first
                for c in ctxs:
                    c.set_target(q.target)
                    c.set_source(src)
                imls_icp.register_frames(ctxs)
            c = ctxs[0]
            for defer in (False, True):
                c.set_defer(defer)
                sd, td = _DevSoa(hip, synth.soa(src)), _DevSoa(hip, synth.soa(q.target))
                bufs += [sd, td]
                c.map_push_device(td.ptr, td.n, count=False)
                c.set_source_device(sd.ptr, sd.n, count=False)
                if not defer:
                    c.synchronize()                   # the stream has passed the loads
                    for b in (sd, td):
                        assert hip.hipMemcpy(C.c_void_p(b.ptr), junk.ctypes.data_as(C.c_void_p), 24 * b.n, 1) == 0
                r = c.register_frame()
                assert np.array_equal(r["pose"], ref["pose"]) and r["iters"] == ref["iters"], (history, defer)
                if defer:                             # first use has run: the context keeps its copy
                    for b in (sd, td):
                        assert hip.hipMemcpy(C.c_void_p(b.ptr), junk.ctypes.data_as(C.c_void_p), 24 * b.n, 1) == 0
                    r = c.register_frame()
                    assert np.array_equal(r["pose"], ref["pose"]), (history, defer)
    finally:
        for c in ctxs:
            c.close()
        for b in bufs:
            b.free()


def _hip():
    """The HIP runtime the product library runs on (tests/gpu_mem.py)."""
    import gpu_mem
    return gpu_mem.product_hip()


class _DevSoa:
    """A (6, n) float32 SoA cloud copied to device memory (tests/gpu_mem.py)."""

    def __init__(self, hip, a):
        import gpu_mem
        self._d = gpu_mem.DevSoa(a, hip)
        self.hip, self.n, self.ptr = hip, self._d.n, self._d.ptr

    def free(self):
        self._d.free()


@pytest.mark.parametrize("packet,iters", [(16, 20), (32, 3)])
def test_traversal_packet_sizes_in_batches(hdl_pair, packet, iters):
    """The traversal packet size (queries per wave, options first_packet / first_packet_iters;
    batched launches too with first_packet_batched) only changes which waves walk which queries: the lists it
    hands k_finish are certified there, so every frame's pose, iterations and trace stay bit-equal
    to the default single-frame path (32-query packets in iteration 0 only)."""
    frames = [(hdl_pair.source, hdl_pair.target),
              (synth.fps_subsample(hdl_pair.source, 40000, seed=11), hdl_pair.target)]
    ref = _single(_params(6), frames)
    poses, its, status, traces = _batched(_params(6), frames,
                                          opts=dict(first_packet=packet, first_packet_iters=iters, first_packet_batched=1))
    for k, r in enumerate(ref):
        assert np.array_equal(r["pose"], poses[k]), (k, np.abs(r["pose"] - poses[k]).max())
        assert (r["iters"], r["status"]) == (its[k], status[k]), k
        assert all(_trace_equal(a, b) for a, b in zip(r["trace"], traces[k])), k
