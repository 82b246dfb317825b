"""Buffer growth while other work is in flight (api.hip devbuf_grow): a replaced device buffer is
retired behind an event on every library stream that still had work — never freed under a pending
kernel, and no device-wide synchronisation.  Results must be bit-equal to the same registrations on
fresh contexts (nothing grown, nothing in flight beside them)."""
import numpy as np
import pytest

from planetary_lidar_odometry_amd import _abi, config, imls_icp, synth

pytestmark = pytest.mark.gpu


def _fresh(p, pair, src=None):
    with imls_icp.ImlsContext(p, device=0) as c:
        c.set_target(pair.target)
        c.set_source(pair.source if src is None else src)
        return c.register_frame()


def _same(a, b):
    return np.array_equal(a["pose"], b["pose"]) and a["iters"] == b["iters"] and a["status"] == b["status"]


def test_grow_beside_a_frame_in_flight():
    """Context A registers a large pair asynchronously; meanwhile context B — sized by a small frame —
    loads a large pair (every per-frame buffer grows, the old ones retired while A's kernels run) and
    registers it; then B goes back to a small frame (the retired buffers may be handed out again)."""
    p = config.bench_params(12)
    big = synth.make_pair("hdl64", map_scans=3, start=8)
    big2 = synth.make_pair("hdl64", map_scans=4, scene_seed=1, start=12)
    small = synth.make_pair("vlp16", map_scans=1, start=6)
    small_src = synth.fps_subsample(small.source, 1200, seed=2)
    want_big, want_big2, want_small = _fresh(p, big), _fresh(p, big2), _fresh(p, small, small_src)
    with imls_icp.ImlsContext(p, device=0) as a, imls_icp.ImlsContext(p, device=0) as b:
        b.set_target(small.target)
        b.set_source(small_src)
        r0 = b.register_frame()
        a.set_target(big.target)
        a.set_source(big.source)
        a.register_frame_async()
        b.set_target(big2.target)                # grows B's target / index buffers beside A's frame
        b.set_source(big2.source)                # and its per-query buffers
        r1 = b.register_frame()
        pa, ia, sa = a.register_frame_result()
        b.set_target(small.target)
        b.set_source(small_src)
        r2 = b.register_frame()
    assert _same(r0, want_small) and _same(r2, want_small)
    assert _same(r1, want_big2)
    assert np.array_equal(pa, want_big["pose"]) and ia == want_big["iters"] and sa == want_big["status"]


@pytest.mark.parametrize("solver", ["LS", "RANSAC"])
def test_pipelined_growing_frames_equal_one_context(solver):
    """LaserOdometry's two pipelined contexts with scans that grow frame by frame: the next map's push
    (upload, NaN filter, index build — all growing their buffers) runs while the other context
    registers.  Poses bit-equal to the one-context loop."""
    p = config.params_from_config(config.load())
    if solver == "LS":
        p.solve_method = _abi.IMLS_SOLVE_LS
    p.max_queue_size = 1
    scene = synth.make_scene(2)
    poses = synth.trajectory(14, 2003)
    sm = synth.vlp16()
    frames = []
    for k in range(7):
        sc = synth.scan(scene, sm, poses[5 + k], seed=4000 + k)
        keep = np.sort(np.random.default_rng(k).choice(len(sc), int(len(sc) * (0.35 + 0.1 * k)), replace=False))
        filtered = sc[keep]
        frames.append((filtered, synth.fps_subsample(filtered, 300 + 250 * k, seed=k)))
    out = {}
    for pipelined in (False, True):
        with imls_icp.LaserOdometry(p, device=0, pipelined=pipelined) as lo:
            for filtered, flat in frames:
                lo.process(filtered, flat)
            out[pipelined] = list(lo.results)
    assert len(out[False]) == len(out[True]) == len(frames) - 1
    for (t0, p0, i0, s0), (t1, p1, i1, s1) in zip(out[False], out[True]):
        assert (i0, s0) == (i1, s1) and np.array_equal(p0, p1)


def test_fifo_mode_switch_needs_empty_map():
    """max_queue_size moving between the concatenated map (1, ≥ 32) and the incremental index
    (2…31) while the FIFO holds scans is refused (IMLS_ERR_STATE); after map_clear it is allowed and
    the incremental map registers like a fresh context."""
    p = config.bench_params(6)
    pair = synth.make_pair("vlp16", map_scans=2, start=9)
    parts = synth.map_parts(pair)
    p.max_queue_size = 1
    with imls_icp.ImlsContext(p, device=0) as c:
        c.map_push(parts[0])
        q = config.bench_params(6)
        q.max_queue_size = 2
        with pytest.raises(_abi.ImlsError) as e:
            c.set_params(q)
        assert e.value.status == _abi.IMLS_ERR_STATE
        c.map_clear()
        c.set_params(q)
        for part in parts:
            c.map_push(part)
        c.set_source(pair.source)
        got = c.register_frame()
    assert _same(got, _fresh(config.bench_params(6), pair))
