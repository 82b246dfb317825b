"""The lone-small-frame path (≤ 4096 queries registered alone: the exact stage fused into the
wave-per-query traversal, k_knn_qwave_f, and the LS in one block, k_solve_small) against the two
other ways the same frame can be registered — alone through the packet traversal (k_knn_wave +
k_finish + the k_project_lane fallback) and in a batch (k_knn_qwave_b + k_finish_b +
k_project_lane_b, k_solve_small_b): the same frame bit for bit.  The correspondences are the same,
and k_solve_small forms the pass-1 normal equations from the rows in one fixed order whichever
kernel produced them.  With every 3rd query uncertified (option force_fallback) the fused path
builds those queries' exact lists in the wave (exact_wave_list) while the other two defer them to
the fallback launch (k_project_lane's search): the same correspondences, so the same poses; frames
registered back to back in one context also check the deferred-query counter's reset.  One path is
also compared with the CPU oracle (imls_icp.cpp:496-745 restated in oracle/imls_oracle.cpp).
A frame of ~8000 queries (wave per query, but above k_solve_small's 4096 rows: k_knn_qwave +
k_finish + the grid solve chain alone, the _b kernels batched) is bit-equal alone and batched too."""
import pathlib

import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi, config, imls_icp, synth

pytestmark = pytest.mark.gpu
GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"


def _frame(ctx, p, force):
    ctx.set_params(p)
    ctx.set_option("force_fallback", 3 if force else 0)
    ctx.enable_stats(True)
    r = ctx.register_frame()
    r["stats"] = ctx.traversal_stats()
    return r


def _batched(p, frames, force):
    """frames registered as one batch (imls_register_frames); returns the first frame's result."""
    ctxs = [imls_icp.ImlsContext(p) for _ in frames]
    try:
        for c, (src, tgt) in zip(ctxs, frames):
            c.set_option("force_fallback", 3 if force else 0)
            c.set_target(tgt)
            c.set_source(src)
        poses, iters, status, traces = imls_icp.register_frames(ctxs)
        return dict(pose=poses[0], iters=iters[0], status=status[0], trace=traces[0])
    finally:
        for c in ctxs:
            c.close()


def _same(r, ref, key):
    assert r["iters"] == ref["iters"] and r["status"] == ref["status"], key
    dp = np.abs(r["pose"] - ref["pose"]).max()
    assert dp == 0, (key, dp)
    for ta, tb in zip(r["trace"], ref["trace"]):
        assert ta.n_valid == tb.n_valid and ta.n_kept == tb.n_kept, key
        assert list(ta.reject) == list(tb.reject), key
        dd = np.abs(np.array(ta.delta) - np.array(tb.delta)).max()
        assert dd == 0, (key, dd)


@pytest.mark.parametrize("name", ["vlp16_pair", "planetary_pair"])
def test_exact_stage_paths_bit_identical(name):
    g = dict(np.load(GOLDEN / f"{name}.npz"))
    src, tgt = np.ascontiguousarray(g["src"]), np.ascontiguousarray(g["tgt"])
    s_pts, t_pts = np.ascontiguousarray(src.T), np.ascontiguousarray(tgt.T)
    p = config.bench_params(10)
    runs = {}
    with imls_icp.ImlsContext(p) as ctx:
        ctx.set_target(t_pts)
        ctx.set_source(s_pts)
        for force in (False, True):
            ctx.set_option("traversal", _abi.IMLS_TRAVERSAL_AUTO)      # ≤ 2000 queries: fused
            runs[("fused", force)] = _frame(ctx, p, force)
            ctx.set_option("traversal", _abi.IMLS_TRAVERSAL_PACKETS)
            runs[("packets", force)] = _frame(ctx, p, force)
    other = (synth.fps_subsample(synth.make_pair("vlp16", map_scans=1, start=9).source, 1500, seed=3), t_pts)
    for force in (False, True):
        runs[("batched", force)] = _batched(p, [(s_pts, t_pts), other], force)
    ref = runs[("fused", False)]
    for key, r in runs.items():
        _same(r, ref, key)
    for path in ("fused", "packets"):
        assert runs[(path, True)]["stats"]["uncertified"] > 0.3 * len(src[0]), (path, runs[(path, True)]["stats"])
    want = oc.register_frame(src, tgt, p)
    assert ref["iters"] == want["iters"] and ref["status"] == want["status"]
    for tg, tw in zip(ref["trace"], want["trace"]):
        assert tg.n_valid == tw.n_valid
        assert list(tg.reject) == list(tw.reject)
    assert np.abs(ref["pose"] - want["pose"]).max() < 1e-6


@pytest.mark.parametrize("force", [False, True], ids=["plain", "forced_fallback"])
def test_mid_size_frame_alone_equals_batched(force):
    """4096 < N ≤ 16384 (auto traversal: one wave per query; the grid solve chain): alone and
    batched give the same frame bit for bit, with and without deferred queries."""
    pair = synth.make_pair("hdl64", map_scans=2, start=3)
    src = synth.fps_subsample(pair.source, 8000, seed=5)
    p = config.bench_params(8)
    with imls_icp.ImlsContext(p) as ctx:
        ctx.set_target(pair.target)
        ctx.set_source(src)
        alone = _frame(ctx, p, force)
    other = (synth.fps_subsample(pair.source, 6000, seed=7), pair.target)
    batched = _batched(p, [(src, pair.target), other], force)
    _same(batched, alone, ("mid", force))
    if force:
        assert alone["stats"]["uncertified"] > 0.3 * 8 * 8000 / 3, alone["stats"]
