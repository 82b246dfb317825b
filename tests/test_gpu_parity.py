"""GPU parity tests: the HIP path (through the C ABI) against the oracle on identical inputs.

Contract (BASELINE north_star: "per-iteration correspondences and final pose match the reference
CPU path on identical inputs to a stated float tolerance"):
  * validity masks, reject counters, transformed points x and normals n: bit-exact;
  * projections y: |Δ| ≤ 1e-5 m (the only non-bit-exact step is the device exp()/acos() vs
    glibc: ≤ 1 ulp in the weights, which moves y by far less than one float ulp except rarely);
  * solver Δ and poses: ≤ 1e-6 (Cholesky of JᵀJ vs Householder QR of J: same solution,
    different rounding; the trim ranks are exact).
Full-size (config B) checks use size-independent properties plus exact comparison on a query
subsample (every query is processed independently, so a subsample is an exact check).
"""
import pathlib

import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi, config, imls_icp, synth

pytestmark = pytest.mark.gpu
GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"
Y_TOL = 1e-5
POSE_TOL = 1e-6


def golden(name):
    return dict(np.load(GOLDEN / f"{name}.npz"))


def gparams(iters=10):
    p = config.bench_params(iters)
    p.delta_dist_threshold = 0.001
    p.delta_angle_threshold = 0.0001745353
    return p


def soa_to_rows(soa6):
    return np.ascontiguousarray(np.asarray(soa6, np.float32).T)


@pytest.fixture(scope="module")
def ctx():
    c = imls_icp.ImlsContext(gparams())
    yield c
    c.close()


def check_projection(got, want_idx, want_rej, want_x, want_y, want_n):
    x, y, n, idx, rej = got
    assert np.array_equal(rej, want_rej), (rej, want_rej)
    assert np.array_equal(idx, want_idx)
    assert np.array_equal(x, want_x)
    assert np.array_equal(n, want_n)
    if len(want_idx) == 0:
        return 1.0
    dy = np.abs(y.astype(np.float64) - want_y.astype(np.float64))
    assert dy.max() <= Y_TOL, dy.max()
    return float((dy == 0).all(axis=1).mean())


@pytest.fixture(params=["auto", "0", "1"], ids=["auto", "packets", "wave_per_query"])
def traversal(request, ctx):
    """Both traversal kernels on the same inputs: packets of 64 queries (k_knn_wave) and one wave
    per query (k_knn_qwave), through the option imls_set_option(IMLS_OPT_TRAVERSAL)."""
    ctx.set_option("traversal", {"auto": _abi.IMLS_TRAVERSAL_AUTO, "0": _abi.IMLS_TRAVERSAL_PACKETS,
                                 "1": _abi.IMLS_TRAVERSAL_WAVE_PER_QUERY}[request.param])
    yield request.param
    ctx.set_option("traversal", _abi.IMLS_TRAVERSAL_AUTO)


@pytest.mark.parametrize("name", ["vlp16_pair", "planetary_pair"])
def test_project_matches_golden(ctx, name, traversal):
    g = golden(name)
    p = gparams()
    ctx.set_params(p)
    ctx.set_target(soa_to_rows(g["tgt"]))
    ctx.set_source(soa_to_rows(g["src"]))
    for k in (0, 1):
        exact = check_projection(ctx.project(g[f"pose{k}"]), g[f"idx{k}"], g[f"rej{k}"], g[f"x{k}"], g[f"y{k}"], g[f"n{k}"])
        assert exact > 0.99, exact
        ok, D = ctx.solve()
        assert ok and np.abs(D - g[f"ls{k}"]).max() < POSE_TOL


@pytest.mark.parametrize("name", ["vlp16_pair", "planetary_pair"])
def test_register_frame_matches_golden(ctx, name, traversal):
    g = golden(name)
    ctx.set_params(gparams())
    ctx.set_target(soa_to_rows(g["tgt"]))
    ctx.set_source(soa_to_rows(g["src"]))
    r = ctx.register_frame()
    assert r["iters"] == int(g["frame_iters"]) and r["status"] == int(g["frame_status"])
    assert np.abs(r["pose"] - g["frame_pose"]).max() < POSE_TOL
    nv = np.array([t.n_valid for t in r["trace"]])
    assert np.array_equal(nv, g["frame_nvalid"][: len(nv)])
    for t, d in zip(r["trace"], g["frame_delta"]):
        assert np.abs(np.array(t.delta).reshape(4, 4) - d).max() < POSE_TOL


def test_solve_correspondences_ls_and_wls(ctx):
    g = golden("vlp16_pair")
    s, d, n = (g[k].astype(np.float64) for k in ("x1", "y1", "n1"))
    p = gparams()
    ctx.set_params(p)
    ok, D = ctx.solve_correspondences(_abi.IMLS_SOLVE_LS, s, d, n)
    assert ok and np.abs(D - oc.solve(_abi.IMLS_SOLVE_LS, s, d, n, p)[1]).max() < POSE_TOL
    w = np.random.default_rng(0).uniform(0.1, 1.0, len(s))
    ok, D = ctx.solve_correspondences(_abi.IMLS_SOLVE_WEIGHTED_LS, s, d, n, w)
    assert ok and np.abs(D - oc.solve(_abi.IMLS_SOLVE_WEIGHTED_LS, s, d, n, p, weights=w)[1]).max() < POSE_TOL
    # reference-shaped free functions
    ok, D2 = imls_icp.SolveMotionEstimationProblemLS(s, d, n, "0", 0.02)
    assert ok and np.abs(D2 - oc.solve(_abi.IMLS_SOLVE_LS, s, d, n, p)[1]).max() < POSE_TOL


def test_trim_with_massive_residual_ties(ctx):
    """Exact-data rows: residuals tie massively → the overflow path of the exact rank select."""
    rng = np.random.default_rng(4)
    N = 30000
    s = rng.uniform(-20, 20, (N, 3))
    n = np.zeros((N, 3))
    n[np.arange(N), rng.integers(0, 3, N)] = 1.0
    d = s + np.array([0.25, -0.5, 0.125])            # exactly representable shifts: r = 0 exactly
    p = gparams()
    ctx.set_params(p)
    ok, D = ctx.solve_correspondences(_abi.IMLS_SOLVE_LS, s, d, n)
    okr, Dr = oc.solve(_abi.IMLS_SOLVE_LS, s, d, n, p)
    assert ok and np.abs(D - Dr).max() < 1e-9


@pytest.mark.parametrize("K", [3, 8, 16, 32])
def test_search_number_variants(ctx, K):
    g = golden("vlp16_pair")
    p = gparams()
    p.search_number = K
    ctx.set_params(p)
    ctx.set_target(soa_to_rows(g["tgt"]))
    ctx.set_source(soa_to_rows(g["src"]))
    want = oc.project(g["src"], g["tgt"], g["pose1"], p)
    check_projection(ctx.project(g["pose1"]), want[3], want[4], want[0], want[1], want[2])


@pytest.mark.parametrize("variant", ["angle_off", "transform_normal", "no_get_normals", "h_small", "r_small"])
def test_option_variants(ctx, variant):
    g = golden("vlp16_pair")
    p = gparams()
    if variant == "angle_off":
        p.normal_angle_constraint = 0
    elif variant == "transform_normal":
        p.transform_normal = 1
    elif variant == "no_get_normals":
        p.get_normals = 0                 # Q1: libnabo semantics → every candidate "invalid normal"
    elif variant == "h_small":
        p.h = 0.05
    elif variant == "r_small":
        p.r = 0.3
    ctx.set_params(p)
    ctx.set_target(soa_to_rows(g["tgt"]))
    ctx.set_source(soa_to_rows(g["src"]))
    want = oc.project(g["src"], g["tgt"], g["pose1"], p)
    check_projection(ctx.project(g["pose1"]), want[3], want[4], want[0], want[1], want[2])
    if variant == "no_get_normals":
        assert len(want[3]) == 0


def test_self_match_and_duplicates(ctx):
    """Queries exactly on map points: NN-1 must skip the zero-distance point (no
    ALLOW_SELF_MATCH, imls_icp.cpp:605-607) while the IMLS kNN keeps it (373); duplicated map
    points exercise exact distance ties (broken by index)."""
    g = golden("vlp16_pair")
    tgt = g["tgt"].copy()
    tgt = np.concatenate([tgt, tgt[:, :500]], axis=1)          # 500 exact duplicates
    src = tgt[:, 1000:1600].copy()                              # queries ON map points
    p = gparams()
    ctx.set_params(p)
    ctx.set_target(soa_to_rows(tgt))
    ctx.set_source(soa_to_rows(src))
    want = oc.project(src, tgt, np.eye(4), p)
    check_projection(ctx.project(np.eye(4)), want[3], want[4], want[0], want[1], want[2])


def test_too_few_correspondences_status(ctx):
    g = golden("vlp16_pair")
    src = g["src"].copy()
    src[:3] += 500.0                                             # far from every map point
    ctx.set_params(gparams())
    ctx.set_target(soa_to_rows(g["tgt"]))
    ctx.set_source(soa_to_rows(src))
    r = ctx.register_frame()
    assert r["status"] == _abi.IMLS_FRAME_TOO_FEW and r["iters"] == 0
    assert np.array_equal(r["pose"], np.eye(4))


def test_bad_arguments_and_state():
    c = imls_icp.ImlsContext(gparams())
    with pytest.raises(_abi.ImlsError) as e:
        c.project(np.eye(4))
    assert e.value.status == _abi.IMLS_ERR_STATE
    with pytest.raises(ValueError):
        c.set_target(np.zeros((0, 5), np.float32))
    p = gparams()
    p.search_number = 64
    with pytest.raises(_abi.ImlsError) as e:
        c.set_params(p)
    assert e.value.status == _abi.IMLS_ERR_UNSUPPORTED
    c.close()


# ------------------------------------------------------------------------------------------------
# Full size: SURVEY §8(d) config B (HDL-64 ~120k-pt scan vs 10-scan map ≈ 1.2M points)
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def config_b():
    pair = synth.make_pair("hdl64", map_scans=10)
    return pair


def test_config_b_projection_exact_on_subsample(ctx, config_b):
    src, tgt = config_b.source, config_b.target
    p = config.bench_params(20)
    ctx.set_params(p)
    ctx.set_target(tgt)
    ctx.set_source(src)
    pose = config_b.true_pose @ synth.pose_xyyaw(0.2, -0.1, 0.003)
    x, y, n, idx, rej = ctx.project(pose)
    assert int(rej.sum()) + len(idx) == src.size
    sub = np.random.default_rng(0).choice(src.size, 3000, replace=False)
    sub.sort()
    want = oc.project(synth.soa(src[sub]), synth.soa(tgt), pose, p)
    pos = {int(i): k for k, i in enumerate(idx)}
    got_valid = np.array([int(i) in pos for i in sub])
    want_valid = np.zeros(len(sub), bool)
    want_valid[want[3]] = True
    assert np.array_equal(got_valid, want_valid)
    rows = np.array([pos[int(sub[j])] for j in want[3]])
    assert np.array_equal(x[rows], want[0]) and np.array_equal(n[rows], want[2])
    assert np.abs(y[rows].astype(np.float64) - want[1]).max() <= Y_TOL


def test_config_b_frame_properties(ctx, config_b):
    p = config.bench_params(20)
    p.delta_dist_threshold = 0.001
    p.delta_angle_threshold = 0.0001745353
    ctx.set_params(p)
    ctx.set_target(config_b.target)
    ctx.set_source(config_b.source)
    r1 = ctx.register_frame()
    r2 = ctx.register_frame()
    assert np.array_equal(r1["pose"], r2["pose"])                 # deterministic
    err = np.linalg.norm(r1["pose"][:3, 3] - config_b.true_pose[:3, 3])
    assert err < 0.05, err                                         # recovers the true motion
    last = np.array(r1["trace"][-1].delta).reshape(4, 4)
    dd = np.linalg.norm(last[:3, 3])
    conv = dd < p.delta_dist_threshold and np.arccos(np.clip((np.trace(last[:3, :3]) - 1) / 2, -1, 1)) < p.delta_angle_threshold
    assert conv == (r1["status"] == _abi.IMLS_FRAME_CONVERGED)
    # target-order invariance: permuting the map leaves every projection unchanged
    perm = np.random.default_rng(1).permutation(config_b.target.size)
    ctx.set_target(config_b.target)
    a = ctx.project(r1["pose"])
    ctx.set_target(config_b.target[perm])
    b = ctx.project(r1["pose"])
    assert np.array_equal(a[3], b[3]) and np.array_equal(a[1], b[1])


def test_non_finite_points_are_dropped_like_the_reference(ctx, traversal):
    """RemoveNANandINFData (imls_icp.cpp:58-78, 80-103): points with a non-finite xyz are erased from
    both clouds in place (order kept) before anything else; normals are not checked there (a NaN map
    normal is rejected later as "invalid normal", 672-679)."""
    g = golden("vlp16_pair")
    src, tgt = g["src"].copy(), g["tgt"].copy()
    rng = np.random.default_rng(11)
    for cloud in (src, tgt):
        bad = rng.choice(cloud.shape[1], 40, replace=False)
        cloud[rng.integers(0, 3, 40), bad] = rng.choice([np.nan, np.inf, -np.inf], 40)
    tgt[3:6, rng.choice(tgt.shape[1], 25, replace=False)] = np.nan          # NaN map normals
    p = gparams()
    ctx.set_params(p)
    assert ctx.set_target(soa_to_rows(tgt)) == int(np.isfinite(tgt[:3]).all(axis=0).sum())
    ctx.set_source(soa_to_rows(src))
    pose = g["pose1"]
    want = oc.project(src[:, np.isfinite(src[:3]).all(axis=0)], tgt, pose, p)
    check_projection(ctx.project(pose), want[3], want[4], want[0], want[1], want[2])
    r = ctx.register_frame()
    o = oc.register_frame(src[:, np.isfinite(src[:3]).all(axis=0)], tgt, p)
    assert r["iters"] == o["iters"] and r["status"] == o["status"]
    assert np.abs(r["pose"] - o["pose"]).max() < POSE_TOL
