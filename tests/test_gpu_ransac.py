"""GPU parity of the RANSAC solve path (solver.cpp:222-385 + common.cpp:19-82 FPS) with its three
final methods LS / Weighted LS / DRPM (solver.cpp:486-603, degeneracy.h:14-131), against the
oracle's restatement on identical inputs and the same glibc rand() seed.

Tolerances: hypothesis selection and inlier sets are integer decisions and must match exactly
(checked through Δ, which would differ by far more than the tolerance otherwise); Δ ≤ 1e-6 as for
the LS path (normal equations on the device vs Householder QR in the oracle), 1e-5 for DRPM (its
probabilities go through erfc, whose device and glibc versions differ in the last ulps).
"""
import pathlib

import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi, config, imls_icp

pytestmark = pytest.mark.gpu
GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"
POSE_TOL = 1e-6
DRPM_TOL = 1e-5
FINALS = {"LS": _abi.IMLS_FINAL_LS, "WLS": _abi.IMLS_FINAL_WEIGHTED_LS, "DRPM": _abi.IMLS_FINAL_DRPM}


def golden(name):
    return dict(np.load(GOLDEN / f"{name}.npz"))


def soa_to_rows(soa6):
    return np.ascontiguousarray(np.asarray(soa6, np.float32).T)


def shipped_params(iters=10, final="DRPM"):
    """The shipped config.json (RANSAC → DRPM) with the chosen final method."""
    p = config.params_from_config(config.load())
    p.iterations = iters
    p.solve_method = _abi.IMLS_SOLVE_RANSAC
    p.ransac_final_method = FINALS[final]
    return p


@pytest.fixture(scope="module")
def ctx():
    c = imls_icp.ImlsContext(shipped_params())
    yield c
    c.close()


def outlier_set(n=4000, frac=0.3, seed=7):
    """Correspondences of a known motion on three plane families, `frac` of them corrupted."""
    rng = np.random.default_rng(seed)
    s = rng.uniform(-15, 15, (n, 3))
    nrm = np.zeros((n, 3))
    nrm[np.arange(n), rng.integers(0, 3, n)] = 1.0
    nrm += rng.normal(0, 0.05, (n, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    a = 0.02
    R = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    d = s @ R.T + np.array([0.3, -0.1, 0.05])
    bad = rng.random(n) < frac
    d[bad] += rng.normal(0, 2.0, (bad.sum(), 3))
    return s, d, nrm


@pytest.mark.parametrize("final", ["LS", "WLS", "DRPM"])
def test_ransac_golden_correspondences(ctx, final):
    g = golden("vlp16_pair")
    s, d, n = (g[k].astype(np.float64) for k in ("x1", "y1", "n1"))
    p = shipped_params(final=final)
    ctx.set_params(p)
    ctx.seed_rng(p.ransac_seed)        # restart the stream: the oracle call starts a fresh one
    ok, D = ctx.solve_correspondences(_abi.IMLS_SOLVE_RANSAC, s, d, n)
    okr, Dr = oc.solve(_abi.IMLS_SOLVE_RANSAC, s, d, n, p)
    assert ok == okr
    assert np.abs(D - Dr).max() < (DRPM_TOL if final == "DRPM" else POSE_TOL)


@pytest.mark.parametrize("final", ["LS", "WLS", "DRPM"])
@pytest.mark.parametrize("pct,iters", [(0.99, 300), (0.75, 5000), (0.5, 40)])
def test_ransac_hypothesis_chunks(ctx, final, pct, iters):
    """Outliers make the early exit late or never: many chunks, the rand() replay across chunks,
    the strict-> first-best choice and the exact draw commit all show in Δ."""
    s, d, n = outlier_set()
    p = shipped_params(final=final)
    p.ransac_min_inliers_percentage = pct
    p.ransac_max_iterations = iters
    ctx.set_params(p)
    ctx.seed_rng(p.ransac_seed)        # restart the stream: the oracle call starts a fresh one
    ok, D = ctx.solve_correspondences(_abi.IMLS_SOLVE_RANSAC, s, d, n)
    okr, Dr = oc.solve(_abi.IMLS_SOLVE_RANSAC, s, d, n, p)
    assert ok == okr
    assert np.abs(D - Dr).max() < (DRPM_TOL if final == "DRPM" else POSE_TOL)


def test_ransac_seed_changes_result(ctx):
    s, d, n = outlier_set(frac=0.45, seed=3)
    out = []
    for seed in (1, 2):
        p = shipped_params(final="LS")
        p.ransac_min_inliers_percentage = 0.99
        p.ransac_max_iterations = 8
        p.ransac_seed = seed
        ctx.set_params(p)
        ctx.seed_rng(p.ransac_seed)
        ok, D = ctx.solve_correspondences(_abi.IMLS_SOLVE_RANSAC, s, d, n)
        okr, Dr = oc.solve(_abi.IMLS_SOLVE_RANSAC, s, d, n, p)
        assert np.abs(D - Dr).max() < POSE_TOL
        out.append(D)
    assert np.abs(out[0] - out[1]).max() > 0   # different draws, different hypotheses


def test_drpm_degenerate_plane(ctx):
    """All correspondences on one plane: H is rank-deficient, min probability < threshold → the
    SNR-weighted branch of SolveWithSnrProbabilities."""
    rng = np.random.default_rng(11)
    n_pts = 3000
    s = np.column_stack([rng.uniform(-10, 10, n_pts), rng.uniform(-10, 10, n_pts), rng.normal(0, 0.01, n_pts)])
    nrm = np.tile([0.0, 0.0, 1.0], (n_pts, 1)) + rng.normal(0, 0.02, (n_pts, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    d = s + np.array([0.2, 0.1, 0.05])
    p = shipped_params(final="DRPM")
    ctx.set_params(p)
    ctx.seed_rng(p.ransac_seed)        # restart the stream: the oracle call starts a fresh one
    ok, D = ctx.solve_correspondences(_abi.IMLS_SOLVE_RANSAC, s, d, nrm)
    okr, Dr = oc.solve(_abi.IMLS_SOLVE_RANSAC, s, d, nrm, p)
    assert ok == okr and np.abs(D - Dr).max() < DRPM_TOL


@pytest.mark.parametrize("name", ["vlp16_pair", "planetary_pair"])
@pytest.mark.parametrize("final", ["LS", "DRPM"])
def test_register_frame_shipped_ransac(ctx, name, final):
    """The shipped solve configuration end to end: every ICP iteration's RANSAC on device."""
    g = golden(name)
    p = shipped_params(iters=8, final=final)
    ctx.set_params(p)
    ctx.seed_rng(p.ransac_seed)        # restart the stream: the oracle call starts a fresh one
    ctx.set_target(soa_to_rows(g["tgt"]))
    ctx.set_source(soa_to_rows(g["src"]))
    r = ctx.register_frame()
    want = oc.register_frame(g["src"], g["tgt"], p)
    tol = DRPM_TOL if final == "DRPM" else POSE_TOL
    assert r["iters"] == want["iters"] and r["status"] == want["status"]
    assert np.abs(r["pose"] - want["pose"]).max() < tol
    for t, u in zip(r["trace"], want["trace"]):
        assert t.n_valid == u.n_valid
        assert np.abs(np.array(t.delta) - np.array(u.delta)).max() < tol


def test_rand_stream_runs_on_across_solves(ctx):
    """the reference never calls srand, so its second RANSAC call draws where the first
    stopped.  Two consecutive stand-alone solves on one context equal two oracle solves sharing one
    carried glibc state; a third after imls_seed_rng equals a fresh oracle solve."""
    s, d, n = outlier_set(frac=0.35, seed=5)
    p = shipped_params(final="LS")
    p.ransac_min_inliers_percentage = 0.99
    p.ransac_max_iterations = 24
    ctx.set_params(p)
    ctx.seed_rng(p.ransac_seed)
    st = oc.rand_state(p.ransac_seed)
    got, want = [], []
    for _ in range(2):
        got.append(ctx.solve_correspondences(_abi.IMLS_SOLVE_RANSAC, s, d, n)[1])
        want.append(oc.solve(_abi.IMLS_SOLVE_RANSAC, s, d, n, p, rand_state=st)[1])
    for a, b in zip(got, want):
        assert np.abs(a - b).max() < POSE_TOL
    assert np.abs(got[0] - got[1]).max() > 0            # the second solve drew other hypotheses
    assert np.array_equal(ctx.rng_state(), st)           # device state == the carried glibc state
    ctx.seed_rng(p.ransac_seed)
    D = ctx.solve_correspondences(_abi.IMLS_SOLVE_RANSAC, s, d, n)[1]
    assert np.abs(D - want[0]).max() < POSE_TOL
    ctx.set_rng_state(st)                                # hand the stream over
    assert np.array_equal(ctx.rng_state(), st)


def test_rand_stream_runs_on_across_frames(ctx):
    """Two consecutive fused frames on one context continue one stream, like the oracle with a
    carried state (the second frame differs from a fresh-stream frame)."""
    g = golden("vlp16_pair")
    p = shipped_params(iters=4, final="LS")
    p.ransac_min_inliers_percentage = 0.999             # no early exit: every frame draws many
    p.ransac_max_iterations = 40
    ctx.set_params(p)
    ctx.seed_rng(p.ransac_seed)
    ctx.set_target(soa_to_rows(g["tgt"]))
    ctx.set_source(soa_to_rows(g["src"]))
    st = oc.rand_state(p.ransac_seed)
    for _ in range(2):
        r = ctx.register_frame()
        want = oc.register_frame(g["src"], g["tgt"], p, rand_state=st)
        assert r["iters"] == want["iters"] and r["status"] == want["status"]
        assert np.abs(r["pose"] - want["pose"]).max() < POSE_TOL
    assert np.array_equal(ctx.rng_state(), st)


def test_standalone_drpm_matches_oracle(ctx):
    """SolveMotionEstimationProblemDRPM (solver.cpp:499-603) on caller rows + weights (RANSAC's
    final step as a free function), well-conditioned and degenerate-plane inputs, unit weights too."""
    rng = np.random.default_rng(21)
    s, d, n = outlier_set(n=2500, frac=0.0, seed=9)
    w = rng.uniform(0.1, 1.0, len(s))
    w /= w.sum()
    p = shipped_params(final="DRPM")
    ctx.set_params(p)
    for weights in (w, None):
        ok, D = ctx.solve_correspondences(_abi.IMLS_SOLVE_DRPM, s, d, n, weights)
        okr, Dr = oc.solve(_abi.IMLS_SOLVE_DRPM, s, d, n, p, weights=weights)
        assert ok and okr and np.abs(D - Dr).max() < DRPM_TOL
    sp = np.column_stack([rng.uniform(-10, 10, 2000), rng.uniform(-10, 10, 2000), rng.normal(0, 0.01, 2000)])
    nn = np.tile([0.0, 0.0, 1.0], (2000, 1)) + rng.normal(0, 0.02, (2000, 3))
    nn /= np.linalg.norm(nn, axis=1, keepdims=True)
    ok, D = ctx.solve_correspondences(_abi.IMLS_SOLVE_DRPM, sp, sp + [0.2, 0.1, 0.05], nn, np.full(2000, 1 / 2000))
    okr, Dr = oc.solve(_abi.IMLS_SOLVE_DRPM, sp, sp + [0.2, 0.1, 0.05], nn, p, weights=np.full(2000, 1 / 2000))
    assert ok == okr and np.abs(D - Dr).max() < DRPM_TOL
    ok, _ = ctx.solve_correspondences(_abi.IMLS_SOLVE_DRPM, s[:0], d[:0], n[:0], w[:0])
    assert not ok                                       # no rows: false, like the oracle
