"""CPU tests of the oracle (test infrastructure): golden vectors, the independent numpy
restatement, glibc rand() itself, and the analytic known-answer tests of SURVEY.md Appendix A.4.
Parity status of the oracle: unpinned (no reference fixtures exist; see oracle/imls_oracle.h)."""
import ctypes
import math
import pathlib

import numpy as np
import pytest

import imls_np
import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi, config, synth

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"


def golden(name):
    return dict(np.load(GOLDEN / f"{name}.npz"))


def gparams(iters=10):
    p = config.bench_params(iters)
    p.delta_dist_threshold = 0.001
    p.delta_angle_threshold = 0.0001745353
    return p


@pytest.mark.parametrize("name", ["vlp16_pair", "planetary_pair"])
def test_oracle_reproduces_golden(name):
    g = golden(name)
    p = gparams()
    for k in (0, 1):
        x, y, n, idx, rej = oc.project(g["src"], g["tgt"], g[f"pose{k}"], p)
        assert np.array_equal(idx, g[f"idx{k}"])
        assert np.array_equal(rej, g[f"rej{k}"])
        assert np.array_equal(x, g[f"x{k}"]) and np.array_equal(y, g[f"y{k}"]) and np.array_equal(n, g[f"n{k}"])
        ok, D = oc.solve(_abi.IMLS_SOLVE_LS, x, y, n, p)
        assert ok and np.abs(D - g[f"ls{k}"]).max() < 1e-12
    fr = oc.register_frame(g["src"], g["tgt"], p)
    assert fr["iters"] == int(g["frame_iters"]) and fr["status"] == int(g["frame_status"])
    assert np.abs(fr["pose"] - g["frame_pose"]).max() < 1e-12


def test_golden_frame_recovers_true_pose():
    g = golden("vlp16_pair")
    err_t = np.linalg.norm(g["frame_pose"][:3, 3] - g["true_pose"][:3, 3])
    assert err_t < 0.1, err_t


def test_nan_points_are_filtered():
    g = golden("vlp16_pair")
    # the golden source carries one NaN x (point 3): dropped (imls_icp.cpp:58-78).  A NaN y
    # drops one more; a NaN NORMAL is not filtered (pcl::isFinite checks xyz only, Q8).
    p = gparams()
    _, _, _, idx_a, rej_a = oc.project(g["src"], g["tgt"], np.eye(4), p)
    assert int(rej_a.sum()) + len(idx_a) == g["src"].shape[1] - 1
    src = g["src"].copy()
    src[1, 5] = np.nan
    _, _, _, idx_b, rej_b = oc.project(src, g["tgt"], np.eye(4), p)
    assert int(rej_b.sum()) + len(idx_b) == g["src"].shape[1] - 2
    src = g["src"].copy()
    src[4, 5] = np.nan
    _, _, _, idx_c, rej_c = oc.project(src, g["tgt"], np.eye(4), p)
    assert int(rej_c.sum()) + len(idx_c) == g["src"].shape[1] - 1


def test_glibc_rand_restatement_matches_libc():
    libc = ctypes.CDLL("libc.so.6")
    for seed in (1, 12345, 2**31 + 7):
        libc.srand(ctypes.c_uint(seed))
        want = [libc.rand() for _ in range(500)]
        got = oc.rand_sequence(seed, 500)
        assert list(got) == want


def test_exact_knn_matches_bruteforce():
    rng = np.random.default_rng(3)
    tgt = np.zeros((6, 3000), np.float32)
    tgt[:3] = rng.uniform(-5, 5, (3, 3000))
    tgt[5] = 1
    q = rng.uniform(-5, 5, (3, 200)).astype(np.float32)
    q[:, 0] = tgt[:3, 17]            # exact duplicate: self-match semantics
    for allow in (0, 1):
        d2, idx = oc.knn(tgt, q, 20, 1.5, allow)
        for j in range(q.shape[1]):
            d = imls_np.exact_d2(q[:, j].astype(np.float64), tgt[:3].T)
            m = d <= 1.5 * 1.5
            if not allow:
                m &= d > np.finfo(np.float64).eps
            cand = np.nonzero(m)[0]
            order = cand[np.lexsort((cand, d[cand]))][:20]
            assert np.array_equal(idx[j, :len(order)], order)
            assert np.all(idx[j, len(order):] == -1) and np.all(np.isinf(d2[j, len(order):]))
            assert np.array_equal(d2[j, :len(order)], d[order])
    d2, idx = oc.knn(tgt, q[:, :1], 1, 1.5, 0)
    assert idx[0, 0] != 17           # NN-1 without ALLOW_SELF_MATCH skips the zero-distance point


# ------------------------------------------------------------------------------------------------
# Analytic known-answer tests
# ------------------------------------------------------------------------------------------------
def plane_map(spacing=0.1, half=3.0, seed=0):
    rng = np.random.default_rng(seed)
    g = np.arange(-half, half + 1e-9, spacing)
    X, Y = np.meshgrid(g, g)
    X = X + rng.uniform(-0.01, 0.01, X.shape)
    Y = Y + rng.uniform(-0.01, 0.01, Y.shape)
    n = X.size
    t = np.zeros((6, n), np.float32)
    t[0], t[1], t[5] = X.ravel(), Y.ravel(), 1.0
    return t


def src_points(pts, normals=None):
    pts = np.atleast_2d(np.asarray(pts, np.float32))
    s = np.zeros((6, len(pts)), np.float32)
    s[:3] = pts.T
    s[3:] = (np.asarray(normals, np.float32).T if normals is not None else np.array([[0], [0], [1]], np.float32))
    return s


def test_kat_plane_height():
    tgt = plane_map()
    p = gparams()
    z0 = 0.35
    x, y, n, idx, rej = oc.project(src_points([[0.123, -0.07, z0]]), tgt, np.eye(4), p)
    assert len(idx) == 1
    # height = z0·Σw/(Σw+1e-5) ⇒ y_z = z0 − height = z0·1e-5/(Σw+1e-5)
    q = np.array([0.123, -0.07, z0], np.float32).astype(np.float64)
    d = imls_np.exact_d2(q, tgt[:3].T)
    order = np.lexsort((np.arange(d.size), d))[:20]
    hmax = math.sqrt(d[order[19]]) / 3
    w = np.exp(-d[order] / hmax / hmax)
    height = float(np.sum(w * z0)) / (float(np.sum(w)) + 1e-5)
    assert abs(float(y[0, 2]) - np.float32(z0 - height)) <= 1e-7
    assert abs(float(y[0, 2]) - z0 * 1e-5 / (float(np.sum(w)) + 1e-5)) <= 1e-7   # the Q4 bias, analytically


def test_kat_pure_translation_ls():
    rng = np.random.default_rng(5)
    t = np.array([0.31, -0.12, 0.05])
    s, n = [], []
    for axis in range(3):
        for _ in range(40):
            pnt = rng.uniform(-10, 10, 3)
            nv = np.zeros(3)
            nv[axis] = 1
            s.append(pnt)
            n.append(nv)
    s, n = np.array(s), np.array(n)
    d = s + t
    p = gparams()
    ok, D = oc.solve(_abi.IMLS_SOLVE_LS, s, d, n, p)
    assert ok
    assert np.abs(D[:3, 3] - t).max() < 1e-12
    assert np.abs(D[:3, :3] - np.eye(3)).max() < 1e-12


@pytest.mark.parametrize("N,kept", [(6, 6), (7, 7), (50, 49), (51, 49), (100, 97)])
def test_kat_trimmed_ls_rank_bounds(N, kept):
    lo, hi = int(0.02 * N), min(int((1 - 0.02) * N), N - 1)
    assert hi - lo + 1 == kept
    rng = np.random.default_rng(N)
    s = rng.uniform(-5, 5, (N, 3))
    n = rng.normal(size=(N, 3))
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    d = s + 0.05 * rng.normal(size=(N, 3))
    ok, D = oc.solve(_abi.IMLS_SOLVE_LS, s, d, n, gparams())
    D2, k2 = imls_np.solve_ls(s, d, n, 0.02)
    assert ok and k2 == kept
    assert np.abs(D - D2).max() < 1e-9


def test_kat_gates_nn_distance():
    p = gparams()
    # map: three points on z = 0 plus the NN candidate; h = 1 → d² = h² passes, just above fails
    base = np.zeros((6, 4), np.float32)
    base[5] = 1
    for eps, expect_valid in ((0.0, True), (1e-6, False)):
        t = base.copy()
        t[0] = [1.0 + eps, 1.5 + eps, 1.6, 1.7]
        t[1] = [0.0, 0.4, -0.4, 0.0]
        x, y, n, idx, rej = oc.project(src_points([[0, 0, 0]]), t, np.eye(4), p)
        assert (len(idx) == 1) == expect_valid, (eps, rej)
        if not expect_valid:
            assert rej[_abi.REJECT_NAMES.index("too_far")] == 1


def test_kat_gates_angle_and_mls_count():
    p = gparams()
    t = np.zeros((6, 3), np.float32)
    t[0] = [0.1, 0.2, -0.15]
    t[1] = [0.0, 0.1, 0.12]

    def with_angle(deg):
        a = math.radians(deg)
        tt = t.copy()
        tt[3], tt[5] = math.sin(a), math.cos(a)
        return tt

    _, _, _, idx, rej = oc.project(src_points([[0, 0, 0.05]]), with_angle(29.9), np.eye(4), p)
    assert len(idx) == 1
    _, _, _, idx, rej = oc.project(src_points([[0, 0, 0.05]]), with_angle(30.1), np.eye(4), p)
    assert len(idx) == 0 and rej[_abi.REJECT_NAMES.index("normal_constraint")] == 1
    # |S| = 2 → MLS failure
    _, _, _, idx, rej = oc.project(src_points([[0, 0, 0.05]]), t[:, :2].copy(), np.eye(4), p)
    assert len(idx) == 0 and rej[_abi.REJECT_NAMES.index("mls_fail")] == 1


def test_kat_hmax_quirk_indexes_sorted_list():
    """Q3: h_max = √L[|S|−1]/3 uses the sorted candidate list, not the accepted set."""
    p = gparams()
    t = np.zeros((6, 5), np.float32)
    t[0] = [0.1, 0.2, 0.3, 0.4, 0.5]
    t[5] = 1.0
    # the second-nearest point's normal violates the angle gate → S = {0, 2, 3, 4}
    t[3, 1], t[5, 1] = 1.0, 0.0
    q = np.array([0.0, 0.0, 0.02], np.float32)
    x, y, n, idx, rej = oc.project(src_points([q]), t, np.eye(4), p)
    assert len(idx) == 1
    qd = q.astype(np.float64)
    d = imls_np.exact_d2(qd, t[:3].T)
    hmax = math.sqrt(d[3]) / 3              # L[|S|−1] = L[3] (not the 4th accepted, which is L[4])
    S = [0, 2, 3, 4]
    w = np.exp(-d[S] / hmax / hmax)
    height = float(np.sum(w * qd[2])) / (float(np.sum(w)) + 1e-5)
    assert float(y[0, 2]) == np.float32(qd[2] - height)


def test_colpiv_qr_basic_solution_3x6():
    rng = np.random.default_rng(11)
    A = rng.normal(size=(3, 6))
    b = rng.normal(size=3)
    x = oc.colpiv_qr_solve(A, b)
    assert np.abs(A @ x - b).max() < 1e-12
    assert np.count_nonzero(x) == 3          # basic solution: non-pivot unknowns are zero
    # full-rank overdetermined: equals the least-squares solution
    A = rng.normal(size=(40, 6))
    b = rng.normal(size=40)
    x = oc.colpiv_qr_solve(A, b)
    assert np.abs(x - np.linalg.lstsq(A, b, rcond=None)[0]).max() < 1e-12


def test_delta_from_x_is_rodrigues():
    from scipy.spatial.transform import Rotation
    for x in ([0, 0, 0, 1, 2, 3], [0.01, -0.02, 0.3, 0, 0, 0], [1.0, 0.5, -0.25, 0.1, 0.1, 0.1]):
        D = oc.delta_from_x(np.array(x, float))
        assert np.abs(D[:3, :3] - Rotation.from_rotvec(x[:3]).as_matrix()).max() < 1e-14
        assert np.array_equal(D[:3, 3], np.array(x[3:], float))


def test_ransac_variants_run_and_are_deterministic():
    g = golden("vlp16_pair")
    s, d, n = g["x1"], g["y1"], g["n1"]
    p = gparams()
    for final in (_abi.IMLS_FINAL_LS, _abi.IMLS_FINAL_WEIGHTED_LS, _abi.IMLS_FINAL_DRPM):
        p.ransac_final_method = final
        ok1, D1 = oc.solve(_abi.IMLS_SOLVE_RANSAC, s, d, n, p)
        ok2, D2 = oc.solve(_abi.IMLS_SOLVE_RANSAC, s, d, n, p)
        okl, DL = oc.solve(_abi.IMLS_SOLVE_LS, s, d, n, p)
        assert ok1 and ok2 and np.array_equal(D1, D2)
        assert np.abs(D1[:3, 3] - DL[:3, 3]).max() < 0.05


def test_weighted_ls_matches_numpy():
    g = golden("vlp16_pair")
    s, d, n = g["x0"].astype(np.float64), g["y0"].astype(np.float64), g["n0"].astype(np.float64)
    w = np.random.default_rng(2).uniform(0.1, 1.0, len(s))
    ok, D = oc.solve(_abi.IMLS_SOLVE_WEIGHTED_LS, s, d, n, gparams(), weights=w)
    assert ok and np.abs(D - imls_np.solve_wls(s, d, n, w)).max() < 1e-9


def picp_dict(p):
    return dict(picp_r=p.picp_r, picp_normal_angle_constraint=p.picp_normal_angle_constraint,
                picp_angle_diff_threshold=p.picp_angle_diff_threshold)


@pytest.mark.parametrize("name", ["vlp16_pair", "planetary_pair"])
@pytest.mark.parametrize("angle", [0, 1])
def test_plane_icp_restatements_agree(name, angle):
    """plane_ICP_proj (laser_odometry.cpp:277-413): C++ oracle vs numpy restatement, bit-exact."""
    g = golden(name)
    p = gparams()
    p.matching_method = _abi.IMLS_MATCH_PLANE_ICP
    p.picp_normal_angle_constraint = angle
    for k in (0, 1):
        x, y, n, idx, rej = oc.project(g["src"], g["tgt"], g[f"pose{k}"], p)
        x2, y2, n2, idx2, rej2 = imls_np.project_plane_icp(g["src"], g["tgt"], g[f"pose{k}"], picp_dict(p))
        assert np.array_equal(rej, rej2) and np.array_equal(idx, idx2)
        assert np.array_equal(x, x2) and np.array_equal(y, y2) and np.array_equal(n, n2)
        assert rej[4] == 0 and rej[5] == 0 and len(idx) > 0.5 * g["src"].shape[1]


def test_plane_icp_kat():
    """Analytic: a query above a z=0 plane projects straight down onto it; beyond picp.r it is
    "no normal" (the reference's bounds check, not "too far"); the h gate does not apply."""
    rng = np.random.default_rng(5)
    m = 4000
    tgt = np.zeros((6, m), np.float32)
    tgt[0] = rng.uniform(-5, 5, m); tgt[1] = rng.uniform(-5, 5, m); tgt[5] = 1.0
    src = np.zeros((6, 3), np.float32)
    src[:3, 0] = (0.3, -0.2, 1.2)     # within picp.r = 1.5 of the plane but beyond h = 1: accepted
    src[:3, 1] = (0.1, 0.4, 0.25)
    src[:3, 2] = (0.0, 0.0, 3.0)      # nothing within 1.5 → no normal
    src[5] = 1.0
    p = gparams()
    p.matching_method = _abi.IMLS_MATCH_PLANE_ICP
    x, y, n, idx, rej = oc.project(src, tgt, np.eye(4), p)
    assert list(idx) == [0, 1] and rej[0] == 1 and rej.sum() == 1
    assert np.allclose(y[:, 2], 0.0, atol=1e-7) and np.allclose(y[:, :2], x[:, :2], atol=1e-7)


# ---- tensor voting (libpointmatcher decompose semantics unpinned) ----------
def tv_params(count_mode=1, k=50, sigma=0.2, thr=0.6):
    p = gparams()
    p.get_normals = 0
    p.recompute_normal_count_mode = count_mode
    p.use_tensor_voting = 1
    p.tensor_k, p.tensor_sigma, p.tensor_distance_threshold = k, sigma, thr
    return p


def test_tv_oracle_reproduces_golden():
    g = golden("tv_pair")
    p = tv_params()
    for k in (0, 1):
        nrm, found, _ = oc.tv_normals(g["tgt"], g["ten"], g[f"tvq{k}"], p)
        assert np.array_equal(found, g[f"tvf{k}"]) and np.array_equal(nrm, g[f"tvn{k}"])
        x, y, n, idx, rej = oc.project(g["src"], g["tgt"], g[f"pose{k}"], p, tensors=g["ten"])
        assert np.array_equal(idx, g[f"idx{k}"]) and np.array_equal(rej, g[f"rej{k}"])
        assert np.array_equal(x, g[f"x{k}"]) and np.array_equal(y, g[f"y{k}"]) and np.array_equal(n, g[f"n{k}"])
    fr = oc.register_frame(g["src"], g["tgt"], p, tensors=g["ten"])
    assert fr["iters"] == int(g["frame_iters"]) and fr["status"] == int(g["frame_status"])
    assert np.abs(fr["pose"] - g["frame_pose"]).max() < 1e-12


@pytest.mark.parametrize("k,sigma,thr", [(8, 0.5, 0.6), (64, 0.4, 1.0), (20, 1.0, 0.3)])
def test_tv_restatements_agree(k, sigma, thr):
    """C++ oracle vs the independent numpy restatement (cKDTree candidates, numpy products,
    LAPACK eigh on the lower triangle), incl. the k-cut of large voting balls."""
    g = golden("tv_pair")
    p = tv_params(k=k, sigma=sigma, thr=thr)
    q = g["tvq1"][:, ::10]
    nrm, found, acc = oc.tv_normals(g["tgt"], g["ten"], q, p)
    nrm2, found2, acc2 = imls_np.tv_normals(g["tgt"], g["ten"], q, dict(tensor_k=k, tensor_sigma=sigma,
                                                                          tensor_distance_threshold=thr))
    assert np.array_equal(found, found2) and found.sum() > 10
    assert np.abs(acc - acc2).max() <= 1e-15 * max(1.0, np.abs(acc).max()) * 10
    assert np.abs(nrm - nrm2).max() <= 1e-10


def test_tv_kat_plane_normal():
    """Known answer: voters on the plane z = 0 whose tensors span the plane (the PCA encoding of
    a flat patch: e1, e2 in-plane) vote into a point of the plane: every r̂ is in-plane, so R and
    R' fix ẑ, the summed tensor has a zero z row/column and its smallest-|λ| eigenvector is ẑ."""
    rng = np.random.default_rng(3)
    M = 400
    tgt = np.zeros((6, M), np.float32)
    tgt[0], tgt[1] = rng.uniform(-0.3, 0.3, M), rng.uniform(-0.3, 0.3, M)
    ev = np.tile(np.array([[0.02, 0.01, 1e-5]], np.float32), (M, 1))
    evecs = np.tile(np.array([[1, 0, 0, 0, 1, 0, 0, 0, 1]], np.float32), (M, 1))
    ten = imls_np.tv_encode_pca(ev, evecs, 50).T
    q = np.array([[0.01], [0.02], [0.0]], np.float32)
    p = tv_params(sigma=0.2, thr=0.6)
    nrm, found, _ = oc.tv_normals(tgt, ten, q, p)
    assert found[0] == 1 and abs(nrm[0, 2] - 1.0) < 1e-12
    far = np.array([[5.0], [5.0], [5.0]], np.float32)       # no voter within thr·σ → zero tensor
    _, found, _ = oc.tv_normals(tgt, ten, far, p)
    assert found[0] == 0


def test_tv_encode_pca_host_helper_matches_restatement():
    """imls_tv_encode_pca (product host helper, scan_registration.cpp:358-381) is pure host float
    arithmetic: bit-identical to the numpy restatement; the unit-ball branch for non-ordered λ."""
    from planetary_lidar_odometry_amd import imls_icp
    g = golden("tv_pair")
    ev, ec = g["evals"], g["evecs"]
    assert np.array_equal(imls_icp.tv_encode_pca(ev, ec, 50), imls_np.tv_encode_pca(ev, ec, 50))
    bad = np.array([[np.nan, 1.0, 0.5]], np.float32)
    assert np.array_equal(imls_icp.tv_encode_pca(bad, ec[:1], 50)[0], np.array([1, 0, 0, 1, 0, 1], np.float32))


def test_threaded_oracle_matches_single_thread():
    """The all-cores CPU baseline (OpenMP over queries) returns the single-thread result exactly."""
    from planetary_lidar_odometry_amd import config, synth
    pair = synth.make_pair("vlp16", map_scans=1, start=5)
    src, tgt = synth.soa(pair.source), synth.soa(pair.target)
    p = config.bench_params(3)
    a = oc.register_frame(src, tgt, p)
    oc.set_threads(4)
    try:
        b = oc.register_frame(src, tgt, p)
    finally:
        oc.set_threads(1)
    assert np.array_equal(a["pose"], b["pose"]) and a["iters"] == b["iters"]
    assert [list(t.reject) for t in a["trace"]] == [list(t.reject) for t in b["trace"]]


def _rot(axis, ang):
    a = np.asarray(axis, float) / np.linalg.norm(axis)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + math.sin(ang) * K + (1 - math.cos(ang)) * K @ K


def test_pose_line_and_chain_match_oracle():
    """savePoseToFile (saver.cpp:46-54) and nowPose = prevLaserPose·rPose (laser_odometry.cpp:652):
    the Python product path and the oracle print byte-identical lines, including the quaternion
    branches taken when trace(R) <= 0 (rotations near π about each axis)."""
    from planetary_lidar_odometry_amd import imls_icp
    rng = np.random.default_rng(7)
    poses = [np.eye(4)]
    for axis in ([1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 1, 0], [0.3, -1, 2]):
        for ang in (1e-9, 0.3, 2.0, math.pi - 1e-3, math.pi):
            P = np.eye(4)
            P[:3, :3] = _rot(axis, ang)
            P[:3, 3] = rng.normal(scale=50, size=3)
            poses.append(P)
    for k, P in enumerate(poses):
        ts = f"{1317384506.0 + 0.1 * k:f}"
        assert imls_icp.format_pose_line(P, ts) == oc.format_pose(P, ts), (k, P)
    prev = np.eye(4)
    for P in poses:
        a = imls_icp.chain_pose(prev, P)
        assert np.array_equal(a, oc.chain_pose(prev, P))
        prev = a


def test_oracle_rand_state_carries_across_frames():
    """A frame with a carried rand() state continues the stream: two RANSAC frames with one carried
    state equal (frame 1 fresh, frame 2 from frame 1's final state), and the state advanced."""
    g = golden("vlp16_pair")
    p = config.params_from_config(config.load())      # shipped: RANSAC -> DRPM
    p.iterations = 2
    st = oc.rand_state(p.ransac_seed)
    st0 = st.copy()
    a = oc.register_frame(g["src"], g["tgt"], p, rand_state=st)
    assert not np.array_equal(st, st0)
    fresh = oc.register_frame(g["src"], g["tgt"], p)
    assert np.array_equal(a["pose"], fresh["pose"])   # first frame: the stream starts at the seed either way


def test_faithful_baseline_mode_is_identical():
    """bench.py's "faithful" CPU baseline (the reference's erase-per-rejection loop, AoS copies and
    per-query allocations) computes exactly what the efficient oracle computes."""
    g = golden("vlp16_pair")
    p = gparams(6)
    a = oc.register_frame(g["src"], g["tgt"], p)
    oc.set_faithful(True)
    try:
        b = oc.register_frame(g["src"], g["tgt"], p)
        x, y, n, idx, rej = oc.project(g["src"], g["tgt"], g["pose1"], p)
    finally:
        oc.set_faithful(False)
    assert np.array_equal(a["pose"], b["pose"]) and a["iters"] == b["iters"]
    assert np.array_equal(idx, g["idx1"]) and np.array_equal(rej, g["rej1"]) and np.array_equal(y, g["y1"])
