"""Independent numpy/scipy restatement of the reference IMLS-ICP path.  TEST INFRASTRUCTURE ONLY.

Second, independent restatement used to pin the C++ oracle (oracle/imls_oracle.cpp): it shares
no code with it — exact kNN comes from scipy's cKDTree (candidates re-ranked by the exact
libnabo metric), least squares from numpy's SVD-based lstsq instead of Householder QR, and
the rotation from scipy's Rotation.from_rotvec instead of the AngleAxis restatement.

PARITY STATUS: parity unpinned (see oracle/imls_oracle.h) — the reference cannot be built or
run here and has no fixtures; agreement of the two restatements plus analytic known-answer
tests is the pin.

Only for small inputs: the per-query logic is a Python loop.
"""
from __future__ import annotations

import math

import numpy as np
from scipy.spatial import cKDTree
from scipy.spatial.transform import Rotation

DBL_EPS = np.finfo(np.float64).eps
REJ_NO_NORMAL, REJ_TOO_FAR, REJ_INVALID_NORMAL, REJ_NORMAL_CONSTRAINT, REJ_MLS_FAIL, REJ_NAN_INF = range(6)


def filter_finite(soa6: np.ndarray) -> np.ndarray:
    """RemoveNANandINFData (imls_icp.cpp:58-72): keep points with finite xyz, in order."""
    keep = np.isfinite(soa6[:3]).all(axis=0)
    return soa6[:, keep]


def exact_d2(q: np.ndarray, P: np.ndarray) -> np.ndarray:
    """libnabo's squared distance, ((dx²+dy²)+dz²) in double from float-valued coordinates."""
    d = q[None, :].astype(np.float64) - P.astype(np.float64)
    return (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]


class ExactKnn:
    """knn(query, K, maxRadius, allowSelfMatch) with libnabo semantics (imls_icp.cpp:372, 605):
    d² ≤ r² inclusive, SORT_RESULTS, self-match (d² ≤ DBL_EPSILON) excluded unless allowed,
    ties broken by index."""

    def __init__(self, pts3: np.ndarray):
        self.P = pts3.T.astype(np.float64)          # (M, 3)
        self.tree = cKDTree(self.P) if len(self.P) else None

    def query(self, q: np.ndarray, K: int, r: float, allow_self: bool):
        if self.tree is None:
            return np.full(K, np.inf), np.full(K, -1)
        r2 = r * r
        extra = 8
        while True:
            kk = min(K + extra, len(self.P))
            _, ii = self.tree.query(q, k=kk, distance_upper_bound=r * (1 + 1e-9) + 1e-12)
            ii = np.atleast_1d(ii)
            ii = ii[ii < len(self.P)]
            d2 = exact_d2(q, self.P[ii]) if ii.size else np.zeros(0)
            m = d2 <= r2
            if not allow_self:
                m &= d2 > DBL_EPS
            d2, ii2 = d2[m], ii[m]
            order = np.lexsort((ii2, d2))
            d2, ii2 = d2[order], ii2[order]
            if len(d2) >= K or kk >= len(self.P) or ii.size < kk:
                break
            extra *= 4
        out_d = np.full(K, np.inf)
        out_i = np.full(K, -1, dtype=np.int64)
        n = min(K, len(d2))
        out_d[:n] = d2[:n]
        out_i[:n] = ii2[:n]
        return out_d, out_i


def _angle_reject(ns, nn, thr):
    # imls_icp.cpp:442-451 / 681-692; NaN passes (Q8)
    dot = (ns[0] * nn[0] + ns[1] * nn[1]) + ns[2] * nn[2]
    n1 = math.sqrt((ns[0] ** 2 + ns[1] ** 2) + ns[2] ** 2)
    n2 = math.sqrt((nn[0] ** 2 + nn[1] ** 2) + nn[2] ** 2)
    with np.errstate(all="ignore"):
        ca = dot / (n1 * n2) if n1 * n2 != 0 else float("nan")
        ang = math.degrees(math.acos(ca)) if -1.0 <= ca <= 1.0 else float("nan")
    return ang > thr


def project(src6: np.ndarray, tgt6: np.ndarray, pose: np.ndarray, p: dict):
    """ProjSourcePtToSurface (imls_icp.cpp:496-745), default branch (get_normals, kd-tree)."""
    src = filter_finite(src6)
    tgt = filter_finite(tgt6)
    knn = ExactKnn(tgt[:3])
    T = np.asarray(pose, dtype=np.float64).reshape(4, 4)
    rej = np.zeros(6, dtype=np.int64)
    xs, ys, ns_out, idx = [], [], [], []
    for i in range(src.shape[1]):
        pt = src[:3, i].astype(np.float64)
        xd = np.array([((T[r, 0] * pt[0] + T[r, 1] * pt[1]) + T[r, 2] * pt[2]) + T[r, 3] for r in range(3)])
        xf = xd.astype(np.float32)
        x = xf.astype(np.float64)
        ns = src[3:, i].astype(np.float64)
        if p.get("transform_normal"):
            ns = (T[:3, :3] @ ns).astype(np.float32).astype(np.float64)
        d1, i1 = knn.query(x, 1, p["r"], allow_self=False)
        if i1[0] < 0 or d1[0] > p["h"] * p["h"]:
            rej[REJ_TOO_FAR] += 1
            continue
        nn = tgt[3:, i1[0]].astype(np.float64)
        if not np.isfinite(nn).all():
            rej[REJ_INVALID_NORMAL] += 1
            continue
        if p["normal_angle_constraint"] and _angle_reject(ns, nn, p["angle_diff_threshold"]):
            rej[REJ_NORMAL_CONSTRAINT] += 1
            continue
        # ImplicitMLSFunction (imls_icp.cpp:301-483)
        K = p["search_number"]
        dk, ik = knn.query(x, K, p["r"], allow_self=True)
        S = []
        for j in range(K):
            if not np.isfinite(dk[j]):
                continue
            q = tgt[:3, ik[j]].astype(np.float64)
            n = tgt[3:, ik[j]].astype(np.float64)
            if not np.isfinite(n).all():
                continue
            if p["normal_angle_constraint"] and _angle_reject(ns, n, p["angle_diff_threshold"]):
                continue
            S.append((q, n))
        if len(S) < 3:
            rej[REJ_MLS_FAIL] += 1
            continue
        hmax = math.sqrt(dk[len(S) - 1]) / 3.0        # Q3
        ws = ps = 0.0
        for q, n in S:
            d = x - q
            dn = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]
            w = math.exp(-dn / hmax / hmax)
            ps += ((w * d[0]) * n[0] + (w * d[1]) * n[1]) + (w * d[2]) * n[2]
            ws += w
        height = ps / (ws + 1e-5)                   # Q4
        if not math.isfinite(height):
            rej[REJ_NAN_INF] += 1
            continue
        y = (x - height * nn).astype(np.float32)
        xs.append(xf)
        ys.append(y)
        ns_out.append(nn.astype(np.float32))
        idx.append(i)
    as3 = lambda a: np.asarray(a, dtype=np.float32).reshape(-1, 3)
    return as3(xs), as3(ys), as3(ns_out), np.asarray(idx, dtype=np.int64), rej


def project_plane_icp(src6: np.ndarray, tgt6: np.ndarray, pose: np.ndarray, p: dict):
    """plane_ICP_proj (laser_odometry.cpp:277-413), kd-tree branch: NN-1 within picp_r (no self
    match), unfound → "no normal", no h gate, y = x − ((x−p)·n)·n."""
    src = filter_finite(src6)
    tgt = filter_finite(tgt6)
    knn = ExactKnn(tgt[:3])
    T = np.asarray(pose, dtype=np.float64).reshape(4, 4)
    rej = np.zeros(6, dtype=np.int64)
    xs, ys, ns_out, idx = [], [], [], []
    for i in range(src.shape[1]):
        pt = src[:3, i].astype(np.float64)
        xd = np.array([((T[r, 0] * pt[0] + T[r, 1] * pt[1]) + T[r, 2] * pt[2]) + T[r, 3] for r in range(3)])
        xf = xd.astype(np.float32)
        x = xf.astype(np.float64)
        ns = src[3:, i].astype(np.float64)
        _, i1 = knn.query(x, 1, p["picp_r"], allow_self=False)
        if i1[0] < 0:
            rej[0] += 1
            continue
        q = tgt[:3, i1[0]].astype(np.float64)
        nn = tgt[3:, i1[0]].astype(np.float64)
        if not np.isfinite(nn).all():
            rej[REJ_INVALID_NORMAL] += 1
            continue
        if p["picp_normal_angle_constraint"] and _angle_reject(ns, nn, p["picp_angle_diff_threshold"]):
            rej[REJ_NORMAL_CONSTRAINT] += 1
            continue
        v = x - q
        pd = (v[0] * nn[0] + v[1] * nn[1]) + v[2] * nn[2]
        xs.append(xf)
        ys.append((x - pd * nn).astype(np.float32))
        ns_out.append(nn.astype(np.float32))
        idx.append(i)
    as3 = lambda a: np.asarray(a, dtype=np.float32).reshape(-1, 3)
    return as3(xs), as3(ys), as3(ns_out), np.asarray(idx, dtype=np.int64), rej


def plane_system(s, d, n):
    """A = [s×n, n], b = n·(d−s) (solver.cpp:89-104)."""
    s, d, n = (np.asarray(a, dtype=np.float64) for a in (s, d, n))
    A = np.concatenate([np.cross(s, n), n], axis=1)
    b = np.einsum("ij,ij->i", n, d - s)
    return A, b


def delta_from_x(x):
    D = np.eye(4)
    D[:3, :3] = Rotation.from_rotvec(x[:3]).as_matrix()
    D[:3, 3] = x[3:]
    return D


def solve_ls(s, d, n, threshold):
    """SolveMotionEstimationProblemLS (solver.cpp:74-166), SVD least squares, ties by index."""
    A, b = plane_system(s, d, n)
    N = len(b)
    x, *_ = np.linalg.lstsq(A, b, rcond=None)
    r = np.abs(A @ x - b)
    order = np.lexsort((np.arange(N), r))
    lo = int(threshold * N)
    hi = min(int((1 - threshold) * N), N - 1)
    keep = order[lo:hi + 1]
    x, *_ = np.linalg.lstsq(A[keep], b[keep], rcond=None)
    return delta_from_x(x), len(keep)


def solve_wls(s, d, n, w):
    A, b = plane_system(s, d, n)
    sw = np.sqrt(np.asarray(w, dtype=np.float64))
    x, *_ = np.linalg.lstsq(A * sw[:, None], b * sw, rcond=None)
    return delta_from_x(x)


def register_frame(src6, tgt6, p: dict):
    """laser_odometry.cpp:478-660 with the LS solver."""
    pose = np.eye(4)
    trace = []
    status = 0
    it = 0
    for it in range(p["iterations"]):
        x, y, n, _, rej = project(src6, tgt6, pose, p)
        if len(x) < p["correspond_number"]:
            status = 2
            break
        D, kept = solve_ls(x, y, n, p["ls_threshold"])
        pose = D @ pose
        trace.append(dict(delta=D, pose=pose.copy(), n_valid=len(x), reject=rej, n_kept=kept))
        dd = math.sqrt(D[0, 3] ** 2 + D[1, 3] ** 2 + D[2, 3] ** 2)
        ct = min(1.0, max((np.trace(D[:3, :3]) - 1.0) / 2.0, -1.0))
        if dd < p["delta_dist_threshold"] and math.acos(ct) < p["delta_angle_threshold"]:
            it += 1
            status = 1
            break
    else:
        it = p["iterations"]
    return pose, it, status, trace


def tv_normals(tgt6: np.ndarray, ten6: np.ndarray, q3: np.ndarray, p: dict):
    """VoteForAny (imls_icp.cpp:171-296) for the query points q3 (3, Q): the voted normal
    ("tangents" — the eigenvector of the smallest |λ| of the summed tensor's lower triangle,
    flipped to +z) and the non-zero flag (Eigen isZero(1e-12)).  ten6: (6, M) input tensors
    (xx, xy, xz, yy, yz, zz) in input order.  libpointmatcher decompose semantics: unpinned."""
    keep = np.isfinite(tgt6[:3]).all(axis=0)
    tgt, ten = tgt6[:, keep], ten6[:, keep].astype(np.float64)
    knn = ExactKnn(tgt[:3])
    P = tgt[:3].T.astype(np.float64)
    sigma, thr, k = p["tensor_sigma"], p["tensor_distance_threshold"], p["tensor_k"]
    Q = q3.shape[1]
    nrm = np.zeros((Q, 3))
    found = np.zeros(Q, dtype=np.int32)
    acc_all = np.zeros((Q, 3, 3))
    I3 = np.eye(3)
    for q in range(Q):
        x = q3[:, q].astype(np.float64)
        dk, ik = knn.query(x, k, np.inf, allow_self=False)
        acc = np.zeros((3, 3))
        for j in ik[ik >= 0]:
            r = x - P[j]
            nr = math.sqrt((r[0] * r[0] + r[1] * r[1]) + r[2] * r[2])
            dist = nr / sigma
            if dist <= 0.0 or dist >= thr:
                continue
            u = r / nr
            w = math.exp(-(nr * nr) / sigma)
            t = ten[:, j]
            T = np.array([[t[0], t[1], t[2]], [t[1], t[3], t[4]], [t[2], t[4], t[5]]])
            R = I3 - 2.0 * np.outer(u, u)
            Rp = (I3 - 0.5 * np.outer(u, u)) @ R
            acc += w * (R @ T @ Rp)
        acc_all[q] = acc
        if np.all(np.abs(acc) <= 1e-12):
            continue
        ev, U = np.linalg.eigh(acc, UPLO="L")      # Eigen SelfAdjointEigenSolver reads the lower triangle
        m = int(np.argmin(np.abs(ev)))
        n = U[:, m]
        if n[2] < 0:
            n = -n
        nrm[q] = n
        found[q] = 1
    return nrm, found, acc_all


def tv_encode_pca(evals: np.ndarray, evecs: np.ndarray, k: int) -> np.ndarray:
    """CustomTensorVoting::myCustomFunctionWithEigen (scan_registration.cpp:358-381) in float32:
    (n, 3) eigenvalues + (n, 9) column-major eigenvectors → (n, 6) tensors (xx xy xz yy yz zz)."""
    a = np.abs(evals.astype(np.float32))
    l1, l3 = a.max(axis=1), a.min(axis=1)
    l2 = ((a[:, 0] + a[:, 1]) + a[:, 2]) - (l1 + l3)
    kf = np.float32(k)
    e1, e2 = evecs[:, 0:3].astype(np.float32), evecs[:, 3:6].astype(np.float32)
    s1, s3 = (l1 - l2) / kf, l3 / kf
    out = np.zeros((len(a), 6), np.float32)
    for m, (r, c) in enumerate(((0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2))):
        S = e1[:, r] * e1[:, c]
        Pm = S + e2[:, r] * e2[:, c]
        out[:, m] = s1 * S + s3 * Pm
    ok = (l1 >= l2) & (l2 >= l3)
    out[~ok] = np.array([1, 0, 0, 1, 0, 1], np.float32)
    return out


def ring_pca_np(xyz, ring_sizes, window_size=3, iter_step=1, knn_distance_threshold=10.0, neighbor_scan="kdtree",
                distance_threshold=0.02, valid_points_threshold=0.8, use_all_points=True, planarity_threshold=0.05):
    """Independent restatement of scan_registration.cpp's "pca" normals (1136-1229; computeNormalPCA
    158-229, findNearestPoint 117-136, checkPlaneValidity 138-156) + computeGeometricFeatures
    (279-327): NN-1 by scipy cKDTree on each line (re-ranked with the float L2 the reference's
    FLANN tree uses), covariance and plane check in float32 numpy, eigen-decomposition by
    numpy.linalg.eigh in float64.  Returns (index, normal, evals, flags, pca_failure, invalid)."""
    xyz = np.asarray(xyz, np.float32)[:, :3]
    sizes = [int(v) for v in ring_sizes]
    start = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    rings = [xyz[start[i]:start[i + 1]] for i in range(len(sizes))]
    trees = [cKDTree(r.astype(np.float64)) if len(r) else None for r in rings]
    num = 3 * (int(2 * window_size / iter_step) + 1)
    out_i, out_n, out_l, out_f = [], [], [], []
    fail = invalid = 0

    def nearest(q, a):
        if neighbor_scan == "index":
            return True, None
        if trees[a] is None:
            return False, None
        k = min(8, len(rings[a]))
        _, cand = trees[a].query(q.astype(np.float64), k=k)
        cand = np.sort(np.atleast_1d(cand))
        d = rings[a][cand] - q                      # float32, ((0 + d0²) + d1²) + d2²
        d2 = ((np.float32(0) + d[:, 0] * d[:, 0]) + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        b = int(np.argmin(d2))                     # first minimum = lowest index among ties
        return bool(d2[b] < np.float32(knn_distance_threshold)), int(cand[b])

    for i in range(1, len(sizes) - 1):
        if sizes[i] == 0 or sizes[i] - 11 < 6 or sizes[i - 1] - 11 < 6 or sizes[i + 1] - 11 < 6:
            continue
        for j in range(5, sizes[i] - 5):
            pts = [rings[i][j + k] for k in range(-window_size, window_size + 1, iter_step) if 0 <= j + k < sizes[i]]
            for a in (i - 1, i + 1):
                ok, nb = nearest(rings[i][j], a)
                if not ok:
                    continue
                nb = j if nb is None else nb
                pts += [rings[a][nb + k] for k in range(-window_size, window_size + 1, iter_step)
                        if 0 <= nb + k < sizes[a]]
            if len(pts) < num:
                fail += 1
                continue
            P = np.array(pts, np.float32)
            c = P.mean(axis=0, dtype=np.float64)
            C = (P - c).T.astype(np.float64) @ (P - c) / (len(P) - 1)
            w, V = np.linalg.eigh(C)
            dist = np.abs((P - c) @ V[:, 0])
            good = np.count_nonzero(dist < distance_threshold) >= valid_points_threshold * len(P)
            if not good:
                invalid += 1
                if not use_all_points:
                    continue
                lam = np.array([-1.0, -1.0, -1.0])
                nrm = V[:, 2]
            else:
                lam = w[::-1]
                nrm = V[:, 0]
            nrm = nrm / np.linalg.norm(nrm)
            if nrm[2] < 0:
                nrm = -nrm
            l1, l2, l3 = lam
            plan = (l2 - l3) / l1
            out_i.append(start[i] + 5 + j)
            out_n.append(nrm); out_l.append(lam)
            out_f.append((1 if not good else 0) | (2 if (good and plan > planarity_threshold) else 0))
    return (np.array(out_i, np.int64), np.array(out_n).reshape(-1, 3), np.array(out_l).reshape(-1, 3),
            np.array(out_f, np.uint8), fail, invalid)
