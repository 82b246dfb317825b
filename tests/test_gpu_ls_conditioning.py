"""GPU: trimmed LS (solver.cpp:74-166) on near-degenerate systems — the geometry degeneracy.h exists
for.  The device forms the normal equations (fp64) and solves them by a pivoted Cholesky; the
reference (and the oracle) use Eigen's column-pivoted Householder QR on A, whose error grows with
cond(A) where the normal equations' grows with cond(A)².  Each case reports both errors against an
extended-precision (80-bit long double) least-squares solution of the same trimmed system, and
asserts the device agrees with the oracle within 1e-6 — or, where the system is so ill-conditioned
that the two fp64 methods disagree by more, that the device is no further from the exact solution
than the oracle is (× 10) — so a conditioning regression shows up here rather than in a pose."""
import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi, config, imls_icp

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-6


@pytest.fixture(scope="module")
def ctx():
    p = config.bench_params(1)
    with imls_icp.ImlsContext(p, device=0) as c:
        yield c


def corridor(n, tilt, seed, length=40.0):
    """Floor z = 0 and walls y = ±2 along x: no normal has an x component when tilt = 0 (x
    translation unobservable); `tilt` (rad) spreads the normals slightly."""
    rng = np.random.default_rng(seed)
    k = rng.integers(0, 3, n)
    s = np.column_stack([rng.uniform(-length / 2, length / 2, n), rng.uniform(-2, 2, n), rng.uniform(0, 3, n)])
    nrm = np.zeros((n, 3))
    s[k == 0, 2] = 0.0
    nrm[k == 0] = (0, 0, 1)
    s[k == 1, 1] = 2.0
    nrm[k == 1] = (0, -1, 0)
    s[k == 2, 1] = -2.0
    nrm[k == 2] = (0, 1, 0)
    nrm += rng.normal(0, tilt, (n, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    return s, nrm


def tilted_plane(n, tilt, seed):
    rng = np.random.default_rng(seed)
    s = np.column_stack([rng.uniform(-20, 20, n), rng.uniform(-20, 20, n), rng.normal(0, 0.02, n)])
    nrm = np.tile([0.0, 0.0, 1.0], (n, 1)) + rng.normal(0, tilt, (n, 3))
    return s, nrm / np.linalg.norm(nrm, axis=1, keepdims=True)


def targets(s, nrm, seed):
    """d = s + motion + noise along the normal (the IMLS projection moves points along n)."""
    rng = np.random.default_rng(seed + 100)
    a = 0.01
    R = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    d = s @ R.T + np.array([0.25, -0.05, 0.03])
    return d + nrm * rng.normal(0, 0.01, (len(s), 1))


def exact_trimmed(s, d, nrm, t):
    """The oracle's trimmed LS (solver.cpp:74-166) with both solves in 80-bit long double (normal
    equations of A in long double are exact enough at these sizes to act as the reference x)."""
    ld = np.longdouble
    S, D, Nn = s.astype(ld), d.astype(ld), nrm.astype(ld)
    A = np.column_stack([Nn[:, 2] * S[:, 1] - Nn[:, 1] * S[:, 2], Nn[:, 0] * S[:, 2] - Nn[:, 2] * S[:, 0],
                         Nn[:, 1] * S[:, 0] - Nn[:, 0] * S[:, 1], Nn[:, 0], Nn[:, 1], Nn[:, 2]])
    b = (Nn * (D - S)).sum(axis=1)

    def lsq(A, b):
        H, g = A.T @ A, A.T @ b
        # Gaussian elimination with partial pivoting in long double
        M = np.column_stack([H, g]).copy()
        for j in range(6):
            p = j + int(np.argmax(np.abs(M[j:, j])))
            M[[j, p]] = M[[p, j]]
            M[j + 1:] -= np.outer(M[j + 1:, j] / M[j, j], M[j])
        x = np.zeros(6, ld)
        for j in range(5, -1, -1):
            x[j] = (M[j, 6] - M[j, j + 1:6] @ x[j + 1:]) / M[j, j]
        return x

    x0 = lsq(A, b)
    r = np.abs(A @ x0 - b).astype(np.float64)
    N = len(b)
    idx = np.lexsort((np.arange(N), r))
    lo, hi = int(t * N), min(int((1 - t) * N), N - 1)
    keep = idx[lo:hi + 1]
    return lsq(A[keep], b[keep]).astype(np.float64)


def x_from_delta(D):
    """(ω, t) of Δ: t exactly, ω by the inverse Rodrigues (small angles)."""
    R = D[:3, :3]
    ang = np.arccos(np.clip((np.trace(R) - 1) / 2, -1, 1))
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    w = w * (ang / (2 * np.sin(ang))) if ang > 1e-12 else w / 2
    return np.concatenate([w, D[:3, 3]])


CASES = {
    "well_conditioned": lambda: tilted_plane(3000, 0.5, 1),
    "corridor_tilt_1e-2": lambda: corridor(4000, 1e-2, 2),
    "corridor_tilt_1e-3": lambda: corridor(4000, 1e-3, 3),
    "plane_tilt_1e-2": lambda: tilted_plane(3000, 1e-2, 4),
    "plane_tilt_1e-3": lambda: tilted_plane(3000, 1e-3, 5),
    "corridor_tilt_1e-5": lambda: corridor(4000, 1e-5, 7),
    "corridor_tilt_1e-6": lambda: corridor(4000, 1e-6, 8),
    "plane_tilt_1e-5": lambda: tilted_plane(3000, 1e-5, 9),
    "short_corridor_tilt_1e-4": lambda: corridor(4000, 1e-4, 10, length=4.0),
}


# fixed target-noise seed per case (reproducible run to run)
TARGET_SEEDS = {case: 101 + k for k, case in enumerate(CASES)}


@pytest.mark.parametrize("case", list(CASES))
def test_near_degenerate_ls(ctx, case):
    s, nrm = CASES[case]()
    d = targets(s, nrm, TARGET_SEEDS[case])
    p = config.bench_params(1)
    ok, D = ctx.solve_correspondences(_abi.IMLS_SOLVE_LS, s, d, nrm)
    okr, Dr = oc.solve(_abi.IMLS_SOLVE_LS, s, d, nrm, p)
    assert ok and okr
    xe = exact_trimmed(s, d, nrm, p.ls_threshold)
    err_gpu = np.abs(x_from_delta(D) - xe).max()
    err_ora = np.abs(x_from_delta(Dr) - xe).max()
    diff = np.abs(D - Dr).max()
    print(f"{case}: |gpu-oracle| {diff:.3e}  gpu err {err_gpu:.3e}  oracle err {err_ora:.3e}")
    # both bounds hold together: Δ equal to the oracle's, and the GPU's distance to the exact trimmed
    # solution no worse than twice the oracle's (measured on MI355X, profiles/r03_experiments: at
    # most 1.23× — corridor tilt 1e-5 — with |gpu − oracle| ≤ 9.1e-13 over every case)
    assert diff < POSE_TOL and err_gpu <= 2 * err_ora + 1e-14, (diff, err_gpu, err_ora)


def test_exactly_degenerate_corridor(ctx):
    """tilt 0: the x translation is unobservable (rank 5).  Eigen's QR returns the basic solution
    (the free column's coordinate 0); the device's pivoted Cholesky must stop at the same rank and
    leave that coordinate 0 too, agreeing with the oracle elsewhere."""
    s, nrm = corridor(4000, 0.0, 6)
    d = targets(s, nrm, 6)
    p = config.bench_params(1)
    ok, D = ctx.solve_correspondences(_abi.IMLS_SOLVE_LS, s, d, nrm)
    okr, Dr = oc.solve(_abi.IMLS_SOLVE_LS, s, d, nrm, p)
    assert ok and okr
    print("degenerate corridor |gpu-oracle|", np.abs(D - Dr).max(), "tx", D[0, 3], Dr[0, 3])
    assert np.abs(D - Dr).max() < POSE_TOL
