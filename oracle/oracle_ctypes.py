"""ctypes binding of the CPU oracle (oracle/liboracle_imls.so).  TEST INFRASTRUCTURE ONLY.

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
Parity status: unpinned (see imls_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import pathlib
import sys

import numpy as np

ORACLE_DIR = pathlib.Path(__file__).resolve().parent
LIB = ORACLE_DIR / "liboracle_imls.so"


def _abi():
    # the params struct lives in the product package's ABI mirror (shared header layout)
    root = ORACLE_DIR.parent
    if str(root) not in sys.path:
        sys.path.insert(0, str(root))
    import plo_amd  # noqa: E402
    return plo_amd.load()._abi


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            raise RuntimeError(f"oracle not built: {LIB} (make -C oracle)")
        L = C.CDLL(str(LIB))
        abi = _abi()
        P, VP, SZ = C.POINTER, C.c_void_p, C.c_size_t
        L.oracle_knn.argtypes = [VP, SZ, VP, SZ, C.c_int, C.c_double, C.c_int, VP, VP]
        L.oracle_project.argtypes = [VP, SZ, VP, SZ, VP, P(abi.ImlsParams), VP, VP, VP, VP, P(SZ), VP]
        L.oracle_solve.argtypes = [C.c_int32, VP, VP, VP, VP, SZ, P(abi.ImlsParams), VP, VP, P(C.c_int)]
        L.oracle_register_frame.argtypes = [VP, SZ, VP, SZ, P(abi.ImlsParams), VP, P(C.c_int), P(C.c_int), VP,
                                            C.c_int, VP, P(SZ), P(C.c_double), P(C.c_double)]
        L.oracle_project_tv.argtypes = [VP, SZ, VP, SZ, VP, VP, P(abi.ImlsParams), VP, VP, VP, VP, P(SZ), VP]
        L.oracle_register_frame_tv.argtypes = [VP, SZ, VP, SZ, VP, P(abi.ImlsParams), VP, P(C.c_int), P(C.c_int), VP,
                                               C.c_int, VP, P(SZ), P(C.c_double), P(C.c_double)]
        L.oracle_register_frame_rs.argtypes = [VP, SZ, VP, SZ, VP, P(abi.ImlsParams), VP, VP, P(C.c_int), P(C.c_int),
                                               VP, C.c_int, VP, P(SZ), P(C.c_double), P(C.c_double)]
        L.oracle_chain_pose.argtypes = [VP, VP, VP]
        L.oracle_format_pose.argtypes = [VP, C.c_char_p, C.c_char_p, SZ]
        L.oracle_format_matched.argtypes = [VP, VP, SZ, C.c_char_p, SZ]
        L.oracle_format_matched.restype = SZ
        L.oracle_tv_normals.argtypes = [VP, SZ, VP, VP, SZ, P(abi.ImlsParams), VP, VP, VP]
        L.oracle_rand_seed.argtypes = [VP, C.c_uint32]
        L.oracle_rand_next.argtypes = [VP]
        L.oracle_set_threads.argtypes = [C.c_int]
        L.oracle_set_faithful.argtypes = [C.c_int]
        L.oracle_rand_next.restype = C.c_int32
        L.oracle_colpiv_qr_solve.argtypes = [VP, C.c_int, C.c_int, VP, VP]
        L.oracle_delta_from_x.argtypes = [VP, VP]
        L.oracle_sym_eig6.argtypes = [VP, VP, VP]
        L.oracle_sample_point_cloud.argtypes = [P(abi.ImlsSampleParams), VP, VP, SZ, SZ, VP, SZ, VP, SZ, SZ, VP,
                                                P(SZ), VP]
        L.oracle_scan_front_end.argtypes = [P(abi.ImlsFrontParams), VP, SZ, SZ, VP, VP, VP, P(SZ)]
        L.oracle_ring_pca.argtypes = [VP, SZ, VP, C.c_int32, P(abi.ImlsPcaParams), VP, VP, VP, VP, VP, VP, VP,
                                      P(SZ), VP]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _soa6(a) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float32)
    assert a.ndim == 2 and a.shape[0] == 6
    return a


def knn(tgt6, q3, K, r, allow_self):
    tgt6 = _soa6(tgt6)
    q3 = np.ascontiguousarray(q3, dtype=np.float32)
    Q = q3.shape[1]
    d2 = np.zeros((Q, K)); idx = np.zeros((Q, K), dtype=np.int32)
    rc = lib().oracle_knn(_ptr(tgt6), tgt6.shape[1], _ptr(q3), Q, K, r, int(allow_self), _ptr(d2), _ptr(idx))
    assert rc == 0
    return d2, idx


def _ten6(t, M):
    if t is None:
        return None
    t = np.ascontiguousarray(t, dtype=np.float32)
    assert t.shape == (6, M)
    return t


def project(src6, tgt6, pose, params, tensors=None):
    src6, tgt6 = _soa6(src6), _soa6(tgt6)
    ten = _ten6(tensors, tgt6.shape[1])
    N = src6.shape[1]
    pose = np.ascontiguousarray(pose, dtype=np.float64).reshape(16)
    x = np.zeros((N, 3), np.float32); y = np.zeros((N, 3), np.float32); n = np.zeros((N, 3), np.float32)
    idx = np.zeros(N, np.uint32); rej = np.zeros(6, np.uint64); nv = C.c_size_t()
    rc = lib().oracle_project_tv(_ptr(src6), N, _ptr(tgt6), tgt6.shape[1], None if ten is None else _ptr(ten),
                                 _ptr(pose), C.byref(params), _ptr(x), _ptr(y), _ptr(n), _ptr(idx), C.byref(nv), _ptr(rej))
    assert rc == 0
    k = nv.value
    return x[:k], y[:k], n[:k], idx[:k], rej


def solve(method, s, d, n, params, weights=None, rand_state=None):
    s, d, n = (np.ascontiguousarray(a, dtype=np.float64).reshape(-1, 3) for a in (s, d, n))
    w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
    D = np.zeros(16); ok = C.c_int()
    rc = lib().oracle_solve(method, _ptr(s), _ptr(d), _ptr(n), None if w is None else _ptr(w), len(s),
                            C.byref(params), None if rand_state is None else _ptr(rand_state), _ptr(D), C.byref(ok))
    assert rc == 0
    return bool(ok.value), D.reshape(4, 4)


def tv_normals(tgt6, tensors, q3, params):
    """VoteForAny per query: (normals (Q,3) double, found (Q,) int32, summed tensors (Q,3,3))."""
    tgt6 = _soa6(tgt6)
    ten = _ten6(tensors, tgt6.shape[1])
    q3 = np.ascontiguousarray(q3, dtype=np.float32)
    Q = q3.shape[1]
    nrm = np.zeros((Q, 3)); found = np.zeros(Q, np.int32); acc = np.zeros((Q, 9))
    rc = lib().oracle_tv_normals(_ptr(tgt6), tgt6.shape[1], _ptr(ten), _ptr(q3), Q, C.byref(params), _ptr(nrm),
                                 _ptr(found), _ptr(acc))
    assert rc == 0
    return nrm, found, acc.reshape(Q, 3, 3)


def register_frame(src6, tgt6, params, corr_iter=-1, tensors=None, rand_state=None):
    """One frame (laser_odometry.cpp:478-660).  rand_state (int32[34], updated in place) carries the
    RANSAC rand() stream across frames; None = a fresh stream from params.ransac_seed."""
    src6, tgt6 = _soa6(src6), _soa6(tgt6)
    ten = _ten6(tensors, tgt6.shape[1])
    abi = _abi()
    it = params.iterations
    trace = (abi.ImlsIterTrace * max(it, 1))()
    pose = np.zeros(16); iters = C.c_int(); status = C.c_int()
    N = src6.shape[1]
    corr = np.zeros((N, 9), np.float32) if corr_iter >= 0 else None
    cn = C.c_size_t(); ti = C.c_double(); tt = C.c_double()
    if rand_state is not None:
        assert rand_state.dtype == np.int32 and rand_state.shape == (34,) and rand_state.flags.c_contiguous
    rc = lib().oracle_register_frame_rs(_ptr(src6), N, _ptr(tgt6), tgt6.shape[1], None if ten is None else _ptr(ten),
                                        C.byref(params), None if rand_state is None else _ptr(rand_state), _ptr(pose),
                                        C.byref(iters), C.byref(status), trace, corr_iter,
                                        None if corr is None else _ptr(corr), C.byref(cn), C.byref(ti), C.byref(tt))
    assert rc == 0
    out = dict(pose=pose.reshape(4, 4), iters=iters.value, status=status.value,
               trace=[trace[k] for k in range(iters.value)], seconds_index=ti.value, seconds_total=tt.value)
    if corr is not None:
        out["corr"] = corr[:cn.value]
    return out


def rand_state(seed=1):
    """glibc srand(seed) state (int32[34])."""
    st = np.zeros(34, np.int32)
    lib().oracle_rand_seed(_ptr(st), seed)
    return st


def chain_pose(prev, rel):
    a = np.ascontiguousarray(prev, dtype=np.float64).reshape(16)
    b = np.ascontiguousarray(rel, dtype=np.float64).reshape(16)
    out = np.zeros(16)
    lib().oracle_chain_pose(_ptr(a), _ptr(b), _ptr(out))
    return out.reshape(4, 4)


def format_pose(pose, timestamp: str) -> str:
    """savePoseToFile's line (saver.cpp:46-54)."""
    P = np.ascontiguousarray(pose, dtype=np.float64).reshape(16)
    buf = C.create_string_buffer(512)
    n = lib().oracle_format_pose(_ptr(P), timestamp.encode(), buf, 512)
    assert 0 < n < 512
    return buf.value.decode()


def format_matched(x3, y3) -> str:
    """saveMatchedPointsToFile's text (saver.cpp:113-133) for float (n, 3) clouds."""
    x3 = np.ascontiguousarray(x3, dtype=np.float32).reshape(-1, 3)
    y3 = np.ascontiguousarray(y3, dtype=np.float32).reshape(-1, 3)
    need = lib().oracle_format_matched(_ptr(x3), _ptr(y3), len(x3), None, 0)
    buf = C.create_string_buffer(need + 1)
    lib().oracle_format_matched(_ptr(x3), _ptr(y3), len(x3), buf, need + 1)
    return buf.value.decode()


def rand_sequence(seed, n):
    st = np.zeros(34, np.int32)
    lib().oracle_rand_seed(_ptr(st), seed)
    return np.array([lib().oracle_rand_next(_ptr(st)) for _ in range(n)], dtype=np.int64)


def colpiv_qr_solve(A, b):
    A = np.ascontiguousarray(A, dtype=np.float64); b = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros(A.shape[1])
    lib().oracle_colpiv_qr_solve(_ptr(A), A.shape[0], A.shape[1], _ptr(b), _ptr(x))
    return x


def delta_from_x(x):
    x = np.ascontiguousarray(x, dtype=np.float64); D = np.zeros(16)
    lib().oracle_delta_from_x(_ptr(x), _ptr(D))
    return D.reshape(4, 4)


def scan_front_end(xyz, front_params):
    """scan_registration.cpp front end (scanreg_oracle.cpp): (xyzi (m, 4), input index (m,), ring sizes)."""
    a = np.ascontiguousarray(xyz, dtype=np.float32)
    n = a.shape[0]
    out = np.zeros((max(n, 1), 4), np.float32); idx = np.zeros(max(n, 1), np.uint32)
    rs = np.zeros(64, np.int32); m = C.c_size_t()
    rc = lib().oracle_scan_front_end(C.byref(front_params), _ptr(a), a.shape[1] if a.ndim == 2 else 3, n, _ptr(out),
                                     _ptr(idx), _ptr(rs), C.byref(m))
    assert rc == 0
    k = m.value
    return out[:k], idx[:k], rs[:front_params.n_scans]


def ring_pca(xyz, ring_sizes, pca_params):
    """scan_registration.cpp pca normals + geometric-features presample (scanreg_oracle.cpp).
    Returns the same dict as ImlsContext.ring_normals_pca plus `margin` (plane-check margin)."""
    a = np.ascontiguousarray(xyz, dtype=np.float32)
    rs = np.ascontiguousarray(ring_sizes, dtype=np.int32)
    n = max(a.shape[0], 1)
    idx = np.zeros(n, np.uint32); nrm = np.zeros((n, 3), np.float32); ev = np.zeros((n, 3), np.float32)
    evec = np.zeros((n, 9), np.float32); feat = np.zeros((n, 8), np.float32); fl = np.zeros(n, np.uint8)
    mg = np.zeros(n, np.float32); cnt = np.zeros(2, np.uint64); nout = C.c_size_t()
    rc = lib().oracle_ring_pca(_ptr(a), a.shape[1], _ptr(rs), len(rs), C.byref(pca_params), _ptr(idx), _ptr(nrm),
                               _ptr(ev), _ptr(evec), _ptr(feat), _ptr(fl), _ptr(mg), C.byref(nout), _ptr(cnt))
    assert rc == 0
    k = nout.value
    return dict(index=idx[:k], normal=nrm[:k], evals=ev[:k], evecs=evec[:k], features=feat[:k], flags=fl[:k],
                margin=mg[:k], pca_failure=int(cnt[0]), plane_invalid=int(cnt[1]))


def sample_point_cloud(xyz, nrm, candidates, last_xyz, sample_params):
    """samplePointCloud "normal" / "major_axis" (scanreg_oracle.cpp): (sampled indices, bin weights)."""
    a = np.ascontiguousarray(xyz, dtype=np.float32); nn = np.ascontiguousarray(nrm, dtype=np.float32)
    assert a.shape == nn.shape and a.shape[1] >= 3
    cand = np.ascontiguousarray(candidates, dtype=np.int32)
    last = np.ascontiguousarray(last_xyz if last_xyz is not None else np.zeros((0, 3)), dtype=np.float32)
    nb = sample_params.azimuth_bins * sample_params.elevation_bins
    out = np.zeros(len(cand) + nb + 1, np.int32); w = np.zeros(nb, np.float32); k = C.c_size_t()
    rc = lib().oracle_sample_point_cloud(C.byref(sample_params), _ptr(a), _ptr(nn), a.shape[1], a.shape[0], _ptr(cand),
                                         len(cand), _ptr(last), last.shape[1] if last.ndim == 2 else 3, last.shape[0],
                                         _ptr(out), C.byref(k), _ptr(w))
    assert rc == 0
    return out[:k.value], w


def set_threads(n: int):
    """Threads of the oracle's per-query projection loop (1 = the reference's single thread)."""
    lib().oracle_set_threads(int(n))


def set_faithful(on: bool):
    """The reference's container costs in the projection loop (erase per rejection, AoS copies,
    per-query allocations); identical results.  CPU baseline only."""
    lib().oracle_set_faithful(int(bool(on)))
