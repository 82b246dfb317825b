"""GPU: the producer's front end (imls_scan_front_end; scan_registration.cpp:862-1069) against the
CPU oracle on raw sweeps in driver order — 16 / 32 / 64 lines, revolutions started anywhere, NaN and
too-close returns, dense and non-dense messages: the surviving points, their ring order, input
indices and ring sizes bit-exact; intensity (= ring + 0.1·relTime) within 2 ulp + 2e-8 (the device
takes atan / atan2 correctly rounded through fp64, the oracle glibc's atanf / atan2f, ≤ 1 ulp apart;
DESIGN §3).  Then the
whole raw-sweep → flat-cloud chain (front end → ring PCA → presample → major_axis sampling) against
the oracle chain, frame by frame."""
import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi, imls_icp, producer, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    with imls_icp.ImlsContext(device=0) as c:
        yield c


@pytest.fixture(scope="module")
def scene():
    return synth.make_scene(3), synth.trajectory(6, 2003)


def _fp(ns, lo=None, hi=None, dense=0):
    p = _abi.default_front_params(ns)
    if lo is not None:
        p.minimum_range = lo
    if hi is not None:
        p.maximum_range = hi
    p.is_dense = dense
    return p


CASES = [("vlp16", 16, 0.0, 0.5, 100.0, 0), ("vlp16", 16, 137.3, 0.5, 100.0, 1), ("hdl64", 64, 0.0, None, None, 0),
         ("hdl64", 64, 251.0, None, None, 1), ("hdl64", 32, 90.0, None, None, 0), ("vlp16", 32, 300.0, 0.5, 100.0, 1)]


@pytest.mark.parametrize("model,ns,start,lo,hi,dense", CASES)
def test_front_end_matches_oracle(ctx, scene, model, ns, start, lo, hi, dense):
    sc, poses = scene
    sm = synth.hdl64() if model == "hdl64" else synth.vlp16()
    raw = synth.raw_sweep(sc, sm, poses[2], 11, start_deg=start, n_nan=7, n_close=5)
    fp = _fp(ns, lo, hi, dense)
    gx, gi, gidx, grs = ctx.scan_front_end(raw, fp)
    ox, oidx, ors = oc.scan_front_end(raw, fp)
    assert np.array_equal(grs, ors) and np.array_equal(gidx, oidx)
    assert np.array_equal(gx, ox[:, :3], equal_nan=True)
    fin = np.isfinite(ox[:, 3])
    assert np.array_equal(np.isfinite(gi), fin)
    # an ulp of the azimuth (~2.4e-7 rad near 2π) moves 0.1·relTime by ≤ 0.1·2·ulp / (endOri − startOri) < 2e-8
    d = np.abs(gi[fin].astype(np.float64) - ox[fin, 3])
    tol = 2 * np.spacing(np.abs(ox[fin, 3]).astype(np.float32)).astype(np.float64) + 2e-8
    assert np.all(d <= tol), (d.max(), float(np.max(d / tol)))
    assert (d == 0).mean() > 0.95


def test_front_end_edge_cases(ctx):
    fp = _fp(16, 0.5, 100.0)
    assert len(ctx.scan_front_end(np.zeros((0, 3), np.float32), fp)[0]) == 0
    assert len(ctx.scan_front_end(np.full((9, 3), 0.01, np.float32), fp)[0]) == 0     # all filtered out
    pts = np.array([[0.5, 0, 0], [0.4999999, 0, 0], [100.0, 0, 0], [100.00001, 0, 0], [3, 0, 0.05]], np.float32)
    assert list(ctx.scan_front_end(pts, fp)[2]) == list(oc.scan_front_end(pts, fp)[1]) == [0, 2, 4]
    with pytest.raises(_abi.ImlsError):
        ctx.scan_front_end(pts, _fp(40))


def test_raw_sweep_chain_matches_oracle(scene):
    """Raw VLP-16 sweeps → GPU front end → ring PCA → presample → major_axis sampling, against the
    oracle's front end → ring_pca → sample_point_cloud on the same sweeps (3 frames: the first sampled
    with "normal", the others against the previous filtered cloud)."""
    sc, poses = scene
    fp = _fp(16, 0.5, 100.0)
    last = None
    with imls_icp.ImlsContext(device=0) as c:
        sr = producer.ScanRegistration(ctx=c, shuffle_seed=4, rand_seed=2)
        for k in range(3):
            raw = synth.raw_sweep(sc, synth.vlp16(), poses[2 + k], 40 + k, start_deg=15.0 * k)
            sp = sr.sample_params()
            filtered, flat = sr.process_raw(raw, fp)
            ox, oidx, ors = oc.scan_front_end(raw, fp)
            o = oc.ring_pca(ox[:, :3], ors, _abi.default_pca_params())
            fxyz = ox[:, :3][o["index"]]
            assert np.array_equal(filtered["x"], fxyz[:, 0]) and np.array_equal(filtered["normal_z"], o["normal"][:, 2])
            cand = np.nonzero(o["flags"] & _abi.IMLS_PCA_CANDIDATE)[0]
            s, _ = oc.sample_point_cloud(fxyz, o["normal"], cand, last, sp)
            assert np.array_equal(fxyz[s][:, 1], flat["y"])
            last = fxyz
