"""GPU: the C++ boundary for real.  tests/cpp/type_swap.cpp runs the reference's per-frame loop
(laser_odometry.cpp:489-647) with only the types swapped — `imls_hip::IMLSICPMatcherHip` for
IMLSICPMatcher and `imls_hip::SolveMotionEstimationProblemLS / RANSAC` with solver.h's argument
lists — linked against the in-tree libimls_gpu.so, in a fresh process (started as a child, never
exec'd from this GPU-initialised one).  Its final rPose, iteration count and per-iteration
correspondence counts must equal the oracle's register_frame on the same frame (LS within 1e-6,
RANSAC→DRPM within 1e-5; the thread context's rand() stream starts at seed 1 like the oracle's)."""
import pathlib
import subprocess

import numpy as np
import pytest

import oracle_ctypes as oc
from planetary_lidar_odometry_amd import _abi, config, synth

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parent.parent
EXE = ROOT / "tests" / "cpp" / "type_swap"
GOLDEN = ROOT / "tests" / "golden"


def write_cloud(path, soa6):
    """uint64 count + 48-byte pcl::PointXYZINormal records."""
    soa6 = np.asarray(soa6, np.float32)
    rec = np.zeros(soa6.shape[1], synth.POINT_DTYPE)
    for k, f in enumerate(("x", "y", "z", "normal_x", "normal_y", "normal_z")):
        rec[f] = soa6[k]
    with open(path, "wb") as f:
        f.write(np.uint64(len(rec)).tobytes())
        f.write(rec.tobytes())


def run_swap(tmp_path, method, iters, name):
    g = dict(np.load(GOLDEN / f"{name}.npz"))
    write_cloud(tmp_path / "src.bin", g["src"])
    write_cloud(tmp_path / "tgt.bin", g["tgt"])
    r = subprocess.run([str(EXE), method, str(iters), str(tmp_path / "src.bin"), str(tmp_path / "tgt.bin")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split("\n")
    nvalid = [int(l.split()[2]) for l in lines if l.startswith("iter ")]
    iters_run = int(next(l for l in lines if l.startswith("iters")).split()[1])
    pose = np.array(next(l for l in lines if l.startswith("pose")).split()[1:], float).reshape(4, 4)
    return g, pose, iters_run, nvalid


@pytest.mark.parametrize("name", ["vlp16_pair", "planetary_pair"])
def test_type_swap_ls(tmp_path, name):
    assert EXE.exists(), "tests/cpp/type_swap not built (run __graft_entry__.build())"
    g, pose, iters, nvalid = run_swap(tmp_path, "LS", 10, name)
    p = config.params_from_config(config.load())
    p.solve_method, p.iterations = _abi.IMLS_SOLVE_LS, 10
    want = oc.register_frame(g["src"], g["tgt"], p)
    assert iters == want["iters"]
    assert nvalid == [int(t.n_valid) for t in want["trace"]]
    assert np.abs(pose - want["pose"]).max() < 1e-6


def test_type_swap_shipped_ransac(tmp_path):
    g, pose, iters, nvalid = run_swap(tmp_path, "RANSAC", 6, "vlp16_pair")
    p = config.params_from_config(config.load())      # RANSAC -> DRPM, shipped values
    p.iterations = 6
    want = oc.register_frame(g["src"], g["tgt"], p)
    assert iters == want["iters"]
    assert nvalid == [int(t.n_valid) for t in want["trace"]]
    assert np.abs(pose - want["pose"]).max() < 1e-5
