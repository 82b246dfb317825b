"""Generates tests/golden/pca_vlp16.npz: the upstream producer's ring-neighbourhood PCA normals +
geometric-features presample (scan_registration.cpp:1136-1229, 279-327, 1481-1489) on the first 9
scan lines of one seeded synthetic VLP-16 sweep (planetary_lidar_odometry_amd/synth.py, scene 0, sensor at the origin,
noise seed 5).

Inputs: the ring-concatenated cloud xyz (laserCloud, 1064-1069) and the ring sizes.  Expected
outputs: the C++ oracle's (oracle/scanreg_oracle.cpp) rows, asserted here against the independent
numpy restatement (oracle/imls_np.py ring_pca_np): identical row indices and failure counters,
flags identical except rows whose plane-check margin is < 1e-6, unit normals |dot| > 1 − 1e-6 on
rows with equal flags.  Parity unpinned (PCL/FLANN and Eigen are not in the container).

usage: python tests/golden/make_pca_golden.py"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import plo_amd  # noqa: E402

plo_amd.load()
import imls_np  # noqa: E402
import oracle_ctypes as oc  # noqa: E402
from planetary_lidar_odometry_amd import _abi, synth  # noqa: E402


def vlp16_rings(scene_seed=0, noise_seed=5, n_rings=9):
    """The first n_rings scan lines of the sweep (ring-major order, so a prefix of the cloud)."""
    cl = synth.scan(synth.make_scene(scene_seed), synth.vlp16(), synth.pose_xyyaw(0, 0, 0), seed=noise_seed)
    ring = np.floor(cl["intensity"]).astype(np.int64)
    sizes = np.bincount(ring, minlength=16)[:n_rings].astype(np.int32)
    xyz = np.stack([cl["x"], cl["y"], cl["z"]], 1).astype(np.float32)[: int(sizes.sum())]
    return xyz, sizes


def check_against_numpy(xyz, sizes, o):
    idx, nrm, lam, fl, fail, inv = imls_np.ring_pca_np(xyz, sizes)
    assert np.array_equal(idx, o["index"].astype(np.int64)), "row indices differ"
    assert fail == o["pca_failure"], (fail, o["pca_failure"])
    flip = fl != o["flags"]
    assert np.all(o["margin"][flip] < 1e-6), "flag flips away from the plane-check boundary"
    assert abs(inv - o["plane_invalid"]) <= int(flip.sum())
    same = ~flip
    dots = np.abs(np.sum(nrm[same] * o["normal"][same], 1))
    assert dots.min() > 1 - 1e-6, dots.min()


def main():
    xyz, sizes = vlp16_rings()
    p = _abi.default_pca_params()
    o = oc.ring_pca(xyz, sizes, p)
    check_against_numpy(xyz, sizes, o)
    out = ROOT / "tests" / "golden" / "pca_vlp16.npz"
    np.savez_compressed(out, xyz=xyz, sizes=sizes, index=o["index"], normal=o["normal"], evals=o["evals"],
                        planarity=o["features"][:, 5], flags=o["flags"], margin=o["margin"],
                        counters=np.array([o["pca_failure"], o["plane_invalid"]], np.int64))
    print(f"wrote {out}: {len(xyz)} points, {len(o['index'])} rows, counters {o['pca_failure']}, {o['plane_invalid']}")


if __name__ == "__main__":
    main()
