"""Generates tests/golden/*.npz — the committed golden vectors of the IMLS-ICP path.

The reference ships no tests or fixtures and cannot be built here, so the
golden outputs come from the CPU oracle (oracle/imls_oracle.cpp) and are accepted only when the
independent numpy/scipy restatement (oracle/imls_np.py) reproduces them (asserted below).
Inputs are seeded synthetic scans (planetary-lidar-odometry_amd/synth.py).

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import plo_amd  # noqa: E402

plo_amd.load()
from planetary_lidar_odometry_amd import config, synth  # noqa: E402
import imls_np  # noqa: E402
import oracle_ctypes as oc  # noqa: E402


def np_params(p):
    return dict(r=p.r, h=p.h, normal_angle_constraint=p.normal_angle_constraint,
                angle_diff_threshold=p.angle_diff_threshold, search_number=p.search_number,
                transform_normal=p.transform_normal, iterations=p.iterations,
                correspond_number=p.correspond_number, ls_threshold=p.ls_threshold,
                delta_dist_threshold=p.delta_dist_threshold, delta_angle_threshold=p.delta_angle_threshold)


def make(name: str, model: str, map_scans: int, start: int, n_src: int, scene_kind: str = "urban"):
    pair = synth.make_pair(model, map_scans=map_scans, start=start, scene_kind=scene_kind)
    src = synth.soa(synth.fps_subsample(pair.source, n_src, seed=7))
    tgt = synth.soa(pair.target)
    # a few NaN points in both clouds exercise RemoveNANandINFData (imls_icp.cpp:58-72)
    src[0, 3] = np.nan
    tgt[1, 10] = np.inf
    p = config.bench_params(10)
    p.delta_dist_threshold = 0.001
    p.delta_angle_threshold = 0.0001745353
    out = dict(src=src, tgt=tgt, true_pose=pair.true_pose)
    poses = [np.eye(4), pair.true_pose @ synth.pose_xyyaw(0.05, -0.03, 0.004)]
    for k, pose in enumerate(poses):
        x, y, n, idx, rej = oc.project(src, tgt, pose, p)
        x2, y2, n2, idx2, rej2 = imls_np.project(src, tgt, pose, np_params(p))
        assert np.array_equal(idx, idx2) and np.array_equal(rej, rej2), f"{name}: restatements disagree (mask)"
        assert np.array_equal(x, x2) and np.array_equal(n, n2) and np.abs(y.astype(np.float64) - y2).max() <= 1e-6
        ok, D = oc.solve(0, x, y, n, p)
        D2, _ = imls_np.solve_ls(x, y, n, p.ls_threshold)
        assert ok and np.abs(D - D2).max() < 1e-9, f"{name}: LS restatements disagree {np.abs(D - D2).max()}"
        out.update({f"pose{k}": pose, f"idx{k}": idx, f"x{k}": x, f"y{k}": y, f"n{k}": n, f"rej{k}": rej, f"ls{k}": D})
    fr = oc.register_frame(src, tgt, p)
    pose_np, it_np, st_np, tr_np = imls_np.register_frame(src, tgt, np_params(p))
    assert fr["iters"] == it_np and fr["status"] == st_np, (fr["iters"], it_np, fr["status"], st_np)
    assert np.abs(fr["pose"] - pose_np).max() < 1e-7, np.abs(fr["pose"] - pose_np).max()
    out.update(frame_pose=fr["pose"], frame_iters=np.int64(fr["iters"]), frame_status=np.int64(fr["status"]),
               frame_nvalid=np.array([t.n_valid for t in fr["trace"]], np.int64),
               frame_rej=np.array([list(t.reject) for t in fr["trace"]], np.int64),
               frame_delta=np.array([np.array(t.delta).reshape(4, 4) for t in fr["trace"]]))
    np.savez_compressed(HERE / f"{name}.npz", **out)
    print(name, "src", src.shape[1], "tgt", tgt.shape[1], "valid", [len(out["idx0"]), len(out["idx1"])],
          "iters", fr["iters"], "status", fr["status"])


def tv_params(iters=10):
    """use_tensor_voting with get_normals=false in count mode (BASELINE config E)."""
    p = config.bench_params(iters)
    p.delta_dist_threshold = 0.001
    p.delta_angle_threshold = 0.0001745353
    p.get_normals = 0
    p.recompute_normal_count_mode = 1
    p.use_tensor_voting = 1
    p.tensor_k, p.tensor_sigma, p.tensor_distance_threshold = 50, 0.2, 0.6
    return p


def make_tv(name: str, n_src: int):
    """Config E fixture: VLP-16 planetary pair + the target's tensor-voting input tensors (the
    reference's PCA encoding, scan_registration.cpp:358-381).  The C++ oracle's voted normals are
    accepted only when the numpy restatement reproduces them (found flags exact, ≤ 1e-12)."""
    pair = synth.make_planetary_pair(map_scans=1, scene_seed=3, start=30)
    src = synth.soa(synth.fps_subsample(pair.source, n_src, seed=7))
    tgt = synth.soa(pair.target)
    ten = np.ascontiguousarray(pair.meta["tensors"].T)                 # (6, M)
    ev, ec = pair.meta["pca"]
    assert np.array_equal(imls_np.tv_encode_pca(ev, ec, 50).T, ten), "encode restatements disagree"
    p = tv_params()
    npp = dict(tensor_sigma=p.tensor_sigma, tensor_distance_threshold=p.tensor_distance_threshold, tensor_k=p.tensor_k)
    out = dict(src=src, tgt=tgt, ten=ten, true_pose=pair.true_pose, evals=ev, evecs=ec)
    poses = [np.eye(4), pair.true_pose @ synth.pose_xyyaw(0.05, -0.03, 0.004)]
    for k, pose in enumerate(poses):
        q = (pose[:3, :3] @ src[:3].astype(np.float64) + pose[:3, 3:]).astype(np.float32)
        nrm, found, _ = oc.tv_normals(tgt, ten, q, p)
        nrm2, found2, _ = imls_np.tv_normals(tgt, ten, q, npp)
        assert np.array_equal(found, found2), f"{name}: TV found flags disagree"
        assert np.abs(nrm - nrm2).max() <= 1e-12, f"{name}: TV normals disagree {np.abs(nrm - nrm2).max()}"
        x, y, n, idx, rej = oc.project(src, tgt, pose, p, tensors=ten)
        out.update({f"pose{k}": pose, f"tvq{k}": q, f"tvn{k}": nrm, f"tvf{k}": found, f"idx{k}": idx, f"x{k}": x,
                    f"y{k}": y, f"n{k}": n, f"rej{k}": rej})
    fr = oc.register_frame(src, tgt, p, tensors=ten)
    out.update(frame_pose=fr["pose"], frame_iters=np.int64(fr["iters"]), frame_status=np.int64(fr["status"]),
               frame_nvalid=np.array([t.n_valid for t in fr["trace"]], np.int64),
               frame_rej=np.array([list(t.reject) for t in fr["trace"]], np.int64))
    np.savez_compressed(HERE / f"{name}.npz", **out)
    print(name, "src", src.shape[1], "tgt", tgt.shape[1], "valid", [len(out["idx0"]), len(out["idx1"])],
          "found", [int(out["tvf0"].sum()), int(out["tvf1"].sum())], "iters", fr["iters"], "status", fr["status"],
          "pose err", np.abs(fr["pose"] - pair.true_pose).max())


if __name__ == "__main__":
    which = sys.argv[1:] or ["vlp16_pair", "planetary_pair", "tv_pair"]
    if "vlp16_pair" in which:
        make("vlp16_pair", "vlp16", 1, 5, 2000)
    if "planetary_pair" in which:
        make("planetary_pair", "vlp16", 1, 8, 1500, scene_kind="planetary")
    if "tv_pair" in which:
        make_tv("tv_pair", 3000)
