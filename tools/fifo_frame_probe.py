"""Tree-quality probe of the FIFO index's quantisation frame (index.hip k_fifo_frame), on the CPU:
config B's map (synth, the bench's pair 0) Morton-sorted under a candidate frame, 64-point leaves,
the implicit binary tree over them; the cost proxy is the number of leaves / nodes whose box meets
each sampled query's ball of its 20th-neighbour distance (what a kNN traversal must visit).  The
full build's frame (origin = bbox min, side = largest extent) is the reference row."""
import pathlib
import sys

import numpy as np
from scipy.spatial import cKDTree

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import plo_amd  # noqa: E402

plo_amd.load()
from planetary_lidar_odometry_amd import synth  # noqa: E402


def spread(v):
    v = v.astype(np.uint64)
    out = np.zeros_like(v)
    for b in range(16):
        out |= ((v >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b)
    return out


def cost(P, Q, R, org, sc, B=64):
    q = np.clip((P - np.asarray(org, np.float32)) * np.float32(sc), 0, 65535).astype(np.uint32)
    k = spread(q[:, 0]) | (spread(q[:, 1]) << np.uint64(1)) | (spread(q[:, 2]) << np.uint64(2))
    X = P[np.argsort(k, kind="stable")]
    L = (len(X) + B - 1) // B
    Xp = np.concatenate([X, np.repeat(X[-1:], L * B - len(X), 0)]).reshape(L, B, 3)
    lo, hi = Xp.min(1), Xp.max(1)
    n = 1
    while n < L:
        n *= 2
    lo = np.concatenate([lo, np.full((n - L, 3), np.inf)])
    hi = np.concatenate([hi, np.full((n - L, 3), -np.inf)])
    leaf = total = 0
    first = True
    while True:
        d = np.maximum(np.maximum(lo[None] - Q[:, None], Q[:, None] - hi[None]), 0)
        hit = ((d * d).sum(2) <= (R * R)[:, None]).sum()
        leaf = hit if first else leaf
        first = False
        total += hit
        if len(lo) == 1:
            return leaf / len(Q), total / len(Q)
        lo, hi = np.minimum(lo[0::2], lo[1::2]), np.maximum(hi[0::2], hi[1::2])


def main():
    pair = synth.make_pairs(1, "hdl64", map_scans=10, scene_seed=0, traj_seed=2000, noise_seed=1000)[0]
    P = np.stack([pair.target["x"], pair.target["y"], pair.target["z"]], 1).astype(np.float32)
    P = P[np.isfinite(P).all(1)]
    S = np.stack([pair.source["x"], pair.source["y"], pair.source["z"]], 1).astype(np.float32)
    S = S[np.isfinite(S).all(1)]
    Q = S[np.random.default_rng(0).choice(len(S), 3000, replace=False)]
    R = np.minimum(cKDTree(P).query(Q, 20)[0][:, -1], 1.0)
    lo, hi = P.min(0), P.max(0)
    e = float((hi - lo).max())
    frames = {
        "full build (bbox min, side e)": (lo, 65535 / e),
        "FIFO: bbox min - e/2, side 2e": (lo - 0.5 * e, 65535 / (2 * e)),
        "1.5e cube centred on the bbox": ((lo + hi) / 2 - 0.75 * e, 65535 / (1.5 * e)),
        "bbox min - e/4, side 1.5e": (lo - 0.25 * e, 65535 / (1.5 * e)),
    }
    for name, (org, sc) in frames.items():
        lf, tot = cost(P, Q, R, org, sc)
        print(f"{name:32s} leaves/query {lf:6.2f}  nodes/query {tot:6.2f}", flush=True)


if __name__ == "__main__":
    main()
