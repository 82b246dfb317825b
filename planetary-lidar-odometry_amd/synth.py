"""Seeded synthetic LiDAR scans for the IMLS-ICP registration path.

The reference has no datasets in-tree and no network is available, so every
benchmark and parity input is generated here, deterministically, from integer seeds.

Scan models:
  * HDL-64: 64 rings evenly spaced over [+2°, −24.33°] (the 64-beam bounds the reference's
    scan_registration.cpp:926-930 uses), 0.18° azimuth step (2000 columns, 128k rays).
  * VLP-16: 16 rings at −15°…+15° step 2° (scan_registration.cpp:948-950), 0.4° azimuth.

Every returned point carries the analytic normal of the primitive it hit plus N(0, 0.01)
noise, renormalised and flipped so that n·z ≥ 0 — the orientation rule of the reference's
PCA normals (scan_registration.cpp:1196-1200).  Points are float32, laid out as the
reference's 48-byte ``pcl::PointXYZINormal`` record (common.h:17):
``x y z pad | nx ny nz pad | intensity curvature pad pad``.

Scenes:
  * ``urban``: ground plane z = −1.73 m (sensor 1.73 m above it), rotated box buildings on
    both sides of a road along +x, parked "cars", poles.
  * ``planetary``: feature-poor terrain (sum of sinusoids + gaussian boulders), no buildings
    (BASELINE config E); ray/heightfield intersection by bisection on the ray.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

# 48-byte AoS record matching pcl::PointXYZINormal (common.h:17).
POINT_DTYPE = np.dtype([
    ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("_p0", "<f4"),
    ("normal_x", "<f4"), ("normal_y", "<f4"), ("normal_z", "<f4"), ("_p1", "<f4"),
    ("intensity", "<f4"), ("curvature", "<f4"), ("_p2", "<f4"), ("_p3", "<f4"),
])
assert POINT_DTYPE.itemsize == 48


@dataclass
class ScanModel:
    rings: np.ndarray          # elevation of each ring, degrees
    azimuth_step_deg: float
    min_range: float
    max_range: float
    range_noise: float = 0.02
    xyz_jitter: float = 1e-4


def hdl64() -> ScanModel:
    return ScanModel(np.linspace(2.0, -24.33, 64), 0.18, 2.0, 120.0)


def vlp16() -> ScanModel:
    return ScanModel(np.arange(-15.0, 15.0 + 1e-9, 2.0), 0.4, 0.5, 100.0)


# --------------------------------------------------------------------------------------------
# Scene
# --------------------------------------------------------------------------------------------
GROUND_Z = -1.73


@dataclass
class Scene:
    kind: str
    boxes: np.ndarray        # (B, 8): cx, cy, cz, hx, hy, hz, yaw, unused
    poles: np.ndarray        # (P, 4): cx, cy, radius, height
    terrain: np.ndarray      # (T, 4) sinusoid terms a, kx, ky, phase   (planetary)
    boulders: np.ndarray     # (Q, 4) cx, cy, amp, sigma                  (planetary)


def make_scene(seed: int = 0, kind: str = "urban", extent: float = 400.0) -> Scene:
    rng = np.random.default_rng(seed)
    boxes, poles = [], []
    terrain = np.zeros((0, 4))
    boulders = np.zeros((0, 4))
    if kind == "urban":
        # buildings on both sides of a road along x ∈ [-150, extent]
        x = -150.0
        while x < extent:
            for side in (-1.0, 1.0):
                w = rng.uniform(8, 25)       # along road
                d = rng.uniform(8, 20)       # depth
                h = rng.uniform(4, 18)
                off = rng.uniform(9, 16)
                yaw = rng.normal(0, 0.12)
                cy = side * (off + d / 2)
                boxes.append([x + w / 2, cy, GROUND_Z + h / 2, w / 2, d / 2, h / 2, yaw, 0])
            x += rng.uniform(14, 32)
        # parked cars
        for _ in range(int((extent + 150) / 9)):
            cx = rng.uniform(-150, extent)
            cy = rng.choice([-1, 1]) * rng.uniform(4.0, 6.5)
            boxes.append([cx, cy, GROUND_Z + 0.75, 2.25, 0.9, 0.75, rng.normal(0, 0.05), 0])
        # poles
        for _ in range(int((extent + 150) / 6)):
            cx = rng.uniform(-150, extent)
            cy = rng.choice([-1, 1]) * rng.uniform(7.0, 8.5)
            poles.append([cx, cy, rng.uniform(0.12, 0.3), rng.uniform(4, 8)])
    elif kind == "planetary":
        n = 3
        terrain = np.stack([rng.uniform(0.2, 1.0, n), rng.uniform(0.02, 0.12, n) * rng.choice([-1, 1], n),
                            rng.uniform(0.02, 0.12, n) * rng.choice([-1, 1], n), rng.uniform(0, 2 * np.pi, n)], 1)
        q = int(extent / 2)
        boulders = np.stack([rng.uniform(-150, extent, q), rng.uniform(-120, 120, q),
                             rng.uniform(0.2, 1.2, q), rng.uniform(0.4, 2.0, q)], 1)
    else:
        raise ValueError(kind)
    b = np.asarray(boxes, dtype=np.float64).reshape(-1, 8)
    p = np.asarray(poles, dtype=np.float64).reshape(-1, 4)
    return Scene(kind, b, p, terrain, boulders)


def _terrain_height(scene: Scene, x, y):
    z = np.full(np.broadcast(x, y).shape, GROUND_Z)
    for a, kx, ky, ph in scene.terrain:
        z = z + a * np.sin(kx * x + ky * y + ph)
    for cx, cy, amp, sg in scene.boulders:
        z = z + amp * np.exp(-((x - cx) ** 2 + (y - cy) ** 2) / (2 * sg * sg))
    return z


def _terrain_grad(scene: Scene, x, y):
    gx = np.zeros(np.broadcast(x, y).shape)
    gy = np.zeros_like(gx)
    for a, kx, ky, ph in scene.terrain:
        c = a * np.cos(kx * x + ky * y + ph)
        gx += c * kx
        gy += c * ky
    for cx, cy, amp, sg in scene.boulders:
        e = amp * np.exp(-((x - cx) ** 2 + (y - cy) ** 2) / (2 * sg * sg))
        gx += -e * (x - cx) / (sg * sg)
        gy += -e * (y - cy) / (sg * sg)
    return gx, gy


def _cast(scene: Scene, o: np.ndarray, d: np.ndarray, max_range: float):
    """Ray cast rays (origin o (3,), unit dirs d (R,3)) → t (R,), normals (R,3). inf = miss."""
    R = d.shape[0]
    t_best = np.full(R, np.inf)
    n_best = np.zeros((R, 3))
    if scene.kind == "urban":
        # ground plane
        with np.errstate(divide="ignore", invalid="ignore"):
            tg = (GROUND_Z - o[2]) / d[:, 2]
        hit = (d[:, 2] < -1e-9) & (tg > 0)
        t_best = np.where(hit, tg, t_best)
        n_best[hit] = (0.0, 0.0, 1.0)
        # boxes (yawed): transform ray to box frame, slab test
        for cx, cy, cz, hx, hy, hz, yaw, _ in scene.boxes:
            c, s = math.cos(yaw), math.sin(yaw)
            ox, oy, oz = o[0] - cx, o[1] - cy, o[2] - cz
            lox, loy = c * ox + s * oy, -s * ox + c * oy
            ldx, ldy = c * d[:, 0] + s * d[:, 1], -s * d[:, 0] + c * d[:, 1]
            ldz = d[:, 2]
            with np.errstate(divide="ignore", invalid="ignore"):
                t1x, t2x = (-hx - lox) / ldx, (hx - lox) / ldx
                t1y, t2y = (-hy - loy) / ldy, (hy - loy) / ldy
                t1z, t2z = (-hz - oz) / ldz, (hz - oz) / ldz
            tminx, tmaxx = np.minimum(t1x, t2x), np.maximum(t1x, t2x)
            tminy, tmaxy = np.minimum(t1y, t2y), np.maximum(t1y, t2y)
            tminz, tmaxz = np.minimum(t1z, t2z), np.maximum(t1z, t2z)
            tmin = np.maximum(np.maximum(tminx, tminy), tminz)
            tmax = np.minimum(np.minimum(tmaxx, tmaxy), tmaxz)
            h = (tmax >= tmin) & (tmin > 0) & (tmin < t_best)
            if not h.any():
                continue
            idx = np.nonzero(h)[0]
            tm = tmin[idx]
            # which face: the axis whose tmin equals tmin
            ax = np.argmax(np.stack([tminx[idx], tminy[idx], tminz[idx]], 1), axis=1)
            ln = np.zeros((idx.size, 3))
            sgn = np.stack([-np.sign(ldx[idx]), -np.sign(ldy[idx]), -np.sign(ldz[idx])], 1)
            ln[np.arange(idx.size), ax] = sgn[np.arange(idx.size), ax]
            wn = np.stack([c * ln[:, 0] - s * ln[:, 1], s * ln[:, 0] + c * ln[:, 1], ln[:, 2]], 1)
            t_best[idx] = tm
            n_best[idx] = wn
        # poles (vertical cylinders from ground up to height)
        for cx, cy, rad, ht in scene.poles:
            ox, oy = o[0] - cx, o[1] - cy
            a = d[:, 0] ** 2 + d[:, 1] ** 2
            b = 2 * (ox * d[:, 0] + oy * d[:, 1])
            cc = ox * ox + oy * oy - rad * rad
            disc = b * b - 4 * a * cc
            ok = (disc > 0) & (a > 1e-12)
            if not ok.any():
                continue
            with np.errstate(invalid="ignore", divide="ignore"):
                tt = (-b - np.sqrt(np.where(ok, disc, 0))) / (2 * a)
            z = o[2] + tt * d[:, 2]
            h = ok & (tt > 0) & (tt < t_best) & (z >= GROUND_Z) & (z <= GROUND_Z + ht)
            if not h.any():
                continue
            idx = np.nonzero(h)[0]
            px = ox + tt[idx] * d[idx, 0]
            py = oy + tt[idx] * d[idx, 1]
            nn = np.stack([px / rad, py / rad, np.zeros(idx.size)], 1)
            t_best[idx] = tt[idx]
            n_best[idx] = nn
    else:
        # heightfield: march then bisect (rays going down only hit reliably; rays up miss).  Only
        # the boulders within reach of this sensor position and only the still-marching rays are
        # evaluated per step (a full scan takes seconds, not minutes).
        bsub = scene.boulders
        if len(bsub):
            reach = max_range + 6.0 * bsub[:, 3] + 2.0     # exp(−d²/2σ²) < 1e-10 beyond
            bsub = bsub[np.hypot(bsub[:, 0] - o[0], bsub[:, 1] - o[1]) < reach]
        sub = Scene(scene.kind, scene.boxes, scene.poles, scene.terrain, bsub)
        t = np.full(R, np.inf)
        fprev = o[2] - _terrain_height(sub, o[0] + 0 * d[:, 0], o[1] + 0 * d[:, 1])
        step = 0.25
        act = np.nonzero(fprev > 0)[0]
        fprev = fprev[act]
        tk = 0.0
        while tk < max_range and act.size:
            tk += step
            p = o[None, :] + tk * d[act]
            f = p[:, 2] - _terrain_height(sub, p[:, 0], p[:, 1])
            cross = f <= 0
            if cross.any():
                ci = act[cross]
                dc = d[ci]
                lo, hi = np.full(ci.size, tk - step), np.full(ci.size, tk)
                for _ in range(30):
                    mid = 0.5 * (lo + hi)
                    pm = o[None, :] + mid[:, None] * dc
                    fm = pm[:, 2] - _terrain_height(sub, pm[:, 0], pm[:, 1])
                    lo = np.where(fm > 0, mid, lo)
                    hi = np.where(fm > 0, hi, mid)
                t[ci] = 0.5 * (lo + hi)
                act, f = act[~cross], f[~cross]
            fprev = f
            step = min(1.0, 0.25 + tk * 0.01)
        hit = np.isfinite(t)
        p = o[None, :] + np.where(hit, t, 0)[:, None] * d
        gx, gy = _terrain_grad(sub, p[:, 0], p[:, 1])
        nn = np.stack([-gx, -gy, np.ones(R)], 1)
        nn /= np.linalg.norm(nn, axis=1, keepdims=True)
        t_best = t
        n_best = nn
    return t_best, n_best


# --------------------------------------------------------------------------------------------
# Poses
# --------------------------------------------------------------------------------------------
def pose_xyyaw(x: float, y: float, yaw: float, z: float = 0.0, roll: float = 0.0, pitch: float = 0.0):
    cr, sr = math.cos(roll), math.sin(roll)
    cp, sp = math.cos(pitch), math.sin(pitch)
    cy, sy = math.cos(yaw), math.sin(yaw)
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    T = np.eye(4)
    T[:3, :3] = Rz @ Ry @ Rx
    T[:3, 3] = (x, y, z)
    return T


def trajectory(n: int, seed: int = 2000, step: float = 1.0, yaw_step_deg: float = 0.5):
    """≈1 m/frame forward with ±yaw_step_deg yaw per frame."""
    rng = np.random.default_rng(seed)
    poses = []
    x = y = yaw = 0.0
    for _ in range(n):
        poses.append(pose_xyyaw(x, y, yaw, 0.0, rng.normal(0, 0.002), rng.normal(0, 0.002)))
        yaw += math.radians(rng.uniform(-yaw_step_deg, yaw_step_deg))
        x += step * math.cos(yaw)
        y += step * math.sin(yaw)
    return poses


# --------------------------------------------------------------------------------------------
# Scans
# --------------------------------------------------------------------------------------------
def raw_sweep(scene: Scene, model: ScanModel, pose: np.ndarray, seed: int, start_deg: float = 0.0,
              n_nan: int = 0, n_close: int = 0) -> np.ndarray:
    """The same sweep as a lidar driver emits it (what scan_registration's front end receives):
    (n, 3) float32 x y z in firing order — azimuth-major (clockwise), every ring at each step — starting at
    azimuth `start_deg`; optionally `n_nan` NaN returns and `n_close` returns inside 0.3 m spread in."""
    cloud, flat = scan(scene, model, pose, seed, return_index=True)
    n_az = len(np.arange(0.0, 360.0, model.azimuth_step_deg))
    ring, az = flat // n_az, flat % n_az
    az0 = int(round(start_deg / model.azimuth_step_deg)) % n_az
    order = np.lexsort((ring, (az0 - az) % n_az))      # clockwise (Velodyne): −atan2(y, x) increases
    xyz = np.stack([cloud["x"], cloud["y"], cloud["z"]], 1)[order].astype(np.float32)
    rng = np.random.default_rng(seed + 17)
    for k in range(n_nan + n_close):
        at = int(rng.integers(0, len(xyz) + 1))
        pt = np.full((1, 3), np.nan, np.float32) if k < n_nan else (rng.normal(0, 0.1, (1, 3))).astype(np.float32)
        xyz = np.concatenate([xyz[:at], pt, xyz[at:]])
    return xyz


def scan(scene: Scene, model: ScanModel, pose: np.ndarray, seed: int, return_index: bool = False):
    """One sweep from sensor pose (4×4 world←sensor), returned in the SENSOR frame as a
    POINT_DTYPE array in ring-major order (like the reference's scan-ring ordering).  return_index:
    also the flat (ring·n_azimuth + azimuth) index of every returned point."""
    rng = np.random.default_rng(seed)
    el = np.radians(model.rings)
    az = np.radians(np.arange(0.0, 360.0, model.azimuth_step_deg))
    E, A = np.meshgrid(el, az, indexing="ij")
    dl = np.stack([np.cos(E) * np.cos(A), np.cos(E) * np.sin(A), np.sin(E)], -1).reshape(-1, 3)
    ring = np.repeat(np.arange(len(el)), len(az)).astype(np.float64)
    rel_t = np.tile(np.arange(len(az)) / len(az), len(el))
    R, t = pose[:3, :3], pose[:3, 3]
    dw = dl @ R.T
    tt, nw = _cast(scene, t, dw, model.max_range)
    ok = np.isfinite(tt) & (tt >= model.min_range) & (tt <= model.max_range)
    tt = tt[ok]
    nl = nw[ok] @ R           # world normal → sensor frame
    dl = dl[ok]
    rng_noise = rng.normal(0.0, model.range_noise, tt.size)
    p = dl * (tt + rng_noise)[:, None] + rng.normal(0.0, model.xyz_jitter, (tt.size, 3))
    nl = nl + rng.normal(0.0, 0.01, nl.shape)
    nl /= np.linalg.norm(nl, axis=1, keepdims=True)
    nl[nl[:, 2] < 0] *= -1.0
    out = np.zeros(tt.size, POINT_DTYPE)
    out["x"], out["y"], out["z"] = p[:, 0], p[:, 1], p[:, 2]
    out["normal_x"], out["normal_y"], out["normal_z"] = nl[:, 0], nl[:, 1], nl[:, 2]
    out["intensity"] = ring[ok] + 0.1 * rel_t[ok]   # scanID + 0.1·relTime (scan_registration.cpp:1042)
    if return_index:
        return out, np.nonzero(ok)[0]
    return out


def transform_cloud(cloud: np.ndarray, T: np.ndarray, rotate_normals: bool = True) -> np.ndarray:
    out = cloud.copy()
    p = np.stack([cloud["x"], cloud["y"], cloud["z"]], 1).astype(np.float64)
    q = p @ T[:3, :3].T + T[:3, 3]
    out["x"], out["y"], out["z"] = q[:, 0], q[:, 1], q[:, 2]
    if rotate_normals:
        n = np.stack([cloud["normal_x"], cloud["normal_y"], cloud["normal_z"]], 1).astype(np.float64)
        m = n @ T[:3, :3].T
        out["normal_x"], out["normal_y"], out["normal_z"] = m[:, 0], m[:, 1], m[:, 2]
    return out


@dataclass
class Pair:
    source: np.ndarray          # POINT_DTYPE, scan k in its own frame
    target: np.ndarray          # POINT_DTYPE, map: scans k-Q..k-1 in the frame of scan k-1
    true_pose: np.ndarray       # 4×4: frame(k-1) ← frame(k), what ICP should recover
    meta: dict


def make_pair(model: str = "hdl64", map_scans: int = 10, scene_seed: int = 0, traj_seed: int = 2000,
              noise_seed: int = 1000, scene_kind: str = "urban", start: int = 30) -> Pair:
    """Scan-to-map pair: the map is the previous ``map_scans`` scans expressed
    in the frame of scan k−1 (the synthetic config-B convention, Q12); source is scan k."""
    sm = hdl64() if model == "hdl64" else vlp16()
    scene = make_scene(scene_seed, scene_kind)
    poses = trajectory(start + 1, traj_seed)
    k = start
    Tk1_inv = np.linalg.inv(poses[k - 1])
    parts = []
    for j in range(k - map_scans, k):
        s = scan(scene, sm, poses[j], noise_seed + j)
        parts.append(transform_cloud(s, Tk1_inv @ poses[j]))
    target = np.concatenate(parts)
    source = scan(scene, sm, poses[k], noise_seed + k)
    true_pose = Tk1_inv @ poses[k]
    return Pair(source, target, true_pose,
                dict(model=model, map_scans=map_scans, scene_seed=scene_seed, traj_seed=traj_seed,
                     noise_seed=noise_seed, scene_kind=scene_kind, start=start,
                     part_sizes=[len(q) for q in parts]))


def make_pairs(n: int, model: str = "hdl64", map_scans: int = 10, scene_seed: int = 0, traj_seed: int = 2000,
               noise_seed: int = 1000, scene_kind: str = "urban", start: int = 30) -> list:
    """`n` consecutive scan-to-map pairs of one trajectory (frames start … start+n−1), generating
    each scan once: pair j registers scan start+j against scans start+j−map_scans … start+j−1
    expressed in the frame of scan start+j−1 (same convention as make_pair)."""
    sm = hdl64() if model == "hdl64" else vlp16()
    scene = make_scene(scene_seed, scene_kind)
    poses = trajectory(start + n, traj_seed)
    scans = {k: scan(scene, sm, poses[k], noise_seed + k) for k in range(start - map_scans, start + n)}
    out = []
    for j in range(n):
        k = start + j
        Tk1_inv = np.linalg.inv(poses[k - 1])
        parts = [transform_cloud(scans[i], Tk1_inv @ poses[i]) for i in range(k - map_scans, k)]
        target = np.concatenate(parts)
        out.append(Pair(scans[k], target, Tk1_inv @ poses[k],
                        dict(model=model, map_scans=map_scans, scene_seed=scene_seed, traj_seed=traj_seed,
                             noise_seed=noise_seed, scene_kind=scene_kind, start=k,
                             part_sizes=[len(q) for q in parts])))
    return out


def map_parts(pair: "Pair") -> list:
    """The map's scans (views into pair.target, oldest first; meta part_sizes), for a device FIFO
    filled scan by scan (accumulateTargetCloud, laser_odometry.cpp:116-136)."""
    sizes = pair.meta.get("part_sizes") or [len(pair.target)]
    return np.split(pair.target, np.cumsum(sizes)[:-1])


def soa(cloud: np.ndarray) -> np.ndarray:
    """(6, N) float32 SoA: x, y, z, nx, ny, nz."""
    return np.stack([cloud[f] for f in ("x", "y", "z", "normal_x", "normal_y", "normal_z")]).astype(np.float32)


def fps_subsample(cloud: np.ndarray, n: int, seed: int = 0) -> np.ndarray:
    """Seeded farthest-point subsample (the realistic ≤2000-query variant, config.json major_axis
    max_total_points)."""
    if cloud.size <= n:
        return cloud.copy()
    rng = np.random.default_rng(seed)
    p = np.stack([cloud["x"], cloud["y"], cloud["z"]], 1).astype(np.float64)
    idx = [int(rng.integers(cloud.size))]
    d = np.linalg.norm(p - p[idx[0]], axis=1)
    for _ in range(n - 1):
        j = int(np.argmax(d))
        idx.append(j)
        d = np.minimum(d, np.linalg.norm(p - p[j], axis=1))
    return cloud[np.sort(np.asarray(idx))]


def pca_features(cloud: np.ndarray, k: int = 15):
    """Per-point PCA features as scan_registration.cpp:158-229 produces them (covariance of the
    neighbourhood / (count − 1), SelfAdjointEigenSolver, eigenvalues re-ordered λ1 ≥ λ2 ≥ λ3 with
    the eigenvector columns swapped to match, 220-226), laid out like 1202-1207: evals (n, 3) and
    evecs (n, 9) = the 3×3 eigenvector matrix column-major (e1 = largest, e2, e3 = normal).
    The neighbourhood here is the k nearest points (the reference takes ring windows of 3 scan
    lines) — synthetic input for config E, not a restatement of the ring search."""
    from scipy.spatial import cKDTree
    p = np.stack([cloud["x"], cloud["y"], cloud["z"]], 1).astype(np.float32)
    _, nb = cKDTree(p.astype(np.float64)).query(p.astype(np.float64), k=min(k, len(p)))
    g = p[nb]                                                    # (n, k, 3) float32
    c = g - g.mean(axis=1, keepdims=True)
    cov = np.einsum("nki,nkj->nij", c, c) / np.float32(g.shape[1] - 1)
    w, v = np.linalg.eigh(cov.astype(np.float64))               # ascending
    w, v = w[:, ::-1].astype(np.float32), v[:, :, ::-1].astype(np.float32)
    evecs = np.transpose(v, (0, 2, 1)).reshape(-1, 9)            # column-major: e1 | e2 | e3
    return np.ascontiguousarray(w), np.ascontiguousarray(evecs)


def make_planetary_pair(map_scans: int = 1, scene_seed: int = 3, start: int = 30, tensor_k: int = 50,
                        pca_k: int = 15):
    """BASELINE config E: sparse VLP-16 scans over the procedural planetary heightfield; the
    target additionally carries tensor-voting input tensors — the reference's own encoding of
    per-point PCA features (CustomTensorVoting, scan_registration.cpp:358-381, restated by
    imls_icp.tv_encode_pca) — that VoteForAny reads through encode(AWARE_TENSOR)."""
    from . import imls_icp
    pr = make_pair("vlp16", map_scans=map_scans, scene_seed=scene_seed, scene_kind="planetary", start=start)
    evals, evecs = pca_features(pr.target, pca_k)
    pr.meta["tensors"] = imls_icp.tv_encode_pca(evals, evecs, tensor_k)
    pr.meta["pca"] = (evals, evecs)
    return pr


def ring_cloud(model: str = "hdl64", scene_seed: int = 0, noise_seed: int | None = None):
    """One sweep at the origin as the upstream producer's input: the ring-concatenated cloud
    `laserCloud` (scan_registration.cpp:1064-1069) as (n, 3) float32 xyz, plus the points per scan
    line (laserCloudScans[i].size())."""
    m = hdl64() if model == "hdl64" else vlp16()
    cl = scan(make_scene(scene_seed), m, pose_xyyaw(0, 0, 0), seed=1000 + scene_seed if noise_seed is None else noise_seed)
    sizes = np.bincount(np.floor(cl["intensity"]).astype(np.int64), minlength=len(m.rings)).astype(np.int32)
    return np.stack([cl["x"], cl["y"], cl["z"]], 1).astype(np.float32), sizes
