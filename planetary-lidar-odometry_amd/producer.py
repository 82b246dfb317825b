"""Upstream producer for the registration path: scan_registration.cpp's per-sweep chain for the
shipped config (config.json scan_registration: compute_normal_method "pca" → presample_method
"geometric_features" → sample_method "major_axis"), on the GPU through the C ABI.

  ScanRegistration.process_raw(raw) the whole handler: scan_front_end (NaN / range filter, ring
                                    assignment and relative time, 862-1069) → process
  ScanRegistration.process(sweep)   laserCloudHandler's tail (scan_registration.cpp:1136-1229 normals,
                                    1448-1461 + 1481-1489 presample, 1494-1503 sampling) → the two
                                    clouds laser_odometry consumes: pcl_cloud (/laser_cloud_filtered,
                                    the map FIFO's input) and pcl_surface_cloud (/laser_cloud_flat,
                                    the registration's source)

The sweep comes in ring-concatenated order (`laserCloud`, 1064-1069) with the points per scan
line.  Sampling follows samplePointCloud's dispatch (761-806): "major_axis" samples its first frame
with the "normal" method (frame == 1, 783) and every later one against the previous pcl_cloud.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from . import _abi
from .imls_icp import ImlsContext
from .synth import POINT_DTYPE


class ScanRegistration:
    def __init__(self, ctx: Optional[ImlsContext] = None, device: int = 0,
                 pca_params: Optional[_abi.ImlsPcaParams] = None, sample_method: str = "major_axis",
                 shuffle_seed: int = 0, rand_seed: int = 1):
        if sample_method not in ("major_axis", "normal"):
            raise ValueError(f"sample_method {sample_method!r}: the GPU producer ships 'major_axis' and 'normal'")
        self._own = ctx is None
        self.ctx = ctx if ctx is not None else ImlsContext(device=device)
        self.pca_params = pca_params if pca_params is not None else _abi.default_pca_params()
        self.sample_method = sample_method
        self.shuffle_seed = shuffle_seed
        self.rand_seed = rand_seed
        self.frame = 1                      # scan_registration.cpp:64
        self.last_xyz: Optional[np.ndarray] = None
        self.last_pca: Optional[dict] = None

    def close(self):
        if self._own:
            self.ctx.close()

    def sample_params(self) -> _abi.ImlsSampleParams:
        first = self.sample_method == "normal" or self.frame == 1
        sp = _abi.default_sample_params(_abi.IMLS_SAMPLE_NORMAL if first else _abi.IMLS_SAMPLE_MAJOR_AXIS)
        sp.shuffle_seed = (self.shuffle_seed + 7919 * self.frame) & 0xFFFFFFFF
        sp.rand_seed = (self.rand_seed + self.frame - 1) & 0xFFFFFFFF
        return sp

    def process_raw(self, raw_xyz, front_params: Optional[_abi.ImlsFrontParams] = None):
        """The whole laserCloudHandler on a raw sweep (driver order, (n, 3+) float32): the front end
        (NaN / range filter, ring assignment, relative time; 862-1069) then process()."""
        xyz, inten, _, sizes = self.ctx.scan_front_end(raw_xyz, front_params)
        return self.process(xyz, sizes, inten)

    def process(self, xyz, ring_sizes, intensity=None):
        """One sweep → (pcl_cloud, pcl_surface_cloud) as POINT_DTYPE arrays (48-byte
        pcl::PointXYZINormal records)."""
        xyz = np.ascontiguousarray(np.asarray(xyz, np.float32)[:, :3])
        o = self.ctx.ring_normals_pca(xyz, ring_sizes, self.pca_params)
        idx = o["index"].astype(np.int64)
        cloud = np.zeros(len(idx), POINT_DTYPE)
        cloud["x"], cloud["y"], cloud["z"] = xyz[idx, 0], xyz[idx, 1], xyz[idx, 2]
        cloud["normal_x"], cloud["normal_y"], cloud["normal_z"] = o["normal"][:, 0], o["normal"][:, 1], o["normal"][:, 2]
        if intensity is not None:
            cloud["intensity"] = np.asarray(intensity, np.float32)[idx]
        cand = np.nonzero(o["flags"] & _abi.IMLS_PCA_CANDIDATE)[0].astype(np.int32)
        fxyz = np.stack([cloud["x"], cloud["y"], cloud["z"]], 1)
        sampled, _ = self.ctx.sample_point_cloud(fxyz, o["normal"], cand, self.last_xyz, self.sample_params())
        surface = cloud[sampled]
        self.frame += 1
        self.last_xyz = fxyz
        self.last_pca = o
        return cloud, surface


def sweep_inputs(cloud: np.ndarray, n_rings: int):
    """A synth.scan sweep (ring-major POINT_DTYPE, intensity = scanID + 0.1·relTime) as the
    producer's inputs: xyz (n, 3) float32, points per ring, intensity."""
    sizes = np.bincount(np.floor(cloud["intensity"]).astype(np.int64), minlength=n_rings).astype(np.int32)
    xyz = np.stack([cloud["x"], cloud["y"], cloud["z"]], 1).astype(np.float32)
    return xyz, sizes, cloud["intensity"].copy()
