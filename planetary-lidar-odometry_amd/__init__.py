"""MI355X-native IMLS-ICP registration path (drop-in for the reference's Matching/Solving loop).

Layout:
  csrc/      hand-written HIP kernels for gfx950 + the C ABI (include/imls_gpu.h) → libimls_gpu.so
  _abi.py    ctypes mirror of the C ABI
  imls_icp.py  host-side mirror of the reference operator interface (IMLSICPMatcher,
             SolveMotionEstimationProblem*, solveMotionEstimationProblem, register_frame)
  config.py  config.json (laser_odometry section) ↔ imls_params
  synth.py   seeded synthetic LiDAR scans (HDL-64 / VLP-16)
"""
from . import _abi  # noqa: F401
from . import config  # noqa: F401
from . import synth  # noqa: F401

__all__ = ["_abi", "config", "synth"]
