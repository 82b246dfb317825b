"""Import shim for the ``planetary-lidar-odometry_amd/`` package directory.

The directory name carries hyphens (it is not a legal Python identifier), so it is loaded under
the module name ``planetary_lidar_odometry_amd``:

    import plo_amd
    pkg = plo_amd.load()           # == sys.modules["planetary_lidar_odometry_amd"]
    from planetary_lidar_odometry_amd import imls_icp
"""
from __future__ import annotations

import importlib.util
import pathlib
import sys

PKG_NAME = "planetary_lidar_odometry_amd"
PKG_DIR = pathlib.Path(__file__).resolve().parent / "planetary-lidar-odometry_amd"


def load():
    mod = sys.modules.get(PKG_NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(PKG_NAME, PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    spec.loader.exec_module(mod)
    return mod
