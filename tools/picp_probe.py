"""Diagnostic: plane_ICP projection (angle gate on) vs the oracle on the committed goldens, per
traversal mode, for the library at IMLS_LIB_PATH (a variant may lack newer symbols: tolerated here).
Prints which outputs differ."""
import ctypes as C
import os
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]
import plo_amd  # noqa: E402

plo_amd.load()
from planetary_lidar_odometry_amd import _abi  # noqa: E402


class _Tolerant(C.CDLL):
    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            class _D:
                pass
            return _D()


_abi.C.CDLL = _Tolerant
from planetary_lidar_odometry_amd import imls_icp  # noqa: E402
import oracle_ctypes as oc  # noqa: E402
from test_gpu_plane_icp import golden, picp_params, soa_to_rows  # noqa: E402

for name in ("vlp16_pair", "planetary_pair"):
    g = golden(name)
    for angle in (0, 1):
        p = picp_params(angle=angle)
        with imls_icp.ImlsContext(p) as ctx:
            ctx.set_target(soa_to_rows(g["tgt"]))
            ctx.set_source(soa_to_rows(g["src"]))
            for k in (0, 1):
                x, y, n, idx, rej = ctx.project(g[f"pose{k}"])
                wx, wy, wn, widx, wrej = oc.project(g["src"], g["tgt"], g[f"pose{k}"], p)
                ok = [np.array_equal(rej, wrej), np.array_equal(idx, widx)]
                if ok[1]:
                    ok += [np.array_equal(x, wx), np.array_equal(y, wy)] + [np.array_equal(n[:, d], wn[:, d]) for d in range(3)]
                print(os.environ.get("IMLS_LIB_PATH", "new"), os.environ.get("IMLS_QWAVE", "auto"), name, angle, k, ok,
                      flush=True)
