"""Latency probe of the shipped solver's deployment call: LaserOdometry.process
one frame at a time with RANSAC → DRPM (config.json's solver), on the config C/D-like stream frames
(≤2000-query flat cloud vs the previous 118k-point filtered scan, 20 ICP iterations).  Prints the
median / p90 wall time per call; run under rocprofv3 --kernel-trace --stats for the per-kernel split
(tools/iter_profile_frame.py groups a trace per frame)."""
import ctypes as C
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (loads the library)
import numpy as np  # noqa: E402
from planetary_lidar_odometry_amd import imls_icp  # noqa: E402

p = bench.solver_params("RANSAC_DRPM", 20)
runner = bench.StreamRunner(1, p, 0, 0, frames_per_seq=6, fuse=False, unique=1, dev=None, resident=False, groups=1)
fr = runner.seqs[0]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
lat, iters = [], []
with imls_icp.LaserOdometry(p, device=0) as lo:
    for j in range(n + 3):
        k = j % len(fr)
        t0 = time.perf_counter()
        r = lo.process(fr[k][0], fr[k][1])
        if j >= 3:
            lat.append((time.perf_counter() - t0) * 1e3)
            if r is not None:
                iters.append(r["iters"])
    print(f"LaserOdometry.process RANSAC->DRPM: median {np.median(lat):.3f} ms  p90 {np.percentile(lat, 90):.3f} ms "
          f"(pipelined {lo.pipelined}, {len(fr[0][1])} queries vs {len(fr[0][0])}-pt scan, iterations {np.mean(iters):.1f})")
lib = runner.ctxs[0].lib if hasattr(runner, "ctxs") else None
runner.close()
if lib is not None and hasattr(lib, "imls_debug_ransac"):   # the DEBUG_WAVE_TRACE build (IMLS_LIB_PATH)
    buf = np.zeros(16, np.uint64)
    lib.imls_debug_ransac(C.c_void_p(buf.ctypes.data))
    nh, nd = max(int(buf[6]), 1), max(int(buf[14]), 1)
    print("  k_ransac_hyp block 0, ticks (100 MHz) per call:",
          {k: round(float(buf[i]) / nh, 1) for i, k in enumerate(["rng+pass1", "pass2", "qr", "delta", "count"])})
    print("  k_drpm_head_small, ticks per call:",
          {k: round(float(buf[8 + i]) / nd, 1) for i, k in enumerate(["select", "compact", "pass1", "slab sum", "eig"])},
          "Jacobi sweeps per call", round(float(buf[13]) / nd, 2))
