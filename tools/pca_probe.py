"""Times imls_ring_normals_pca (the upstream producer's ring PCA normals) on one synthetic HDL-64
sweep: k_ring_pca's average duration from HIP events on its stream (timing kind 5) and the whole
call (H2D + kernels + compaction + D2H).  usage: python tools/pca_probe.py [reps]"""
import json, pathlib, sys, time
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import plo_amd
plo_amd.load()
import numpy as np
from planetary_lidar_odometry_amd import _abi, imls_icp, synth

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
xyz, sizes = synth.ring_cloud("hdl64", 0)
with imls_icp.ImlsContext(device=0) as c:
    for _ in range(3):
        r = c.ring_normals_pca(xyz, sizes)
    c.enable_timing(True); c.reset_timing()
    t = time.perf_counter()
    for _ in range(reps):
        r = c.ring_normals_pca(xyz, sizes)
    wall = (time.perf_counter() - t) / reps
    ms, n = c.kernel_timing(5)
pairs = sum(2 * int(sizes[i]) * (int(sizes[i - 1]) + int(sizes[i + 1])) / 2 for i in range(1, len(sizes) - 1))
out = {"points": int(len(xyz)), "rows": int(len(r["index"])), "kernel_ms": ms / max(n, 1), "launches": n,
       "call_ms": wall * 1e3, "points_per_s_kernel": len(xyz) / (ms / max(n, 1) / 1e3),
       "nn_pairs_per_launch": pairs, "nn_Gpairs_per_s": pairs / (ms / max(n, 1) / 1e3) / 1e9}
print(json.dumps(out))
