"""Times the upstream producer on the GPU for one synthetic HDL-64 frame pair: ring PCA normals +
presample (imls_ring_normals_pca, k_ring_pca) on both sweeps, then major_axis sampling of frame 1
against frame 0 (imls_sample_point_cloud, k_major_avg + k_fps).  Kernel averages from HIP events on
the context stream (timing kinds 5 and 6); call times include host bookkeeping and PCIe.
usage: python tools/producer_probe.py [reps]"""
import json, pathlib, sys, time
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import plo_amd
plo_amd.load()
import numpy as np
from planetary_lidar_odometry_amd import _abi, imls_icp, synth

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
m = synth.hdl64()
sc = synth.make_scene(0)
frames = []
for k in (0, 1):
    cl = synth.scan(sc, m, synth.pose_xyyaw(k * 1.0, 0, np.radians(0.5 * k)), seed=100 + k)
    sizes = np.bincount(np.floor(cl["intensity"]).astype(np.int64), minlength=len(m.rings))
    frames.append((np.stack([cl["x"], cl["y"], cl["z"]], 1).astype(np.float32), sizes))
with imls_icp.ImlsContext(device=0) as c:
    def run():
        out = []
        for xyz, sizes in frames:
            r = c.ring_normals_pca(xyz, sizes)
            out.append((xyz[r["index"]], r["normal"], np.nonzero(r["flags"] & _abi.IMLS_PCA_CANDIDATE)[0]))
        (x0, n0, c0), (x1, n1, c1) = out
        t = time.perf_counter()
        s, w = c.sample_point_cloud(x1, n1, c1, x0, _abi.default_sample_params(_abi.IMLS_SAMPLE_MAJOR_AXIS))
        return s, time.perf_counter() - t, len(c1), len(x0)
    for _ in range(2):
        run()
    c.enable_timing(True); c.reset_timing()
    ts = []
    for _ in range(reps):
        s, dt, ncand, mlast = run()
        ts.append(dt)
    pca_ms, pca_n = c.kernel_timing(5)
    avg_ms, avg_n = c.kernel_timing(6)
print(json.dumps({"points": [int(len(f[0])) for f in frames], "candidates": ncand, "last_cloud": mlast,
                  "sampled": int(len(s)), "k_ring_pca_ms": pca_ms / max(pca_n, 1),
                  "k_major_avg_ms": avg_ms / max(avg_n, 1), "sample_call_ms": 1e3 * float(np.median(ts))}))
