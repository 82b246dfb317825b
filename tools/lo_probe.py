"""Latency probe of the deployment call: LaserOdometry.process one frame at a time (pipelined for
max_queue_size 1) on the config C/D-like stream frames (≤2000-query flat cloud, 118k-point filtered
scan, 20 ICP iterations); prints the median / p90 wall time per call.  Run under rocprofv3
--kernel-trace --hip-trace to see where a frame's time goes between its launches."""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (loads the library)
import numpy as np  # noqa: E402
from planetary_lidar_odometry_amd import config, imls_icp  # noqa: E402

p = config.bench_params(20)
runner = bench.StreamRunner(1, p, 0, 0, frames_per_seq=6, fuse=False, unique=1, dev=None, resident=False, groups=1)
fr = runner.seqs[0]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
if "counted" in sys.argv[2:]:          # A/B: the flat cloud loaded with its count (host waits for it)
    _orig = imls_icp.ImlsContext.set_source
    imls_icp.ImlsContext.set_source = lambda self, cloud, count=True: _orig(self, cloud, True)
lat = []
with imls_icp.LaserOdometry(p, device=0) as lo:
    for j in range(n + 3):
        k = j % len(fr)
        t0 = time.perf_counter()
        lo.process(fr[k][0], fr[k][1])
        if j >= 3:
            lat.append((time.perf_counter() - t0) * 1e3)
    print(f"LaserOdometry.process{' (counted)' if 'counted' in sys.argv[2:] else ''}: median {np.median(lat):.3f} ms  p90 {np.percentile(lat, 90):.3f} ms "
          f"(pipelined {lo.pipelined}, {len(fr[0][1])} queries vs {len(fr[0][0])}-pt scan)")
runner.close()
