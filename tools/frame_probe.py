"""Debug probe of the config C/D single-frame latency (a ≤2000-query flat cloud vs its previous
118k-point filtered scan, 20 ICP iterations, one frame at a time): per-kind kernel time per frame
(HIP events) and, with the DEBUG_WAVE_TRACE build (IMLS_LIB_PATH=…/debug/libimls_gpu.so), the
k_solve_small phase clocks per solve."""
import ctypes as C
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (loads the library)
import numpy as np  # noqa: E402
from planetary_lidar_odometry_amd import config, imls_icp  # noqa: E402

p = config.bench_params(20)
runner = bench.StreamRunner(1, p, 0, 0, frames_per_seq=3, fuse=False, unique=1, dev=None, resident=False, groups=1)
fr = runner.seqs[0]
lib = runner.ctxs[0].lib
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
with imls_icp.ImlsContext(p, device=0) as c:
    lat = []
    for j in range(n + 3):
        c.map_push(fr[j % 2][0], count=False)
        c.set_source(fr[1 - j % 2][1], count=False)
        t0 = time.perf_counter()
        c.register_frame()
        if j >= 3:
            lat.append((time.perf_counter() - t0) * 1e3)
    print(f"register_frame alone: median {np.median(lat):.3f} ms  p90 {np.percentile(lat, 90):.3f} ms "
          f"({len(fr[1][1])} queries vs {len(fr[0][0])}-pt map)")
    c.enable_timing(True)
    c.reset_timing()
    for j in range(n):
        c.map_push(fr[j % 2][0], count=False)
        c.set_source(fr[1 - j % 2][1], count=False)
        c.register_frame()
    for i, name in enumerate(("projection", "index", "solve", "k_knn_wave", "k_finish")):
        ms, k = c.kernel_timing(i)
        print(f"  {name:12s} {ms / n:.3f} ms per frame ({k / n:.0f} launches)")
    if hasattr(lib, "imls_debug_solve"):
        buf = np.zeros(8, np.uint64)
        lib.imls_debug_solve(C.c_void_p(buf.ctypes.data))
        solves = (2 * n + 3) * 20          # every k_solve_small call of this process (fixed 20 iterations)
        ph = ["partials+sum", "solve6+gate", "residuals", "hist+bitonic", "kept sums", "solve6", "delta", "finish"]
        print("  k_solve_small phases, ticks (100 MHz) per solve:",
              {k: round(float(v) / solves, 1) for k, v in zip(ph, buf)})
runner.close()
