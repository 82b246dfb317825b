"""Per-wave records of the fused wave-per-query kernel (k_knn_qwave_f) of a lone small frame, from the
DEBUG_WAVE_TRACE build (IMLS_LIB_PATH=…/debug/libimls_gpu.so): for the last launch of a 20-iteration
frame (steady state) and of a 1-iteration frame (iteration 0): wave start spread, per-wave traversal
and exact-stage durations, and what the last-finishing waves were doing (µs, 100 MHz clock)."""
import ctypes as C
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import numpy as np  # noqa: E402
from planetary_lidar_odometry_amd import config, imls_icp  # noqa: E402

runner = bench.StreamRunner(1, config.bench_params(20), 0, 0, frames_per_seq=3, fuse=False, unique=1, dev=None,
                            resident=False, groups=1)
fr = runner.seqs[0]
for iters in (20, 1):
    p = config.bench_params(iters)
    with imls_icp.ImlsContext(p, device=0) as c:
        lib = c.lib
        for j in range(4):
            c.map_push(fr[j % 2][0], count=False)
            c.set_source(fr[1 - j % 2][1], count=False)
            c.register_frame()
        n = len(fr[1 - 3 % 2][1])
        buf = np.zeros((n, 16), np.uint32)
        got = lib.imls_debug_waves(C.c_void_p(buf.ctypes.data), n)
    r = buf[:got].astype(np.int64)
    t0 = r[:, 0].min()
    st, mid, en = (r[:, 0] - t0) / 100.0, (r[:, 1] - t0) / 100.0, (r[:, 2] - t0) / 100.0
    trav, fin, life = mid - st, en - mid, en - st
    print(f"== iteration {iters - 1} of a {iters}-iteration frame: {got} waves, launch span {en.max():.1f} us")
    for name, v in (("start", st), ("traversal", trav), ("exact stage", fin), ("lifetime", life), ("end", en)):
        q = np.percentile(v, [0, 10, 50, 90, 99, 100])
        print(f"  {name:12s} " + " ".join(f"{x:7.2f}" for x in q) + "   (min p10 p50 p90 p99 max)")
    sk = r[:, 3] == 1
    print(f"  Verlet skips {sk.sum()} / {got}; greedy {int(r[:, 6].sum())}; leaves mean {r[:, 4].mean():.1f} max {r[:, 4].max()}, "
          f"inner mean {r[:, 5].mean():.1f} max {r[:, 5].max()}")
    last = np.argsort(-en)[:8]
    for k in last:
        print(f"  late wave slot {k}: start {st[k]:.2f} traversal {trav[k]:.2f} exact {fin[k]:.2f} skip {r[k, 3]} "
              f"leaves {r[k, 4]} inner {r[k, 5]} hw {r[k, 7]:#x}")
    hist, edges = np.histogram(st, bins=10)
    print("  start histogram: " + " ".join(f"{e:.1f}:{h}" for e, h in zip(edges[:-1], hist)))
runner.close()
