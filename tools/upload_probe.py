"""Host-time probe of the deferred per-frame uploads (map_push / set_source with count=False)."""
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import plo_amd  # noqa: E402

plo_amd.load()
from planetary_lidar_odometry_amd import config, imls_icp, synth  # noqa: E402

pair = synth.make_pair("hdl64", map_scans=1, start=5)
tgt = pair.target
src = synth.fps_subsample(pair.source, 1900, seed=1)
print("target", tgt.size, "source", src.size, flush=True)
ctxs = [imls_icp.ImlsContext(config.bench_params(20)) for _ in range(8)]
for rep in range(3):
    t = {"map_push": 0.0, "set_source": 0.0, "set_target": 0.0, "build": 0.0}
    for it in range(5):
        for c in ctxs:
            t0 = time.perf_counter(); c.map_push(tgt, count=False); t1 = time.perf_counter()
            c.set_source(src, count=False); t2 = time.perf_counter()
            t["map_push"] += t1 - t0; t["set_source"] += t2 - t1
        t0 = time.perf_counter()
        for c in ctxs:
            c.index_stats()                      # forces the deferred builds
        t["build"] += time.perf_counter() - t0
        for c in ctxs:
            t0 = time.perf_counter(); c.set_target(tgt, count=False); t["set_target"] += time.perf_counter() - t0
        for c in ctxs:
            c.synchronize()
    print({k: round(v / 40 * 1e3, 3) for k, v in t.items()}, "ms per frame", flush=True)
a = np.empty((tgt.size, 6), np.float32)
t0 = time.perf_counter()
for _ in range(20):
    for k, f in enumerate(("x", "y", "z", "normal_x", "normal_y", "normal_z")):
        a[:, k] = tgt[f]
print("numpy field gather", round((time.perf_counter() - t0) / 20 * 1e3, 3), "ms", flush=True)
