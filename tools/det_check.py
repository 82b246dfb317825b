"""Determinism check: imls_register_batch (3 contexts) vs one context on 5 stream pairs — poses bit-identical?"""
import sys; sys.path.insert(0, '.')
import plo_amd; plo_amd.load()
import numpy as np
from planetary_lidar_odometry_amd import config, imls_icp, synth
pairs = synth.make_pairs(5, "vlp16", map_scans=1, scene_seed=3, traj_seed=2003, noise_seed=1003)
pairs = [(synth.fps_subsample(q.source, 1500, seed=k), q.target) for k, q in enumerate(pairs)]
p = config.bench_params(8)
with imls_icp.ImlsBatch(p, streams=3) as b:
    a, _, _ = b.register(pairs)
with imls_icp.ImlsContext(p) as c:
    out = []
    for src, tgt in pairs:
        c.enable_stats(True); c.set_target(tgt); c.set_source(src); out.append(c.register_frame()["pose"])
        st = c.traversal_stats()
print("bit-identical:", all(np.array_equal(x, y) for x, y in zip(a, out)), "max diff", max(np.abs(x - y).max() for x, y in zip(a, out)), st)
