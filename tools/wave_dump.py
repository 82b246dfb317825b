"""Debug: per-wave records of the last k_knn_wave launch (DEBUG_WAVE_TRACE=1 build) for a config-B
pair registered with `iters` iterations: prints the distribution and the slowest waves."""
import ctypes as C, pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import plo_amd
plo_amd.load()
import numpy as np, torch
from planetary_lidar_odometry_amd import config, imls_icp, synth
pair = synth.make_pairs(1, "hdl64", map_scans=10, scene_seed=0, traj_seed=2000, noise_seed=1000)[0]
sd = torch.from_numpy(np.ascontiguousarray(synth.soa(pair.source))).cuda()
td = torch.from_numpy(np.ascontiguousarray(synth.soa(pair.target))).cuda()
cols = ["seed_t", "trav_t", "leaves", "inner", "bc_events", "sparse_lv", "bcast_lv", "greedy", "W_inf", "W>1", "Wmax",
        "sp_lanes", "sp_ins", "bc_ins", "seed_steps", "seed_pts"]
for iters in [int(a) for a in sys.argv[1:]] or [1]:
    c = imls_icp.ImlsContext(config.bench_params(iters), device=0)
    c.set_target_device(td.data_ptr(), pair.target.size)
    c.set_source_device(sd.data_ptr(), pair.source.size)
    c.register_frame_async()
    c.register_frame_result()
    nw = (c.N + 63) // 64 if hasattr(c, "N") else 1972
    buf = np.zeros((8192, 16), np.uint32)
    n = c.lib.imls_debug_waves(C.c_void_p(buf.ctypes.data), 8192)
    a = buf[:1972, :16].astype(np.float64)
    a[:, 10] = buf[:1972, 10].view(np.float32)
    t = a[:, 0] + a[:, 1]
    print(f"== launch {iters - 1}: waves {n}; total ticks mean {t.mean():.0f} p50 {np.median(t):.0f} p99 {np.percentile(t, 99):.0f} max {t.max():.0f}")
    print("   mean:", {k: round(float(v), 1) for k, v in zip(cols, a.mean(0))})
    for i in np.argsort(-t)[:10]:
        print(f"   w{i:5d}", {k: (round(float(v), 3) if k == 'Wmax' else int(v)) for k, v in zip(cols, a[i])})
    c.close()
fin = np.zeros(12, np.uint64)
lib = imls_icp.ImlsContext(config.bench_params(1), device=0).lib
if lib.imls_debug_final(C.c_void_p(fin.ctypes.data)) == 0 and fin[0]:
    print(f"== trimmed-LS boundary bins over {int(fin[0])} solves: mean n_lo {fin[1] / fin[0]:.1f}, "
          f"mean n_hi {fin[2] / fin[0]:.1f}, max {int(fin[3])}")
    ph = ["load", "bitonic", "add_rows", "partials+sum", "solve6", "delta", "finish"]
    print("   k_solve_final phases, clock ticks per solve:", {k: round(float(fin[4 + i]) / float(fin[0]), 0) for i, k in enumerate(ph)})
