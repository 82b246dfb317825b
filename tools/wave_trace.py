"""Debug: run one config-B pair against a DEBUG_WAVE_TRACE=1 build of libimls_gpu.so and print
the traversal counters, including the insert counters of that build (slots 6, 7)."""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import plo_amd
plo_amd.load()
import numpy as np, torch
from planetary_lidar_odometry_amd import config, imls_icp, synth
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
pair = synth.make_pairs(1, "hdl64", map_scans=10, scene_seed=0, traj_seed=2000, noise_seed=1000)[0]
sd = torch.from_numpy(np.ascontiguousarray(synth.soa(pair.source))).cuda()
td = torch.from_numpy(np.ascontiguousarray(synth.soa(pair.target))).cuda()
keys = ("sum_kq", "nn_found", "leaves", "inner", "waves", "uncertified", "insert_events", "lane_inserts", "seed_clk_sum", "seed_clk_max", "trav_clk_sum", "trav_clk_max", "leaf_sum", "leaf_max", "events_max", "greedy_lanes")
for iters in [int(a) for a in (sys.argv[1:] or ['1', '2', '3', '20'])]:
    c = imls_icp.ImlsContext(config.bench_params(iters), device=0)
    c.set_target_device(td.data_ptr(), pair.target.size)
    c.set_source_device(sd.data_ptr(), pair.source.size)
    c.register_frame_async()
    r = c.register_frame_result()
    raw = np.zeros(16, np.uint64)
    c.lib.imls_traversal_stats(c.ctx, raw.ctypes.data)
    print(iters, {k: int(v) for k, v in zip(keys, raw)}, "pose", np.round(r[0][:3, 3], 4).tolist(), flush=True)
    c.close()
