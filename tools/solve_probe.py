"""Debug: phase timings of k_solve_small (DEBUG_WAVE_TRACE=1 build) over one stream frame."""
import ctypes as C, pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import plo_amd
plo_amd.load()
import numpy as np, torch
from planetary_lidar_odometry_amd import config, imls_icp, synth
pair = synth.make_pairs(1, "hdl64", map_scans=1, scene_seed=0, traj_seed=2000, noise_seed=1000)[0]
src = synth.fps_subsample(pair.source, 2000, seed=0)
sd = torch.from_numpy(np.ascontiguousarray(synth.soa(src))).cuda()
td = torch.from_numpy(np.ascontiguousarray(synth.soa(pair.target))).cuda()
c = imls_icp.ImlsContext(config.bench_params(20), device=0)
for rep in range(3):
    c.set_target_device(td.data_ptr(), pair.target.size)
    c.set_source_device(sd.data_ptr(), src.size)
    c.register_frame_async()
    c.register_frame_result()
out = np.zeros(8, np.uint64)
c.lib.imls_debug_solve(C.c_void_p(out.ctypes.data))
print("k_solve_small phase ticks (sum over 60 launches, 100 MHz):", out.tolist())
print("per launch us:", [round(float(v) / 60 / 100, 2) for v in out])
