"""bench.py's host hand-over mode for the pair workloads (`--host-inputs`, SURVEY §8(d) `t_pair`):
each context keeps its map as a device FIFO of the map's scans (max_queue_size = their number,
accumulateTargetCloud laser_odometry.cpp:116-136) and every registration pushes the newest scan
and sets the source from host memory, as the reference's 48-B PointXYZINormal records.  The pushed
scan cycles through the map's scans, so the FIFO always holds the same points from a rotating first
scan.  Every result must be bit-equal to the pair registered alone on a fresh context whose map is
the same scans concatenated in the same rotation (single-frame kernels), and the rotation-0 result
must match the CPU oracle on the pair's own target (iterations, valid counts, reject counters
exact; pose within 1e-6)."""
import sys
import pathlib

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

pytestmark = pytest.mark.gpu


def test_pair_runner_host_fifo_rotation():
    import bench
    import oracle_ctypes as oc
    from planetary_lidar_odometry_amd import config, synth
    pairs = synth.make_pairs(2, "vlp16", map_scans=3, scene_seed=1, traj_seed=2001, noise_seed=1001)
    p = config.bench_params(6)
    runner = bench.PairRunner(pairs, p, None, 0, fuse=True, groups=2, host=True)
    try:
        assert runner.p.max_queue_size == 3
        rots = {}

        def tagging(idx, orig=runner._prep):
            orig(idx)
            for k in idx:
                rots.setdefault(k, []).append(runner.rot[k])
        runner.pipe.prep = tagging
        res = []
        for _ in range(4):
            res += runner.step()
        res += runner.drain()
        assert len(res) == 8
        seen = {}
        for r in res:
            k = r[0]
            j = seen.get(k, 0)
            seen[k] = j + 1
            ref = runner.single_fresh(k, rots[k][j])
            assert bench.same_result(r, ref), (k, j, rots[k][j])
        assert sorted(set(rots[0])) == [0, 1, 2]      # every rotation of the FIFO occurred
        k0 = runner.single_fresh(0, 0)
        want = oc.register_frame(synth.soa(pairs[0].source), synth.soa(pairs[0].target), p)
        assert k0[2] == want["iters"] and k0[3] == want["status"]
        for tg, tw in zip(k0[4], want["trace"]):
            assert tg.n_valid == tw.n_valid and list(tg.reject) == list(tw.reject)
        assert np.abs(np.asarray(k0[1]) - want["pose"]).max() < 1e-6
    finally:
        runner.close()
