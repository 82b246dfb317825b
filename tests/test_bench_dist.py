"""CPU (gloo, world size 2): bench.py's own multi-rank path — rank setup (dist_setup with
--backend gloo), the timed region (barrier + sync on both sides, max-over-ranks elapsed),
the one pose exchange (all-gather in unit order) and the trajectory chaining — driven through
the functions bench.main uses.  The device leg is replaced, in this test only, by the CPU oracle
registering a small golden pair, so the poses are real registration results."""
import os
import pathlib
import socket
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def marker(rank, k):
    from planetary_lidar_odometry_amd import synth
    return synth.pose_xyyaw(0.01 * rank, 0.001 * k, 0.0001 * (rank * 10 + k))


def _worker(rank, world, port, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import bench
    import oracle_ctypes as oc
    from planetary_lidar_odometry_amd import config
    import torch.distributed as dist
    w, r, _, dev = bench.dist_setup("gloo")
    assert (w, r) == (world, rank) and dev.type == "cpu"
    g = dict(np.load(ROOT / "tests" / "golden" / "vlp16_pair.npz"))
    p = config.bench_params(2)
    counter = [0]

    def step():           # one unit per step on this rank: a real (oracle) registration, tagged
        res = oc.register_frame(g["src"], g["tgt"], p)
        k = counter[0]
        counter[0] += 1
        return [(res["pose"] @ marker(rank, k), res["iters"], res["status"])]

    elapsed, per, out = bench.timed_steps(step, steps, world, dev)
    # this rank's units form one sequence (seq 0 locally), in step order
    recs, trajs = bench.exchange_poses([(0, k, o[0]) for k, o in enumerate(out)], world, rank)
    # the per-rank roofline inputs (bench.main gathers them before ranks != 0 return): rank-specific
    # synthetic busy pass / probe so the gathered rows are checkable
    busy = {"projection_busy_ms": 2.0 * (rank + 1) * steps}
    probe = {"kernel_avg_ms": {"k_knn_wave": 0.1 * (rank + 1), "k_finish": 0.05}}
    vals = bench.rank_roofline(1e9 * (rank + 1), busy, steps, per, probe, 5e7)
    roof = bench.gather_rank_roofline(vals, world, dev)
    q.put((rank, elapsed, sum(per), recs, {s: (o.tolist(), t) for s, (o, t) in trajs.items()}, roof))
    dist.destroy_process_group()


def test_bench_dist_path_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, steps, world = _free_port(), 3, 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle_ctypes as oc
    from planetary_lidar_odometry_amd import config
    g = dict(np.load(ROOT / "tests" / "golden" / "vlp16_pair.npz"))
    base = oc.register_frame(g["src"], g["tgt"], config.bench_params(2))["pose"]
    want = np.array([base @ marker(r, k) for r in range(world) for k in range(steps)])   # rank-major records
    elapsed = [t[1] for t in res]
    assert elapsed[0] == elapsed[1]                          # max over ranks, identical on every rank
    assert all(elapsed[0] >= t[2] for t in res)              # ≥ each rank's own time in its steps
    for r, (_, _, _, _, _, roof) in enumerate(res):
        assert [d["rank"] for d in roof] == list(range(world))          # every rank's row, on every rank
        for k, d in enumerate(roof):
            assert d["algorithmic_bytes_per_step"] == 1e9 * (k + 1)
            assert d["busy_projection_ms_per_step"] == 2.0 * (k + 1)
            assert abs(d["achieved"] - 1e9 * (k + 1) / (2e-3 * (k + 1)) / 1e9) < 1e-6   # 500 GB/s
            assert abs(d["frac"] - d["achieved"] / 8000.0) < 1e-12          # bench.HBM_PEAK_GBS
            assert abs(d["serialised_launch_ms"] - (0.1 * (k + 1) + 0.05)) < 1e-12
            assert d["serialised_frac"] > 0 and d["ms_per_step"] > 0
        assert roof == res[0][5]                                         # identical on both ranks
    for _, _, _, (seq, order, poses), trajs, _ in res:
        assert np.array_equal(poses, want)
        assert list(seq) == [r << 20 for r in range(world) for _ in range(steps)]
        assert list(order) == [k for _ in range(world) for k in range(steps)]
        # every rank's sequence chained on its own (laser_odometry.cpp:652-655 per sequence)
        assert sorted(trajs) == [r << 20 for r in range(world)]
        for r in range(world):
            orders, traj = trajs[r << 20]
            T, chained = np.eye(4), []
            for k in range(steps):
                T = T @ want[r * steps + k]
                chained.append(T)
            assert orders == list(range(steps))
            assert np.array_equal(traj, np.array(chained))
