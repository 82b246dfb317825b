"""CPU (gloo, world size 2): one long sequence split over ranks: each rank registers
a contiguous block of frames after pushing the `max_queue_size` filtered scans before its block
into its map FIFO as a halo (accumulateTargetCloud, laser_odometry.cpp:116-136; frame 0 only seeds
the map, Q13).  Every frame then sees exactly the map it sees on one rank, so after the one
all-gather of relative poses the chained trajectory (652-655) equals the single-rank stream bit for
bit.  The device is replaced, in this test only, by the CPU oracle (a map FIFO over
oracle register_frame), so the poses are real registrations."""
import os
import pathlib
import socket
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

N_FRAMES = 12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _frames():
    """A 12-frame VLP-16 drive: (filtered cloud = the full scan, flat cloud = 400 FPS samples)."""
    from planetary_lidar_odometry_amd import synth
    sm = synth.vlp16()
    scene = synth.make_scene(11)
    poses = synth.trajectory(N_FRAMES, 2011)
    out = []
    for k in range(N_FRAMES):
        sc = synth.scan(scene, sm, poses[k], 3011 + k)
        out.append((sc, synth.fps_subsample(sc, 400, seed=k)))
    return out


class OracleOdometry:
    """Device stand-in (test only): LaserOdometry's map FIFO + registration, on the CPU oracle."""

    def __init__(self, queue, iters=4):
        from planetary_lidar_odometry_amd import config
        self.queue = queue
        self.fifo = []
        self.p = config.bench_params(iters)
        self.p.max_queue_size = queue

    def map_push(self, filtered):
        self.fifo.append(filtered)
        if len(self.fifo) > self.queue:          # the reference's `if` (drops once)
            self.fifo.pop(0)

    def register(self, flat):
        import oracle_ctypes as oc
        from planetary_lidar_odometry_amd import synth
        tgt = np.concatenate(self.fifo)
        return oc.register_frame(synth.soa(flat), synth.soa(tgt), self.p)["pose"]


def _single_rank(frames, queue):
    from planetary_lidar_odometry_amd import sequences
    halo, block = sequences.halo_block(len(frames), 0, 1, queue)
    assert len(halo) == 1 and block == range(1, len(frames))
    rel = sequences.run_halo_block(OracleOdometry(queue), frames, halo, block)
    return rel, sequences.chain_trajectory(rel)


def _worker(rank, world, port, queue, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import plo_amd
    plo_amd.load()
    import torch.distributed as dist
    from planetary_lidar_odometry_amd import sequences
    dist.init_process_group("gloo")
    frames = _frames()
    halo, block = sequences.halo_block(len(frames), rank, world, queue)
    rel = sequences.run_halo_block(OracleOdometry(queue), frames, halo, block)
    allp = sequences.gather_relative_poses(rel, len(frames) - 1)
    q.put((rank, list(halo), list(block), allp, sequences.chain_trajectory(allp)))
    dist.destroy_process_group()


def test_halo_block_ranges():
    from planetary_lidar_odometry_amd import sequences
    for n, world, queue in [(12, 2, 1), (12, 2, 3), (12, 3, 3), (5, 4, 2), (2, 3, 1)]:
        seen = []
        for r in range(world):
            halo, block = sequences.halo_block(n, r, world, queue)
            if len(block):
                assert list(halo) == list(range(max(0, block.start - queue), block.start))
            seen += list(block)
        assert seen == list(range(1, n))          # every frame but the first, once, in order


@pytest.mark.parametrize("queue", [1, 3])
def test_halo_split_gloo_world2(queue):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    qu = ctx.Queue()
    port, world = _free_port(), 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, queue, qu)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([qu.get(timeout=150) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rel1, traj1 = _single_rank(_frames(), queue)
    assert res[1][1] == list(range(res[1][2][0] - queue, res[1][2][0]))   # rank 1's halo precedes its block
    for _, _, _, allp, traj in res:
        assert np.array_equal(allp, rel1)          # same relative poses, bit for bit
        assert np.array_equal(traj, traj1)         # same chained trajectory


def test_halo_split_refuses_ransac():
    """A halo split is exact only for solvers without random draws: RANSAC's rand() stream runs
    across the sequence's frames (common.cpp:49, never seeded), so run_halo_block refuses it."""
    from planetary_lidar_odometry_amd import _abi, sequences
    odo = OracleOdometry(1)
    odo.p.solve_method = _abi.IMLS_SOLVE_RANSAC
    with pytest.raises(ValueError, match="RANSAC"):
        sequences.run_halo_block(odo, [], range(0), range(1, 2))
