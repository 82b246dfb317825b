"""CPU tests: config.json key paths / method names, and the multi-rank pair sharding + pose
all-gather (torch.distributed gloo, world size 2) that bench.py uses over RCCL on the GPU node."""
import copy
import os
import socket

import pathlib
import sys

import numpy as np
import pytest

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent.parent))
import plo_amd  # noqa: E402  (spawned workers import this module without conftest)

plo_amd.load()
from planetary_lidar_odometry_amd import _abi, config, sequences, synth  # noqa: E402


def test_config_method_names():
    cfg = config.load()
    p = config.params_from_config(cfg)
    assert p.matching_method == _abi.IMLS_MATCH_IMLS and p.solve_method == _abi.IMLS_SOLVE_RANSAC
    assert p.ransac_final_method == _abi.IMLS_FINAL_DRPM
    for name, val in (("LS", _abi.IMLS_SOLVE_LS), ("RANSAC", _abi.IMLS_SOLVE_RANSAC)):
        c = copy.deepcopy(cfg)
        c["laser_odometry"]["solve_method"]["method"] = name
        assert config.params_from_config(c).solve_method == val
    # "Weighted LS" is a RANSAC final method only: as a top-level name the reference's dispatcher
    # prints "Invalid SOLVE_METHOD!" (laser_odometry.cpp:269-272), so the config is rejected
    for bad in ("Ceres", "ICP", "Teaser", "nope", "Weighted LS"):
        c = copy.deepcopy(cfg)
        c["laser_odometry"]["solve_method"]["method"] = bad
        with pytest.raises(config.ConfigError):
            config.params_from_config(c)
    c = copy.deepcopy(cfg)
    c["laser_odometry"]["matching_method"]["method"] = "ICP"
    with pytest.raises(config.ConfigError, match="Invalid MATCHING_METHOD"):
        config.params_from_config(c)
    with pytest.raises(FileNotFoundError):
        config.load("/nonexistent/config.json")


def test_bench_params():
    p = config.bench_params(20)
    assert p.iterations == 20 and p.solve_method == _abi.IMLS_SOLVE_LS and p.delta_dist_threshold < 0


@pytest.mark.parametrize("n,world", [(10, 3), (8, 8), (3, 4), (0, 2)])
def test_shard_range_partitions(n, world):
    seen = []
    for r in range(world):
        seen.extend(sequences.shard_range(n, r, world))
    assert seen == list(range(n))


def test_chain_trajectory():
    rel = [synth.pose_xyyaw(1.0, 0.0, 0.01 * k) for k in range(5)]
    T = sequences.chain_trajectory(np.array(rel))
    ref = np.eye(4)
    for k, d in enumerate(rel):
        ref = ref @ d
        assert np.allclose(T[k], ref)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_units, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = sequences.shard_range(n_units, rank, world)
    local = np.array([synth.pose_xyyaw(0.1 * k, 0.0, 0.001 * k) for k in mine]).reshape(-1, 4, 4)
    allp = sequences.gather_relative_poses(local, n_units)
    q.put((rank, allp))
    dist.destroy_process_group()


def test_gather_relative_poses_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n_units = 7
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_units, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=60) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.array([synth.pose_xyyaw(0.1 * k, 0.0, 0.001 * k) for k in range(n_units)])
    for _, allp in res:
        assert np.array_equal(allp, want)


def test_weighted_ls_top_level_rejected_but_final_accepted():
    cfg = config.load()
    c = copy.deepcopy(cfg)
    c["laser_odometry"]["solve_method"]["method"] = "Weighted LS"
    with pytest.raises(config.ConfigError, match="Invalid SOLVE_METHOD"):
        config.params_from_config(c)
    for name, val in config.FINAL.items():
        c = copy.deepcopy(cfg)
        c["laser_odometry"]["solve_method"]["RANSAC"]["final_solve_method"] = name
        assert config.params_from_config(c).ransac_final_method == val


def test_chain_pose_is_eigen_order():
    from planetary_lidar_odometry_amd import imls_icp
    rng = np.random.default_rng(3)
    a, b = rng.normal(size=(4, 4)), rng.normal(size=(4, 4))
    got = imls_icp.chain_pose(a, b)
    want = np.array([[((a[i, 0] * b[0, j] + a[i, 1] * b[1, j]) + a[i, 2] * b[2, j]) + a[i, 3] * b[3, j]
                      for j in range(4)] for i in range(4)])
    assert np.array_equal(got, want)
