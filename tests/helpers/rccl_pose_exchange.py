"""Child process of tests/test_gpu_rccl.py: bench.py's own distributed path on ONE GPU over RCCL.

Started as a fresh process (no GPU call before dist_setup) with RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 and
MASTER_ADDR/PORT, i.e. exactly what `torch.distributed.run --nproc-per-node 1` hands bench.py:
bench.dist_setup("nccl") initialises the process group, bench.StreamRunner / Pipeline register
`--seqs` independent stream sequences (one batched launch sequence per step) for `--steps` timed
steps (barrier + max-over-ranks timing through the group), and bench.exchange_poses all-gathers the
tagged relative poses over RCCL and chains every sequence on its own
(laser_odometry.cpp:652-655).  Prints one JSON line; exits non-zero on any mismatch.
"""
import argparse
import json
import os
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=16)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    import bench                                   # loads the HIP library; no GPU call yet
    import torch
    import torch.distributed as dist
    from planetary_lidar_odometry_amd import config, sequences
    world, rank, local, dev = bench.dist_setup("nccl")
    assert dist.is_initialized() and dist.get_backend() == "nccl", "no RCCL process group"
    p = config.bench_params(a.iters)
    runner = bench.StreamRunner(a.seqs, p, local, rank, frames_per_seq=3, fuse=True, unique=2, dev=dev,
                                resident=True, groups=1)
    bench.timed_steps(runner.step, 1, world, dev, torch.cuda.synchronize)      # warm-up
    runner.drain()
    elapsed, per, res = bench.timed_steps(runner.step, a.steps, world, dev, torch.cuda.synchronize)
    res += runner.drain()
    tags = [(k, j, r[1]) for j, r in enumerate(res) for k in [r[0]]]
    (seq, order, poses), trajs = bench.exchange_poses(tags, world, rank)
    # the same records and trajectories computed locally, without the collective
    lseq = np.array([rank * (1 << 20) + t[0] for t in tags], dtype=np.int64)
    lorder = np.array([t[1] for t in tags], dtype=np.int64)
    lposes = np.asarray([t[2] for t in tags], dtype=np.float64).reshape(-1, 4, 4)
    want = sequences.chain_per_sequence(lseq, lorder, lposes)
    ok_rec = (np.array_equal(seq, lseq) and np.array_equal(order, lorder) and np.array_equal(poses, lposes))
    ok_traj = sorted(trajs) == sorted(want) and all(
        np.array_equal(trajs[s][0], want[s][0]) and np.array_equal(trajs[s][1], want[s][1]) for s in want)
    out = dict(backend=dist.get_backend(), world=world, results=len(res), sequences=len(trajs),
               records_equal=bool(ok_rec), trajectories_equal=bool(ok_traj), elapsed_s=elapsed,
               frames_per_s=len(res) / elapsed if elapsed > 0 else None,
               nccl_version=".".join(map(str, torch.cuda.nccl.version())) if hasattr(torch.cuda, "nccl") else None)
    print(json.dumps(out), flush=True)
    runner.close()
    dist.destroy_process_group()
    sys.exit(0 if ok_rec and ok_traj and len(res) == a.seqs * a.steps else 1)


if __name__ == "__main__":
    main()
