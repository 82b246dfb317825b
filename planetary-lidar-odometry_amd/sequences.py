"""Multi-GPU sharding of scan registration.

Every frame's registration restarts from rPose = I (laser_odometry.cpp:484-485) and uses only
the raw source cloud and the raw previous `max_queue_size` clouds (116-136, Q12), so frames are
independent units once their map is known:

* many sequences (config D): whole sequences per rank, each chained on its own;
* one long sequence: contiguous blocks of frames per rank, each block preceded by a halo of the
  `max_queue_size` filtered scans before it, pushed into the rank's map FIFO and not registered
  (halo_block) — every frame then sees the same map as on one rank, so its relative pose is the
  same bits, for solvers that draw no random numbers (LS, Weighted LS).  RANSAC draws from ONE
  rand() stream across the whole sequence (the reference's process-wide, never-seeded rand(),
  common.cpp:49; LaserOdometry keeps its context's stream across frames): a rank starting
  mid-sequence would need the stream's state after every earlier frame's draws, which only a
  sequential run produces, so run_halo_block refuses RANSAC (split many sequences instead: each
  sequence on one rank keeps its stream).

The only exchange is ONE all-gather of the 4×4 relative poses (16 doubles per frame, 128 B) over
RCCL/xGMI; every rank then chains each sequence T_k = T_{k−1}·ΔT_k (laser_odometry.cpp:652-655).
The exchange is latency-bound, not bandwidth-bound.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_units: int, rank: int, world: int) -> range:
    """Contiguous block of units for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n_units, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def halo_block(n_frames: int, rank: int, world: int, queue: int):
    """One long sequence of n_frames over `world` ranks: (halo, block).  Frame 0 only seeds the map
    (Q13, laser_odometry.cpp:478), so the registered frames 1 … n_frames−1 are split into contiguous
    blocks; `halo` = the frames whose filtered scans the rank pushes into its FIFO before its block
    (the max_queue_size scans preceding it, accumulateTargetCloud 116-136), none registered."""
    blk = shard_range(max(n_frames - 1, 0), rank, world)
    block = range(blk.start + 1, blk.stop + 1)
    if len(block) == 0:
        return range(0), block
    return range(max(0, block.start - max(queue, 0)), block.start), block


def run_halo_block(odo, frames, halo, block):
    """Drive a LaserOdometry-shaped object (map_push(filtered) / register(flat) → rPose) over one
    rank's share of a sequence: the halo scans join the FIFO unregistered, then each block frame is
    registered against the FIFO and its filtered scan pushed, as processData orders them
    (laser_odometry.cpp:478-670).  Returns the block's relative poses in frame order.  RANSAC is
    refused (module docstring: its rand() stream runs across the sequence's frames)."""
    from . import _abi
    params = (getattr(odo, "params", None) or getattr(odo, "p", None)
              or getattr(getattr(odo, "ctx", None), "params", None))
    if params is not None and int(getattr(params, "solve_method", 0)) == _abi.IMLS_SOLVE_RANSAC:
        raise ValueError("run_halo_block: RANSAC draws one rand() stream across the sequence; a halo "
                         "split is exact only for LS / Weighted LS — split whole sequences instead")
    for k in halo:
        odo.map_push(frames[k][0])
    rel = []
    for k in block:
        rel.append(np.asarray(odo.register(frames[k][1]), dtype=np.float64).reshape(4, 4))
        odo.map_push(frames[k][0])
    return np.array(rel).reshape(-1, 4, 4)


def chain_trajectory(rel_poses: np.ndarray, start: np.ndarray | None = None) -> np.ndarray:
    """Prefix product nowPose_k = prevLaserPose · rPose_k (laser_odometry.cpp:652-655)."""
    T = np.eye(4) if start is None else np.asarray(start, dtype=np.float64)
    out = np.empty((len(rel_poses), 4, 4))
    for k, d in enumerate(rel_poses):
        T = T @ d
        out[k] = T
    return out


def chain_per_sequence(seq_ids, orders, rel_poses) -> dict:
    """Trajectories of independent sequences (config D: one prevLaserPose per sequence,
    laser_odometry.cpp:652-655): {seq: (orders ascending, chained poses)} — each sequence's frames
    are chained in their own order, never into another sequence's."""
    seq_ids, orders = np.asarray(seq_ids), np.asarray(orders)
    rel_poses = np.asarray(rel_poses, dtype=np.float64).reshape(-1, 4, 4)
    out = {}
    for s in np.unique(seq_ids):
        idx = np.nonzero(seq_ids == s)[0]
        idx = idx[np.argsort(orders[idx], kind="stable")]
        out[int(s)] = (orders[idx], chain_trajectory(rel_poses[idx]))
    return out


def _dist_device(group):
    import torch
    import torch.distributed as dist
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")


def gather_relative_poses(local: np.ndarray, n_units: int, group=None) -> np.ndarray:
    """All-gather every rank's relative poses (block-sharded by shard_range) into the global
    (n_units, 4, 4) array, in unit order.  Uses torch.distributed (RCCL on GPU, gloo on CPU)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = _dist_device(group)
    maxn = -(-n_units // world)
    buf = torch.zeros((maxn, 16), dtype=torch.float64, device=dev)
    mine = shard_range(n_units, rank, world)
    assert len(local) == len(mine)
    if len(mine):
        buf[: len(mine)] = torch.as_tensor(np.asarray(local, dtype=np.float64).reshape(-1, 16), device=dev)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = np.empty((n_units, 4, 4))
    for r in range(world):
        rr = shard_range(n_units, r, world)
        out[rr.start:rr.stop] = parts[r][: len(rr)].cpu().numpy().reshape(-1, 4, 4)
    return out


def gather_tagged_poses(seq_ids, orders, rel_poses, group=None):
    """All-gather of (sequence id, frame order, relative pose) records of every rank (counts may
    differ: one small all-gather of the counts, then one of the padded records).  Returns the
    concatenation over ranks (rank-major): (seq_ids, orders, poses (n, 4, 4))."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dev = _dist_device(group)
    n = len(seq_ids)
    cnt = torch.tensor([n], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    maxn = max(max(counts), 1)
    buf = torch.zeros((maxn, 18), dtype=torch.float64, device=dev)
    if n:
        rec = np.concatenate([np.asarray(seq_ids, np.float64).reshape(-1, 1), np.asarray(orders, np.float64).reshape(-1, 1),
                              np.asarray(rel_poses, np.float64).reshape(-1, 16)], axis=1)
        buf[:n] = torch.as_tensor(rec, device=dev)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    rec = np.concatenate([parts[r][: counts[r]].cpu().numpy() for r in range(world)], axis=0)
    return rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64), rec[:, 2:].reshape(-1, 4, 4)
