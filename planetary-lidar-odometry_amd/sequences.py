"""Multi-GPU sharding of independent scan pairs.

Every frame's registration restarts from rPose = I (laser_odometry.cpp:484-485) and uses only
the raw source cloud and the raw previous `max_queue_size` clouds (116-136, Q12), so scan pairs
are independent units: ranks take contiguous blocks of pairs (one sequence per rank for config D),
register them with no data-path collective, and ONE all-gather of the 4×4 relative poses
(16 doubles per pair, 128 B) over RCCL/xGMI lets every rank chain the trajectory
T_k = T_{k−1}·ΔT_k (laser_odometry.cpp:652-655).  The exchange is latency-bound, not bandwidth-bound.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_units: int, rank: int, world: int) -> range:
    """Contiguous block of units for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n_units, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def chain_trajectory(rel_poses: np.ndarray, start: np.ndarray | None = None) -> np.ndarray:
    """Prefix product nowPose_k = prevLaserPose · rPose_k (laser_odometry.cpp:652-655)."""
    T = np.eye(4) if start is None else np.asarray(start, dtype=np.float64)
    out = np.empty((len(rel_poses), 4, 4))
    for k, d in enumerate(rel_poses):
        T = T @ d
        out[k] = T
    return out


def gather_relative_poses(local: np.ndarray, n_units: int, group=None) -> np.ndarray:
    """All-gather every rank's relative poses (block-sharded by shard_range) into the global
    (n_units, 4, 4) array, in unit order.  Uses torch.distributed (RCCL on GPU, gloo on CPU)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
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
