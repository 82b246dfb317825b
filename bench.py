"""Benchmark: IMLS-ICP scan-pairs/s on BASELINE config B.

Workload (one "step" = one scan-pair registration, inputs already resident in HBM):
  synthetic HDL-64 scan (~126k points, all used as queries) vs a 10-scan local map (~1.26M
  points); index build (NaN filter, Morton sort, tree) + 20 ICP iterations (fixed: delta
  thresholds −1), each = fused transform/kNN/IMLS projection + trimmed-LS solve + pose update,
  all on device, one host sync per pair.  LS, t = 0.02; shipped IMLS parameters (h=1, r=3, K=20,
  30° normal gate).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process per
GPU, each registers its own independent pairs (weak scaling); the only exchange is
one RCCL all-gather of the relative poses for trajectory chaining; max-over-ranks timing.

Prints ONE JSON line (rank 0).  Progress goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
# One HIP stream per pair in flight: give the runtime 8 hardware queues (its default is 4) so the
# 4 pair streams never share a queue with each other or the runtime's own copies.  Read by the HIP
# runtime at initialisation, i.e. before torch touches the GPU.
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("IMLS_BENCH_HW_QUEUES", "8")
import plo_amd  # noqa: E402

plo_amd.load()
from planetary_lidar_odometry_amd import config, imls_icp, sequences, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E nominal (MI355X_MICROARCH.md chip table)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def soa_tensor(cloud, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(synth.soa(cloud))).to(dev).contiguous()


def algorithmic_bytes_per_launch(stats: dict, trace, iters: int) -> float:
    """B_q = 24 (query xyz+n) + 24·[NN found] + 24·k_q + 40·[valid], summed over
    the queries of one projection launch (k_q from the kernel's own counts)."""
    n_valid = float(np.mean([t.n_valid for t in trace])) if trace else 0.0
    return 24.0 * stats["queries"] + 24.0 * stats["nn_found"] / iters + 24.0 * stats["sum_kq"] / iters + 40.0 * n_valid


def cpu_baseline(pair, iters_full: int, min_seconds: float = 10.0, max_pairs: int = 4):
    """The oracle (C++ restatement, -O3, 1 thread) on the same pair: whole registrations (index
    build + `iters_full` ICP iterations, the same fixed-iteration parameters as the GPU leg),
    repeated until at least `min_seconds` of CPU work (bounded sample)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_ctypes as oc
    p = config.bench_params(iters_full)
    src, tgt = synth.soa(pair.source), synth.soa(pair.target)
    total, n, t_idx = 0.0, 0, 0.0
    while n < max_pairs and (n == 0 or total < min_seconds):
        r = oc.register_frame(src, tgt, p)
        total += r["seconds_total"]
        t_idx += r["seconds_index"]
        n += 1
    # secondary: the same oracle with its per-query projection loop on all host cores
    # this process may use (OpenMP; the index build and the solver stay sequential)
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)))
    oc.set_threads(threads)
    try:
        r2 = oc.register_frame(src, tgt, p)
    finally:
        oc.set_threads(1)
    return dict(value=n / total, unit="scan-pairs/s", cores=1, kind="port",
                sample=f"{n} whole pair registration(s) ({pair.source.size} queries vs {pair.target.size}-pt map, "
                       f"{r['iters']} ICP iterations each) in {total:.1f} s, index build {t_idx / n:.2f} s/pair; "
                       f"oracle/imls_oracle.cpp -O3, 1 thread",
                seconds_per_pair=total / n,
                all_cores={"value": 1.0 / r2["seconds_total"], "cores": threads,
                           "sample": f"1 whole pair registration, projection loop OpenMP over {threads} threads"})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--queries", type=int, default=0, help="0 = all source points; else FPS subsample")
    ap.add_argument("--inflight", type=int, default=4, help="independent scan pairs in flight (one stream each)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU-baseline leg")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    ap.add_argument("--workload", choices=["B", "stream"], default="B",
                    help="B: config B (the headline); stream: config C-like frames — 2000 FPS queries "
                         "(config.json major_axis max_total_points) vs the previous scan")
    args = ap.parse_args()
    stream = args.workload == "stream"
    map_scans = 1 if stream else 10
    if stream and args.queries <= 0:
        args.queries = 2000

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    t0 = time.time()
    P = max(1, args.inflight)
    pairs = synth.make_pairs(P, "hdl64", map_scans=map_scans, scene_seed=rank, traj_seed=2000 + rank,
                             noise_seed=1000 + 97 * rank)
    if args.queries > 0:
        pairs = [synth.Pair(synth.fps_subsample(q.source, args.queries, seed=rank), q.target, q.true_pose, q.meta)
                 for q in pairs]
    log(f"[rank {rank}] {P} pair(s) generated in {time.time() - t0:.1f}s: "
        f"{[q.source.size for q in pairs]} queries, maps {[q.target.size for q in pairs]}")
    s_dev = [soa_tensor(q.source, dev) for q in pairs]
    t_dev = [soa_tensor(q.target, dev) for q in pairs]
    torch.cuda.synchronize()

    p = config.bench_params(args.iters)
    ctxs = [imls_icp.ImlsContext(p, device=local) for _ in range(P)]   # one context (= stream) per pair in flight

    def step():
        # P independent pairs in flight: each context's index build + fused 20-iteration loop is
        # enqueued on its own stream; results are collected after all are enqueued
        for c, q, sd, td in zip(ctxs, pairs, s_dev, t_dev):
            c.set_target_device(td.data_ptr(), q.target.size)
            c.set_source_device(sd.data_ptr(), q.source.size)
            c.register_frame_async()
        return [c.register_frame_result() for c in ctxs]

    for _ in range(args.warmup):
        res = step()
    errs = [np.linalg.norm(r[0][:3, 3] - q.true_pose[:3, 3]) for r, q in zip(res, pairs)]
    err = float(max(errs))
    log(f"[rank {rank}] warmup done; max pose error vs truth {err * 100:.2f} cm")

    for c in ctxs:
        c.enable_timing(True)
        c.reset_timing()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    poses = []
    for _ in range(args.steps):
        res = step()
        poses.extend(r[0] for r in res)
    if world > 1:
        n_units = world * args.steps * P
        allp = sequences.gather_relative_poses(np.array(poses), n_units)   # the one RCCL exchange
        traj = sequences.chain_trajectory(allp)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dist.barrier()
        elapsed = float(tt.item())
    for c in ctxs:
        c.enable_timing(False)

    def tsum(k):
        ms = sum(c.kernel_timing(k)[0] for c in ctxs)
        n = sum(c.kernel_timing(k)[1] for c in ctxs)
        return ms, n
    proj_ms, proj_n = tsum(0)
    idx_ms, idx_n = tsum(1)
    sol_ms, sol_n = tsum(2)
    knn_ms, knn_n = tsum(3)
    fin_ms, fin_n = tsum(4)
    ctx = ctxs[0]
    stats = ctx.index_stats()
    trav = ctx.traversal_stats()
    log(f"[rank {rank}] traversal (last frame of pair 0, {args.iters} iterations): {trav}")
    # n_valid per iteration of pair 0's last frame for the byte count
    bytes_launch = algorithmic_bytes_per_launch(stats, ctx.last_trace, args.iters)
    avg_proj_s = proj_ms / max(proj_n, 1) / 1e3
    achieved = bytes_launch / avg_proj_s / 1e9 if avg_proj_s > 0 else 0.0
    n_pairs = args.steps * P
    aggregate = bytes_launch * args.iters * n_pairs / elapsed / 1e9

    if rank != 0:
        for c in ctxs:
            c.close()
        if world > 1:
            dist.destroy_process_group()
        return

    # HBM traffic per projection launch from the committed PMC pass (tools/pmc_traffic.py):
    # 2·FETCH_SIZE + WRITE_SIZE of k_knn_wave + k_finish (gfx950 FETCH_SIZE counts ½ of wide reads)
    traffic = None
    tj = pathlib.Path(args.traffic_json)
    if tj.exists():
        try:
            tdat = json.loads(tj.read_text())
            if tdat.get("queries") == stats["queries"] and tdat.get("iters") == args.iters:
                traffic = tdat.get("bytes_per_launch")
        except (ValueError, OSError):
            traffic = None

    cpu = None
    if world == 1 and not args.no_cpu:
        log("[rank 0] CPU baseline (oracle, 1 thread) ...")
        cpu = cpu_baseline(pairs[0], args.iters)
        log(f"[rank 0] CPU baseline {cpu['value']:.4f} pairs/s")

    value = world * n_pairs / elapsed
    ms_step = elapsed / args.steps * 1e3
    out = {
        "metric": ("IMLS-ICP frames/s (config C-like stream: 2000 FPS queries of an HDL-64 scan vs the previous scan, "
                   "20 ICP iterations)") if stream else
                  "IMLS-ICP scan-pairs/s (HDL-64 ~120k-pt scan vs 10-scan map, 20 ICP iterations)",
        "value": value,
        "unit": "frames/s" if stream else "scan-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "ms_per_pair": elapsed / n_pairs * 1e3,
        "pairs_in_flight": P,
        "ms_per_iteration": (elapsed / n_pairs * 1e3 - idx_ms / max(idx_n, 1)) / args.iters,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded HDL-64 ray-cast urban scene, planetary-lidar-odometry_amd/synth.py)",
        "config": {
            "workload": (f"config C-like stream: {args.queries} FPS queries vs the previous scan; a step = {P} frames "
                         f"in flight") if stream else
                        f"config B: HDL-64 scan vs 10-scan local map; a step = {P} independent scan pairs in flight",
            "queries": int(stats["queries"]),
            "map_points": int(stats["points"]),
            "icp_iterations": args.iters,
            "solver": "LS (trimmed, t=0.02)",
            "search_number": p.search_number,
            "parallelism": f"pairs sharded over {world} GPU(s), RCCL pose all-gather" if world > 1 else "1 GPU",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "projection step = k_knn_wave (packet traversal) + k_finish (exact re-rank, gates, IMLS, "
                      "pass-1 normal equations) + k_project_lane (fallback, normally 0 queries)",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "algorithmic_bytes_per_launch": bytes_launch,
            "avg_launch_ms": avg_proj_s * 1e3,
            "launches": int(proj_n),
            "kernel_avg_ms": {"k_knn_wave": knn_ms / max(knn_n, 1), "k_finish": fin_ms / max(fin_n, 1)},
            "aggregate_algorithmic_GBps": aggregate,
        },
        "breakdown_ms_per_pair": {     # summed per-pair stream time (overlaps across pairs in flight)
            "index_build": idx_ms / max(n_pairs, 1),
            "projection": proj_ms / max(n_pairs, 1),
            "solve_chain": sol_ms / max(n_pairs, 1),
        },
        "traversal_per_launch": {k: v / args.iters for k, v in trav.items()},
        "cpu_baseline": cpu,
        "final_pose_error_cm": float(err * 100),
    }
    print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
