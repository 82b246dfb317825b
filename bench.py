"""Benchmark: IMLS-ICP scan-pairs/s on BASELINE config B, plus the other configs.

Workloads (--workload):
  B       (default, the headline)  synthetic HDL-64 scan (~126k points, all used as queries) vs a
          10-scan local map (~1.26M points); one "step" = `--inflight` independent scan pairs in
          flight, each = index build + 20 ICP iterations (fixed: delta thresholds −1), inputs already
          resident in HBM, one host sync per pair.  Shipped IMLS parameters (h=1, r=3, K=20, 30°).
  stream  config C/D-like: `--inflight` independent sequences, each a seeded HDL-64 drive through
          the GPU producer (ring PCA → geometric-features presample → major_axis sampling, ≤ 2000
          flat points); a step = one frame per sequence: the previous filtered scan joins the
          device map FIFO (map_push: only that scan crosses PCIe), the flat cloud is uploaded, and
          the frame is registered — host buffers in, pose out (PCIe included).
  A       config A: VLP-16 scan (~13k queries) vs the previous scan, inputs resident in HBM.
--solver LS (default) or RANSAC_DRPM (the shipped config.json solver: RANSAC → DRPM).

Measurement: the timed region (barrier + synchronize on both sides, max over ranks) carries no
instrumentation.  A separate probe afterwards registers `--latency-pairs` pairs ONE AT A TIME with
HIP events around every projection launch (on the stream it runs on): single-pair latency
(median / p90), single-pair ms per ICP iteration, and the dominant kernel's serialised duration,
which is what roofline.achieved divides the algorithmic bytes by (and what rocprofv3 --stats of the
same command reports).  The CPU baseline (rank 0, N = 1) is the oracle — test infrastructure, timed
here only as the reported baseline.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process per
GPU, each registers its own independent pairs (weak scaling); the only exchange is one
all-gather of the relative poses for trajectory chaining (RCCL; --backend gloo for CPU rehearsal).

Prints ONE JSON line (rank 0).  Progress goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import platform
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
from planetary_lidar_odometry_amd import _abi, config, imls_icp, sequences, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E nominal (MI355X_MICROARCH.md chip table)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------------------------------------
# distributed plumbing (shared with tests/test_bench_dist.py, which runs it on gloo)
# ------------------------------------------------------------------------------------------------
def dist_setup(backend: str = "auto"):
    """(world, rank, local_rank, torch device); initialises the process group when WORLD_SIZE > 1."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "auto":
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    use_cuda = backend == "nccl" or torch.cuda.is_available()
    if use_cuda:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    return world, rank, local, dev


def timed_steps(step, steps: int, world: int, dev, sync=None):
    """Run `steps` calls of step() between barrier + sync on both sides.  Returns (elapsed = max over
    ranks, per-step seconds of this rank, the concatenated per-step results)."""
    import torch.distributed as dist
    sync = sync or (lambda: None)
    if world > 1:
        dist.barrier()
    sync()
    per, out = [], []
    t0 = time.perf_counter()
    for _ in range(steps):
        ts = time.perf_counter()
        out.extend(step())
        per.append(time.perf_counter() - ts)
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dist.barrier()
        elapsed = float(tt.item())
    return elapsed, per, out


def exchange_poses(local_poses, world: int):
    """The one collective: all-gather of every rank's relative poses (unit order = rank-major blocks,
    sequences.shard_range) and the chained trajectory nowPose_k = prevLaserPose·rPose_k."""
    local_poses = np.asarray(local_poses, dtype=np.float64).reshape(-1, 4, 4)
    if world == 1:
        allp = local_poses
    else:
        allp = sequences.gather_relative_poses(local_poses, world * len(local_poses))
    return allp, sequences.chain_trajectory(allp)


# ------------------------------------------------------------------------------------------------
# CPU baseline (oracle: test infrastructure, used here only as the timed reported baseline)
# ------------------------------------------------------------------------------------------------
def host_info() -> dict:
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    allowed = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    return dict(cpu_model=model, os_cpu_count=os.cpu_count(), affinity_cpus=len(allowed),
                omp_num_threads=os.environ.get("OMP_NUM_THREADS"))


class _Pinned:
    """Pin this process to one CPU for the 1-thread leg (restored on exit)."""

    def __enter__(self):
        self.prev = os.sched_getaffinity(0)
        self.cpu = min(self.prev)
        os.sched_setaffinity(0, {self.cpu})
        return self

    def __exit__(self, *a):
        os.sched_setaffinity(0, self.prev)


def cpu_baseline(src, tgt, p, label: str, min_seconds: float = 10.0, max_pairs: int = 4, faithful_iters: int = 2,
                 tensors=None):
    """The oracle on the same pair (same parameters): (1) "efficient" port, 1 thread pinned: whole
    registrations repeated to >= min_seconds (<= max_pairs); (2) "faithful": the reference's
    container costs (erase per rejection, AoS copies, per-query heap vectors), 1 thread pinned, on
    the first `faithful_iters` ICP iterations, extrapolated per pair; (3) all cores: the per-query
    loop on every CPU this process may use (OpenMP)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_ctypes as oc
    info = host_info()
    iters = p.iterations
    with _Pinned() as pin:
        total, n, t_idx = 0.0, 0, 0.0
        while n < max_pairs and (n == 0 or total < min_seconds):
            r = oc.register_frame(src, tgt, p, tensors=tensors)
            total += r["seconds_total"]
            t_idx += r["seconds_index"]
            n += 1
        pf = _abi.ImlsParams.from_buffer_copy(p)
        pf.iterations = min(faithful_iters, iters)
        oc.set_faithful(True)
        try:
            rf = oc.register_frame(src, tgt, pf, tensors=tensors)
        finally:
            oc.set_faithful(False)
    t_iter_f = (rf["seconds_total"] - rf["seconds_index"]) / max(rf["iters"], 1)
    faithful_pair = rf["seconds_index"] + iters * t_iter_f
    threads = max(1, min(info["affinity_cpus"], int(os.environ.get("OMP_NUM_THREADS") or 10 ** 6)))
    oc.set_threads(threads)
    try:
        r2 = oc.register_frame(src, tgt, p, tensors=tensors)
    finally:
        oc.set_threads(1)
    return dict(
        value=n / total, unit="scan-pairs/s", cores=1, kind="port",
        sample=f"{n} whole registration(s) of the {label} pair ({src.shape[1]} queries vs {tgt.shape[1]}-pt map, "
               f"{r['iters']} ICP iterations each) in {total:.1f} s, index build {t_idx / n:.2f} s/pair; "
               f"oracle/imls_oracle.cpp -O3 (efficient port: stable compaction), 1 thread pinned to CPU {pin.cpu}",
        seconds_per_pair=total / n,
        faithful={"value": 1.0 / faithful_pair, "cores": 1, "seconds_per_pair": faithful_pair,
                  "sample": f"index build + {rf['iters']} of {iters} ICP iterations with the reference's container "
                            f"costs (erase per rejected point, AoS copy per iteration, per-query heap vectors), "
                            f"{rf['seconds_total']:.1f} s, extrapolated to {iters} iterations"},
        all_cores={"value": 1.0 / r2["seconds_total"], "cores": threads,
                   "sample": f"1 whole registration, per-query projection loop OpenMP over {threads} threads "
                             f"(index build and solver sequential)"},
        host=info)


# ------------------------------------------------------------------------------------------------
# workloads
# ------------------------------------------------------------------------------------------------
def soa_tensor(cloud, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(synth.soa(cloud))).to(dev).contiguous()


def algorithmic_bytes_per_launch(stats: dict, trace, iters: int) -> float:
    """B_q = 24 (query xyz+n) + 24·[NN found] + 24·k_q + 40·[valid], summed over
    the queries of one projection launch (k_q from the kernel's own counts)."""
    n_valid = float(np.mean([t.n_valid for t in trace])) if trace else 0.0
    return 24.0 * stats["queries"] + 24.0 * stats["nn_found"] / iters + 24.0 * stats["sum_kq"] / iters + 40.0 * n_valid


def solver_params(solver: str, iters: int) -> _abi.ImlsParams:
    p = config.bench_params(iters)                      # LS, fixed iteration count
    if solver == "RANSAC_DRPM":
        shipped = config.params_from_config(config.load())
        p.solve_method = shipped.solve_method           # RANSAC
        p.ransac_final_method = shipped.ransac_final_method   # DRPM
    return p


class Pipeline:
    """Fused steps: the contexts are split into `groups` parts, each registered as ONE launch
    sequence (register_frames_async).  A part is re-loaded (deferred uploads and NaN filters: no
    host wait, enqueued behind its running batch), collected and launched again while the other
    parts' batches still run, so batches
    overlap on the GPU (one fills another's tail) and the host work hides behind them (groups = 1:
    one batch per step, collected at the next step).  A step registers every context once and
    returns the results collected during it; the batches launched last stay in flight into the
    next step (the timed region's device-wide synchronize on both sides covers them)."""

    def __init__(self, ctxs, prep, groups=2):
        g = max(1, min(groups, len(ctxs)))
        bounds = [round(k * len(ctxs) / g) for k in range(g + 1)]
        self.halves = [ctxs[bounds[k]:bounds[k + 1]] for k in range(g)]
        self.prep = prep                  # prep(list of context indices)
        self.offs = bounds[:g]
        self.inflight = [False] * len(self.halves)
        self.t_wait = self.t_launch = 0.0   # host time in result waits / in register_frames_async

    def _collect(self, h):
        if not self.inflight[h]:
            return []
        self.inflight[h] = False
        t0 = time.perf_counter()
        poses, iters, st, _ = imls_icp.register_frames_result(self.halves[h])
        self.t_wait += time.perf_counter() - t0
        return list(zip(poses, iters, st))

    def step(self):
        out = []
        for h, half in enumerate(self.halves):
            # the part's next inputs are enqueued while its previous batch still runs (each
            # context's stream is ordered after the batch: set_target / map_push / set_source
            # touch nothing the batch reads before it ends), then its results are collected
            self.prep(range(self.offs[h], self.offs[h] + len(half)))
            out += self._collect(h)
            t0 = time.perf_counter()
            imls_icp.register_frames_async(half)    # builds (after the filter counts) + the batch's launches
            self.t_launch += time.perf_counter() - t0
            self.inflight[h] = True
        return out

    def drain(self):
        out = []
        for h in range(len(self.halves)):
            out += self._collect(h)
        return out


class PairRunner:
    """Configs A / B: independent pairs, inputs resident in HBM, one context per pair.  fuse: the
    step's pairs are registered as ONE launch sequence (imls_register_frames); else one launch
    sequence per pair, each on its context's stream."""

    def __init__(self, pairs, p, dev, local, fuse=True, groups=2, tensors=False):
        self.fuse = fuse
        self.pairs = pairs
        self.s_dev = [soa_tensor(q.source, dev) for q in pairs]
        self.t_dev = [soa_tensor(q.target, dev) for q in pairs]
        # config E: the targets' tensor-voting input tensors, SoA (6, M) in HBM
        self.ten_dev = None
        if tensors:
            import torch
            self.ten_dev = [torch.from_numpy(np.ascontiguousarray(q.meta["tensors"].T)).to(dev).contiguous() for q in pairs]
        self.ctxs = [imls_icp.ImlsContext(p, device=local) for _ in pairs]
        self.pipe = Pipeline(self.ctxs, self._prep, groups) if fuse else None

    def _prep(self, idx):
        for k in idx:
            q, c = self.pairs[k], self.ctxs[k]
            c.set_target_device(self.t_dev[k].data_ptr(), q.target.size, count=False)
            if self.ten_dev:
                c.set_target_tensors_device(self.ten_dev[k].data_ptr(), q.target.size)
            c.set_source_device(self.s_dev[k].data_ptr(), q.source.size, count=False)

    def step(self, ctxs=None, idx=None, fuse=None):
        fuse = self.fuse if fuse is None else fuse
        if fuse and ctxs is None:
            return self.pipe.step()
        ctxs = ctxs or self.ctxs
        idx = idx if idx is not None else range(len(self.pairs))
        for c, k in zip(ctxs, idx):
            q = self.pairs[k]
            c.set_target_device(self.t_dev[k].data_ptr(), q.target.size)
            if self.ten_dev:
                c.set_target_tensors_device(self.ten_dev[k].data_ptr(), q.target.size)
            c.set_source_device(self.s_dev[k].data_ptr(), q.source.size)
            if not fuse:
                c.register_frame_async()
        if fuse:
            poses, iters, st, _ = imls_icp.register_frames(ctxs)
            return list(zip(poses, iters, st))
        return [c.register_frame_result() for c in ctxs]

    def close(self):
        if self.pipe:
            self.pipe.drain()
        for c in self.ctxs:
            c.close()


class StreamRunner:
    """Config C/D-like: `n_seq` independent sequences (one context each); each step processes one
    frame per sequence exactly as LaserOdometry.process does (map_push of the previous filtered
    scan, set_source of the flat cloud, register), host buffers in.  A sequence ping-pongs over its
    F produced frames (0 … F−1 … 0 …) so every step registers two adjacent frames."""

    def __init__(self, n_seq, p, local, rank, frames_per_seq=5, fuse=True, unique=8, dev=None, resident=True, groups=2):
        from planetary_lidar_odometry_amd import producer
        self.fuse = fuse
        sm = synth.hdl64()
        self.seqs = []
        with imls_icp.ImlsContext(device=local) as pctx:
            for q in range(min(n_seq, max(unique, 1))):
                scene = synth.make_scene(17 * rank + q)
                poses = synth.trajectory(frames_per_seq + 3, 2000 + 31 * rank + q)
                sr = producer.ScanRegistration(ctx=pctx, shuffle_seed=q, rand_seed=1 + q)
                frames = []
                for k in range(frames_per_seq):
                    sw = synth.scan(scene, sm, poses[3 + k], seed=5000 + 100 * q + k)
                    xyz, sizes, inten = producer.sweep_inputs(sw, len(sm.rings))
                    frames.append(sr.process(xyz, sizes, inten))
                self.seqs.append(frames)
        # sequences beyond `unique` replay the produced ones (each still its own context and map
        # FIFO, at its own phase): producing every HDL-64 sweep on the host would dominate set-up
        u = len(self.seqs)
        # resident: every produced cloud already in HBM as SoA6 (the timed region starts with the
        # inputs resident, like config B; a step pushes / loads them device-to-device); else host
        # buffers cross PCIe inside the timed region (the reference's host-side hand-over)
        self.resident = resident
        self.dev_frames = ([[(soa_tensor(f, dev), soa_tensor(g, dev)) for f, g in fr] for fr in self.seqs]
                           if resident else None)
        self.seqs = [self.seqs[q % u] for q in range(n_seq)]
        self.dseq = [q % u for q in range(n_seq)]
        self.ctxs = [imls_icp.ImlsContext(p, device=local) for _ in range(n_seq)]
        self.pos = [(q // u) % frames_per_seq for q in range(n_seq)]
        self.dir = [1] * n_seq
        # frame 0 only seeds the map (Q13); afterwards each registered frame's filtered scan joins
        # the FIFO at the start of that sequence's next step, as LaserOdometry.process orders it
        self.pending = [fr[self.pos[q]][0] for q, fr in enumerate(self.seqs)]
        self.pending_k = list(self.pos)
        self.t_prep = self.t_reg = 0.0        # host time in the per-frame uploads / in registration
        self.pipe = Pipeline(self.ctxs, self._prep, groups) if fuse else None

    def _prep(self, idx):
        """One frame of each sequence in idx, as LaserOdometry.process orders it: the previous
        filtered scan joins the device map FIFO (only it crosses PCIe), the flat cloud is loaded;
        deferred (no host wait for the NaN-filtered counts)."""
        t0 = time.perf_counter()
        for q in idx:
            c = self.ctxs[q]
            k = self._advance(q)
            if self.resident:
                filt, _ = self.dev_frames[self.dseq[q]][self.pending_k[q]]
                _, flat = self.dev_frames[self.dseq[q]][k]
                c.map_push_device(filt.data_ptr(), filt.shape[1], count=False)
                c.set_source_device(flat.data_ptr(), flat.shape[1], count=False)
            else:
                c.map_push(self.pending[q], count=False)
                c.set_source(self.seqs[q][k][1], count=False)
            self.pending[q] = self.seqs[q][k][0]
            self.pending_k[q] = k
            self.pos[q] = k
        self.t_prep += time.perf_counter() - t0

    def _advance(self, q):
        F = len(self.seqs[q])
        nxt = self.pos[q] + self.dir[q]
        if nxt < 0 or nxt >= F:
            self.dir[q] = -self.dir[q]
            nxt = self.pos[q] + self.dir[q]
        return nxt

    def step(self):
        if self.pipe:
            t0 = time.perf_counter()
            p0 = self.t_prep
            out = self.pipe.step()
            self.t_reg += time.perf_counter() - t0 - (self.t_prep - p0)
            return out
        self._prep(range(len(self.ctxs)))               # one launch sequence per frame, own stream each
        t1 = time.perf_counter()
        for c in self.ctxs:
            c.register_frame_async()
        out = [c.register_frame_result() for c in self.ctxs]
        self.t_reg += time.perf_counter() - t1
        return out

    @property
    def queries(self):
        return int(np.mean([len(f[1]) for s in self.seqs for f in s]))

    @property
    def map_points(self):
        return int(np.mean([len(f[0]) for s in self.seqs for f in s]))

    def close(self):
        if self.pipe:
            self.pipe.drain()
        for c in self.ctxs:
            c.close()


def latency_probe(run_one, ctx, n_pairs: int, iters: int):
    """Pairs registered one at a time with per-launch HIP events (on the context's stream)."""
    ctx.enable_timing(True)
    ctx.reset_timing()
    lat = []
    for _ in range(n_pairs):
        t = time.perf_counter()
        run_one()
        lat.append(time.perf_counter() - t)
    ctx.enable_timing(False)
    # one more pair with the traversal / neighbour counters on (Σk_q, NN found: the algorithmic
    # bytes) — counted apart from the timed pairs, whose kernels then carry no counter atomics
    ctx.enable_stats(True)
    run_one()
    ctx.enable_stats(False)
    k = {name: ctx.kernel_timing(i) for i, name in enumerate(("projection", "index", "solve", "k_knn_wave", "k_finish"))}
    lat = np.array(lat) * 1e3
    idx_ms = k["index"][0] / max(k["index"][1], 1)
    return dict(pairs=n_pairs, median_ms=float(np.median(lat)), p90_ms=float(np.percentile(lat, 90)),
                ms_per_iteration=float((np.median(lat) - idx_ms) / iters),
                kernel_avg_ms={n: v[0] / max(v[1], 1) for n, v in k.items()},
                launches={n: int(v[1]) for n, v in k.items()})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--queries", type=int, default=0, help="config B: 0 = all source points; else FPS subsample")
    ap.add_argument("--inflight", type=int, default=0,
                    help="independent pairs / sequences per step (0 = workload default: B 4, A 256, stream 1024)")
    ap.add_argument("--no-fuse", action="store_true",
                    help="one launch sequence per pair on its own stream instead of one for the whole step")
    ap.add_argument("--unique-seqs", type=int, default=8, help="stream: distinct produced sequences")
    ap.add_argument("--groups", type=int, default=0,
                    help="fused: launch sequences the step's pairs are split into, kept in flight together "
                         "(0 = workload default: B 4, A 1, stream 1)")
    ap.add_argument("--host-inputs", action="store_true",
                    help="stream: frames handed over in host memory (PCIe inside the timed region)")
    ap.add_argument("--latency-pairs", type=int, default=50, help="single-pair latency / roofline probe size")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU-baseline leg")
    ap.add_argument("--backend", choices=["auto", "nccl", "gloo"], default="auto")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    ap.add_argument("--workload", choices=["B", "stream", "A", "E"], default="B")
    ap.add_argument("--solver", choices=["LS", "RANSAC_DRPM"], default="LS")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    world, rank, local, dev = dist_setup(args.backend)
    # config B: each pair already fills the GPU; 4 in flight as 4 one-pair launch sequences measured
    # best (pairs per sequence × sequences: 1×4 264.7, 2×2 252.4, 2×4 255.7, 3×2 237.2, 4×2 231,
    # 8×2 205 pairs/s: more per launch only adds cache pressure).  The ~1900-query stream frames
    # need many per launch: 64 per sequence × 2 → 2819 frames/s (32 × 4: 1841)
    # measured (profiles/r02_final): B pairs fill the GPU alone and run best as 4 one-pair launch
    # sequences in flight; the small A / stream frames run best as ONE large batch per step (two
    # half batches in flight share hardware queues, so a filter of one half can wait behind the
    # other half's launch sequence)
    P = args.inflight if args.inflight > 0 else {"B": 4, "A": 256, "stream": 1024, "E": 256}[args.workload]
    if args.groups <= 0:
        args.groups = {"B": 4, "A": 1, "stream": 1, "E": 1}[args.workload]
    fuse = not args.no_fuse
    p = solver_params(args.solver, args.iters)
    if args.workload == "E":
        # config E: normals by tensor voting (VoteForAny, k 50, σ 0.2, threshold 0.6) on the targets'
        # input tensors; the map's IMLS normals recomputed in count mode (get_normals false)
        p.get_normals, p.recompute_normal_count_mode = 0, 1
        p.use_tensor_voting, p.tensor_k, p.tensor_sigma, p.tensor_distance_threshold = 1, 50, 0.2, 0.6
    t0 = time.time()
    if args.workload == "stream":
        runner = StreamRunner(P, p, local, rank, fuse=fuse, unique=args.unique_seqs, dev=dev,
                              resident=not args.host_inputs, groups=args.groups)
        probe_ctx = runner.ctxs[0]
        queries, map_points = runner.queries, runner.map_points
        single = None
    else:
        if args.workload == "E":
            # sparse VLP-16 scans over the planetary heightfield (synth.make_planetary_pair: ~10 s of
            # host ray casting each): two distinct pairs, replayed by the step's contexts
            uniq = [synth.make_planetary_pair(scene_seed=3 + rank, start=30 + k) for k in range(min(P, 2))]
            pairs = [uniq[k % len(uniq)] for k in range(P)]
        else:
            model, map_scans = ("vlp16", 1) if args.workload == "A" else ("hdl64", 10)
            pairs = synth.make_pairs(P, model, map_scans=map_scans, scene_seed=rank, traj_seed=2000 + rank,
                                     noise_seed=1000 + 97 * rank)
        if args.queries > 0:
            pairs = [synth.Pair(synth.fps_subsample(q.source, args.queries, seed=rank), q.target, q.true_pose, q.meta)
                     for q in pairs]
        runner = PairRunner(pairs, p, dev, local, fuse=fuse, groups=args.groups, tensors=args.workload == "E")
        probe_ctx = runner.ctxs[0]
        queries, map_points = pairs[0].source.size, pairs[0].target.size
        # the probe runs the one-frame launch sequence: its events separate k_knn_wave and k_finish
        single = lambda: runner.step([probe_ctx], [0], fuse=False)   # noqa: E731
    log(f"[rank {rank}] workload {args.workload} set up in {time.time() - t0:.1f}s: {P} in flight, "
        f"~{queries} queries vs ~{map_points}-pt maps, solver {args.solver}")
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        res = runner.step()
    if args.workload != "stream":
        if runner.pipe:                  # pipelined results arrive out of pair order: check one plain pass
            runner.pipe.drain()
            res = runner.step(runner.ctxs, range(P), fuse=False)
        errs = [np.linalg.norm(r[0][:3, 3] - q.true_pose[:3, 3]) for r, q in zip(res, runner.pairs)]
        log(f"[rank {rank}] warmup done; max pose error vs truth {max(errs) * 100:.2f} cm")

    if hasattr(runner, "t_prep"):
        runner.t_prep = runner.t_reg = 0.0
    if getattr(runner, "pipe", None):
        runner.pipe.t_wait = runner.pipe.t_launch = 0.0
    elapsed, per_step, res = timed_steps(runner.step, args.steps, world, dev, torch.cuda.synchronize)
    if getattr(runner, "pipe", None):
        res += runner.pipe.drain()        # the batches still in flight (already finished: synchronized)
    if hasattr(runner, "t_prep"):
        log(f"[rank {rank}] host time per step: uploads (+ filters) {runner.t_prep / args.steps * 1e3:.2f} ms, "
            f"rest (builds, launches, waits) {runner.t_reg / args.steps * 1e3:.2f} ms")
    if getattr(runner, "pipe", None):
        log(f"[rank {rank}] pipeline host time per step: result waits {runner.pipe.t_wait / args.steps * 1e3:.2f} ms, "
            f"register_frames_async (builds + launches) {runner.pipe.t_launch / args.steps * 1e3:.2f} ms")
    poses = [r[0] for r in res]
    allp, traj = exchange_poses(poses, world)          # the one RCCL exchange (trajectory chaining)
    n_pairs = args.steps * P
    value = world * n_pairs / elapsed

    # single-pair latency + serialised per-launch kernel durations (roofline), outside the timed region
    probe = latency_probe(single, probe_ctx, args.latency_pairs, args.iters) if single else None
    stats = probe_ctx.index_stats()
    trav = probe_ctx.traversal_stats()
    bytes_launch = algorithmic_bytes_per_launch(stats, probe_ctx.last_trace, args.iters)

    if rank != 0:
        runner.close()
        if world > 1:
            dist.destroy_process_group()
        return

    traffic = None
    tj = pathlib.Path(args.traffic_json)
    if tj.exists() and args.workload == "B":
        try:
            tdat = json.loads(tj.read_text())
            if tdat.get("queries") == stats["queries"] and tdat.get("iters") == args.iters:
                traffic = tdat.get("bytes_per_launch")
        except (ValueError, OSError):
            traffic = None

    cpu = None
    if world == 1 and not args.no_cpu and args.workload != "stream":
        log("[rank 0] CPU baseline (oracle) ...")
        q0 = runner.pairs[0]
        cpu = cpu_baseline(synth.soa(q0.source), synth.soa(q0.target), p, f"config {args.workload}",
                           tensors=np.ascontiguousarray(q0.meta["tensors"].T) if args.workload == "E" else None)
        log(f"[rank 0] CPU baseline {cpu['value']:.4f} pairs/s (faithful {cpu['faithful']['value']:.4f}, "
            f"{cpu['all_cores']['cores']} cores {cpu['all_cores']['value']:.3f})")

    roof = None
    if probe:
        kd = probe["kernel_avg_ms"]
        dom_ms = kd["k_knn_wave"] + kd["k_finish"]
        achieved = bytes_launch / (dom_ms / 1e3) / 1e9 if dom_ms > 0 else 0.0
        roof = {
            "bound": "hbm",
            "kernel": "projection step = k_knn_wave (packet traversal) + k_finish (exact re-rank, gates, IMLS, "
                      "pass-1 normal equations); serialised per-launch HIP-event duration, one pair in flight",
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "algorithmic_bytes_per_launch": bytes_launch,
            "avg_launch_ms": dom_ms,
            "kernel_avg_ms": kd,
            "aggregate_algorithmic_GBps": bytes_launch * args.iters * n_pairs * world / elapsed / 1e9,
            "aggregate_frac": bytes_launch * args.iters * n_pairs * world / elapsed / 1e9 / HBM_PEAK_GBS,
        }
    solver_txt = "LS (trimmed, t=0.02)" if args.solver == "LS" else "RANSAC -> DRPM (shipped config.json solver)"
    if args.workload == "B":
        metric = "IMLS-ICP scan-pairs/s (HDL-64 ~120k-pt scan vs 10-scan map, 20 ICP iterations)"
        workload = f"config B: HDL-64 scan vs 10-scan local map; a step = {P} independent scan pairs" + (" in one launch sequence" if fuse else " in flight, one stream each")
        unit = "scan-pairs/s"
    elif args.workload == "E":
        metric = ("IMLS-ICP scan-pairs/s (config E: tensor-voting normals + IMLS on sparse VLP-16 planetary scans, "
                  "20 ICP iterations)")
        workload = f"config E: planetary VLP-16 scan vs the previous scan, tensor voting; a step = {P} independent pairs" + (" in one launch sequence" if fuse else " in flight, one stream each")
        unit = "scan-pairs/s"
    elif args.workload == "A":
        metric = "IMLS-ICP scan-pairs/s (config A: VLP-16 scan vs 1-scan map, 20 ICP iterations)"
        workload = f"config A: VLP-16 scan vs the previous scan; a step = {P} independent pairs" + (" in one launch sequence" if fuse else " in flight, one stream each")
        unit = "scan-pairs/s"
    else:
        metric = ("IMLS-ICP frames/s (config C/D-like stream: producer-sampled <=2000-pt flat clouds of HDL-64 "
                  "sweeps vs the device map FIFO, 20 ICP iterations" +
                  (", host hand-over: PCIe of the new scan included)" if args.host_inputs else
                   ", frames resident in HBM)"))
        workload = f"config C/D-like: {P} independent sequences, one frame each per step" + (" in one launch sequence" if fuse else ", one stream each")
        unit = "frames/s"
    per = np.array(per_step) * 1e3
    out = {
        "metric": metric,
        "value": value,
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "ms_per_step_median": float(np.median(per)),
        "ms_per_step_p90": float(np.percentile(per, 90)),
        "ms_per_pair": elapsed / n_pairs * 1e3,
        "pairs_in_flight": P,
        "ms_per_iteration": elapsed / n_pairs * 1e3 / args.iters,
        "single_pair": probe,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded HDL-64 / VLP-16 ray-cast urban scene, planetary-lidar-odometry_amd/synth.py)",
        "config": {
            "workload": workload,
            "queries": int(stats["queries"]) if args.workload != "stream" else queries,
            "map_points": int(stats["points"]) if args.workload != "stream" else map_points,
            "icp_iterations": args.iters,
            "solver": solver_txt,
            "search_number": p.search_number,
            "fused_launch": fuse,
            "launch_groups": args.groups if fuse else P,
            "parallelism": f"independent pairs per GPU over {world} GPU(s), RCCL pose all-gather" if world > 1 else "1 GPU",
        },
        "roofline": roof,
        "traversal_per_launch": {k: v / args.iters for k, v in trav.items()},
        "trajectory_end": traj[-1][:3, 3].tolist() if len(traj) else None,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    runner.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
