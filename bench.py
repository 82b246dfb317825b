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
B_HOST_DEFAULT = False  # config B: host hand-over by default (else --host-inputs)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------------------------------------
# distributed plumbing (shared with tests/test_bench_dist.py, which runs it on gloo)
# ------------------------------------------------------------------------------------------------
def dist_setup(backend: str = "auto"):
    """(world, rank, local_rank, torch device).  Under a launcher (torch.distributed.run sets
    WORLD_SIZE, even at N = 1) the process group is initialised, so the launched bench always runs
    its collectives — barrier, max-over-ranks timing, the pose all-gather — over RCCL (nccl) or gloo;
    a plain `python bench.py` (no WORLD_SIZE) stays single-process without a group."""
    import torch
    import torch.distributed as dist
    launched = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "auto":
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    use_cuda = backend == "nccl" or torch.cuda.is_available()
    if use_cuda:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    if (launched or world > 1) and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    return world, rank, local, dev


def _grouped() -> bool:
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def timed_steps(step, steps: int, world: int, dev, sync=None):
    """Run `steps` calls of step() between barrier + sync on both sides.  Returns (elapsed = max over
    ranks, per-step seconds of this rank, the concatenated per-step results)."""
    import torch.distributed as dist
    sync = sync or (lambda: None)
    grouped = _grouped()
    if grouped:
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
    if grouped:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dist.barrier()
        elapsed = float(tt.item())
    return elapsed, per, out


def exchange_poses(results, world: int, rank: int = 0):
    """The one collective: all-gather of every rank's (sequence, frame order, relative pose) records
    and each sequence's trajectory nowPose_k = prevLaserPose·rPose_k chained on its own
    (laser_odometry.cpp:652-655; config D: 8 independent sequences, never one trajectory).
    results: [(seq, order, pose 4×4)], seq ids local to the rank (made global as rank·2^20 + seq).
    Returns (records (seq, order, pose) of every rank, {seq: (orders, trajectory)})."""
    seq = np.array([rank * (1 << 20) + int(r[0]) for r in results], dtype=np.int64)
    order = np.array([int(r[1]) for r in results], dtype=np.int64)
    poses = np.asarray([r[2] for r in results], dtype=np.float64).reshape(-1, 4, 4)
    if world > 1 or _grouped():           # over the process group whenever there is one (RCCL on GPU)
        seq, order, poses = sequences.gather_tagged_poses(seq, order, poses)
    return (seq, order, poses), sequences.chain_per_sequence(seq, order, poses)


RANK_ROOF_FIELDS = ("algorithmic_bytes_per_step", "busy_projection_ms_per_step", "ms_per_step",
                    "serialised_launch_ms", "algorithmic_bytes_per_launch")


def rank_roofline(bytes_per_step: float, busy, busy_steps: int, per_step, probe, bytes_per_launch: float) -> list:
    """This rank's roofline inputs (RANK_ROOF_FIELDS order): its own step's algorithmic bytes, the
    time its projection kernels were busy per step (HIP-event union, busy pass; 0 without one), its
    own mean timed step, and its serialised single-pair launch (k_knn_wave + k_finish, 0 without)."""
    busy_ms = busy["projection_busy_ms"] / busy_steps if busy and busy_steps > 0 else 0.0
    dom = 0.0
    if probe:
        kd = probe["kernel_avg_ms"]
        dom = kd.get("k_knn_wave", 0.0) + kd.get("k_finish", 0.0)
    return [float(bytes_per_step), float(busy_ms), float(np.mean(per_step) * 1e3) if len(per_step) else 0.0,
            float(dom), float(bytes_per_launch)]


def gather_rank_roofline(vals: list, world: int, dev) -> list:
    """All-gather of every rank's rank_roofline() values (one collective, every rank calls it — before
    any rank leaves main), expanded per rank with its achieved HBM GB/s and fraction of the peak: the
    busy-pass figure (bytes per step / busy projection time) and the serialised single-pair one.
    SURVEY §8(e): the per-GPU achieved HBM fraction of the multi-GPU run."""
    import torch
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    if _grouped() and world > 1:
        import torch.distributed as dist
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        rows = [o.cpu().tolist() for o in out]
    else:
        rows = [t.cpu().tolist()]
    recs = []
    for r, row in enumerate(rows):
        d = dict(zip(RANK_ROOF_FIELDS, row), rank=r)
        busy = d["busy_projection_ms_per_step"]
        d["achieved"] = d["algorithmic_bytes_per_step"] / (busy / 1e3) / 1e9 if busy > 0 else None
        d["frac"] = d["achieved"] / HBM_PEAK_GBS if d["achieved"] is not None else None
        ser = d["serialised_launch_ms"]
        d["serialised_achieved"] = d["algorithmic_bytes_per_launch"] / (ser / 1e3) / 1e9 if ser > 0 else None
        d["serialised_frac"] = d["serialised_achieved"] / HBM_PEAK_GBS if ser > 0 else None
        recs.append(d)
    return recs


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
                omp_num_threads=os.environ.get("OMP_NUM_THREADS"), cpu_quota=cpu_quota())


def cpu_quota() -> dict:
    """The CPU bandwidth limit of this process's cgroup, read where the kernel exposes it: cgroup v2
    cpu.max ("<quota> <period>" or "max <period>") or v1 cpu.cfs_quota_us / cpu.cfs_period_us
    (−1 = unlimited).  cpus = quota / period (null when unlimited or unreadable)."""
    def rd(path):
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            return None
    v2 = rd("/sys/fs/cgroup/cpu.max")
    if v2:
        q, per = (v2.split() + ["100000"])[:2]
        cpus = None if q == "max" else int(q) / int(per)
        return dict(source="/sys/fs/cgroup/cpu.max", raw=v2, cpus=cpus)
    q = rd("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") or rd("/sys/fs/cgroup/cpu,cpuacct/cpu.cfs_quota_us")
    per = rd("/sys/fs/cgroup/cpu/cpu.cfs_period_us") or rd("/sys/fs/cgroup/cpu,cpuacct/cpu.cfs_period_us")
    if q is not None:
        cpus = None if int(q) < 0 or not per else int(q) / int(per)
        return dict(source="/sys/fs/cgroup/cpu/cpu.cfs_quota_us", raw=f"{q} {per}", cpus=cpus)
    return dict(source=None, raw=None, cpus=None)


class _Pinned:
    """Pin this process to one CPU for the 1-thread leg (restored on exit)."""

    def __enter__(self):
        self.prev = os.sched_getaffinity(0)
        self.cpu = min(self.prev)
        os.sched_setaffinity(0, {self.cpu})
        return self

    def __exit__(self, *a):
        os.sched_setaffinity(0, self.prev)


def cpu_baseline(src, tgt, p, label: str, min_seconds: float = 10.0, max_pairs: int = 4, tensors=None,
                 faithful: bool = True):
    """The oracle on the same pair (same parameters).  Returns (baseline dict, the oracle's first
    result — the parity reference of that pair).
      (1) "efficient" port, 1 thread pinned: whole registrations repeated to >= min_seconds;
      (2) "faithful": the reference's container costs (erase per rejection, AoS copies, per-query heap
          vectors), 1 thread pinned, one whole registration (every ICP iteration);
      (3) "host_share": the per-query loop OpenMP over this process's CPU share (OMP_NUM_THREADS on
          the GPU box: 16 of its 256 CPUs per GPU — the box's rule for worker pools), plus the
          perfect-scaling bound of the 1-thread figure over every CPU the process may run on (an
          upper bound for the whole socket pair: the index build and solver are sequential)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_ctypes as oc
    info = host_info()
    iters = p.iterations
    first = None
    with _Pinned() as pin:
        total, n, t_idx = 0.0, 0, 0.0
        while n < max_pairs and (n == 0 or total < min_seconds):
            r = oc.register_frame(src, tgt, p, tensors=tensors)
            first = first or r
            total += r["seconds_total"]
            t_idx += r["seconds_index"]
            n += 1
        rf = None
        if faithful:
            oc.set_faithful(True)
            try:
                rf = oc.register_frame(src, tgt, p, tensors=tensors)
            finally:
                oc.set_faithful(False)
    # SURVEY §8(d)'s secondary baseline is the per-query loop on every host core.  The process's CPU
    # share is the smallest of: its affinity set, the cgroup CPU quota, and OMP_NUM_THREADS (the GPU
    # pool sets 16 per GPU and requires worker pools sized to it) — measured at that share, with the
    # thread-scaling curve below it; all cores are measured only when nothing caps the share
    q = info["cpu_quota"]
    omp = int(os.environ.get("OMP_NUM_THREADS") or 10 ** 6)
    share = max(1, min(info["affinity_cpus"], omp, int(q["cpus"]) if q["cpus"] else 10 ** 6))
    threads = share
    curve = {}
    for t in sorted({k for k in (2, 4, 8) if k < threads} | {threads}):
        oc.set_threads(t)
        try:
            r2 = oc.register_frame(src, tgt, p, tensors=tensors)
        finally:
            oc.set_threads(1)
        curve[t] = 1.0 / r2["seconds_total"]
    one = n / total
    capped_by = [name for name, v in (("affinity", info["affinity_cpus"]), ("OMP_NUM_THREADS", omp),
                                      ("cgroup quota", int(q["cpus"]) if q["cpus"] else 10 ** 6)) if v == share]
    all_cores = dict(measured=share >= info["affinity_cpus"], value=curve[threads] if share >= info["affinity_cpus"] else None,
                     cores=share, affinity_cpus=info["affinity_cpus"], capped_by=capped_by,
                     quota={"cgroup": q, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
                            "source": "cgroup cpu.max / cpu.cfs_quota_us as read; OMP_NUM_THREADS from the environment "
                                      "(the GPU pool: 16 CPUs per GPU, worker pools sized to it)"},
                     scaling={str(k): v for k, v in curve.items()},
                     scaling_efficiency=curve[threads] / (threads * one) if threads > 1 else 1.0)
    out = dict(
        value=one, unit="scan-pairs/s", cores=1, kind="port",
        sample=f"{n} whole registration(s) of the {label} pair ({src.shape[1]} queries vs {tgt.shape[1]}-pt map, "
               f"{r['iters']} ICP iterations each) in {total:.1f} s, index build {t_idx / n:.2f} s/pair; "
               f"oracle/imls_oracle.cpp -O3 (efficient port: stable compaction), 1 thread pinned to CPU {pin.cpu}",
        seconds_per_pair=total / n,
        host_share={"value": curve[threads], "cores": threads,
                    "sample": f"1 whole registration, per-query projection loop OpenMP over {threads} threads "
                              f"(this process's CPU share; index build and solver sequential)"},
        all_cores=all_cores,
        all_cpus_linear_bound={"value": one * info["affinity_cpus"], "cores": info["affinity_cpus"],
                               "sample": "1-thread value x every CPU in sched_getaffinity (perfect scaling: an "
                                         "upper bound, not a measurement)"},
        host=info)
    if rf is not None:
        out["faithful"] = {"value": 1.0 / rf["seconds_total"], "cores": 1, "seconds_per_pair": rf["seconds_total"],
                           "sample": f"1 whole registration (index build + all {rf['iters']} ICP iterations) with the "
                                     f"reference's container costs (erase per rejected point, AoS copy per iteration, "
                                     f"per-query heap vectors), {rf['seconds_total']:.1f} s"}
    return out, first


def parity_vs_oracle(got: dict, want: dict, truth=None) -> dict:
    """The GPU's single-frame result of a pair against the oracle's (DESIGN §3 contract: iterations,
    status, per-iteration valid counts and reject counters exact; pose within 1e-6 (1e-5 through
    DRPM's device erfc)).  truth: the synthetic relative pose — both results' translation error
    against it shows whether a large error is the algorithm's (shared) or the kernels'."""
    tg, tw = got["trace"], want["trace"]
    d = {
        "max_pose_diff_vs_oracle": float(np.abs(np.asarray(got["pose"]) - np.asarray(want["pose"])).max()),
        "iters_equal": int(got["iters"]) == int(want["iters"]),
        "status_equal": int(got["status"]) == int(want["status"]),
        "n_valid_equal": len(tg) == len(tw) and all(a.n_valid == b.n_valid for a, b in zip(tg, tw)),
        "rejects_equal": len(tg) == len(tw) and all(list(a.reject) == list(b.reject) for a, b in zip(tg, tw)),
        "iters": int(got["iters"]),
    }
    if truth is not None:
        d["gpu_truth_err_cm"] = float(np.linalg.norm(np.asarray(got["pose"])[:3, 3] - truth[:3, 3]) * 100)
        d["oracle_truth_err_cm"] = float(np.linalg.norm(np.asarray(want["pose"])[:3, 3] - truth[:3, 3]) * 100)
    return d


# ------------------------------------------------------------------------------------------------
# workloads
# ------------------------------------------------------------------------------------------------
def soa_tensor(cloud, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(synth.soa(cloud))).to(dev).contiguous()


def frame_bytes(stats: dict, n_queries: int, trace) -> float:
    """SURVEY §8(d) algorithmic bytes of one frame's projections, summed over the iterations it ran:
    Σ_it Σ_q [24 (query xyz+n) + 24·[NN found] + 24·k_q + 40·[valid]] (k_q and NN-found from the
    kernels' own counters, accumulated over the frame)."""
    its = len(trace)
    return (24.0 * n_queries * its + 24.0 * stats["nn_found"] + 24.0 * stats["sum_kq"]
            + 40.0 * float(sum(t.n_valid for t in trace)))


def solver_params(solver: str, iters: int) -> _abi.ImlsParams:
    p = config.bench_params(iters)                      # LS, fixed iteration count
    if solver == "RANSAC_DRPM":
        shipped = config.params_from_config(config.load())
        p.solve_method = shipped.solve_method           # RANSAC
        p.ransac_final_method = shipped.ransac_final_method   # DRPM
    return p


class Pipeline:
    """Fused steps: the contexts are split into `groups` parts, each registered as ONE launch
    sequence (register_frames_async).  A part is re-loaded (count-less uploads: no host wait,
    enqueued behind its running batch), collected and launched again while the other parts' batches
    still run, so batches overlap on the GPU (one fills another's tail) and the host work hides
    behind them (groups = 1: one batch per step, collected at the next step).  A step registers
    every context once and returns the results collected during it, tagged with the context index:
    (k, pose, iterations, status, trace); the batches launched last stay in flight into the next
    step (the timed region's device-wide synchronize on both sides covers them)."""

    def __init__(self, ctxs, prep, groups=2):
        g = max(1, min(groups, len(ctxs)))
        bounds = [round(k * len(ctxs) / g) for k in range(g + 1)]
        self.halves = [ctxs[bounds[k]:bounds[k + 1]] for k in range(g)]
        self.prep = prep                  # prep(list of context indices)
        self.offs = bounds[:g]
        self.inflight = [False] * len(self.halves)
        self.t_wait = self.t_launch = 0.0   # host time in result waits / in register_frames_async
        self.t_prep = self.t_tag = 0.0      # host time in the parts' input loads / in tagging the results

    def _order(self, h):
        """Part h's contexts in the order handed to register_frames_async: rotated by h, so that the
        parts' lead contexts — whose streams carry their launch sequences — are consecutive contexts
        (consecutively created streams land on different hardware queues; equal-sized parts' first
        contexts can share one, and one part's filter then waits behind the other's batch)."""
        half = self.halves[h]
        r = h % len(half)
        return half[r:] + half[:r]

    def _collect(self, h):
        if not self.inflight[h]:
            return []
        self.inflight[h] = False
        t0 = time.perf_counter()
        poses, iters, st, tr = imls_icp.register_frames_result(self._order(h))
        self.t_wait += time.perf_counter() - t0
        n, r = len(self.halves[h]), h % len(self.halves[h])
        return [(self.offs[h] + (r + j) % n, poses[j], int(iters[j]), int(st[j]), tr[j]) for j in range(len(poses))]

    def step(self):
        out = []
        for h, half in enumerate(self.halves):
            # the part's next inputs are enqueued while its previous batch still runs (each
            # context's stream is ordered after the batch: set_target / map_push / set_source
            # touch nothing the batch reads before it ends), then its results are collected
            t0 = time.perf_counter()
            self.prep(range(self.offs[h], self.offs[h] + len(half)))
            t1 = time.perf_counter()
            self.t_prep += t1 - t0
            got = self._collect(h)
            t2 = time.perf_counter()
            out += got
            self.t_tag += time.perf_counter() - t2
            t0 = time.perf_counter()
            imls_icp.register_frames_async(self._order(h))   # builds (after the filter counts) + the batch's launches
            self.t_launch += time.perf_counter() - t0
            self.inflight[h] = True
        return out

    def drain(self):
        out = []
        for h in range(len(self.halves)):
            out += self._collect(h)
        return out


class PairRunner:
    """Configs A / B / E: independent pairs, inputs resident in HBM, one context per pair.  fuse:
    the step's pairs are registered as `groups` launch sequences in flight (Pipeline); else one
    launch sequence per pair, each on its context's stream.  RANSAC: every registration starts its
    context's rand() stream from params.ransac_seed (each pair is an independent registration, the
    reference's first frame), so a result depends on its pair alone."""

    def __init__(self, pairs, p, dev, local, fuse=True, groups=2, tensors=False, alloc=None, host=False):
        self.fuse = fuse
        self.pairs = pairs
        self.ransac = p.solve_method == _abi.IMLS_SOLVE_RANSAC
        # host: the deployment hand-over (SURVEY §8(d) t_pair) — every context keeps its map as a
        # device FIFO of the map's scans (max_queue_size = their number, accumulateTargetCloud
        # laser_odometry.cpp:116-136), and each registration takes the NEWEST scan and the source
        # from host memory as the reference's 48-B PointXYZINormal records (map_push + set_source:
        # pack + PCIe inside the timed region).  The pushed scan cycles through the pair's map
        # scans, so the FIFO always holds the same points, concatenated from a rotating first scan
        # (self.rot[k] = that scan's index for the context's last load).
        self.host = host
        self.local = local
        self.p = type(p).from_buffer_copy(p)             # (host mode sets its max_queue_size)
        p = self.p
        if host:
            self.parts = [synth.map_parts(q) for q in pairs]
            self.p.max_queue_size = len(self.parts[0])
            self.tick = [0] * len(pairs)
            self.rot = [0] * len(pairs)
        # device copies (anything with data_ptr()): torch tensors, or `alloc(float32 array)`
        to_dev = alloc or (lambda a: __import__("torch").from_numpy(np.ascontiguousarray(a)).to(dev).contiguous())
        self.s_dev = [to_dev(synth.soa(q.source)) for q in pairs] if not host else None
        self.t_dev = [to_dev(synth.soa(q.target)) for q in pairs] if not host else None
        # config E: the targets' tensor-voting input tensors, SoA (6, M) in HBM
        self.ten_dev = None
        if tensors:
            self.ten_dev = [to_dev(np.ascontiguousarray(q.meta["tensors"].T)) for q in pairs]
        self.ctxs = [imls_icp.ImlsContext(p, device=local) for _ in pairs]
        self.seed_state = self.ctxs[0].rng_state()        # a fresh context's stream (params.ransac_seed)
        if host:
            for k, c in enumerate(self.ctxs):             # the FIFO's steady state: every map scan once
                for part in self.parts[k]:
                    c.map_push(part, count=False)
        # deferred reads of the count-less device loads: a large batch filters all its members in
        # three launches (the inputs stay resident and unchanged for the whole run)
        per_group = len(pairs) / max(1, groups)
        for c in self.ctxs:
            c.set_defer(fuse and per_group >= 8)
        self.pipe = Pipeline(self.ctxs, self._prep, groups) if fuse else None

    def _load(self, c, k, count):
        q = self.pairs[k]
        if self.ransac:
            c.set_rng_state(self.seed_state)
        if self.host:
            parts = self.parts[k]
            i = self.tick[k] % len(parts)
            self.tick[k] += 1
            c.map_push(parts[i], count=count)             # the new scan: host records → FIFO
            self.rot[k] = (i + 1) % len(parts)            # the FIFO now starts at scan i + 1
            c.set_source(q.source, count=count)
            return
        c.set_target_device(self.t_dev[k].data_ptr(), q.target.size, count=count)
        if self.ten_dev:
            c.set_target_tensors_device(self.ten_dev[k].data_ptr(), q.target.size)
        c.set_source_device(self.s_dev[k].data_ptr(), q.source.size, count=count)

    def _prep(self, idx):
        for k in idx:
            self._load(self.ctxs[k], k, False)

    def step(self):
        if self.fuse:
            return self.pipe.step()
        return self.single()

    def single(self, idx=None):
        """Each pair (or pairs idx) registered alone, one launch sequence per pair on its own
        context's stream (imls_register_frame: the single-frame kernels), tagged like Pipeline."""
        idx = list(range(len(self.pairs)) if idx is None else idx)
        for k in idx:
            self._load(self.ctxs[k], k, True)
            self.ctxs[k].register_frame_async()
        out = []
        for k in idx:
            pose, it, st = self.ctxs[k].register_frame_result()
            out.append((k, pose, it, st, self.ctxs[k].last_trace))
        return out

    def single_fresh(self, k: int, rot: int = 0):
        """Pair k registered alone on a fresh context whose map is the pair's scans from scan `rot`
        on (host mode: the same FIFO content — the scans pushed in that order, so its incremental
        index is the one the timed context built; else the pair's target): the single-frame kernels,
        tagged like Pipeline."""
        with imls_icp.ImlsContext(self.p, device=self.local) as c:
            if self.ransac:
                c.set_rng_state(self.seed_state)
            if self.host:
                parts = self.parts[k]
                for part in parts[rot:] + parts[:rot]:
                    c.map_push(part, count=False)
            else:
                c.set_target(self.pairs[k].target)
            c.set_source(self.pairs[k].source)
            r = c.register_frame()
        return (k, r["pose"], r["iters"], r["status"], r["trace"])

    def drain(self):
        return self.pipe.drain() if self.pipe else []

    def close(self):
        self.drain()
        for c in self.ctxs:
            c.close()


class StreamRunner:
    """Config C/D-like: `n_seq` independent sequences (one context each); each step processes one
    frame per sequence in LaserOdometry.process's order (map_push of the previous filtered scan,
    set_source of the flat cloud, register).  One difference, for RANSAC only: every frame restarts
    its context's rand() stream from params.ransac_seed (_prep), so a frame's result depends on that
    frame alone and can be verified by re-registering it on a fresh context; LaserOdometry and the
    reference instead run one stream across the sequence's frames.  The draws per frame are the same
    in number and kind, so the stream-RANSAC frames/s measures the same work.  A sequence ping-pongs over its F produced frames
    (0 … F−1 … 0 …) so every step registers two adjacent frames.  Results are tagged with the
    context index; self.last[q] = (map frame, source frame) of the frame most recently loaded."""

    def __init__(self, n_seq, p, local, rank, frames_per_seq=5, fuse=True, unique=8, dev=None, resident=True, groups=2):
        from planetary_lidar_odometry_amd import producer
        self.fuse = fuse
        self.p = p
        self.local = local
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
        self.unique_seqs = u
        # resident: every produced cloud already in HBM as SoA6 (the timed region starts with the
        # inputs resident, like config B; a step pushes / loads them device-to-device); else host
        # buffers cross PCIe inside the timed region (the reference's host-side hand-over)
        self.resident = resident
        self.dev_frames = ([[(soa_tensor(f, dev), soa_tensor(g, dev)) for f, g in fr] for fr in self.seqs]
                           if resident else None)
        self.seqs = [self.seqs[q % u] for q in range(n_seq)]
        self.dseq = [q % u for q in range(n_seq)]
        self.ctxs = [imls_icp.ImlsContext(p, device=local) for _ in range(n_seq)]
        for c in self.ctxs:
            c.set_defer(fuse and n_seq / max(1, groups) >= 8)
        self.seed_state = self.ctxs[0].rng_state()
        self.ransac = p.solve_method == _abi.IMLS_SOLVE_RANSAC
        self.pos = [(q // u) % frames_per_seq for q in range(n_seq)]
        self.dir = [1] * n_seq
        # frame 0 only seeds the map (Q13); afterwards each registered frame's filtered scan joins
        # the FIFO at the start of that sequence's next step, as LaserOdometry.process orders it
        self.pending = [fr[self.pos[q]][0] for q, fr in enumerate(self.seqs)]
        self.pending_k = list(self.pos)
        self.last = [None] * n_seq
        self.t_prep = self.t_reg = 0.0        # host time in the per-frame uploads / in registration
        self.pipe = Pipeline(self.ctxs, self._prep, groups) if fuse else None

    def _prep(self, idx):
        """One frame of each sequence in idx, as LaserOdometry.process orders it: the previous
        filtered scan joins the device map FIFO (only it crosses PCIe), the flat cloud is loaded;
        count-less (no host wait for the NaN-filtered counts)."""
        t0 = time.perf_counter()
        for q in idx:
            c = self.ctxs[q]
            k = self._advance(q)
            if self.ransac:
                c.set_rng_state(self.seed_state)
            if self.resident:
                filt, _ = self.dev_frames[self.dseq[q]][self.pending_k[q]]
                _, flat = self.dev_frames[self.dseq[q]][k]
                c.map_push_device(filt.data_ptr(), filt.shape[1], count=False)
                c.set_source_device(flat.data_ptr(), flat.shape[1], count=False)
            else:
                c.map_push(self.pending[q], count=False)
                c.set_source(self.seqs[q][k][1], count=False)
            self.last[q] = (self.pending_k[q], k)
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
        out = []
        for q, c in enumerate(self.ctxs):
            pose, it, st = c.register_frame_result()
            out.append((q, pose, it, st, c.last_trace))
        self.t_reg += time.perf_counter() - t1
        return out

    def single(self, q, frames):
        """Frame (map frame m, source frame k) of sequence q registered alone on a fresh context
        (set_target of the map scan — max_queue_size 1 — + set_source + register_frame)."""
        m, k = frames
        fr = self.seqs[q]
        with imls_icp.ImlsContext(self.p, device=self.local) as c:
            c.set_target(fr[m][0])
            c.set_source(fr[k][1])
            return c.register_frame()

    @property
    def queries(self):
        return int(np.mean([len(f[1]) for s in self.seqs for f in s]))

    @property
    def map_points(self):
        return int(np.mean([len(f[0]) for s in self.seqs for f in s]))

    def drain(self):
        return self.pipe.drain() if self.pipe else []

    def close(self):
        self.drain()
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
    k = {name: ctx.kernel_timing(i) for i, name in enumerate(("projection", "index", "solve", "k_knn_wave", "k_finish"))}
    lat = np.array(lat) * 1e3
    idx_ms = k["index"][0] / max(k["index"][1], 1)
    return dict(pairs=n_pairs, median_ms=float(np.median(lat)), p90_ms=float(np.percentile(lat, 90)),
                ms_per_iteration=float((np.median(lat) - idx_ms) / iters),
                kernel_avg_ms={n: v[0] / max(v[1], 1) for n, v in k.items()},
                launches={n: int(v[1]) for n, v in k.items()})


def stream_frame_probe(runner, n_frames: int = 40, warm: int = 3) -> dict:
    """One LaserOdometry.process frame alone — the deployment shape: the ROS node registers one frame
    at a time, inside the reference's timer "2. Matching and solving in flat points"
    (laser_odometry.cpp:482, 660; tic_toc.h:28-38).  Host inputs as the node holds them (48-B
    PointXYZINormal records): the previous filtered scan joins the device map FIFO (map_push), the
    flat cloud is set, the fused registration runs and its pose returns to the host — one context
    kept across frames, sequence 0 ping-ponged over its produced frames.  Wall time per frame
    (median / p90), the host hand-over part (pack + enqueue + filter waits), and the per-kind kernel
    split from a second pass with HIP events around every launch."""
    fr = runner.seqs[0]
    F = len(fr)

    def idx(j):
        if F == 1:
            return 0, 0
        r, ph = divmod(j, F - 1)
        k = ph if r % 2 == 0 else F - 1 - ph
        k2 = k + 1 if r % 2 == 0 else k - 1
        return k, k2                       # map frame, source frame (adjacent)
    with imls_icp.ImlsContext(runner.p, device=runner.local) as c:
        def frame(j):
            m, k = idx(j)
            t0 = time.perf_counter()
            # count-less loads: the host does not wait for the NaN-filtered counts (the build waits
            # for them at the first use, inside register_frame) — one host sync per frame
            c.map_push(fr[m][0], count=False)
            c.set_source(fr[k][1], count=False)
            t1 = time.perf_counter()
            r = c.register_frame()
            return t1 - t0, time.perf_counter() - t0, r
        for j in range(warm):
            frame(j)
        lat, hand = [], []
        for j in range(n_frames):
            h, t, _ = frame(warm + j)
            lat.append(t)
            hand.append(h)
        c.enable_timing(True)
        c.reset_timing()
        nt = max(n_frames // 2, 1)
        for j in range(nt):
            frame(warm + n_frames + j)
        c.enable_timing(False)
        kinds = ("projection", "index", "solve", "k_knn_wave", "k_finish")
        split = {}
        for i, name in enumerate(kinds):
            ms, n = c.kernel_timing(i)
            split[name] = {"ms_per_frame": ms / nt, "launches_per_frame": n / nt}
    lat, hand = np.array(lat) * 1e3, np.array(hand) * 1e3
    # the product's own per-frame call: LaserOdometry.process (pipelined for max_queue_size 1 — the
    # frame registers on the context holding the previous scan's index while its own filtered scan is
    # pushed to the other), one frame at a time, wall clock of each call
    plat = []
    with imls_icp.LaserOdometry(runner.p, device=runner.local) as lo:
        for j in range(warm + n_frames + 1):
            m, k = idx(j)
            t0 = time.perf_counter()
            lo.process(fr[k][0], fr[k][1])
            if j > warm:
                plat.append(time.perf_counter() - t0)
        pipelined = lo.pipelined
    plat = np.array(plat) * 1e3
    return dict(frames=n_frames, median_ms=float(np.median(plat)), p90_ms=float(np.percentile(plat, 90)),
                pipelined=pipelined,
                rule="LaserOdometry.process(filtered scan, flat cloud) per frame, host inputs, one frame at a time, "
                     "wall clock: set_source + the fused registration (20 ICP iterations) against the previous scan's "
                     "index + this frame's map_push (accumulateTargetCloud) — on the other context, overlapping the "
                     "registration, when pipelined",
                unpipelined={"median_ms": float(np.median(lat)), "p90_ms": float(np.percentile(lat, 90)),
                             "host_handover_median_ms": float(np.median(hand)),
                             "rule": "one context: map_push(previous filtered scan) + set_source(flat cloud), both "
                                     "count-less, + register_frame"},
                host_handover_median_ms=float(np.median(hand)), kernel_split=split,
                queries=int(np.mean([len(f[1]) for f in fr])), map_points=int(np.mean([len(f[0]) for f in fr])))


def same_result(a, b) -> bool:
    """Bit equality of two tagged results (pose, iterations, status, every trace record)."""
    if not (np.array_equal(np.asarray(a[1]), np.asarray(b[1])) and a[2] == b[2] and a[3] == b[3]):
        return False
    ta, tb = a[4], b[4]
    return len(ta) == len(tb) and all(
        list(x.delta) == list(y.delta) and list(x.pose) == list(y.pose) and list(x.reject) == list(y.reject)
        and x.n_valid == y.n_valid and x.n_kept == y.n_kept for x, y in zip(ta, tb))


def union_ms(iv) -> float:
    """Length of the union of [start, end) intervals (ms)."""
    if len(iv) == 0:
        return 0.0
    iv = sorted(map(tuple, iv))
    busy, cs, ce = 0.0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return busy + ce - cs


def busy_pass(runner, steps: int, sync):
    """A second timed pass with light HIP-event timing (projection and solve launches only, every
    launch sequence's own stream; imls_enable_timing 2) on one device-wide clock: returns its wall
    time and the union of the projection / solve intervals — the time the GPU spent with at least
    one projection (or solve) kernel running, the denominator of roofline.frac."""
    ctxs = runner.ctxs
    runner.drain()
    sync()
    for c in ctxs:
        c.reset_timing()
        c.enable_timing(2)
    ctxs[0].timing_origin()
    t0 = time.perf_counter()
    for _ in range(steps):
        runner.step()
    runner.drain()
    sync()
    wall = time.perf_counter() - t0
    proj = np.concatenate([c.timing_intervals(0) for c in ctxs] + [np.zeros((0, 2))])
    solve = np.concatenate([c.timing_intervals(2) for c in ctxs] + [np.zeros((0, 2))])
    for c in ctxs:
        c.enable_timing(0)
    return dict(wall_ms=wall * 1e3, projection_busy_ms=union_ms(proj), solve_busy_ms=union_ms(solve),
                any_busy_ms=union_ms(np.concatenate([proj, solve])), projection_launches=int(len(proj)))


def stats_pass(runner):
    """One step with the neighbour counters on for every context (then off): each frame's
    algorithmic bytes (frame_bytes).  Returns {context: bytes}."""
    runner.drain()
    for c in runner.ctxs:
        c.enable_stats(True)
    res = runner.step() + runner.drain()
    out = {}
    for k, pose, it, st, tr in res:
        c = runner.ctxs[k]
        out[k] = frame_bytes(c.index_stats(), c.index_stats()["queries"], tr)
    for c in runner.ctxs:
        c.enable_stats(False)
    return out


def host_leg(pairs, p, dev, local, args, world, fuse):
    """Config B's host hand-over leg beside the headline (SURVEY §8(d) t_pair): the same pairs, each
    context's map a device FIFO of the pair's 10 scans with its incremental index, and every
    registration taking the NEWEST scan and the source from host memory (pack + PCIe inside the
    timed region).  The headline `value` stays the resident-input rate (inputs in HBM when the timed
    region starts); this is the PCIe-inclusive rate of the same workload, every timed result checked
    bit for bit against its pair registered alone on a fresh context holding the same FIFO content."""
    import torch
    hr = PairRunner(pairs, p, dev, local, fuse=fuse, groups=args.groups, host=True)
    loads = {}
    orig_load = hr._load

    def tagging_load(c, k, count):
        orig_load(c, k, count)
        loads.setdefault(k, []).append(hr.rot[k])
    for _ in range(args.warmup):
        hr.step()
    hr.drain()
    torch.cuda.synchronize()
    hr._load = tagging_load
    elapsed, per_step, res = timed_steps(hr.step, args.steps, world, dev, torch.cuda.synchronize)
    res += hr.drain()
    hr._load = orig_load
    seen, cache, mism = {}, {}, 0
    for r in res:
        k = r[0]
        j = seen.get(k, 0)
        seen[k] = j + 1
        if args.no_verify:
            continue
        key = (k, loads[k][j])
        if key not in cache:
            cache[key] = hr.single_fresh(*key)
        mism += 0 if same_result(r, cache[key]) else 1
    probe = latency_probe(lambda: hr.single([0]), hr.ctxs[0], max(1, min(args.latency_pairs, 20)), args.iters)
    hr.close()
    if mism:
        raise SystemExit(f"bench: host leg: {mism} timed result(s) differ from the single-frame path")
    n = args.steps * len(pairs)
    return {"value": world * n / elapsed, "unit": "scan-pairs/s",
            "inputs": "host memory (PCIe inside the timed region)",
            "ms_per_step": elapsed / args.steps * 1e3,
            "index_ms_per_registration": probe["kernel_avg_ms"].get("index"),
            "single_pair_median_ms": probe["median_ms"],
            "verify": {"timed_results": len(res), "checked": 0 if args.no_verify else len(res), "mismatches": mism,
                       "rule": "every timed result vs its pair registered alone on a fresh context holding the same "
                               "FIFO content (single-frame kernels), bit for bit"}}


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
                    help="inputs handed over in host memory, PCIe inside the timed region (stream: the new map "
                         "scan + flat cloud per frame; A/B: each pair's map is a device FIFO of its scans, the newest "
                         "scan + the source cross PCIe per registration, SURVEY §8(d) t_pair)")
    ap.add_argument("--resident-inputs", action="store_true",
                    help="B: inputs already resident in HBM" + (" (the default for B is the host hand-over: "
                         "--host-inputs)" if B_HOST_DEFAULT else " (already the default for B; the host "
                         "hand-over is --host-inputs, and the headline line carries it as host_handover)"))
    ap.add_argument("--latency-pairs", type=int, default=50, help="single-pair latency / roofline probe size")
    ap.add_argument("--busy-steps", type=int, default=5, help="steps of the HIP-event busy-time pass (0 = skip)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU-baseline leg")
    ap.add_argument("--no-host-leg", action="store_true", help="config B: skip the host hand-over leg")
    ap.add_argument("--no-verify", action="store_true", help="skip the bit-equality check of the timed results")
    ap.add_argument("--backend", choices=["auto", "nccl", "gloo"], default="auto")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    ap.add_argument("--workload", choices=["B", "stream", "A", "E"], default="B")
    ap.add_argument("--solver", choices=["LS", "RANSAC_DRPM"], default="LS")
    args = ap.parse_args()
    # config B's headline includes SURVEY §8(d)'s t_pair hand-over: the newest map scan and the source
    # cross PCIe per registration (the map a device FIFO with its incremental index)
    if args.workload == "B" and B_HOST_DEFAULT and not args.resident_inputs:
        args.host_inputs = True

    import torch
    import torch.distributed as dist
    world, rank, local, dev = dist_setup(args.backend)
    # measured (profiles/r02_final): B pairs fill the GPU alone and run best as 4 one-pair launch
    # sequences in flight (1x4 264.7, 2x2 252.4, 2x4 255.7, 4x2 231, 8x2 205 pairs/s: more per launch
    # only adds cache pressure); the small A / stream frames run best as ONE large batch per step
    # (two half batches in flight share hardware queues, so a filter of one half can wait behind
    # the other half's launch sequence)
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
    stream = args.workload == "stream"
    if stream:
        runner = StreamRunner(P, p, local, rank, fuse=fuse, unique=args.unique_seqs, dev=dev,
                              resident=not args.host_inputs, groups=args.groups)
        queries, map_points = runner.queries, runner.map_points
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
        if args.host_inputs and args.workload == "E":
            raise SystemExit("--host-inputs: config E's tensor inputs stay device-resident (not supported)")
        runner = PairRunner(pairs, p, dev, local, fuse=fuse, groups=args.groups, tensors=args.workload == "E",
                            host=args.host_inputs)
        queries, map_points = pairs[0].source.size, pairs[0].target.size
    probe_ctx = runner.ctxs[0]
    log(f"[rank {rank}] workload {args.workload} set up in {time.time() - t0:.1f}s: {P} in flight, "
        f"~{queries} queries vs ~{map_points}-pt maps, solver {args.solver}")
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        runner.step()
    runner.drain()

    if hasattr(runner, "t_prep"):
        runner.t_prep = runner.t_reg = 0.0
    if getattr(runner, "pipe", None):
        runner.pipe.t_wait = runner.pipe.t_launch = runner.pipe.t_prep = runner.pipe.t_tag = 0.0
    # the stream's frame of each result: the (map, source) frames loaded when its batch was prepared
    # (host-input pairs: the FIFO rotation of each result's load)
    frames_at_launch = {}
    tag_loads = stream or (args.host_inputs and not stream)
    if tag_loads and stream:
        orig_prep = runner._prep

        def tagging_prep(idx):
            orig_prep(idx)
            for q in idx:
                frames_at_launch.setdefault(q, []).append(runner.last[q])
        runner._prep = tagging_prep
        if runner.pipe:
            runner.pipe.prep = tagging_prep
    elif tag_loads:
        # host-input pairs: every load (pipelined or single-frame) records its FIFO rotation
        orig_load = runner._load

        def tagging_load(c, k, count):
            orig_load(c, k, count)
            frames_at_launch.setdefault(k, []).append(runner.rot[k])
        runner._load = tagging_load
    elapsed, per_step, res = timed_steps(runner.step, args.steps, world, dev, torch.cuda.synchronize)
    res += runner.drain()                 # the batches still in flight (already finished: synchronized)
    if tag_loads and stream:
        runner._prep = orig_prep
        if runner.pipe:
            runner.pipe.prep = orig_prep
    elif tag_loads:
        runner._load = orig_load
    if hasattr(runner, "t_prep"):
        log(f"[rank {rank}] host time per step: uploads (+ filters) {runner.t_prep / args.steps * 1e3:.2f} ms, "
            f"rest (builds, launches, waits) {runner.t_reg / args.steps * 1e3:.2f} ms")
    if getattr(runner, "pipe", None):
        log(f"[rank {rank}] pipeline host time per step: result waits {runner.pipe.t_wait / args.steps * 1e3:.2f} ms, "
            f"register_frames_async (builds + launches) {runner.pipe.t_launch / args.steps * 1e3:.2f} ms, "
            f"input loads {runner.pipe.t_prep / args.steps * 1e3:.2f} ms, result tagging {runner.pipe.t_tag / args.steps * 1e3:.2f} ms, "
            f"rest {(elapsed - runner.pipe.t_wait - runner.pipe.t_launch - runner.pipe.t_prep - runner.pipe.t_tag) / args.steps * 1e3:.2f} ms")
    n_pairs = args.steps * P
    value = world * n_pairs / elapsed

    # ---- outside the timed region -------------------------------------------------------------
    # (1) every timed result bit-equal to its pair registered alone (single-frame kernels)
    verify = None
    worst = 0
    if stream:
        # each context's results in launch order ↔ the frames loaded for those launches (the warm-up
        # launches were drained before the timed region: the first result per context is the first
        # timed launch); EVERY timed result is compared with its frame registered alone on a fresh
        # context — the sequences beyond `unique` replay the produced ones, so the distinct
        # (produced sequence, map frame, source frame) registrations are cached
        seen, cache = {}, {}
        checked = mism = 0
        seqs_checked = set()
        for k, pose, it, st, tr in res:
            j = seen.get(k, 0)
            seen[k] = j + 1
            if args.no_verify:
                continue
            key = (runner.dseq[k],) + tuple(frames_at_launch[k][j])
            if key not in cache:
                cache[key] = runner.single(k, frames_at_launch[k][j])
            ref = cache[key]
            ok = same_result((k, pose, it, st, tr), (k, ref["pose"], ref["iters"], ref["status"], ref["trace"]))
            checked += 1
            seqs_checked.add(k)
            mism += 0 if ok else 1
        verify = dict(timed_results=len(res), checked=checked, mismatches=mism, sequences=len(seqs_checked),
                      distinct_frames=len(cache),
                      rule="every timed result of every sequence vs a fresh context registering that frame alone "
                           "(single-frame kernels), bit for bit")
    elif args.host_inputs:
        # each result vs its pair registered alone on a fresh context whose map is the FIFO's content
        # at that load (same scans, same rotation), single-frame kernels, bit for bit
        seen, cache, mism = {}, {}, 0
        for r in res:
            k = r[0]
            j = seen.get(k, 0)
            seen[k] = j + 1
            key = (k, frames_at_launch[k][j])
            if args.no_verify:
                continue
            if key not in cache:
                cache[key] = runner.single_fresh(*key)
            mism += 0 if same_result(r, cache[key]) else 1
        ref = {k: runner.single_fresh(k, 0) for k in range(len(runner.pairs))}
        verify = dict(timed_results=len(res), checked=0 if args.no_verify else len(res), mismatches=mism,
                      distinct_maps=len(cache),
                      rule="every timed result vs its pair registered alone on a fresh context holding the same FIFO "
                           "content (single-frame kernels), bit for bit")
        errs = [np.linalg.norm(ref[k][1][:3, 3] - q.true_pose[:3, 3]) for k, q in enumerate(runner.pairs)]
        worst = int(np.argmax(errs))
        log(f"[rank {rank}] max pose error vs synthetic truth {max(errs) * 100:.2f} cm (pair {worst})")
    else:
        ref = {r[0]: r for r in runner.single()}
        mism = 0 if args.no_verify else sum(0 if same_result(r, ref[r[0]]) else 1 for r in res)
        verify = dict(timed_results=len(res), checked=0 if args.no_verify else len(res), mismatches=mism,
                      rule="every timed result vs its pair registered alone (single-frame kernels), bit for bit")
        errs = [np.linalg.norm(ref[k][1][:3, 3] - q.true_pose[:3, 3]) for k, q in enumerate(runner.pairs)]
        worst = int(np.argmax(errs))      # the parity leg checks this pair against the oracle
        log(f"[rank {rank}] max pose error vs synthetic truth {max(errs) * 100:.2f} cm (pair {worst})")
    log(f"[rank {rank}] timed results checked {verify['checked']}, mismatches {verify['mismatches']}")
    if verify["mismatches"]:
        raise SystemExit(f"bench: {verify['mismatches']} timed result(s) differ from the single-frame path")

    # (2) per-sequence trajectories (one all-gather of tagged relative poses)
    if stream:
        tags = [(k, j, r[1]) for j, r in enumerate(res) for k in [r[0]]]
    else:
        tags = [(0, r[0], r[1]) for r in res[-P:]] if len(res) >= P else []   # the last step: pairs 0..P-1 in order
    allp, trajs = exchange_poses(tags, world, rank)

    # (3) single-pair latency + serialised per-launch kernel durations, algorithmic bytes, busy time
    probe = single_frame = None
    if not stream:
        probe = latency_probe(lambda: runner.single([0]), probe_ctx, args.latency_pairs, args.iters)
    elif args.latency_pairs > 0:
        single_frame = stream_frame_probe(runner, args.latency_pairs)
        log(f"[rank {rank}] single frame: median {single_frame['median_ms']:.3f} ms, p90 {single_frame['p90_ms']:.3f} ms, "
            f"host hand-over {single_frame['host_handover_median_ms']:.3f} ms")
    fb = stats_pass(runner)
    bytes_per_step = float(sum(fb.values())) if not stream else float(np.mean(list(fb.values()))) * P
    busy = busy_pass(runner, args.busy_steps, torch.cuda.synchronize) if args.busy_steps > 0 else None
    trav = probe_ctx.traversal_stats()
    want_leg = args.workload == "B" and not args.host_inputs and not args.no_host_leg
    # every rank's roofline inputs, gathered before ranks ≠ 0 leave (per-GPU fraction)
    per_rank = gather_rank_roofline(
        rank_roofline(bytes_per_step, busy, args.busy_steps, per_step, probe,
                      (fb[0] / max(args.iters, 1)) if not stream and fb else 0.0), world, dev)

    def run_leg():
        # after the resident runner is closed: with its contexts (and their streams) alive, the leg's
        # launch sequences shared hardware queues and measured ~45 % slower
        leg = host_leg(runner.pairs, p, dev, local, args, world, fuse)
        log(f"[rank {rank}] host hand-over leg: {leg['value']:.1f} pairs/s, index {leg['index_ms_per_registration']} ms "
            f"per registration, {leg['verify']['checked']} results checked")
        return leg

    if rank != 0:
        runner.close()
        if want_leg:
            run_leg()
        if _grouped():
            dist.destroy_process_group()
        return

    # PMC traffic per launch (rocprofv3 counters cannot be read from inside this process): the
    # pmc_traffic.json of a PMC pass of this same workload — tools/measure_round.sh runs its passes
    # first and hands this run the fresh file; the driver's plain run reads the round's committed one
    traffic = traffic_meta = None
    tj = pathlib.Path(args.traffic_json)
    stats0 = probe_ctx.index_stats()
    if tj.exists() and args.workload == "B":
        try:
            tdat = json.loads(tj.read_text())
            if tdat.get("queries") == stats0["queries"] and tdat.get("iters") == args.iters:
                traffic = tdat.get("bytes_per_launch")
                traffic_meta = {"source": str(tj), "fetch_factor": tdat.get("fetch_factor", 2.0),
                                "ratio_vs_algorithmic": tdat.get("ratio_vs_algorithmic"),
                                "calibrated": "calibration" in tdat, "scope": tdat.get("scope")}
        except (ValueError, OSError):
            traffic = None

    # (4) CPU baseline + parity of one pair (frame) vs the oracle
    cpu = parity = None
    if world == 1 and not args.no_cpu:
        log("[rank 0] CPU baseline (oracle) ...")
        if stream:
            m, k = frames_at_launch[0][0]
            fr = runner.seqs[0]
            src, tgt, ten, truth = synth.soa(fr[k][1]), synth.soa(fr[m][0]), None, None
            got = runner.single(0, (m, k))
            label = f"stream (sequence 0, frame {k} vs frame {m}'s filtered scan)"
        else:
            q0 = runner.pairs[worst]
            src, tgt, truth = synth.soa(q0.source), synth.soa(q0.target), q0.true_pose
            ten = np.ascontiguousarray(q0.meta["tensors"].T) if args.workload == "E" else None
            k0, pose0, it0, st0, tr0 = runner.single_fresh(worst, 0) if args.host_inputs else runner.single([worst])[0]
            got = dict(pose=pose0, iters=it0, status=st0, trace=tr0)
            label = f"config {args.workload}, pair {worst} (the step's largest error vs the synthetic truth)"
        cpu, want = cpu_baseline(src, tgt, p, label, tensors=ten, faithful=True)
        parity = parity_vs_oracle(got, want, truth)
        parity["pair"] = label
        log(f"[rank 0] CPU baseline {cpu['value']:.4f} pairs/s (faithful {cpu['faithful']['value']:.4f}, "
            f"{cpu['host_share']['cores']} cores {cpu['host_share']['value']:.3f}); parity {parity}")
        if stream:
            cpu["unit"] = "frames/s"

    # (5) roofline of the projection step (HBM-bound by the survey's accounting)
    roof = None
    ms_step = elapsed / args.steps * 1e3
    agg = bytes_per_step / (ms_step / 1e3) / 1e9
    roof = {
        "bound": "hbm",
        "kernel": "projection step = k_knn_wave (packet traversal) + k_finish (exact re-rank, gates, IMLS, pass-1 "
                  "normal equations) [+ k_project_lane fallback]: algorithmic bytes of every projection launch of a "
                  "step / the time at least one projection kernel ran (union of HIP-event intervals of all launch "
                  "sequences on one device clock, busy pass)",
        "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "traffic": traffic,
        "traffic_meta": traffic_meta,
        "algorithmic_bytes_per_step": bytes_per_step,
        "aggregate_GBps": agg,
        "aggregate_frac": agg / HBM_PEAK_GBS,
    }
    if busy:
        bsteps = args.busy_steps
        busy_step = busy["projection_busy_ms"] / bsteps
        roof.update(achieved=bytes_per_step / (busy_step / 1e3) / 1e9 if busy_step > 0 else 0.0,
                    busy_projection_ms_per_step=busy_step,
                    busy_solve_ms_per_step=busy["solve_busy_ms"] / bsteps,
                    busy_any_ms_per_step=busy["any_busy_ms"] / bsteps,
                    busy_pass_ms_per_step=busy["wall_ms"] / bsteps,
                    busy_pass_launches_per_step=busy["projection_launches"] / bsteps)
        roof["frac"] = roof["achieved"] / HBM_PEAK_GBS
    else:
        roof.update(achieved=agg, frac=agg / HBM_PEAK_GBS)
    roof["per_rank"] = per_rank
    if world > 1:
        fr = [d["frac"] for d in per_rank if d["frac"] is not None]
        roof["per_rank_frac_min_max"] = [min(fr), max(fr)] if fr else None
    if probe:
        kd = probe["kernel_avg_ms"]
        dom_ms = kd["k_knn_wave"] + kd["k_finish"]
        b_launch = fb[0] / max(args.iters, 1)
        roof["serialised_single_pair"] = {
            "avg_launch_ms": dom_ms, "kernel_avg_ms": kd, "algorithmic_bytes_per_launch": b_launch,
            "achieved": b_launch / (dom_ms / 1e3) / 1e9 if dom_ms > 0 else 0.0,
            "frac": b_launch / (dom_ms / 1e3) / 1e9 / HBM_PEAK_GBS if dom_ms > 0 else 0.0}

    solver_txt = "LS (trimmed, t=0.02)" if args.solver == "LS" else "RANSAC -> DRPM (shipped config.json solver)"
    if args.workload == "B":
        metric = "IMLS-ICP scan-pairs/s (HDL-64 ~120k-pt scan vs 10-scan map, 20 ICP iterations)"
        workload = f"config B: HDL-64 scan vs 10-scan local map; a step = {P} independent scan pairs" + (f" as {args.groups} launch sequences in flight" if fuse else " in flight, one stream each")
        if args.host_inputs:
            workload += ("; host hand-over: each pair's map is a device FIFO of its 10 scans, the newest scan and the "
                         "source cross PCIe as 48-B PointXYZINormal records in every registration")
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
    first_traj = next(iter(trajs.values()), None)
    out = {
        "metric": metric,
        "value": value,
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "ms_per_step_median": float(np.median(per)),
        "ms_per_step_p90": float(np.percentile(per, 90)),
        "ms_per_pair": elapsed / n_pairs * 1e3,
        "pairs_in_flight": P,
        "ms_per_iteration": elapsed / n_pairs * 1e3 / args.iters,
        "single_pair": probe,
        "single_frame": single_frame,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded HDL-64 / VLP-16 ray-cast urban scene, planetary-lidar-odometry_amd/synth.py)",
        "config": {
            "workload": workload,
            "queries": int(stats0["queries"]) if not stream else queries,
            "map_points": int(stats0["points"]) if not stream else map_points,
            "icp_iterations": args.iters,
            "solver": solver_txt,
            "search_number": p.search_number,
            "inputs": "host memory (PCIe inside the timed region)" if args.host_inputs else "resident in HBM",
            "fused_launch": fuse,
            "launch_groups": args.groups if fuse else P,
            "parallelism": (f"independent pairs per GPU over {world} GPU(s), {dist.get_backend()} "
                            f"({'RCCL' if dist.get_backend() == 'nccl' else 'CPU'}) pose all-gather"
                            if _grouped() else "1 GPU, no process group"),
        },
        "verify": verify,
        "parity": parity,
        "roofline": roof,
        "busy_pass": busy,
        "traversal_per_launch": {k: v / args.iters for k, v in trav.items()},
        "sequences": len(trajs),
        "trajectory_end_seq0": first_traj[1][-1][:3, 3].tolist() if first_traj is not None and len(first_traj[1]) else None,
        "cpu_baseline": cpu,
        "host_handover": None,
    }
    runner.close()
    if want_leg:
        out["host_handover"] = run_leg()
    print(json.dumps(out), flush=True)
    if _grouped():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
