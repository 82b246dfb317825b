"""GPU: parity on the path the headline number times.  bench.py's config B registers 10-scan
HDL-64 pairs (~126k queries vs ~1.26M map points) through PairRunner's Pipeline: count-less device
loads, deferred builds, several launch sequences in flight, the batched `_b` kernels.  Here the
same runner registers two such pairs (one per launch sequence, and both in one) and every result
must be
  (a) bit-equal — pose, iterations, status, every trace record — to the pair registered alone
      through imls_register_frame (the single-frame kernels), and
  (b) equal to the CPU oracle (oracle/imls_oracle.cpp, laser_odometry.cpp:478-660 /
      imls_icp.cpp:496-745 / solver.cpp:74-166): iterations and status equal, per-iteration valid
      counts and reject counters exact, pose within 1e-6."""
import os
import pathlib
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import oracle_ctypes as oc  # noqa: E402
from planetary_lidar_odometry_amd import synth  # noqa: E402

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-6


@pytest.fixture(scope="module")
def bench_mod():
    import bench
    return bench


@pytest.fixture(scope="module")
def pairs():
    # bench.py's own pair set for rank 0 (synth.make_pairs(P, "hdl64", 10, scene 0, traj 2000, noise 1000))
    return synth.make_pairs(2, "hdl64", map_scans=10, scene_seed=0, traj_seed=2000, noise_seed=1000)


@pytest.fixture(scope="module")
def oracle_results(pairs, bench_mod):
    p = bench_mod.solver_params("LS", 20)
    oc.set_threads(min(16, len(os.sched_getaffinity(0))))
    try:
        return [oc.register_frame(synth.soa(q.source), synth.soa(q.target), p) for q in pairs]
    finally:
        oc.set_threads(1)


@pytest.mark.parametrize("groups", [2, 1], ids=["one_pair_per_sequence", "two_pairs_one_sequence"])
def test_bench_pipeline_matches_single_and_oracle(bench_mod, pairs, oracle_results, groups):
    import gpu_mem                                     # device copies on the product's HIP runtime
    p = bench_mod.solver_params("LS", 20)
    bufs = []

    def alloc(a):
        bufs.append(gpu_mem.DevSoa(a))
        return bufs[-1]
    runner = bench_mod.PairRunner(pairs, p, None, 0, fuse=True, groups=groups, alloc=alloc)
    try:
        res = []
        for _ in range(2):                              # two pipelined steps, as the timed region runs them
            res += runner.step()
        res += runner.drain()
        assert sorted(r[0] for r in res) == [0, 0, 1, 1]
        ref = {r[0]: r for r in runner.single()}
        for r in res:
            assert bench_mod.same_result(r, ref[r[0]]), r[0]
        for k, want in enumerate(oracle_results):
            _, pose, iters, status, trace = ref[k]
            assert iters == want["iters"] == 20 and status == want["status"]
            for tg, tw in zip(trace, want["trace"]):
                assert tg.n_valid == tw.n_valid
                assert list(tg.reject) == list(tw.reject)
            assert np.abs(pose - want["pose"]).max() < POSE_TOL, np.abs(pose - want["pose"]).max()
    finally:
        runner.close()
        for b in bufs:
            b.free()
