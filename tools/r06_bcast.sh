#!/bin/bash
# Round 6: broadcast leaf scan by scalar loads (IMLS_BCAST_SCALAR) — projection tests, then a same-box
# A/B against the v_readlane scan (var_oldbc) and 8-point groups (var_bc8), and one SQ pass each.
set -u
O=gpurun_out/${OUT:-r06_bcast}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_bench_path.py \
    tests/test_gpu_frames.py tests/test_gpu_batch.py tests/test_gpu_qfuse.py tests/test_gpu_plane_icp.py tests/test_gpu_bucket.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
OUT=${OUT:-r06_bcast}/ab VARS="oldbc bc8" ROUNDS=2 bash tools/ab_libs.sh || exit 1
for v in product oldbc; do
  lib=""; [ $v = product ] || lib=planetary-lidar-odometry_amd/csrc/var_$v/libimls_gpu.so
  for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY"; do
    IMLS_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex 'k_knn_wave|k_finish' --output-format csv \
      --pmc $pass -d $O/sq_$v -o run -- python3 bench.py --no-host-leg --steps 2 --warmup 1 --no-cpu --inflight 1 --no-fuse --latency-pairs 2 > $O/sq_$v.out 2> $O/sq_$v.err
    echo "sq $v rc=$?"
  done
done
echo done
