#!/bin/bash
# Round 6: search radius (1 + skin)·r (underfull lists reusable) — projection / stream tests, then a
# same-box A/B against skin 0 (var_noskin) and the per-iteration split of one pair in flight.
set -u
O=gpurun_out/${OUT:-r06_skin}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_bench_path.py \
    tests/test_gpu_frames.py tests/test_gpu_batch.py tests/test_gpu_qfuse.py tests/test_gpu_plane_icp.py tests/test_gpu_bucket.py \
    tests/test_gpu_stream.py tests/test_gpu_tv.py tests/test_gpu_projected.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
OUT=${OUT:-r06_skin}/ab VARS="noskin" ROUNDS=2 bash tools/ab_libs.sh
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_single -o run -- python3 bench.py --no-cpu --no-host-leg --inflight 1 --no-fuse --steps 5 --warmup 1 --latency-pairs 3 > $O/kt_single.out 2> $O/kt_single.err
echo "kt rc=$?"
f=$(find $O/kt_single -name '*kernel_trace.csv' | head -1)
python3 tools/iter_profile.py $f > $O/per_iteration.txt; cat $O/per_iteration.txt
timeout -k 10 300 python3 tools/lo_probe.py 30 > $O/lo_probe.out 2>&1; echo "lo rc=$?"; cat $O/lo_probe.out
IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/var_noskin/libimls_gpu.so timeout -k 10 300 python3 tools/lo_probe.py 30 > $O/lo_probe_noskin.out 2>&1; echo "lo noskin rc=$?"; cat $O/lo_probe_noskin.out
echo done
