#!/bin/bash
# Round 6: breadth-first top of the packet walk in the first ICP iterations (MODE 3, IMLS_BFS_ITERS)
# — projection tests, then a same-box A/B against var_nobfs, and the per-iteration split of one pair.
set -u
O=gpurun_out/${OUT:-r06_bfs}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_bench_path.py \
    tests/test_gpu_frames.py tests/test_gpu_batch.py tests/test_gpu_bucket.py tests/test_gpu_plane_icp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
OUT=${OUT:-r06_bfs}/ab VARS="nobfs" ROUNDS=2 bash tools/ab_libs.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_single -o run -- python3 bench.py --no-cpu --no-host-leg --inflight 1 --no-fuse --steps 5 --warmup 1 --latency-pairs 3 > $O/kt_single.out 2> $O/kt_single.err
echo "kt rc=$?"
f=$(find $O/kt_single -name '*kernel_trace.csv' | head -1)
python3 tools/iter_profile.py $f > $O/per_iteration.txt; cat $O/per_iteration.txt
echo done
