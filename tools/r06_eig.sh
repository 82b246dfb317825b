#!/bin/bash
# Round 6: round-robin Jacobi for the DRPM eigendecomposition — RANSAC / stream / batched tests, the
# phase clocks (debug build) and the lone-frame probe + stream RANSAC leg (product build)
set -u
O=gpurun_out/${OUT:-r06_eig}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_ransac.py tests/test_gpu_stream.py tests/test_gpu_frames.py \
    tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/var_dbg/libimls_gpu.so timeout -k 10 300 python3 tools/ransac_probe.py 20 > $O/phase.out 2> $O/phase.err; echo "phase rc=$?"; cat $O/phase.out
timeout -k 10 300 python3 tools/ransac_probe.py 30 > $O/ransac_probe.out 2> $O/ransac_probe.err; echo "probe rc=$?"; cat $O/ransac_probe.out
timeout -k 10 400 python3 bench.py --workload stream --solver RANSAC_DRPM --no-cpu > $O/bench_stream_ransac.json 2> $O/bench_stream_ransac.err
echo "bench rc=$?"; python3 -c "
import json;d=json.loads(open('$O/bench_stream_ransac.json').read().strip().splitlines()[-1]);print(d['value'], d['single_frame']['median_ms'])"
echo done
