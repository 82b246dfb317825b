#!/bin/bash
# Batched RANSAC -> DRPM: the frames / RANSAC / stream GPU tests, then the shipped-solver bench legs
# (stream and config A) and a kernel-trace of the stream leg.
set -u
O=gpurun_out/${OUT:-rb}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_ransac.py tests/test_gpu_stream.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload stream --no-cpu --solver RANSAC_DRPM > $O/stream_ransac.json 2> $O/stream_ransac.err
rc=$?; echo "stream rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload A --no-cpu --solver RANSAC_DRPM > $O/A_ransac.json 2> $O/A_ransac.err
rc=$?; echo "A rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --workload stream --no-cpu --solver RANSAC_DRPM --steps 3 --warmup 1 > $O/kt.json 2> $O/kt.err
rc=$?; echo "kt rc=$rc"; exit $rc
