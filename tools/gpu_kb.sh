#!/bin/bash
# Traversal-kernel iteration: parity tests that exercise it, a one-pair-in-flight kernel trace of
# config B (per-ICP-iteration durations: tools/iter_profile.py) and the default B bench.
set -u
O=gpurun_out/${OUT:-kb}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_frames.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --inflight 1 --steps 4 --warmup 1 --latency-pairs 3 --no-cpu --no-fuse > $O/kt.json 2> $O/kt.err
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu --latency-pairs 5 > $O/B.json 2> $O/B.err
rc=$?; echo "B rc=$rc"; exit $rc
