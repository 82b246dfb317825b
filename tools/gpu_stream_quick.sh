#!/bin/bash
# Stream / frames GPU tests, then the stream legs (LS, RANSAC) at their defaults.
set -u
O=gpurun_out/${OUT:-sq}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_batch.py tests/test_gpu_stream.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for solver in LS RANSAC_DRPM; do
  timeout -k 10 300 python3 bench.py --workload stream --no-cpu --solver $solver > $O/stream_$solver.json 2> $O/stream_$solver.err
  rc=$?; echo "stream $solver rc=$rc $(python3 -c "import json;print(json.loads(open('$O/stream_$solver.json').read().strip().splitlines()[-1])['value'])")"; grep "host time" $O/stream_$solver.err; [ $rc -eq 0 ] || exit $rc
done
