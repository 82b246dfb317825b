#!/bin/bash
# XCD-grouped batched projection: frames tests, then the stream legs with IMLS_XCD=0 / auto.
set -u
O=gpurun_out/${OUT:-xcd}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for x in 0 -1; do
  for solver in LS RANSAC_DRPM; do
    IMLS_XCD=$x timeout -k 10 300 python3 bench.py --workload stream --no-cpu --solver $solver > $O/s_${x}_$solver.json 2> $O/s_${x}_$solver.err
    rc=$?; echo "xcd $x $solver rc=$rc $(python3 -c "import json;print(json.loads(open('$O/s_${x}_$solver.json').read().strip().splitlines()[-1])['value'])")"; [ $rc -eq 0 ] || exit $rc
  done
  IMLS_XCD=$x timeout -k 10 300 python3 bench.py --workload A --no-cpu > $O/a_$x.json 2> $O/a_$x.err
  rc=$?; echo "xcd $x A rc=$rc $(python3 -c "import json;print(json.loads(open('$O/a_$x.json').read().strip().splitlines()[-1])['value'])")"; [ $rc -eq 0 ] || exit $rc
done
