#!/bin/bash
# Broadcast-leaf lockstep insertion (IMLS_BCAST_LOCK 0/1/2): parity with it always on, the B bench
# for each setting and a one-pair-in-flight kernel trace per setting (per-iteration knn durations).
set -u
O=gpurun_out/${OUT:-bc}
mkdir -p $O
export TMPDIR=/tmp
IMLS_BCAST_LOCK=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for b in 0 1 2; do
  IMLS_BCAST_LOCK=$b timeout -k 10 300 python3 bench.py --no-cpu --latency-pairs 2 > $O/B_$b.json 2> $O/B_$b.err
  rc=$?; echo "B bcast=$b rc=$rc $(python3 -c "import json;print(json.loads(open('$O/B_$b.json').read().strip().splitlines()[-1])['value'])")"; [ $rc -eq 0 ] || exit $rc
done
for b in 0 2; do
  IMLS_BCAST_LOCK=$b timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt$b -o run -- python3 bench.py --inflight 1 --steps 4 --warmup 1 --latency-pairs 1 --no-cpu --no-fuse > $O/kt$b.json 2> $O/kt$b.err
  rc=$?; echo "kt $b rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
