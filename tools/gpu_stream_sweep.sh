#!/bin/bash
# Stream RANSAC -> DRPM: launch-group / in-flight sweep.
set -u
O=gpurun_out/${OUT:-ss}
mkdir -p $O
export TMPDIR=/tmp
for cfg in "128 2" "192 3" "256 4" "256 2" "128 4"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --workload stream --no-cpu --solver RANSAC_DRPM --inflight $1 --groups $2 > $O/s_$1_$2.json 2> $O/s_$1_$2.err
  rc=$?; echo "inflight $1 groups $2 rc=$rc $(python3 -c "import json;print(json.loads(open('$O/s_$1_$2.json').read().strip().splitlines()[-1])['value'])")"; [ $rc -eq 0 ] || exit $rc
done
