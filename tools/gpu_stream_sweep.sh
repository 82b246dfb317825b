#!/bin/bash
# Stream leg: in-flight / launch-group sweep.  CFGS="inflight:groups ...", SOLVER=LS|RANSAC_DRPM.
set -u
O=gpurun_out/${OUT:-ss}
mkdir -p $O
export TMPDIR=/tmp
for cfg in ${CFGS:-128:2 192:3 256:4 256:2 128:4}; do
  i=${cfg%%:*}; g=${cfg##*:}
  timeout -k 10 300 python3 bench.py --workload ${WL:-stream} --no-cpu --solver ${SOLVER:-RANSAC_DRPM} --inflight $i --groups $g > $O/s_${i}_$g.json 2> $O/s_${i}_$g.err
  rc=$?; echo "inflight $i groups $g rc=$rc $(python3 -c "import json;print(json.loads(open('$O/s_${i}_$g.json').read().strip().splitlines()[-1])['value'])")"; [ $rc -eq 0 ] || exit $rc
done
