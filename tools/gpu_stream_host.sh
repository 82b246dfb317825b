#!/bin/bash
# Stream legs (LS and RANSAC -> DRPM) with the pipeline's host-time split.
set -u
O=gpurun_out/${OUT:-sh}
mkdir -p $O
export TMPDIR=/tmp
for solver in LS RANSAC_DRPM; do
  timeout -k 10 300 python3 bench.py --workload stream --no-cpu --solver $solver > $O/stream_$solver.json 2> $O/stream_$solver.err
  rc=$?; echo "$solver rc=$rc"; grep "host time" $O/stream_$solver.err; [ $rc -eq 0 ] || exit $rc
done
