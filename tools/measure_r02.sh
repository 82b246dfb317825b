#!/bin/bash
# Round-2 measurement set: headline bench (config B, CPU baselines), config C/D-like stream, the
# shipped solver (RANSAC -> DRPM) on config A and on the stream, and a rocprofv3 kernel trace of
# the one-pair-in-flight config B run.  Outputs under gpurun_out/${OUT:-m2}/.  Stops at the first
# failing step.
set -u
O=gpurun_out/${OUT:-m2}
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
[ "${SKIP_B:-0}" = 1 ] || run bench_B 400
run bench_stream 300 --workload stream --no-cpu
[ "${SKIP_RANSAC:-0}" = 1 ] || run bench_A_ransac 300 --workload A --solver RANSAC_DRPM
[ "${SKIP_RANSAC:-0}" = 1 ] || run bench_stream_ransac 300 --workload stream --solver RANSAC_DRPM --no-cpu
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run \
     -- python3 bench.py --inflight 1 --steps 5 --warmup 1 --latency-pairs 20 --no-cpu > $O/kt.json 2> $O/kt.err
  rc=$?; echo "kt rc=$rc"; exit $rc
fi
