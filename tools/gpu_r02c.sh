#!/bin/bash
# Stream / B fused-pipeline variants (no test suite).
set -u
O=gpurun_out/${OUT:-r02c}
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; grep "host time" $O/$name.err; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
run stream64 300 --workload stream --no-cpu
IMLS_QWAVE=0 run stream64_packets 300 --workload stream --no-cpu
run stream128 300 --workload stream --no-cpu --inflight 128
run B8 300 --no-cpu --latency-pairs 3
run B4 300 --no-cpu --latency-pairs 3 --inflight 4
