#!/bin/bash
set -u
O=gpurun_out/${OUT:-r02g}
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; grep "host time" $O/$name.err; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
#run s64 300 --workload stream --no-cpu
#run s128 300 --workload stream --no-cpu --inflight 128
#run s256 300 --workload stream --no-cpu --inflight 256
run B8 300 --no-cpu --latency-pairs 3
run B16 300 --no-cpu --latency-pairs 3 --inflight 16
run B4 300 --no-cpu --latency-pairs 3 --inflight 4
