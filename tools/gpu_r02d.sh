#!/bin/bash
set -u
O=gpurun_out/${OUT:-r02d}
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; grep "host time" $O/$name.err; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
run stream64 300 --workload stream --no-cpu
IMLS_QWAVE=0 run stream64_packets 300 --workload stream --no-cpu
IMLS_BENCH_HW_QUEUES=16 run stream64_q16 300 --workload stream --no-cpu
run B8 300 --no-cpu --latency-pairs 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --workload stream --no-cpu --steps 5 --warmup 1 > $O/kt.json 2> $O/kt.err
echo "kt rc=$?"
