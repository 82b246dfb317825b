#!/bin/bash
set -u
O=gpurun_out/${OUT:-r02e}
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; grep "host time" $O/$name.err; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
IMLS_VERLET=1 run s64_qverlet 300 --workload stream --no-cpu
IMLS_QWAVE=0 run s64_packets 300 --workload stream --no-cpu
IMLS_QWAVE=0 run s128_packets 300 --workload stream --no-cpu --inflight 128
IMLS_VERLET=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_qv -o run -- python3 bench.py --workload stream --no-cpu --steps 5 --warmup 1 > $O/kt_qv.json 2> $O/kt_qv.err
echo "kt_qv rc=$?"
IMLS_QWAVE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_pk -o run -- python3 bench.py --workload stream --no-cpu --steps 5 --warmup 1 > $O/kt_pk.json 2> $O/kt_pk.err
echo "kt_pk rc=$?"
