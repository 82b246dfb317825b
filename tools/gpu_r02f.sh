#!/bin/bash
set -u
O=gpurun_out/${OUT:-r02f}
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; grep "host time" $O/$name.err; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
run s64 300 --workload stream --no-cpu
run s128 300 --workload stream --no-cpu --inflight 128
run s256 300 --workload stream --no-cpu --inflight 256
run s64_host 300 --workload stream --no-cpu --host-inputs
run s4_streams 300 --workload stream --no-cpu --no-fuse --inflight 4
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_batch.py tests/test_gpu_stream.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?"; tail -2 $O/tests.log
