#!/bin/bash
# Round-2 batched-launch check: full GPU suite, then fused vs per-stream benches (B, stream, A).
set -u
O=gpurun_out/${OUT:-r02b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/gpu_tests.log | head -20; exit $rc; }
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
run B_fused8 300 --no-cpu --latency-pairs 5 ${B_EXTRA:-}
run B_fused16 300 --no-cpu --latency-pairs 5 --inflight 16
run B_streams4 300 --no-cpu --latency-pairs 5 --no-fuse --inflight 4
run stream_fused64 300 --workload stream --no-cpu
run stream_fused256 300 --workload stream --no-cpu --inflight 256
run stream_streams4 300 --workload stream --no-cpu --no-fuse --inflight 4
run A_fused16 300 --workload A --no-cpu --latency-pairs 5
