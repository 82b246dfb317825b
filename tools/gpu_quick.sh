#!/bin/bash
# quick GPU iteration: GPU tests (optionally a subset) → bench (4 in flight) → bench (1 in flight)
# → kernel trace of the 1-in-flight bench.  Outputs under gpurun_out/q/.
set -u
O=gpurun_out/q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/gpu_tests.log; case $rc in 0|1|5) ;; *) echo stop; exit $rc;; esac
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_EXTRA:-} > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --inflight 1 ${BENCH_EXTRA:-} > $O/bench1.json 2> $O/bench1.err
rc=$?; echo "bench1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run \
   -- python3 bench.py --steps 3 --warmup 1 --no-cpu --inflight 1 ${BENCH_EXTRA:-} > $O/kt.json 2> $O/kt.err
rc=$?; echo "kt rc=$rc"; exit $rc
