#!/bin/bash
# One GPU-box session: smoke → GPU parity tests → short bench.  Stops at the first crash,
# abort or time limit (test FAILURES, exit 1, do not stop the bench).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"
case $rc in 0|1) ;; *) echo "stop"; exit $rc;; esac
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) echo "stop"; exit $rc;; esac
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 5 --warmup 1} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; exit $rc
