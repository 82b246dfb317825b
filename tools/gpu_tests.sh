#!/bin/bash
# GPU test suite only (optionally a subset: TESTS=...), verbose, per-test timeout.
set -u
O=gpurun_out/t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/gpu_tests.log; exit $rc
