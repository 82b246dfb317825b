#!/bin/bash
set -u
O=gpurun_out/front
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_front_end.py tests/test_gpu_wire.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 $O/tests.log; exit $rc
