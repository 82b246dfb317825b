#!/bin/bash
# Round-3 GPU check (outputs under gpurun_out/${OUT:-check}/): the GPU test suite (or TESTS=...),
# smoke, and the headline bench (BENCH_ARGS).  Each step under its own time limit; stops at the
# first failure.
set -u
O=gpurun_out/${OUT:-check}
mkdir -p $O
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -25 $O/$name.out; tail -15 $O/$name.err; exit $rc; }
}
[ "${SKIP_TESTS:-0}" = 1 ] || step gpu_tests 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python3 bench.py ${BENCH_ARGS:-}
echo done
