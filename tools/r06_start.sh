#!/bin/bash
# Round-6 first measurement: GPU suite (the retire-instead-of-free change), smoke, the driver's B
# line, and the SQ counters of the batched projection kernels at 4 pairs in flight (the "old" side).
set -u
O=gpurun_out/${OUT:-r06_start}
mkdir -p $O
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
step gpu_tests 800 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_B 600 python3 bench.py
OUT=${OUT:-r06_start}/sq4 bash tools/gpu_sq4.sh > $O/sq4.log 2>&1; echo "sq4 rc=$?"
echo done
