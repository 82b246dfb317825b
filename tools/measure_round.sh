#!/bin/bash
# Round measurement: GPU tests, the headline bench (with CPU baseline), rocprofv3 kernel-trace/stats
# of the same bench command, and the PMC traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs,
# --kernel-trace only — never combined with other traces).  Outputs under gpurun_out/measure/.
set -u
O=gpurun_out/measure
mkdir -p $O
export TMPDIR=/tmp
BENCH="bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-2}"
timeout -k 10 700 python -m pytest tests -m gpu -q > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; case $rc in 0|1) ;; *) echo stop; exit $rc;; esac
timeout -k 10 600 python3 $BENCH > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $BENCH --no-cpu \
    > $O/kt_bench.json 2> $O/kt_bench.err
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --kernel-trace --kernel-include-regex 'k_knn_wave|k_finish' --output-format csv \
      --pmc $c -d $O/pmc_$c -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --inflight 1 \
      > $O/pmc_$c.json 2> $O/pmc_$c.err
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo done
