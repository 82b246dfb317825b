#!/bin/bash
# quick iteration: GPU tests → bench (no CPU leg) → one SQ counter pass on the wave kernel
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; case $rc in 0|1) ;; *) echo stop; exit $rc;; esac
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_EXTRA:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; case $rc in 0) ;; *) echo stop; exit $rc;; esac
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu --inflight 1 ${BENCH_EXTRA:-} > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?; echo "bench1 rc=$rc"; case $rc in 0) ;; *) echo stop; exit $rc;; esac
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run \
   -- python3 bench.py --steps 3 --warmup 1 --no-cpu --inflight 1 > gpurun_out/kt.json 2> gpurun_out/kt.err
rc=$?; echo "kt rc=$rc"; case $rc in 0) ;; *) echo stop; exit $rc;; esac
timeout -k 10 400 rocprofv3 --kernel-trace --kernel-include-regex 'k_knn_wave|k_finish' --output-format csv \
   --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
   -d gpurun_out/pmc/sq1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --inflight 1 > gpurun_out/pmc/sq1.json 2> gpurun_out/pmc/sq1.err
rc=$?; echo "pmc rc=$rc"; exit $rc
