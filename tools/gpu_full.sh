#!/bin/bash
# smoke → GPU tests → bench → rocprof kernel trace of a short bench.  Stops on crash/timeout.
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; case $rc in 0|1) ;; *) echo stop; exit $rc;; esac
timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; case $rc in 0|1) ;; *) echo stop; exit $rc;; esac
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; case $rc in 0) ;; *) echo stop; exit $rc;; esac
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
rc=$?; echo "rocprof rc=$rc"; exit $rc
