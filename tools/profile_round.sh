#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench (no PMC counters here).
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
rc=$?; echo "rocprof rc=$rc"; exit $rc
