#!/bin/bash
# parameter sweep of the seed heuristics: tests once, then kernel-trace per setting
set -u
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; case $rc in 0|1) ;; *) echo stop; exit $rc;; esac
for cfg in ${SWEEP:-"1:0.25"}; do
  sh=${cfg%%:*}; rs=${cfg##*:}
  IMLS_SEED_HALF=$sh IMLS_RESEED=$rs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sweep/s${sh}_r${rs} -o run \
     -- python3 bench.py --steps 3 --warmup 1 --no-cpu --inflight 1 > gpurun_out/sweep/s${sh}_r${rs}.json 2> gpurun_out/sweep/s${sh}_r${rs}.err
  rc=$?; echo "cfg $cfg rc=$rc"; case $rc in 0) ;; *) echo stop; exit $rc;; esac
done
