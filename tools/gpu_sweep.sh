#!/bin/bash
# parameter sweep of the traversal heuristics: tests once, then a kernel trace per setting
# SWEEP="VAR=v,VAR2=v2 VAR=v3 ..."   (each item: comma-separated environment assignments; "base" = defaults)
set -u
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; case $rc in 0|1) ;; *) echo stop; exit $rc;; esac
for cfg in ${SWEEP:-base}; do
  tag=$(echo "$cfg" | tr ',=' '_-')
  envs=""
  [ "$cfg" != base ] && envs=$(echo "$cfg" | tr ',' ' ')
  ( [ -n "$envs" ] && export $envs; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d gpurun_out/sweep/$tag -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --inflight 1 > gpurun_out/sweep/$tag.json 2> gpurun_out/sweep/$tag.err )
  rc=$?; echo "cfg $cfg rc=$rc"; case $rc in 0) ;; *) echo stop; exit $rc;; esac
done
