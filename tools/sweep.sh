#!/bin/bash
# Traversal knob sweep without the test suite: a kernel trace per setting of a short one-pair-in-
# flight bench.  SWEEP="VAR=v,VAR2=v2 VAR=v3 ..." (comma-separated env assignments; "base" = defaults)
set -u
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
for cfg in ${SWEEP:-base}; do
  tag=$(echo "$cfg" | tr ',=' '_-')
  envs=""
  [ "$cfg" != base ] && envs=$(echo "$cfg" | tr ',' ' ')
  ( [ -n "$envs" ] && export $envs; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
     -d gpurun_out/sweep/$tag -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --inflight 1 --latency-pairs 3 ${BENCH_EXTRA:-} > gpurun_out/sweep/$tag.json 2> gpurun_out/sweep/$tag.err )
  rc=$?; echo "cfg $cfg rc=$rc"; case $rc in 0) ;; *) echo stop; exit $rc;; esac
done
python3 tools/sweep_summary.py
