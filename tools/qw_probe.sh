#!/bin/bash
# GPU tests, then the stream workload and config B with per-iteration kernel timings
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?"
for p in 4 8; do
  timeout -k 10 300 python bench.py --workload stream --steps 20 --warmup 3 --inflight $p --no-cpu > gpurun_out/s_p$p.json 2> gpurun_out/s_p$p.err || exit 1
done
export SWEEP='base'
bash tools/gpu_sweep.sh
