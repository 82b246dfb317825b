#!/bin/bash
set -u
O=gpurun_out/statsexp
mkdir -p $O
export TMPDIR=/tmp
for v in 0 1; do
  if [ $v = 1 ]; then export IMLS_NO_STATS=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt$v -o run -- python3 bench.py --inflight 1 --steps 3 --warmup 1 --latency-pairs 2 --no-cpu --no-fuse > $O/kt$v.json 2> $O/kt$v.err
  echo "kt$v rc=$?"
done
