#!/bin/bash
# SQ instruction counters of k_knn_wave / k_finish per ICP iteration, one pair in flight (outputs
# under gpurun_out/${OUT:-sqi}/): one --pmc pass per VARIANTS entry ("base" or NAME=VALUE[+...]);
# tools/sq_iter.py prints VALU / SALU / LDS instructions and wave cycles per wave by iteration.
set -u
O=gpurun_out/${OUT:-sqi}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-verify --inflight 1 --no-fuse --latency-pairs 3 --busy-steps 0"
for v in ${VARIANTS:-base}; do
  envs=""; [ "$v" = base ] || envs="${v//+/ }"
  for e in $envs; do export "$e"; done
  timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex 'k_knn_wave|k_finish' --output-format csv \
      --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_WAIT_ANY \
      -d $O/$v -o run -- $B > $O/$v.json 2> $O/$v.err
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for e in $envs; do unset "${e%%=*}"; done
  python3 tools/sq_iter.py $O/$v > $O/$v.txt && cat $O/$v.txt
done
echo done
