#!/bin/bash
# Traversal diagnostics (outputs under gpurun_out/${OUT:-diag}/): per-wave records of k_knn_wave at
# ICP iterations 0, 1, 2, 5 (debug build, tools/wave_dump.py) and a knob sweep of the config-B
# throughput bench (KNOBS: space-separated NAME=VALUE env settings, "base" = defaults).
set -u
O=gpurun_out/${OUT:-diag}
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_DUMP:-0}" != 1 ]; then
  IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/debug/libimls_gpu.so timeout -k 10 300 python3 tools/wave_dump.py 1 2 3 6 > $O/wave_dump.txt 2> $O/wave_dump.err
  rc=$?; echo "wave_dump rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/wave_dump.err; exit $rc; }
fi
for k in ${KNOBS:-base}; do
  if [ "$k" = base ]; then envs=""; else envs="$k"; fi
  env $envs timeout -k 10 240 python3 bench.py --no-cpu --no-verify --latency-pairs 3 --busy-steps 3 --steps 8 > $O/bench_$k.json 2> $O/bench_$k.err
  rc=$?; echo "bench $k rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_$k.err; exit $rc; }
done
echo done
