#!/bin/bash
# Same-box A/B of the lone-small-frame latency (tools/frame_probe.py: a ≤2000-query flat cloud vs its
# previous 118k-point scan, 20 ICP iterations, one frame at a time) between the product library and
# csrc/variant/libimls_gpu.so (make variant VARIANT_FLAGS=...), ROUNDS alternations; outputs under
# gpurun_out/${OUT:-lone_ab}/.
set -u
O=gpurun_out/${OUT:-lone_ab}
mkdir -p $O
V=planetary-lidar-odometry_amd/csrc/variant/libimls_gpu.so
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 200 python3 tools/frame_probe.py 30 > $O/base_$r.txt 2> $O/base_$r.err || { tail -5 $O/base_$r.err; exit 1; }
  echo "base $r: $(head -1 $O/base_$r.txt)"
  IMLS_LIB_PATH=$V timeout -k 10 200 python3 tools/frame_probe.py 30 > $O/var_$r.txt 2> $O/var_$r.err || { tail -5 $O/var_$r.err; exit 1; }
  echo "variant $r: $(head -1 $O/var_$r.txt)"
done
echo done
