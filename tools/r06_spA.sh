#!/bin/bash
# Round 6: sparse-lane threshold 20 (product) vs 32 (var_sp32) on config A (LS and RANSAC) and E
set -u
O=gpurun_out/${OUT:-r06_spA}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in product sp32; do
    lib=""; [ $v = product ] || lib=planetary-lidar-odometry_amd/csrc/var_$v/libimls_gpu.so
    for w in "A LS" "A RANSAC_DRPM" "E LS"; do
      set -- $w
      env ${lib:+IMLS_LIB_PATH=$lib} timeout -k 10 300 python3 bench.py --no-cpu --workload $1 --solver $2 > $O/${v}_$1_$2_$r.json 2> $O/${v}_$1_$2_$r.err || { tail -3 $O/${v}_$1_$2_$r.err; exit 1; }
      python3 -c "
import json;d=json.loads(open('$O/${v}_$1_$2_$r.json').read().strip().splitlines()[-1]);print('$v $1 $2 $r', round(d['value'],1))"
    done
  done
done
echo done
