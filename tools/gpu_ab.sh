#!/bin/bash
# A/B of csrc/variant/libimls_gpu.so (IMLS_LIB_PATH) against the product library: projection parity
# tests on the variant, then config B alternated twice (pairs/s, one-pair k_knn_wave / k_finish).
set -u
O=gpurun_out/${OUT:-ab}
mkdir -p $O
export TMPDIR=/tmp
V=planetary-lidar-odometry_amd/csrc/variant/libimls_gpu.so
IMLS_LIB_PATH=$V timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_plane_icp.py \
    tests/test_gpu_tv.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "variant tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
show() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);s=d['single_pair']['kernel_avg_ms'];print('$2', round(d['value'],1), 'knn', round(s['k_knn_wave']*1e3,1), 'finish', round(s['k_finish']*1e3,1))"; }
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu --steps 6 > $O/base_$r.json 2> $O/base_$r.err || exit $?
  show $O/base_$r.json "base $r"
  IMLS_LIB_PATH=$V timeout -k 10 300 python3 bench.py --no-cpu --steps 6 > $O/var_$r.json 2> $O/var_$r.err || exit $?
  show $O/var_$r.json "variant $r"
done
