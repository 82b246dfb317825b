#!/bin/bash
# Same-box A/B of csrc/variant/libimls_gpu.so (IMLS_LIB_PATH) against the product library (outputs
# under gpurun_out/${OUT:-ab}/): optional projection parity tests on the variant (VARIANT_TESTS=1),
# then config B alternated ROUNDS times (pairs/s, busy-pass projection time, one-pair k_knn_wave /
# k_finish); then, unless SKIP_DUMP=1, the per-wave traversal records of the debug build.
set -u
O=gpurun_out/${OUT:-ab}
mkdir -p $O
export TMPDIR=/tmp
V=planetary-lidar-odometry_amd/csrc/variant/libimls_gpu.so
if [ "${PRODUCT_TESTS:-0}" = 1 ]; then
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_plane_icp.py \
      tests/test_gpu_tv.py tests/test_gpu_bench_path.py ${PRODUCT_TESTS_EXTRA:-} -m gpu -x -q --timeout 120 --timeout-method thread > $O/product_tests.log 2>&1
  rc=$?; echo "product tests rc=$rc"; tail -2 $O/product_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${VARIANT_TESTS:-0}" = 1 ]; then
  IMLS_LIB_PATH=$V timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_verlet.py tests/test_gpu_plane_icp.py \
      tests/test_gpu_tv.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "variant tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
show() { python3 -c "
import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];s=r.get('serialised_single_pair',{}).get('kernel_avg_ms',{})
print('$2', round(d['value'],1), 'busy_proj', round(r.get('busy_projection_ms_per_step',0),2), 'knn', round(s.get('k_knn_wave',0)*1e3,1), 'finish', round(s.get('k_finish',0)*1e3,1), 'single', round(d['single_pair']['median_ms'],2))"; }
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 python3 bench.py --no-cpu --steps 8 --latency-pairs 10 ${BENCH_ARGS:-} > $O/base_$r.json 2> $O/base_$r.err || { tail -5 $O/base_$r.err; exit 1; }
  show $O/base_$r.json "base $r"
  IMLS_LIB_PATH=$V timeout -k 10 300 python3 bench.py --no-cpu --steps 8 --latency-pairs 10 ${BENCH_ARGS:-} > $O/var_$r.json 2> $O/var_$r.err || { tail -5 $O/var_$r.err; exit 1; }
  show $O/var_$r.json "variant $r"
done
kn=0
for k in ${KNOBS:-}; do   # product library with NAME=VALUE knobs (several joined by '+')
  f=$O/knob_$(echo "$k" | tr '/' '_')_$((++kn))
  timeout -k 10 300 env ${k//+/ } python3 bench.py --no-cpu --steps 8 --latency-pairs 10 ${BENCH_ARGS:-} > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  show $f.json "$k"
done
if [ "${SKIP_DUMP:-0}" != 1 ]; then
  IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/debug/libimls_gpu.so timeout -k 10 300 python3 tools/wave_dump.py 1 2 3 6 > $O/wave_dump.txt 2> $O/wave_dump.err
  rc=$?; echo "wave_dump rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/wave_dump.err; exit $rc; }
fi
echo done
