#!/bin/bash
# Round 6: LDS tile sort + merge passes for the ≤ 256k-key index sorts (IMLS_SMALL_SORT) — index /
# FIFO / parity / stream tests, then a same-box A/B (host hand-over leg: index ms per registration)
# against var_cubsort (hipcub's merge sort).
set -u
O=gpurun_out/${OUT:-r06_sort}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python3 -u -m pytest tests/test_gpu_fifo_index.py tests/test_gpu_parity.py tests/test_gpu_verlet.py \
    tests/test_gpu_bench_path.py tests/test_gpu_frames.py tests/test_gpu_batch.py tests/test_gpu_stream.py tests/test_gpu_host_inputs.py \
    tests/test_gpu_bucket.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in product cubsort; do
    lib=""; [ $v = product ] || lib=planetary-lidar-odometry_amd/csrc/var_$v/libimls_gpu.so
    env ${lib:+IMLS_LIB_PATH=$lib} timeout -k 10 300 python3 bench.py --no-cpu --steps 8 --latency-pairs 5 > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]);h=d['host_handover']
print('$v $r', round(d['value'],1), 'host', round(h['value'],1), 'idx_ms', round(h['index_ms_per_registration'],4), 'single', round(d['single_pair']['median_ms'],3), 'index', round(d['single_pair']['kernel_avg_ms']['index'],4))"
  done
done
timeout -k 10 300 python3 tools/lo_probe.py 30 > $O/lo_probe.out 2>&1; echo "lo rc=$?"; cat $O/lo_probe.out
IMLS_LIB_PATH=planetary-lidar-odometry_amd/csrc/var_cubsort/libimls_gpu.so timeout -k 10 300 python3 tools/lo_probe.py 30 > $O/lo_probe_cub.out 2>&1; echo "lo cub rc=$?"; cat $O/lo_probe_cub.out
echo done
